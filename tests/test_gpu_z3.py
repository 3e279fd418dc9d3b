"""The reference's own constraint objects through the GPU path (z3 stand-in: tests/fake_z3.py).

LASER's prune filter reads ``Constraints.is_possible`` on lists of laser.smt Bools whose
``.raw`` are z3 expressions (constraints.py:10-126).  Here such lists (built with the
stand-in z3) go through ``batch_is_possible``: lowered by mythril_amd.z3_lower, decided by
GPU witnesses that Z3Backend re-checks with the stand-in's evaluator before they are
trusted, refuted on the host, or handed to the fallback with the original expressions.
"""
import pytest

from mythril_amd import solver as SV
from mythril_amd.z3_backend import Z3Backend

from . import fake_z3 as z3

pytestmark = pytest.mark.gpu


class Wrapped:
    """laser.smt.Bool stand-in: the z3 expression is `.raw` (smt/bool.py)."""

    def __init__(self, raw):
        self.raw = raw


class RefConstraints(list):
    """constraints.py:10-126 surface the prune filter reads."""

    def __init__(self, items):
        super().__init__(items)
        self._is_possible = None
        self._default_timeout = 100
        self.witness = None


def test_reference_constraints_through_gpu_with_z3_recheck(mgp_ctx):
    be = Z3Backend(z3, recheck_refutations=1.0)  # every host refutation is audited by z3
    old = SV.set_backend(be)
    SV.SolverStatistics().reset()
    SV.unsat_cores().reset()
    SV.enable_gpu(True)
    try:
        size = z3.BitVec("9_calldatasize", 256)
        cd = z3.Array("9_calldata", z3.BitVecSort(256), z3.BitVecSort(8))
        sender = z3.BitVec("sender_9", 256)
        word = z3.Concat([z3.If(z3.BitVecVal(4 + i, 256) < size, cd[4 + i], z3.BitVecVal(0, 8)) for i in range(32)])
        actors = z3.Or(sender == 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,
                       sender == 0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE)
        items = [
            RefConstraints([Wrapped(actors), Wrapped(z3.UGT(word, 0)), Wrapped(z3.ULE(word, 20))]),
            RefConstraints([Wrapped(actors), z3.ULT(word, 5), z3.UGT(word, 9)]),          # UNSAT (host)
            RefConstraints([Wrapped(actors), Wrapped(word == 7)]),
        ]
        res = SV.batch_is_possible(items)
        st = SV.SolverStatistics()
        assert res == [True, False, True]
        assert st.gpu_sat == 2 and st.refuted == 1 and st.query_count == 0
        assert st.rechecks == 2 and st.recheck_rejects == 0 and be.rechecks == 2
        assert st.refute_rechecks == 1 and st.refute_disagreements == 0
        w = items[2].witness
        assert w["sender_9"] in (0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF, 0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE)
        # an unlowerable constraint keeps the whole query on z3 with the original objects
        fp = z3._mk(z3.FuncDeclRef(z3.Z3_OP_FP_ADD, "fp.add"), z3.BitVecSort(256), [sender, sender])
        more = RefConstraints([Wrapped(sender == 5), Wrapped(fp == sender)])
        assert SV.batch_is_possible([more]) == [True]  # unknown counts as possible (constraints.py:50)
        assert st.not_lowerable == 1 and st.query_count == 1
    finally:
        SV.set_backend(old)
