"""The z3 boundary (mythril_amd/z3_lower.py, z3_backend.py) against a stand-in z3 module.

z3 is absent here and on the GPU box, so tests/fake_z3.py reproduces z3py's expression
surface and evaluates it from the SMT-LIB semantics.  The walker's terms, flattened by
the native front end and evaluated by the oracle (oracle/bvsem.py), must give the same
truth value as the stand-in's own evaluation of the original expression, on random
assignments of every constant, function and array.  Parity with real z3 is unpinned.
"""
import random

import numpy as np
import pytest

from mythril_amd import dag as D
from mythril_amd import front as F
from mythril_amd import solver as SV
from mythril_amd import z3_lower as ZL
from oracle import bvsem as S

from . import fake_z3 as z3

M256 = (1 << 256) - 1


def _slot_values(B, s, lw, env, funcs):
    """Candidate row of state s that realises env / funcs: named variables by name, every
    UF application and base-array read by the interpretation at its argument."""
    out = []
    v0, v1 = int(B.var_off[s]), int(B.var_off[s + 1])
    names = B.var_names(s)
    i = 0
    while i < v1 - v0:
        full = int(B.var_full[v0 + i])
        k = max(1, (full + 255) // 256)
        kind = int(B.var_kind[v0 + i])
        if kind == 0:
            value = env.get(names[i], 0)
        else:
            e = lw.origin[int(B.var_tid[v0 + i])]
            if isinstance(e, tuple):
                name, arg = "array:" + e[0].decl().name(), z3.evaluate(e[1], env, funcs)
            else:
                name, arg = e.decl().name(), z3.evaluate(e.children()[0], env, funcs)
            value = funcs.get(name, {}).get(arg, 0)
        for j in range(k):
            out.append((value >> (256 * j)) & M256)
        i += k
    return out


def _check(exprs, envs, funcs_of):
    lw = ZL.lowering_for(exprs[0])
    terms = [lw.lower_constraints([e]) for e in exprs]
    B = F.Batch(terms)
    dags = [D.build_state(t) for t in terms]
    n_true = 0
    for env in envs:
        funcs = funcs_of(env)
        for s, (e, d) in enumerate(zip(exprs, dags)):
            want = bool(z3.evaluate(e, env, funcs))
            got = S.eval_root(d.nodes, d.consts, _slot_values(B, s, lw, env, funcs))
            assert got == want, (s, env)
            n_true += want
    B.close()
    return n_true


def test_operator_zoo_matches_stand_in_semantics():
    rng = random.Random(5)
    x, y, z = z3.BitVec("zx", 256), z3.BitVec("zy", 256), z3.BitVec("zz", 64)
    b = z3.Bool("zb")
    exprs = [
        z3.ULT(x + y * 3, x - y), z3.UGE(z3.UDiv(x, y), z3.URem(x, y)), (x / y) == (x % y),
        z3.SRem(x, y) < 5, (x & y | ~x) ^ y == z3.LShR(x, 3), (x << 7) >= (x >> 250),
        z3.Extract(63, 0, x) == z, z3.Concat(z, z3.Extract(191, 0, y)) == x, z3.ZeroExt(192, z) == y,
        z3.SignExt(192, z) == x, z3.RepeatBitVec(4, z) == x, z3.RotateLeft(z, 5) == z3.RotateRight(z, 59),
        z3.BVComp(x, y) == z3.BVRedOr(z), z3.BVRedAnd(z) == 1, z3.Not(z3.BVMulNoOverflow(x, y, False)),
        z3.Distinct(x, y, x + 1), z3.Implies(b, z3.ULT(x, 10)), z3.Xor(b, x == y), b == z3.ULT(y, x),
        z3.If(b, x, y) == x + 1, z3.And(z3.Or(b, x == 3), z3.Not(b)), -x == y, z3.UGT(x, 5) == b,
    ]

    def env_gen():
        for _ in range(60):
            pick = lambda w: rng.choice([0, 1, 2, 3, 5, (1 << w) - 1, 1 << (w - 1), rng.getrandbits(w),
                                         rng.getrandbits(8)])
            yield {"zx": pick(256), "zy": pick(256), "zz": pick(64), "zb": rng.getrandbits(1)}

    assert _check(exprs, list(env_gen()), lambda env: {}) > 0


def test_laser_shapes_calldata_keccak_storage():
    """calldata bytes (calldata.py:219-232: If(i < size, calldata[i], 0), signed <),
    a keccak256_512 pair with the manager's condition (keccak_function_manager.py:118-146),
    a Storage Store chain read back (array.py:16-63), a constant array (K)."""
    rng = random.Random(9)
    size = z3.BitVec("1_calldatasize", 256)
    cd = z3.Array("1_calldata", z3.BitVecSort(256), z3.BitVecSort(8))
    sender = z3.BitVec("sender_1", 256)
    word = z3.Concat([z3.If(z3.BitVecVal(4 + i, 256) < size, cd[4 + i], z3.BitVecVal(0, 8)) for i in range(32)])
    f = z3.Function("keccak256_512", z3.BitVecSort(512), z3.BitVecSort(256))
    inv = z3.Function("keccak256_512-1", z3.BitVecSort(256), z3.BitVecSort(512))
    key = z3.Concat(sender, z3.BitVecVal(263, 256))
    h = f(key)
    cond = z3.And(inv(h) == key, z3.ULE(1000, h), z3.ULT(h, 1 << 200), z3.URem(h, 64) == 0)
    st = z3.Array("Storage", z3.BitVecSort(256), z3.BitVecSort(256))
    st2 = z3.Store(z3.Store(st, h, 1), 2, word)
    kk = z3.Store(z3.K(z3.BitVecSort(256), z3.BitVecVal(7, 256)), word, 9)
    exprs = [z3.And(cond, st2[h] == 1), z3.And(st2[2] == word, z3.ULE(word, 20)), kk[sender] == 7,
             z3.And(cond, z3.Select(st2, sender + 1) == 0), z3.Or(cond, word == 0)]

    envs = []
    for _ in range(40):
        envs.append({"1_calldatasize": rng.choice([0, 4, 20, 36, 100, 1 << 255]),
                     "sender_1": rng.choice([2, 1000, 1 << 100, rng.getrandbits(256)])})

    def funcs_of(env):
        kval = (env["sender_1"] << 256) | 263
        hv = rng.choice([1024, 1000 + 64 * rng.getrandbits(8), rng.getrandbits(256)])
        cdv = {i: rng.choice([0, 1, rng.getrandbits(8)]) for i in range(40)}
        return {"keccak256_512": {kval: hv}, "keccak256_512-1": {hv: kval}, "array:1_calldata": cdv,
                "array:Storage": {hv: rng.choice([0, 1]), 2: 5}}

    assert _check(exprs, envs, funcs_of) > 0


def test_unsupported_constructs_go_to_the_fallback(monkeypatch):
    x = z3.BitVec("ux", 256)
    fp = z3._mk(z3.FuncDeclRef(z3.Z3_OP_FP_ADD, "fp.add"), z3.BitVecSort(256), [x, x])
    assert ZL.to_terms([fp == x]) is None
    with pytest.raises(SV.NotLowerable):
        SV._terms([fp == x])
    f2 = z3.Function("g2", z3.BitVecSort(8), z3.BitVecSort(8), z3.BitVecSort(8))
    assert ZL.to_terms([f2(z3.BitVecVal(1, 8), z3.BitVecVal(2, 8)) == 0]) is None


def test_z3_backend_check_and_recheck():
    from mythril_amd.z3_backend import Z3Backend

    be = Z3Backend(z3)
    x, y = z3.BitVec("rx", 256), z3.BitVec("ry", 256)
    cd = z3.Array("2_calldata", z3.BitVecSort(256), z3.BitVecSort(8))
    cs = [z3.ULT(x, y), cd[x] == 5, y == 9]
    terms = SV._terms(cs)
    B = F.Batch([terms])
    lw = ZL.lowering_for(x)
    # a witness row as the GPU would return it: rx = 3, ry = 9, calldata[3] = 5
    names = B.var_names(0)
    words = np.zeros((B.n_vars(0), 8), np.uint32)
    for i, nm in enumerate(names):
        v = {"rx": 3, "ry": 9}.get(nm, 5)
        words[i, 0] = v
    w = B.witness(0, words)
    assert be.recheck(terms, w) is True
    words[names.index("rx"), 0] = 12  # violates rx < ry
    assert be.recheck(terms, B.witness(0, words)) is False
    assert be.rechecks == 2 and be.recheck_failures == 1
    # terms without a z3 origin cannot be re-checked
    from mythril_amd.smt import symbol_factory
    assert be.recheck([(symbol_factory.BitVecSym("m", 256) == 1).raw], w) is None
    # the fallback on the original constraints: pinned -> decided by the stand-in
    r, m = be.check(SV._terms([x == 3, y == 9, z3.ULT(x, y)]), 100)
    assert r == SV.sat and m.raw is not None
    # Model.eval on a mirror term of a z3 model: mapped back to the z3 expression
    # (ADVICE r2); both kinds of model answer with a value that has .as_long()
    tx = ZL.lowering_for(x).lower(x)
    assert m.eval(tx).as_long() == 3
    gm = SV.Model([{"rx": 7}])
    assert gm.eval(tx).as_long() == 7 and gm.eval(ZL.lowering_for(y).lower(y)) is None
    r, _ = be.check(SV._terms([x == 3, y == 2, z3.ULT(x, y)]), 100)
    assert r == SV.unsat
    B.close()


class _AllUnsat:
    """A pre-filter stand-in that refutes everything (a deliberately unsound pre-check)."""

    def check_states(self, states, parents=None):
        return [(SV.unsat, None)] * len(states)


def test_refutation_audit_counts_disagreements(monkeypatch):
    """Z3Backend(recheck_refutations=f) puts a deterministic fraction f of the host's
    refutations to z3; a z3 `sat` is counted as a disagreement and z3's answer wins
    (VERDICT r2 item 4)."""
    from mythril_amd.z3_backend import Z3Backend

    x, y = z3.BitVec("ax", 256), z3.BitVec("ay", 256)

    class RC(list):
        def __init__(self, items):
            super().__init__(items)
            self._is_possible, self._default_timeout, self.witness = None, 100, None

    be = Z3Backend(z3, recheck_refutations=1.0)
    old = SV.set_backend(be)
    monkeypatch.setattr(SV, "prefilter", lambda: _AllUnsat())
    try:
        st = SV.SolverStatistics()
        st.reset()
        SV.unsat_cores().reset()
        items = [RC([x == 3, y == 2, z3.ULT(x, y)]), RC([x == 3, y == 9, z3.ULT(x, y)])]
        with pytest.warns(RuntimeWarning, match="soundness"):
            assert SV.batch_is_possible(items) == [False, True]
        assert st.refute_rechecks == 2 and st.refute_disagreements == 1
        s = SV.Solver()
        s.add(x == 1, y == 2)
        with pytest.warns(RuntimeWarning):
            assert s.check() == SV.sat  # the refutation is overridden with z3's model
        assert s.model().raw is not None and st.refute_disagreements == 2
        # a fraction: every other refutation is audited
        be.recheck_refutations, be._refutations_seen = 0.5, 0
        st.reset()
        SV.batch_is_possible([RC([x == k, y == k + 1, z3.ULT(y, x)]) for k in range(6)])
        assert st.refute_rechecks == 3 and st.refute_disagreements == 0
        # off by default
        assert Z3Backend(z3).recheck_refutation([]) is None
        with pytest.raises(ValueError):
            Z3Backend(z3, recheck_refutations=2.0)
    finally:
        SV.set_backend(old)
