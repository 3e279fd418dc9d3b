"""The mixed contract corpus (corpus.py: suicide.sol, BECToken.sol, WalletLibrary.sol shapes)
through the GPU-first front end: every GPU witness is a model of its constraints (checked by
the oracle), no shape expected UNSAT gets a witness, no shape expected SAT is refuted, and
the outcome counts per contract are reported.  Expectations are by reading (corpus.py);
issue-level parity with `myth analyze` stays unpinned (no solc / z3 / mythril)."""
import collections

import pytest

import corpus
from mythril_amd import dag as D
from mythril_amd import solver as SV
from oracle import bvsem as S

pytestmark = pytest.mark.gpu


def test_mixed_corpus_soundness_and_counts(mgp_ctx):
    SV.unsat_cores().reset()
    SV.SolverStatistics().reset()
    SV.enable_gpu(True)
    items = corpus.corpus(240)
    res = SV.prefilter().check_states([c[1] for c in items])
    counts = collections.defaultdict(collections.Counter)
    for (label, terms, expected), (kind, model) in zip(items, res):
        counts[label][kind] += 1
        if kind == SV.sat:
            assert expected != "unsat", f"{label}: witness for a shape that is UNSAT by construction"
            st = D.build_state(list(terms))
            assert S.eval_root(st.nodes, st.consts, D.model_to_slots(st, dict(model))), label
        if kind == SV.unsat:
            assert expected != "sat", f"{label}: refuted a shape that is SAT by construction"
    print({k: dict(v) for k, v in counts.items()})
    total = collections.Counter()
    for v in counts.values():
        total.update(v)
    assert total[SV.sat] > 0 and total[SV.unsat] > 0
    # suicide.sol: the attacker query is refuted on the host, no fallback (suicide.py:76-99)
    assert counts["suicide:attacker query"][SV.unsat] == sum(counts["suicide:attacker query"].values())
