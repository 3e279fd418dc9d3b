"""The product policy over restated `myth analyze` queries, on the CPU (no GPU): the LASER
restatement of two solidity_examples contracts (corpus.laser, corpus.contracts) answered
by tests/fe_emulate.py's CPU restatement of Prefilter (first round, pre-check, seeded
decision rows, case-split refutation), counted as corpus.account counts z3 calls.

The held-out contracts (corpus.held_out) are not used here: no policy knob is checked
against them.
"""
import collections

from oracle.keccak_ref import keccak256

import corpus
from mythril_amd import _native as N
from mythril_amd import front as F
from tests import fe_emulate as E


def _queries(names):
    return corpus.suite(hasher=keccak256, contracts=set(names))


def test_calls_and_returnvalue_restatement_no_contradiction():
    """calls.sol / returnvalue.sol: no answer contradicts a by-reading expectation, and the
    z3 calls stay at the round-4 level (ether_thief's balance comparisons after zero-value
    transfers are refuted by the two-level case split, ether_thief.py:55-95)."""
    qs = _queries(["calls", "returnvalue"])
    assert not set(q[0] for q in qs) & corpus.held_out()
    ans = E.suite_answers(qs)
    acc = corpus.account(qs, ans)
    assert acc["all"]["contradicted"] == 0
    assert acc["all"]["z3_calls"] <= 22, acc["by_contract"]
    thief = collections.Counter(a for q, a in zip(qs, ans) if "ether_thief" in q[2] and q[4] == "unsat")
    assert thief["unsat"] >= 19 and thief["sat"] == 0, thief


def test_case_split_refutes_what_plain_analysis_leaves():
    """mgp_refute_split on the expected-unsat ether_thief queries: one level refutes strictly
    more than mgp_refute and two levels strictly more than one, each a superset of the
    last; it never refutes an expected-sat query of the two contracts."""
    qs = _queries(["calls", "returnvalue"])
    B = F.Batch([list(q[3]) for q in qs])
    packed = B.packed()[:4]
    plain = N.refute(*packed)
    split = N.refute_split(*packed, max_splits=8)
    split2 = N.refute_split(*packed, max_splits=8, depth=2)
    B.close()
    assert ((plain == 1) & (split != 1)).sum() == 0
    assert ((split == 1) & (split2 != 1)).sum() == 0
    exp = [q[4] for q in qs]
    assert not any(s == 1 and e == "sat" for s, e in zip(split2, exp))
    thief = [k for k, q in enumerate(qs) if "ether_thief" in q[2] and q[4] == "unsat"]
    n0, n1, n2 = (sum(r[k] == 1 for k in thief) for r in (plain, split, split2))
    assert n0 < n1 < n2, (n0, n1, n2)


def test_no_refutation_of_a_witnessed_query():
    """The UNSAT side on real contract shapes, on the CPU: every query of
    calls.sol / returnvalue.sol / etherstore.sol that the CPU restatement of the witness
    rounds answers with a model (checked by the C oracle there) is refuted neither by
    mgp_refute nor by mgp_refute_split at the product's settings (case splits and interval
    bisection); and every refuted query's sat-if-reachable expectation has a refuted ancestor."""
    from mythril_amd import solver as SV

    qs = _queries(["calls", "returnvalue", "etherstore"])
    ans, _ = E.suite_answers(qs, witnesses=True)
    sat = [k for k, a in enumerate(ans) if a == "sat"]
    assert len(sat) > 100
    B = F.Batch([list(qs[k][3]) for k in sat])
    packed = B.packed()[:4]
    plain = N.refute(*packed)
    split = N.refute_split(*packed, max_splits=SV.Prefilter.SPLIT_REFUTE, depth=SV.Prefilter.SPLIT_DEPTH)
    B.close()
    bad = [qs[k][2] for k, p, r in zip(sat, plain, split) if p == 1 or r == 1]
    assert not bad, bad[:5]
    acc = corpus.account(qs, ans)
    assert acc["all"]["refuted_with_sat_expectation_if_reachable"] == 0, acc["all"]
    assert acc["all"]["contradicted"] == 0 and acc["all"]["sat_expectations_dropped"] == 0, acc["all"]


def test_refute_cache_matches_the_refuter():
    """corpus/refute_cache.json (the stream generator's refutations by state content key) was
    written by the refuter as it is now: its version is the hash of the refuter's sources and
    settings, and a stale file would make every suite() run (GPU tests, bench) recompute its
    decisions live.  A sample of its entries must agree with a live mgp_refute_split run."""
    import json

    from corpus import laser as L

    with open(L._CACHE_PATH) as f:
        blob = json.load(f)
    assert blob["version"] == L._refuter_version(), "stale corpus/refute_cache.json: run python -m corpus.laser"
    assert len(blob["decisions"]) > 1000
    # live agreement on the queries of two small contracts (keys recomputed from their terms)
    qs = _queries(["suicide", "origin", "calls"])
    from mythril_amd.solver import Prefilter

    seen = 0
    for q in qs:
        B = F.Batch([list(q[3])])
        key = f"{int(B.state_key[0]):016x}"
        if key in blob["decisions"]:
            live = int(N.refute_split(*B.packed()[:4], max_splits=Prefilter.SPLIT_REFUTE,
                                      depth=Prefilter.SPLIT_DEPTH)[0]) == 1
            assert live == bool(blob["decisions"][key]), q[2]
            seen += 1
        B.close()
    assert seen >= 5, seen


def test_account_counts_a_refuted_sat_if_reachable_query():
    """corpus.account: a child expected sat under an unlabelled parent keeps
    its expectation (label suffix SAT_IF_REACHABLE); its refutation is a contradiction unless
    an ancestor is refuted too; under a parent expected unsat the expectation is dropped."""
    T = (object(),)
    R = corpus.SAT_IF_REACHABLE
    qs = [("c", "prune", "c:root", T, None, -1),              # 0 unlabelled
          ("c", "prune", "c:child" + R, T, "sat", 0),         # 1 sat if 0 is reachable
          ("c", "prune", "c:grandchild" + R, T, "sat", 1),    # 2 sat if 1 is reachable
          ("c", "prune", "c:bad", T, "unsat", -1),            # 3
          ("c", "prune", "c:under unsat" + corpus.UNDER_UNSAT_PARENT, T, None, 3)]
    # 1 refuted under an undecided root: a contradiction; 2 refuted under refuted 1: consistent
    acc = corpus.account(qs, ["undecided", "unsat", "unsat", "unsat", "undecided"])
    c = acc["by_contract"]["c"]
    assert c["contradicted"] == 1 and c["refuted_with_sat_expectation_if_reachable"] == 1
    assert c["refuted_if_reachable_ancestor_refuted"] == 1 and c["sat_expectations_dropped"] == 1
    # the root refuted as well: no contradiction left
    acc = corpus.account(qs, ["unsat", "unsat", "unsat", "unsat", "undecided"])
    assert acc["by_contract"]["c"]["contradicted"] == 0


def test_suite_marks_expectations_by_parent():
    """corpus.suite(): no sat expectation is dropped (the stream never follows a parent
    expected unsat); children of unlabelled parents carry the SAT_IF_REACHABLE suffix."""
    qs = _queries(["bectoken"])
    assert not any(q[2].endswith(corpus.UNDER_UNSAT_PARENT) for q in qs)
    marked = [k for k, q in enumerate(qs) if q[2].endswith(corpus.SAT_IF_REACHABLE)]
    assert marked and all(qs[k][4] == "sat" for k in marked)
    for k in marked:   # the parent is unlabelled or itself sat-if-reachable
        p = qs[k][5]
        assert qs[p][4] is None or qs[p][2].endswith(corpus.SAT_IF_REACHABLE)
