"""Deterministic answers and the second witness round on the GPU.

* explicit (decision) rows land in the device candidates exactly where the host
  restatement (tests/fe_emulate.apply_xrows) puts them;
* a state's answer does not depend on its batch: the mixed corpus in two orders, a
  subset alone, and Prefilter(devices=[0, 0]) (two contexts, two host threads, hash
  shards by content key) give the same sat / unsat / undecided vector and witnesses;
* the whole two-round policy on the 1024-state corpus leaves for z3 exactly the states
  the CPU restatement of the same rounds (C oracle over the same candidates) leaves,
  at most 20 (>= 50x fewer solver calls), and contradicts no expectation.
"""
import collections

import numpy as np
import pytest

from mythril_amd import _native as N
from mythril_amd import dag as D
from mythril_amd import front as F
from mythril_amd import solver as SV

pytestmark = pytest.mark.gpu


def _corpus(n):
    import corpus

    return corpus.corpus(n)


@pytest.fixture()
def clean():
    SV.SolverStatistics().reset()
    SV.unsat_cores().reset()
    yield
    SV.unsat_cores().reset()


@pytest.mark.parametrize("n_states", [64, 200])
def test_explicit_rows_in_device_candidates(mgp_ctx, n_states):
    """64 states (<= 16 384 rows of hundreds of variables): a workgroup per row
    (mgp_fe_cands_rowblock_kernel); 200 states x 256: a thread per row."""
    from tests.fe_emulate import apply_xrows

    states = [c[1] for c in _corpus(n_states)]
    B = F.Batch(states)
    nv = B.n_vars() + 1
    rows, mask, _ = N.decision_rows(*B.packed(), nv, 77, 4, None, state_keys=B.state_key)
    _, dom = N.refute_domains(*B.packed(), B.var_off)
    for n_cand in (64, 256):
        dev = B.device_candidates(mgp_ctx, n_cand, nv, 77, dom=dom, xrows=(rows, mask))
        host = N.make_candidates(n_cand, nv, 77, B.var_off, B.var_width, B.hint_off, B.hints, B.alias_off, B.aliases,
                                 B.const_off, B.consts, D._FIXED_LIMBS, np.zeros(B.n_states, np.uint8),
                                 var_kind=B.var_kind, dom=dom, state_keys=B.state_key)
        apply_xrows(B, host, rows, mask)
        bad = np.nonzero((dev != host).any(axis=(1, 2, 3)))[0]
        assert bad.size == 0, f"n_cand={n_cand}: {bad.size} states differ, first {bad[:5]}"
    B.close()


def _kinds(res):
    return [r[0] for r in res]


def _same_answers(a, b):
    assert _kinds(a) == _kinds(b)
    for (ka, wa), (kb, wb) in zip(a, b):
        if ka == SV.sat:
            assert dict(wa) == dict(wb)


def test_answers_do_not_depend_on_the_batch(clean):
    pf = SV.Prefilter(0)
    try:
        cs = [c[1] for c in _corpus(240)]
        base = pf.check_states(cs)
        SV.unsat_cores().reset()
        perm = np.random.default_rng(7).permutation(len(cs))
        got = pf.check_states([cs[i] for i in perm])
        _same_answers([base[i] for i in perm], got)
        SV.unsat_cores().reset()
        sub = list(range(3, len(cs), 11))
        _same_answers([base[i] for i in sub], pf.check_states([cs[i] for i in sub]))
        SV.unsat_cores().reset()
        _same_answers([base[17]], pf.check_states([cs[17]]))
    finally:
        pf.close()


def test_two_contexts_answer_like_one(clean):
    """Prefilter(devices=[0, 0]): two contexts on one GPU, one host thread each, states
    hash-sharded by content key -- the same answers as Prefilter(0)."""
    one, two = SV.Prefilter(0), SV.Prefilter(devices=[0, 0])
    try:
        cs = [c[1] for c in _corpus(300)]
        owner = two.shard(cs)
        assert set(owner.tolist()) == {0, 1}
        a = one.check_states(cs)
        SV.unsat_cores().reset()
        b = two.check_states(cs)
        _same_answers(a, b)
    finally:
        one.close()
        two.close()


def test_two_pipelines_answer_like_one(clean):
    """Prefilter(pipelines=2): two contexts on one GPU with half the OpenMP threads each, a
    batch of >= PIPELINE_MIN states hash-sharded over them, a smaller one on the first --
    the same answers and witnesses as one pipeline, both ways."""
    one, two = SV.Prefilter(0), SV.Prefilter(0, pipelines=2)
    try:
        assert len(two.ctxs) == 2
        for n in (300, 40):
            cs = [c[1] for c in _corpus(n)]
            SV.unsat_cores().reset()
            a = one.check_states(cs)
            SV.unsat_cores().reset()
            b = two.check_states(cs)
            _same_answers(a, b)
            assert (two.last_profile or {}).get("shards", 1) == (2 if n >= two.PIPELINE_MIN else 1)
    finally:
        one.close()
        two.close()


def test_corpus_undecided_equals_cpu_restatement(clean):
    """The 1024-state mixed corpus through the product Prefilter (two rounds, decision rows)
    leaves exactly the states the CPU restatement of the same rounds leaves."""
    from tests import fe_emulate

    C = _corpus(1024)
    pf = SV.Prefilter(0)
    try:
        res = pf.check_states([c[1] for c in C])
    finally:
        pf.close()
    kinds = _kinds(res)
    undecided = [i for i, k in enumerate(kinds) if k == "undecided"]
    want, _ = fe_emulate.run(1024)
    assert undecided == sorted(want), (collections.Counter(C[i][0] for i in undecided), len(want))
    assert len(undecided) <= 20
    for (lab, _, exp), k in zip(C, kinds):
        assert not (exp == "unsat" and k == SV.sat) and not (exp == "sat" and k == SV.unsat), lab
    assert sum(1 for (_, _, e), k in zip(C, kinds) if e == "unsat" and k == SV.unsat) == \
        sum(1 for _, _, e in C if e == "unsat")


def test_submit_finish_equals_check_batch(mgp_ctx):
    """mgp_check_submit / mgp_check_finish (two rounds in flight on one context, finished in
    order) give what mgp_check_batch gives for each batch; a third submit is refused while
    two are in flight, and the context works on afterwards."""
    cs = [c[1] for c in _corpus(200)]
    B1, B2 = F.Batch(cs[:120]), F.Batch(cs[120:])
    want = [B.check(mgp_ctx, 256, 99) for B in (B1, B2)]
    p1 = B1.submit(mgp_ctx, 256, 99)
    p2 = B2.submit(mgp_ctx, 256, 99)
    with pytest.raises(N.MgpError):
        B1.submit(mgp_ctx, 256, 99)
    got = [p1.finish(), p2.finish()]
    for (f, w, r, _), (gf, gw, gr, _) in zip(want, got):
        assert np.array_equal(f, gf) and np.array_equal(r, gr)
        sat = f >= 0
        assert np.array_equal(w[sat], gw[sat])
    f3 = B2.check(mgp_ctx, 256, 99)[0]
    assert np.array_equal(f3, want[1][0])
    B1.close()
    B2.close()


def test_grouped_pipelined_call_answers_like_one_group(clean):
    """A call cut into several candidate-memory groups (Batch.select of the one build), their
    first and second rounds pipelined two in flight: the same answers and witnesses as the
    call in one group."""
    pf = SV.Prefilter(0)
    try:
        cs = [c[1] for c in _corpus(300)]
        a = pf.check_states(cs)
        assert pf.last_profile.get("groups", 1) == 1
        SV.unsat_cores().reset()
        pf.cand_bytes = 48 * pf.n_cand * 64 * 32
        b = pf.check_states(cs)
        assert pf.last_profile.get("groups", 1) >= 3
        assert pf.last_profile["pipelined_rounds"] > pf.last_profile["groups"]
        _same_answers(a, b)
    finally:
        pf.close()
