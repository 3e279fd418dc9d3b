"""Solver front end with the host UNSAT pre-check — CPU only.

The GPU stage is replaced by a stub context that finds no witness, so every
state reaches mgp_refute and then, if not refuted, the fallback backend.  The
contracts checked are the reference's: Constraints.is_possible
(constraints.py:34-51: unsat -> False, unknown -> True), get_model
(analysis/solver.py:27-61: UnsatError on unsat/unknown) and
SolverStatistics.query_count (one per fallback check, solver_statistics.py).
"""
import numpy as np
import pytest

from mythril_amd import _native as N
from mythril_amd import solver as SV
from mythril_amd.smt import And, Not, Or, ULT, UGT, symbol_factory

BVV = symbol_factory.BitVecVal
BVS = symbol_factory.BitVecSym


class NoWitnessContext:
    """Stands in for the GPU context: no candidate satisfies any state."""

    def __init__(self, device=0):
        self.batches = 0

    def eval_batch(self, words, po, cands):
        self.batches += 1
        n = len(po) - 1
        return np.full(n, -1, dtype=np.int32), np.zeros((n, cands.shape[2], 8), dtype=np.uint32)

    def check_batch(self, batch, n_cand, seed, parents=None, refute=True, xrows=None):
        """mgp_check_batch without a GPU: no witness; the host pre-check as in the pipeline."""
        self.batches += 1
        n = batch.n_states
        ref = N.refute(*batch.packed()) if refute else np.zeros(n, np.int8)
        return (np.full(n, -1, dtype=np.int32), np.zeros((n, max(1, batch.n_vars()), 8), dtype=np.uint32), ref,
                np.zeros(5))

    def close(self):
        pass


class CountingBackend(SV.Backend):
    def __init__(self):
        self.calls = 0

    def check(self, terms, timeout_ms, minimize=(), maximize=()):
        self.calls += 1
        return SV.unknown, None


@pytest.fixture()
def fe(monkeypatch):
    monkeypatch.setattr(N, "Context", NoWitnessContext)
    monkeypatch.setattr(SV, "_prefilter", None)
    SV.enable_gpu(True)
    b = CountingBackend()
    old = SV.set_backend(b)
    SV.SolverStatistics().reset()
    SV.unsat_cores().reset()
    SV.get_model.cache_clear()
    yield b
    SV.set_backend(old)
    SV.get_model.cache_clear()


def test_is_possible_refuted_without_fallback(fe):
    x, size = BVS("x", 256), BVS("calldatasize", 256)
    items = [
        SV.Constraints([x == BVV(1, 256), x == BVV(2, 256)]),
        SV.Constraints([ULT(size, BVV(4, 256)), UGT(size, BVV(35, 256))]),
        SV.Constraints([x == BVV(3, 256), Not(x == BVV(3, 256))]),
        SV.Constraints([x * x == BVV(5, 256)]),  # UNSAT, but not by bits and ranges
        SV.Constraints([Or(x == BVV(1, 256), x == BVV(2, 256))]),  # SAT; the stub finds no witness
    ]
    assert SV.batch_is_possible(items) == [False, False, False, True, True]
    st = SV.SolverStatistics()
    assert st.refuted == 3 and st.query_count == 2 and fe.calls == 2
    assert [c._is_possible for c in items] == [False, False, False, True, True]


def test_get_model_and_optimize(fe):
    x = BVS("x", 256)
    with pytest.raises(SV.UnsatError):
        SV.get_model((x == BVV(5, 256), ULT(x, BVV(5, 256))))
    assert fe.calls == 0
    with pytest.raises(SV.UnsatError):  # minimize: still no model exists, no fallback needed
        SV.get_model((And(x == BVV(5, 256), x == BVV(7, 256)),), minimize=(x,))
    assert fe.calls == 0
    with pytest.raises(SV.UnsatError):  # satisfiable but minimised -> fallback (unknown here)
        SV.get_model((ULT(x, BVV(5, 256)),), minimize=(x,))
    assert fe.calls == 1
    s = SV.Solver()
    s.add(x == BVV(9, 256), UGT(x, BVV(9, 256)))
    assert s.check() == SV.unsat and fe.calls == 1
    assert SV.SolverStatistics().query_count == 1


def test_refute_off_restores_reference_path(fe):
    x = BVS("x", 256)
    pf = SV.prefilter()
    pf.refute = False
    items = [SV.Constraints([x == BVV(1, 256), x == BVV(2, 256)])]
    assert SV.batch_is_possible(items) == [True]  # unknown -> possible, via the fallback
    assert fe.calls == 1 and SV.SolverStatistics().refuted == 0


def test_unsat_core_cache(fe):
    x, y, z, w = (BVS(n, 256) for n in ("cx", "cy", "cz", "cw"))
    a = [x == BVV(1, 256), ULT(y, BVV(5, 256)), x == BVV(2, 256), UGT(z, BVV(3, 256))]
    assert SV.batch_is_possible([SV.Constraints(a)]) == [False]
    st = SV.SolverStatistics()
    assert st.refuted == 1 and st.core_hits == 0
    # refuted lists are shrunk in batches (Prefilter.core_batch); flush the pending one
    assert SV.unsat_cores().sets == [] and len(SV.unsat_cores().pending) == 1
    SV.prefilter().flush_cores()
    # the stored core is the contradiction alone, not the whole path
    assert SV.unsat_cores().sets == [frozenset({a[0].raw, a[2].raw})]
    # another path repeating the contradiction: UNSAT from the cache, no analysis, no fallback
    b = [w == BVV(7, 256), x == BVV(2, 256), UGT(z, BVV(9, 256)), x == BVV(1, 256)]
    assert SV.batch_is_possible([SV.Constraints(b), SV.Constraints(b[:3])]) == [False, True]
    assert st.refuted == 1 and st.core_hits == 1 and fe.calls == 1


def test_fallback_unsat_feeds_the_cache(fe):
    class UnsatBackend(SV.Backend):
        calls = 0

        def check(self, terms, timeout_ms, minimize=(), maximize=()):
            UnsatBackend.calls += 1
            return SV.unsat, None

    SV.set_backend(UnsatBackend())
    x = BVS("fx", 256)
    base = [x * x == BVV(5, 256)]  # UNSAT for the solver, not for the pre-check
    assert SV.batch_is_possible([SV.Constraints(base)]) == [False]
    assert SV.batch_is_possible([SV.Constraints(base + [ULT(x, BVV(100, 256))])]) == [False]
    assert UnsatBackend.calls == 1 and SV.SolverStatistics().core_hits == 1


class SecondRoundContext(NoWitnessContext):
    """No witness among the first round's candidates; in the second round (the one that
    carries host decision rows) the first decision row 'satisfies'."""

    def check_batch(self, batch, n_cand, seed, parents=None, refute=True, xrows=None):
        f, w, ref, t = super().check_batch(batch, n_cand, seed, parents, refute, xrows)
        if xrows is None:
            return f, w, ref, t
        rows, mask = xrows
        nv = w.shape[1]
        w[:, : rows.shape[2]] = rows[:, 0, :nv]
        return np.where(mask[:, 0].any(axis=1), 0, -1).astype(np.int32), w, ref, t


def test_second_candidate_round(fe, monkeypatch):
    monkeypatch.setattr(N, "Context", SecondRoundContext)
    x, y = BVS("rx", 256), BVS("ry", 256)
    items = [SV.Constraints([ULT(x, y)]), SV.Constraints([x == BVV(1, 256), x == BVV(2, 256)])]
    assert SV.batch_is_possible(items) == [True, False]
    st = SV.SolverStatistics()
    assert st.gpu_retry == 1 and st.gpu_sat == 1 and st.refuted == 1 and fe.calls == 0
    # the first round (no witness from the stub), then ONE second round for the open state
    # whose decision rows the stub satisfies
    assert SV.prefilter().ctx.batches == 2
    w = items[0].witness
    assert set(w) == {"rx", "ry"} and w["rx"] < w["ry"]  # decision row 0 is a model of rx < ry


def test_decision_rows_per_state_rule():
    """Decision rows per state depend on the state alone (variables x nodes x rows against
    Prefilter.decide_max_units), not on a wall-clock budget or on the rest of the batch."""
    import types

    import corpus
    from mythril_amd.front import Batch
    from corpus.keccak_manager import KeccakFunctionManager

    kfm = KeccakFunctionManager()
    states = [list(t) for _, t, _ in corpus.wallet_states(0, kfm)[:4]]
    states += [list(corpus.bectoken_states(k, kfm)[1]) for k in range(4)]
    B = Batch(states)
    units = np.diff(B.var_off).astype(float) * np.diff(B.node_off)
    fake = types.SimpleNamespace(decide_rows=4, decide_max_units=SV.Prefilter.DECIDE_MAX_UNITS,
                                 DECIDE_MIN_ROWS=SV.Prefilter.DECIDE_MIN_ROWS)
    assert (SV.Prefilter.rows_per_state(fake, B) == 4).all()  # the corpus fits the default cap
    fake.decide_max_units = float(units[4:].max()) * 4      # BECToken fits four, WalletLibrary not
    r = SV.Prefilter.rows_per_state(fake, B)
    assert (r[4:] == 4).all() and all(r[i] in (0, 2) for i in range(4))
    B2 = Batch(states[::-1])  # the same states in another batch order: the same rule per state
    assert np.array_equal(SV.Prefilter.rows_per_state(fake, B2), r[::-1])
    B.close()
    B2.close()


def test_core_shrink_halving_finds_a_core_of_a_redundant_list():
    """A list reaching its contradiction twice (no single deletion alone breaks it) still
    shrinks: a halving round keeps the half that is refuted alone (the newer half is tried
    first: a path's older constraints are its parent's), and without halvings the greedy
    deletions (mgp_refute_cores, round 5: each deletion that keeps the list refuted is kept)
    end on one of the two contradictions (UnsatCores.shrink_many)."""
    v = [BVS(f"h{i}", 256) for i in range(12)]
    x, y = BVS("hx", 256), BVS("hy", 256)
    # first half: one contradiction on x among fillers; second half: another on y
    first = [ULT(v[0], BVV(9, 256)), x == BVV(1, 256), UGT(v[1], BVV(2, 256)), x == BVV(2, 256),
             ULT(v[2], BVV(7, 256)), UGT(v[3], BVV(1, 256)), ULT(v[4], BVV(5, 256)), UGT(v[5], BVV(4, 256))]
    second = [ULT(v[6], BVV(9, 256)), y == BVV(3, 256), UGT(v[7], BVV(2, 256)), ULT(v[8], BVV(7, 256)),
              y == BVV(4, 256), UGT(v[9], BVV(1, 256)), ULT(v[10], BVV(5, 256)), UGT(v[11], BVV(4, 256))]
    terms = [c.raw for c in first + second]
    from mythril_amd.front import Batch

    B = Batch([terms, terms[:8], terms[8:]])
    assert list(N.refute(*B.packed())) == [1, 1, 1]  # the list, and each half alone
    B.close()
    old = SV.UnsatCores.HALVINGS
    try:
        SV.UnsatCores.HALVINGS = 0  # greedy deletions alone: one of the two contradictions
        greedy = set(SV.UnsatCores.shrink(N, terms))
        assert greedy in ({first[1].raw, first[3].raw}, {second[1].raw, second[4].raw}), greedy
        SV.UnsatCores.HALVINGS = old
        core = SV.UnsatCores.shrink(N, terms)
    finally:
        SV.UnsatCores.HALVINGS = old
    assert set(core) == {second[1].raw, second[4].raw}


def test_retry_round_groups(fe):
    """The second round's open states in one group (its grouping batch reused as the round's
    batch) or, past cand_bytes, in several (one batch per group): same answers, every open
    state retried once."""
    def items():
        return [SV.Constraints([ULT(BVS(f"rg{i}_{j}", 256), BVV(7 + j, 256)) for j in range(1 + i % 5)])
                for i in range(24)]

    pf = SV.prefilter()
    got = {}
    old = pf.cand_bytes
    try:
        # the second cap holds the first round (24 states x n_cand x 5 variables) but not
        # the second round's larger candidate block
        pf.retry_cand = 2 * pf.n_cand
        for cap in (old, 24 * pf.n_cand * 5 * 32):
            pf.cand_bytes = cap
            SV.SolverStatistics().reset()
            got[cap] = SV.batch_is_possible(items())
            assert SV.SolverStatistics().gpu_retry == 24
    finally:
        pf.cand_bytes = old
        pf.retry_cand = pf.RETRY_CAND
    assert list(got.values())[0] == list(got.values())[1] == [True] * 24


def test_core_shrink_halves_a_list_longer_than_max_terms():
    """A 48-constraint refuted list (past max_terms = 32, no single-deletion pass) halves
    into range and shrinks to its two-constraint core."""
    fill = [ULT(BVS(f"lf{i}", 256), BVV(100 + i, 256)) for i in range(46)]
    x = BVS("lx", 256)
    terms = [c.raw for c in fill[:5] + [x == BVV(5, 256)] + fill[5:9] + [x == BVV(6, 256)] + fill[9:]]
    assert len(terms) == 48
    old = SV.UnsatCores.HALVINGS
    try:
        SV.UnsatCores.HALVINGS = 0
        assert SV.UnsatCores.shrink(N, terms) == terms  # too long: stored whole
        SV.UnsatCores.HALVINGS = old
        core = SV.UnsatCores.shrink(N, terms)
    finally:
        SV.UnsatCores.HALVINGS = old
    assert set(core) == {terms[5], terms[10]}
