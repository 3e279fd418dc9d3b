"""The native front-end pipeline on the GPU (mgp_check_batch), against the host reference.

* GPU-generated candidates (mgp_fe_cands_kernel) are bit-identical to the host generator
  mgp_make_candidates on the same tables and seed;
* first-SAT of mgp_check_batch equals the C oracle's first-SAT over exactly those
  candidates, on the GPU program (padded key equalities strengthened), and its
  refutations equal mgp_refute on the original nodes;
* a child state gets its parent's witness as candidate row 0.
"""
import numpy as np
import pytest

from mythril_amd import _native as N
from mythril_amd import dag as D
from mythril_amd import front as F
from mythril_amd.smt import UGT, ULT, symbol_factory
from oracle import coracle

pytestmark = pytest.mark.gpu

BVV, BVS = symbol_factory.BitVecVal, symbol_factory.BitVecSym


def _contract_batch(n):
    import corpus

    return [c[1] for c in corpus.corpus(n)]  # suicide, BECToken, WalletLibrary shapes (pinned constants too)


def test_device_candidates_equal_host_generator(mgp_ctx):
    states = _contract_batch(96)
    B = F.Batch(states)
    n_vars = B.n_vars() + 2  # padding variables are filled too
    _, dom = N.refute_domains(*B.packed(), B.var_off)
    for n_cand, seed, d in ((64, 5, None), (256, 0x4D595448, dom), (37, 11, dom)):
        dev = B.device_candidates(mgp_ctx, n_cand, n_vars, seed, dom=d)
        host = N.make_candidates(n_cand, n_vars, seed, B.var_off, B.var_width, B.hint_off, B.hints, B.alias_off,
                                 B.aliases, B.const_off, B.consts, D._FIXED_LIMBS, np.zeros(B.n_states, np.uint8),
                                 var_kind=B.var_kind, dom=d, state_keys=B.state_key)
        bad = np.nonzero((dev != host).any(axis=(1, 2, 3)))[0]
        assert bad.size == 0, f"n_cand={n_cand}: {bad.size} states differ, first {bad[:5]}"
    B.close()


def test_check_batch_matches_oracle_and_refute(mgp_ctx):
    states = _contract_batch(200)
    x, y = BVS("x", 256), BVS("y", 256)
    states += [(ULT(x, BVV(5, 256)).raw, UGT(x, BVV(9, 256)).raw),  # refuted
               ((x * x == BVV(5, 256)).raw,), ((x == y + 1).raw, (y == BVV(7, 256)).raw)]
    B = F.Batch(states)
    seed, n_cand = 1234, 256
    first, wit, ref, times = B.check(mgp_ctx, n_cand, seed)
    n_vars = max(1, B.n_vars())
    _, dom = N.refute_domains(*B.packed(), B.var_off)  # the pipeline draws domain rows from these
    cands = B.device_candidates(mgp_ctx, n_cand, n_vars, seed, dom=dom)
    want = coracle.first_sat(*B.packed(gpu=True), cands)
    _, _, status = N.lower(*B.packed(gpu=True))
    assert (status == 0).all()  # every corpus shape lowers (spill slots, Bool demotion, 255-entry pools)
    assert np.array_equal(first, want)
    assert np.array_equal(ref, N.refute(*B.packed()))
    assert ref[200] == 1 and first[200] == -1
    assert first[202] >= 0
    for s in np.nonzero(first >= 0)[0]:
        assert (wit[s, : B.n_vars(s)] == cands[s, first[s], : B.n_vars(s)]).all()
    w = B.witness(202, wit[202])
    assert w["y"] == 7 and w["x"] == 8
    assert len(times) == 5 and (times >= 0).all()
    B.close()


def test_parent_witness_is_row_zero(mgp_ctx):
    x, y, z = BVS("x", 256), BVS("y", 256), BVS("z", 256)
    parent = [(x * y == BVV(391, 256)).raw, UGT(x, BVV(1, 256)).raw, UGT(y, BVV(1, 256)).raw]  # 17 x 23
    P = F.Batch([parent])
    pf, pw, _, _ = P.check(mgp_ctx, 64, 7, parents=[{"x": 17, "y": 23}])
    assert pf[0] == 0  # the dict parent (a fallback solver's model) is row 0
    pwit = P.witness(0, pw[0])
    P.close()
    assert dict(pwit) == {"x": 17, "y": 23}
    child = parent + [ULT(x, y).raw, (z != x).raw]
    C = F.Batch([child])
    cf, cw, _, _ = C.check(mgp_ctx, 64, 8, parents=[pwit])
    assert cf[0] == 0  # row 0 = the parent's x and y (SlotWitness keys); z is the child's own
    w = C.witness(0, cw[0])
    assert w["x"] == 17 and w["y"] == 23
    C.close()


def test_check_batch_program_cache(mgp_ctx):
    """mgp_check_batch keeps the programs it lowered (keyed by the exact node list and
    constants): a second call on the same states, and a call on a subset in another
    order (the retry round's shape), give the results of a fresh lowering."""
    states = _contract_batch(120)
    B = F.Batch(states)
    f1, w1, r1, _ = B.check(mgp_ctx, 256, 77)
    f2, w2, r2, _ = B.check(mgp_ctx, 256, 77)
    assert np.array_equal(f1, f2) and np.array_equal(w1, w2) and np.array_equal(r1, r2)
    sub = list(range(len(states) - 1, -1, -3))
    S = F.Batch([states[i] for i in sub])
    fs, _, rs, _ = S.check(mgp_ctx, 256, 5)
    n_vars = max(1, S.n_vars())
    _, dom = N.refute_domains(*S.packed(), S.var_off)
    cands = S.device_candidates(mgp_ctx, 256, n_vars, 5, dom=dom)
    want = coracle.first_sat(*S.packed(gpu=True), cands)
    _, _, status = N.lower(*S.packed(gpu=True))
    ok = status == 0
    assert np.array_equal(fs[ok], want[ok]) and (fs[~ok] == N.MGP_UNDECIDED).all()
    assert np.array_equal(rs, r1[sub])
    B.close()
    S.close()
