"""Decision rows on the GPU (mythril_amd/csrc/mgp_decide.hip) against the host's.

The device kernel runs the same propagation code as the host (mgp_domain.h compiled for
gfx950), one wave per (state, row) task; its rows, masks and statuses must be
bit-identical to mgp_decision_rows on the mixed contract corpus (suicide, BECToken,
WalletLibrary states: relaxed wide values, UF congruence, Or case splits, pair
orderings), on the synthetic batch, with per-state row counts, and through the
Prefilter's second witness round (the answers do not depend on where the rows ran).
"""
import time

import numpy as np
import pytest

from mythril_amd import _native as N
from mythril_amd import front as F
from mythril_amd import solver as SV

pytestmark = pytest.mark.gpu


def _both(packed, nv, seed, n_decide, rps, keys, ctx):
    t = time.perf_counter()
    h = N.decision_rows(*packed, nv, seed, n_decide, rps, state_keys=keys)
    th = time.perf_counter() - t
    t = time.perf_counter()
    d = N.decision_rows(*packed, nv, seed, n_decide, rps, state_keys=keys, ctx=ctx)
    td = time.perf_counter() - t
    return h, d, th, td


def _assert_same(h, d):
    rows_h, mask_h, st_h = h
    rows_d, mask_d, st_d = d
    assert np.array_equal(st_h, st_d)
    assert np.array_equal(mask_h, mask_d)
    m = mask_h.astype(bool)
    bad = np.nonzero((rows_h[m] != rows_d[m]).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} of {int(m.sum())} decided slots differ"


def test_device_rows_bit_identical_on_corpus(mgp_ctx):
    import corpus

    states = [c[1] for c in corpus.corpus(1024)]
    B = F.Batch(states)
    fake = type("P", (), {"decide_rows": 4, "decide_max_units": SV.Prefilter.DECIDE_MAX_UNITS,
                          "DECIDE_MIN_ROWS": SV.Prefilter.DECIDE_MIN_ROWS})()
    rps = SV.Prefilter.rows_per_state(fake, B)
    h, d, th, td = _both(B.packed(decide=True), max(1, B.n_vars()), 0x4D595448 + 0x7F4A7C15, 4, rps,
                         B.state_key, mgp_ctx)
    _assert_same(h, d)
    assert int(h[1].sum()) > 100_000  # the rows really decide slots
    print(f"corpus 1024 x 4 rows: host {th * 1e3:.1f} ms, device {td * 1e3:.1f} ms")
    B.close()


@pytest.mark.parametrize("n_decide", [1, 8])
def test_device_rows_bit_identical_on_synthetic(mgp_ctx, n_decide):
    b = N.synth_generate(0x4D595448, 99, 512, 64, 16)
    packed = (b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
    rps = np.array([(s % 9) for s in range(512)], np.uint8)  # 0..8 rows, some states none
    keys = np.arange(512, dtype=np.uint64) * 0x9E3779B97F4A7C15
    h, d, th, td = _both(packed, b["n_vars"], 77, n_decide, rps, keys, mgp_ctx)
    _assert_same(h, d)
    print(f"synthetic 512 x {n_decide} rows: host {th * 1e3:.1f} ms, device {td * 1e3:.1f} ms")


def test_prefilter_answers_do_not_depend_on_where_rows_run(mgp_ctx):
    """Prefilter(decide_on_gpu=always) and (never) give the same answers and witnesses."""
    import corpus

    states = [c[1] for c in corpus.corpus(256)]
    res = []
    for where in ("never", "always"):
        SV.unsat_cores().reset()
        pf = SV.Prefilter()
        pf.decide_on_gpu = where
        res.append(pf.check_states(states))
        pf.close()
    assert [r[0] for r in res[0]] == [r[0] for r in res[1]]
    for (k0, w0), (k1, w1) in zip(*res):
        if k0 == SV.sat:
            assert dict(w0) == dict(w1)
    SV.unsat_cores().reset()
