"""CPU emulation of the pre-filter's witness rounds (test infrastructure; uses the C oracle).

The GPU evaluates candidates; here the C oracle does, over exactly the candidates the
device generator would produce (mgp_make_candidates is bit-identical to it,
tests/test_gpu_front.py).  Used to study which corpus states stay undecided without a
GPU:  python -m tests.fe_emulate [n_states]
"""
from __future__ import annotations

import collections
import sys
import time

import numpy as np

from mythril_amd import _native as N
from mythril_amd import dag as D
from mythril_amd import front as F
from oracle import coracle


def host_round(B, n_cand, seed, dom=None, xrows=None):
    """The candidates mgp_check_batch evaluates (content-keyed device mixture, domain rows,
    explicit rows in the first mixture rows), evaluated by the C oracle."""
    nv = max(1, B.n_vars())
    c = N.make_candidates(n_cand, nv, seed, B.var_off, B.var_width, B.hint_off, B.hints, B.alias_off, B.aliases,
                          B.const_off, B.consts, D._FIXED_LIMBS, np.zeros(B.n_states, np.uint8),
                          var_kind=B.var_kind, dom=dom, state_keys=B.state_key)
    if xrows is not None:
        apply_xrows(B, c, *xrows)
    _, _, status = N.lower(*B.packed(gpu=True))
    f = coracle.first_sat(*B.packed(gpu=True), c)
    f[status != 0] = -2
    f[(B.flags & F.FE_SAT_UNSAFE) != 0] = -1
    return f


def first_round_rows(B, seed, parents=None, decide_rows: int = 4, seed_rows: int = 0x3):
    """Prefilter._first_round_rows restated: decision rows (seed + ROWS_FIRST_SEED) of the
    states above ROWS_FIRST_NODES nodes, parent-seeded like the retry round's; None if none."""
    from mythril_amd import solver as SV

    big = np.diff(B.node_off) > SV.Prefilter.ROWS_FIRST_NODES
    if not big.any():
        return None
    fake = type("P", (), {"decide_rows": decide_rows, "decide_max_units": SV.Prefilter.DECIDE_MAX_UNITS,
                          "DECIDE_MIN_ROWS": SV.Prefilter.DECIDE_MIN_ROWS})()
    row0 = min(SV.Prefilter.ROWS_FIRST_FROM, max(0, decide_rows - 1))
    n_rows = min(decide_rows - row0, SV.Prefilter.ROWS_FIRST_ROWS)
    rps = np.where(big, np.minimum(SV.Prefilter.rows_per_state(fake, B), n_rows), 0).astype(np.uint8)
    gv = max(1, B.n_vars())
    seeds = None
    if parents is not None and any(p is not None for p in parents):
        seeds = F.seed_arrays(B, parents)
        if seeds[0].shape[1] != gv:
            seeds = None
    rows, mask, _ = N.decision_rows(*B.packed(decide=True), gv, (seed + SV.Prefilter.ROWS_FIRST_SEED) & (2 ** 64 - 1),
                                    n_rows, rps, state_keys=B.state_key, seeds=seeds, seed_rows=seed_rows,
                                    row0=row0)
    return rows, mask


def apply_xrows(B, cands, rows, mask, first_row=2):
    """Host restatement of mgp_fe_cands_kernel's explicit rows: mixture row k (candidate
    first_row + k) takes the masked slots of row k; pinned constants stay."""
    for s in range(B.n_states):
        V = B.n_vars(s)
        kind = B.var_kind[int(B.var_off[s]): int(B.var_off[s + 1])]
        for k in range(rows.shape[1]):
            c = first_row + k
            if c >= cands.shape[1]:
                break
            m = mask[s, k, :V].astype(bool) & (kind != 2)
            cands[s, c, :V][m] = rows[s, k, :V][m]
            # the slot-width mask of the kernel (decision values are inside their width already)
    return cands


def run(n: int = 1024, seed: int = 0x4D595448, decide_rows: int = 4, n2: int = 256):
    import corpus

    from mythril_amd import solver as SV

    C = corpus.corpus(n)
    states = [c[1] for c in C]
    t = time.time()
    B = F.Batch(states)
    ref, dom = N.refute_domains(*B.packed(), B.var_off)
    f1 = host_round(B, 256, seed, dom=dom, xrows=first_round_rows(B, seed, decide_rows=decide_rows))
    B.close()
    open_ = [i for i in range(n) if f1[i] < 0 and ref[i] != 1]
    print(f"first round: sat {int((f1 >= 0).sum())} refuted {int((ref == 1).sum())} open {len(open_)} "
          f"({time.time() - t:.1f}s)")
    t = time.time()
    SB = F.Batch([states[i] for i in open_])
    seed2 = seed + 0x7F4A7C15
    fake = type("P", (), {"decide_rows": decide_rows, "decide_max_units": SV.Prefilter.DECIDE_MAX_UNITS,
                          "DECIDE_MIN_ROWS": SV.Prefilter.DECIDE_MIN_ROWS})()
    rps = SV.Prefilter.rows_per_state(fake, SB)
    td = time.time()
    rows, mask, _ = N.decision_rows(*SB.packed(decide=True), max(1, SB.n_vars()), seed2, decide_rows, rps,
                                    state_keys=SB.state_key)
    td = time.time() - td
    _, dom2 = N.refute_domains(*SB.packed(), SB.var_off)
    f2 = host_round(SB, n2, seed2, dom=dom2, xrows=(rows, mask))
    SB.close()
    open2 = [i for k, i in enumerate(open_) if f2[k] < 0]
    if open2:  # the product's case-split refutation of what both rounds leave open
        LB = F.Batch([states[i] for i in open2])
        rs = N.refute_split(*LB.packed()[:4], max_splits=SV.Prefilter.SPLIT_REFUTE,
                                depth=SV.Prefilter.SPLIT_DEPTH)
        LB.close()
        open2 = [i for k, i in enumerate(open2) if rs[k] != 1]
    print(f"second round: +{len(open_) - len(open2)} open {len(open2)} (decisions {td:.2f}s, "
          f"{time.time() - t:.1f}s)")
    cnt = collections.Counter(C[i][0] for i in open2)
    for k, v in sorted(cnt.items()):
        print(f"  {v:4d}  {k}  (expected {next(c[2] for c in C if c[0] == k)})")
    return open2, C


if __name__ == "__main__":
    run(int(sys.argv[1]) if len(sys.argv) > 1 else 1024)


def suite_answers(queries, seed: int = 0x4D595448, decide_rows: int = 4, n2: int = 256, seed_rows: int = 0x3,
                  witnesses: bool = False):
    """The product policy over corpus.suite() queries on the CPU, level by level along the
    parent links as corpus.answer feeds the GPU Prefilter: first round (parent witness in
    row 0, device mixture with domain rows), host pre-check, second round with (parent-
    seeded) decision rows.  -> list of 'sat' / 'unsat' / 'undecided' (test infrastructure:
    the C oracle evaluates the candidates)."""
    from mythril_amd import solver as SV

    n = len(queries)
    depth = [0] * n
    for i, q in enumerate(queries):
        depth[i] = depth[q[5]] + 1 if q[5] >= 0 else 0
    ans = ["undecided"] * n
    wit = [None] * n     # (slot keys, values) of a SAT query's witness
    levels = collections.defaultdict(list)
    for i, d in enumerate(depth):
        levels[d].append(i)
    fake = type("P", (), {"decide_rows": decide_rows, "decide_max_units": SV.Prefilter.DECIDE_MAX_UNITS,
                          "DECIDE_MIN_ROWS": SV.Prefilter.DECIDE_MIN_ROWS})()
    for d in sorted(levels):
        idx = levels[d]
        B = F.Batch([list(queries[i][3]) for i in idx])
        par = [wit[queries[i][5]] if queries[i][5] >= 0 else None for i in idx]
        ref, dom = N.refute_domains(*B.packed(), B.var_off)
        nv = max(1, B.n_vars())
        has = np.array([p is not None for p in par], np.uint8)
        c = N.make_candidates(256, nv, seed, B.var_off, B.var_width, B.hint_off, B.hints, B.alias_off, B.aliases,
                              B.const_off, B.consts, D._FIXED_LIMBS, has, var_kind=B.var_kind, dom=dom,
                              state_keys=B.state_key)
        pw = [None if p is None else dict_to_witness(p) for p in par]
        sv, sm = F.seed_arrays(B, pw)
        for s in range(B.n_states):
            m = sm[s].astype(bool)
            c[s, 0, m] = sv[s, m]
        xr = first_round_rows(B, seed, pw, decide_rows=decide_rows, seed_rows=seed_rows)
        if xr is not None:
            apply_xrows(B, c, *xr)
        _, _, status = N.lower(*B.packed(gpu=True))
        f1 = coracle.first_sat(*B.packed(gpu=True), c)
        f1[status != 0] = -2
        f1[(B.flags & F.FE_SAT_UNSAFE) != 0] = -1
        open_ = [k for k in range(len(idx)) if f1[k] < 0 and ref[k] != 1]
        rows = None
        if open_:
            SB = F.Batch([list(queries[idx[k]][3]) for k in open_])
            rps = SV.Prefilter.rows_per_state(fake, SB)
            spar = [par[k] for k in open_]
            seeds = F.seed_arrays(SB, [None if p is None else dict_to_witness(p) for p in spar]) \
                if any(p is not None for p in spar) else None
            seed2 = seed + 0x7F4A7C15
            rows, mask, _ = N.decision_rows(*SB.packed(decide=True), max(1, SB.n_vars()), seed2, decide_rows, rps,
                                            state_keys=SB.state_key, seeds=seeds, seed_rows=seed_rows)
            _, dom2 = N.refute_domains(*SB.packed(), SB.var_off)
            nv2 = max(1, SB.n_vars())
            c2 = N.make_candidates(n2, nv2, seed2, SB.var_off, SB.var_width, SB.hint_off, SB.hints, SB.alias_off,
                                   SB.aliases, SB.const_off, SB.consts, D._FIXED_LIMBS, np.zeros(SB.n_states, np.uint8),
                                   var_kind=SB.var_kind, dom=dom2, state_keys=SB.state_key)
            apply_xrows(SB, c2, rows, mask)
            _, _, st2 = N.lower(*SB.packed(gpu=True))
            f2 = coracle.first_sat(*SB.packed(gpu=True), c2)
            f2[st2 != 0] = -2
            f2[(SB.flags & F.FE_SAT_UNSAFE) != 0] = -1
            for j, k in enumerate(open_):
                if f2[j] >= 0:
                    i = idx[k]
                    ans[i] = "sat"
                    v0, v1 = int(SB.var_off[j]), int(SB.var_off[j + 1])
                    wit[i] = (np.array(SB.var_key[v0:v1]), c2[j, f2[j], : v1 - v0].copy())
            SB.close()
        for k, i in enumerate(idx):
            if f1[k] >= 0:
                ans[i] = "sat"
                v0, v1 = int(B.var_off[k]), int(B.var_off[k + 1])
                wit[i] = (np.array(B.var_key[v0:v1]), c[k, f1[k], : v1 - v0].copy())
            elif ref[k] == 1:
                ans[i] = "unsat"
        left = [i for i in idx if ans[i] == "undecided"]
        if left:  # the product's case-split refutation of what both rounds leave open
            LB = F.Batch([list(queries[i][3]) for i in left])
            rs = N.refute_split(*LB.packed()[:4], max_splits=SV.Prefilter.SPLIT_REFUTE,
                                depth=SV.Prefilter.SPLIT_DEPTH)
            LB.close()
            for k, i in enumerate(left):
                if rs[k] == 1:
                    ans[i] = "unsat"
        B.close()
    return (ans, wit) if witnesses else ans


class dict_to_witness:
    """A (slot keys, values) pair in the shape front.parent_arrays accepts."""

    def __init__(self, kv):
        self.kv = kv


def _parent_arrays_kv(p, _orig=F.parent_arrays):
    if isinstance(p, dict_to_witness):
        return np.asarray(p.kv[0], np.uint64), np.ascontiguousarray(p.kv[1], np.uint32).reshape(-1, 8)
    return _orig(p)


F.parent_arrays = _parent_arrays_kv
