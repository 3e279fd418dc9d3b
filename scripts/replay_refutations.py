"""Replay every refutation of the restated suite with the independent checker.

    python scripts/replay_refutations.py [out.json] [--workers N] [--tier1] [--contracts a,b]

For every query of corpus.suite() (all 13 contracts) that the product's split refuter refutes
at the product's settings (mgp_refute_split, Prefilter.SPLIT_REFUTE / SPLIT_DEPTH), the
refuter's UNSAT core (mgp_refute_cores) is re-proved by oracle.refute_check -- reasoning of its
own over the term DAG, written apart from mgp_domain.h (its docstring).  Writes per-contract
counts of replayed / unreplayed refutations and the labels of the unreplayed ones (default
profiles/refute_replay_r6.json).  An unreplayed refutation is one the checker's search did not
close, not one it found wrong: a checker cannot find a refutation wrong, only a model can (the
GPU witness checks of tests/test_gpu_suite.py).  CPU only; test infrastructure.
"""
import collections
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import corpus  # noqa: E402
from mythril_amd import _native as N  # noqa: E402
from mythril_amd import front as F  # noqa: E402
from mythril_amd.solver import Prefilter  # noqa: E402
from oracle import refute_check as RC  # noqa: E402
from oracle.keccak_ref import keccak256  # noqa: E402

_CORES = None   # refuted query index -> its core (inherited by the forked workers)
_TIERS = None


def _one(k):
    t = time.perf_counter()
    ok = RC.refute(_CORES[k], tiers=_TIERS)
    return k, bool(ok), time.perf_counter() - t


def main():
    global _CORES, _TIERS
    args = [a for k, a in enumerate(sys.argv[1:]) if not a.startswith("--")
            and sys.argv[k] not in ("--workers", "--contracts")]
    out_path = args[0] if args else "profiles/refute_replay_r6.json"
    workers = 7
    if "--workers" in sys.argv:
        workers = int(sys.argv[sys.argv.index("--workers") + 1])
    if "--tier1" in sys.argv:   # the cheap search alone (a quick look)
        _TIERS = RC.TIERS[:1]
    t0 = time.perf_counter()
    names = None
    if "--contracts" in sys.argv:   # a subset of the suite (a quick look)
        names = set(sys.argv[sys.argv.index("--contracts") + 1].split(","))
    qs = corpus.suite(hasher=keccak256, contracts=names)
    B = F.Batch([list(q[3]) for q in qs])
    p = B.packed()[:4]
    split = N.refute_split(*p, max_splits=Prefilter.SPLIT_REFUTE, depth=Prefilter.SPLIT_DEPTH)
    keep, st = N.refute_cores(*p, np.array([len(q[3]) for q in qs], np.uint32))
    B.close()
    refuted = [k for k in range(len(qs)) if split[k] == 1]
    cores = {}
    for k in refuted:
        cs = list(qs[k][3])
        cores[k] = [c for c, m in zip(cs, keep[k]) if m] if st[k] == 1 else cs
    _CORES = cores
    t_suite = time.perf_counter() - t0
    t1 = time.perf_counter()
    with mp.get_context("fork").Pool(workers) as pool:
        res = pool.map(_one, refuted, chunksize=4)
    by = collections.defaultdict(lambda: {"refuted": 0, "replayed": 0, "unreplayed": []})
    secs = []
    for k, ok, dt in res:
        c = by[qs[k][0]]
        c["refuted"] += 1
        c["replayed"] += ok
        if not ok:
            c["unreplayed"].append(qs[k][2])
        secs.append(dt)
    tot = {"queries": len(qs), "refuted": len(refuted), "replayed": sum(ok for _, ok, _ in res),
           "core_constraints_mean": float(np.mean([len(cores[k]) for k in refuted])) if refuted else 0.0,
           "suite_seconds": round(t_suite, 1), "replay_seconds": round(time.perf_counter() - t1, 1),
           "workers": workers, "tiers": [list(t) for t in (_TIERS or RC.TIERS)],
           "state_seconds_max": round(max(secs), 2) if secs else 0.0}
    blob = {"all": tot, "by_contract": {c: {**v, "unreplayed_kinds": dict(collections.Counter(
        lab.split(":")[1].split("@")[0] for lab in v["unreplayed"]))} for c, v in sorted(by.items())}}
    with open(out_path, "w") as f:
        json.dump(blob, f, indent=1)
    print(json.dumps(tot))


if __name__ == "__main__":
    main()
