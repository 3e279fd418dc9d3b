"""A/B in one process: the first-round decision rows of a large batch run before the
lowering (default) or beside it on half the host threads each (rows_overlap_split).
Cold calls interleaved per repetition, medians.

    python3 profiles/fe_overlap_ab.py > gpurun_out/fe_overlap_ab.json
"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import corpus  # noqa: E402
from mythril_amd import solver as SV  # noqa: E402


def main():
    cs = [c[1] for c in corpus.corpus(1024)]
    a, b = SV.Prefilter(0), SV.Prefilter(0)
    b.rows_overlap_split = True
    pfs = {"sequential": a, "overlap_half": b}
    out = {}
    for n, reps in ((64, 12), (128, 10), (512, 6), (1024, 6)):
        walls = {k: [] for k in pfs}
        for r in range(reps):
            sub = cs[(r * 37) % max(1, len(cs) - n):][:n]
            for k in (list(pfs) if r % 2 == 0 else list(reversed(list(pfs)))):
                SV.unsat_cores().reset()
                pfs[k]._N.program_cache_clear()
                t = time.perf_counter()
                res = pfs[k].check_states(sub)
                walls[k].append(1e3 * (time.perf_counter() - t))
        out[str(n)] = {k: float(np.median(w)) for k, w in walls.items()}
        print(n, out[str(n)], file=sys.stderr, flush=True)
    for pf in pfs.values():
        pf.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
