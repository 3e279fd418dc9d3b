"""A/B of Prefilter's small-batch policies in one process on one box (host speed varies by
+-25 % across boxes): speculative retry rows (speculate_rows_max) and the overlap of the
first-round rows with lowering, cold calls interleaved per repetition, medians.

    python3 profiles/fe_spec_ab.py > gpurun_out/fe_spec_ab.json
"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import corpus  # noqa: E402
from mythril_amd import solver as SV  # noqa: E402


def main():
    C = corpus.corpus(1024)
    cs = [c[1] for c in C]
    wal = [c[1] for c in C if c[0].startswith("wallet")]
    bec = [c[1] for c in C if c[0].startswith("bectoken")]
    configs = {"spec16": 16, "spec0": 0}
    pfs = {}
    for k, v in configs.items():
        pf = SV.Prefilter(0)
        pf.speculate_rows_max = v
        pfs[k] = pf
    out = {}
    for label, pool, n, reps in (("mixed", cs, 1, 60), ("mixed", cs, 2, 60), ("wallet", wal, 2, 40),
                                 ("bectoken", bec, 2, 40), ("mixed", cs, 16, 20)):
        walls = {k: [] for k in configs}
        for r in range(reps):
            sub = pool[(r * n * 7) % max(1, len(pool) - n):][:n]
            for k in (configs if r % 2 == 0 else reversed(list(configs))):
                SV.unsat_cores().reset()
                pfs[k]._N.program_cache_clear()
                t = time.perf_counter()
                pfs[k].check_states(sub)
                walls[k].append(1e3 * (time.perf_counter() - t))
        out[f"{label}_{n}"] = {k: float(np.median(w)) for k, w in walls.items()}
        print(label, n, out[f"{label}_{n}"], file=sys.stderr, flush=True)
    for pf in pfs.values():
        pf.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
