"""Front-end latency probe (profiling aid): Prefilter.check_states on 1, 2 and 16 states of
the mixed corpus, repeated, with the per-stage split; run under rocprofv3 to see where a
small batch's time goes (profiles/run_fe_prof.sh)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import corpus  # noqa: E402
from mythril_amd import solver as SV  # noqa: E402


def main():
    items = [c[1] for c in corpus.corpus(512) if not c[0].startswith("wallet")]
    pf = SV.Prefilter(device=0)
    pf.check_states(items[:4])
    for n in [int(x) for x in os.environ.get("FE_SIZES", "1,2,16").split(",")]:
        rows = []
        for r in range(20):
            SV.unsat_cores().reset()
            t = time.perf_counter()
            pf.check_states(items[r % 8: r % 8 + n])
            rows.append((1e3 * (time.perf_counter() - t), pf.last_profile))
        rows.sort(key=lambda x: x[0])
        ms, prof = rows[len(rows) // 2]
        print(json.dumps({"states": n, "ms": ms, **{k: round(v, 3) for k, v in prof.items() if k.endswith("_ms")}}),
              flush=True)


if __name__ == "__main__":
    main()
