"""Front-end kernel trace probe (profiling aid): Prefilter.check_states on the 1 024-state
mixed corpus, cold (program cache cleared, no UNSAT core cached), a few times, printing the
stage split of each call; run it under `rocprofv3 --kernel-trace --stats` to see which
kernels make up the call's GPU wait:
    rocprofv3 --kernel-trace --stats -d gpurun_out/fe_trace -o run --output-format csv -- \
        python3 profiles/fe_trace.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import corpus  # noqa: E402
from mythril_amd import solver as SV  # noqa: E402


def main():
    n = int(os.environ.get("FE_STATES", "1024"))
    cs = [c[1] for c in corpus.corpus(n)]
    pf = SV.Prefilter(device=0)
    pf.check_states(cs[:8])
    for r in range(int(os.environ.get("FE_REPS", "4"))):
        SV.unsat_cores().reset()
        pf._N.program_cache_clear()
        t = time.perf_counter()
        pf.check_states(cs)
        ms = 1e3 * (time.perf_counter() - t)
        prof = pf.last_profile or {}
        print(json.dumps({"rep": r, "states": n, "ms": round(ms, 2),
                          **{k: round(v, 3) for k, v in prof.items() if k.endswith("_ms")}}), flush=True)


if __name__ == "__main__":
    main()
