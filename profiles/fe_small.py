"""Small-batch front-end calls (LASER's JUMPI fork: 2 successors) in a loop, for a
rocprofv3 kernel trace of where a 2-state call's time goes.
    python profiles/fe_small.py [n_states] [reps]"""
import sys
import time

sys.path.insert(0, ".")
import corpus  # noqa: E402
from mythril_amd import solver as SV  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
cs = [c[1] for c in corpus.corpus(1024)]
pf = SV.Prefilter()
pf.check_states(cs[:64])
walls = []
for r in range(reps):
    SV.unsat_cores().reset()
    pf._N.program_cache_clear()
    sub = cs[(r * n) % (len(cs) - n):][:n]
    t = time.perf_counter()
    pf.check_states(sub)
    walls.append(1e3 * (time.perf_counter() - t))
walls.sort()
print(f"{n} states: median {walls[len(walls) // 2]:.3f} ms, p10 {walls[len(walls) // 10]:.3f}, p90 {walls[9 * len(walls) // 10]:.3f}")
print("last profile", pf.last_profile)
pf.close()
