#!/bin/bash
# A/B of the interpreter's chunks-per-wave loop: GPU parity suite, then the default
# bench workload (eval only) at chunks_per_wave 1 and the default (outputs under gpurun_out/cpw_<tag>/)
set -euo pipefail
TAG=${1:-a}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/cpw_${TAG}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -2 "$OUT/tests.log"
ARGS="--steps 10 --warmup 3 --keccak 0 --no-cpu --refute-sample 0 --frontend 0"
for c in 1 0; do
  if [ "$c" = 0 ]; then unset MGP_CHUNKS_PER_WAVE; else export MGP_CHUNKS_PER_WAVE=$c; fi
  timeout -k 10 200 python -u bench.py $ARGS > "$OUT/bench_cpw$c.json" 2> "$OUT/bench_cpw$c.err"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['ms_per_step'], d['roofline']['frac_spec'])" "$OUT/bench_cpw$c.json" "cpw=$c"
done
