#!/bin/bash
# Where a small front-end batch's time goes: kernel + HIP API trace of
# profiles/fe_latency.py (1, 2 and 16 states, repeated).   bash profiles/run_fe_prof.sh <tag>
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${1:-fe}
OUT=gpurun_out/feprof_${TAG}
mkdir -p "$OUT"
timeout -k 10 200 python3 -u profiles/fe_latency.py > "$OUT/plain.jsonl" 2> "$OUT/plain.err"
cat "$OUT/plain.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 -u profiles/fe_latency.py > "$OUT/traced.jsonl" 2> "$OUT/traced.err"
cat "$OUT/traced.jsonl"
