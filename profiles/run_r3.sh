#!/bin/bash
# Round-3 box run: GPU suite then the default bench line.   bash profiles/run_r3.sh <tag>
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${1:-r3a}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  cat gpurun_out/${TAG}_bench.json | head -c 600
fi
