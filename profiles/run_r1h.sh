#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1h_tests.log 2>&1
tail -3 gpurun_out/r1h_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1h_smoke.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r1h_bench.json 2> gpurun_out/r1h_bench.err
cat gpurun_out/r1h_bench.json
bash profiles/collect.sh r1h
