#!/bin/bash
# GPU check of the spill / Bool-demotion work: the parity tests (both engines), the
# front-end and corpus tests, then the default bench.   bash profiles/run_spill.sh <tag>
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${1:-r2s}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "spilled or long_programs or synthetic_vs" -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_spill.log 2>&1
tail -3 gpurun_out/${TAG}_spill.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
