#!/bin/bash
# GPU-box round check: gpu tests, smoke, default bench; with a second argument "prof"
# also the rocprofv3 collection (profiles/collect.sh).   bash profiles/run_round.sh <tag> [prof]
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${1:-r1}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
if [ "${2:-}" = "prof" ]; then bash profiles/collect.sh ${TAG}; fi
