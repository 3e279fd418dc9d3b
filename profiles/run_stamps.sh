#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread -m gpu > gpurun_out/st3_tests.log 2>&1 || { tail -40 gpurun_out/st3_tests.log; exit 1; }
tail -1 gpurun_out/st3_tests.log
timeout -k 10 200 python -u profiles/stamps.py > gpurun_out/stamps3.txt 2>&1 || { tail -20 gpurun_out/stamps3.txt; exit 1; }
cat gpurun_out/stamps3.txt
