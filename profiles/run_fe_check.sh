#!/bin/bash
# Front-end checks after a front-end change: the front-end / corpus / solver GPU tests,
# then the latency probe with a kernel + HIP API trace.   bash profiles/run_fe_check.sh <tag>
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${1:-fe}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_front.py tests/test_gpu_corpus.py tests/test_gpu_solver.py tests/test_gpu_z3.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_fe_tests.log 2>&1
tail -3 gpurun_out/${TAG}_fe_tests.log
bash profiles/run_fe_prof.sh ${TAG}
