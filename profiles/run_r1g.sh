#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/r1g_bench.json 2> gpurun_out/r1g_bench.err
cat gpurun_out/r1g_bench.json
bash profiles/collect.sh r1g
