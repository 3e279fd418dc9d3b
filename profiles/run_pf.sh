#!/bin/bash
# candidate prefetch distance A/B (quarter workload):  bash profiles/run_pf.sh <tag>
set -e
TAG=${1:-pf}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread -m gpu > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for d in ${DISTS:-0 64 256 1024}; do
  MGP_PREFETCH_DIST=$d timeout -k 10 200 python -u bench.py --states ${QS:-262144} --steps 5 --warmup 2 --keccak 0 --no-cpu > gpurun_out/${TAG}_$d.json 2> gpurun_out/${TAG}_$d.err
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_$d.json')); print('dist $d', '%.4g evals/s' % d['value'], '%.3f ms' % d['ms_per_step'])"
done
