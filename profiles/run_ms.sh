#!/bin/bash
# bucket launches on one stream vs spread over auxiliary streams (quarter and full workload)
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread -m gpu > gpurun_out/ms_tests.log 2>&1 || { tail -40 gpurun_out/ms_tests.log; exit 1; }
tail -1 gpurun_out/ms_tests.log
for qs in 262144 1048576; do
for m in 0 1; do
  MGP_BUCKET_STREAMS=$m timeout -k 10 200 python -u bench.py --states $qs --steps 5 --warmup 2 --keccak 0 --no-cpu > gpurun_out/ms_${qs}_$m.json 2> gpurun_out/ms_${qs}_$m.err
  python3 -c "import json; d=json.load(open('gpurun_out/ms_${qs}_$m.json')); print('states $qs streams $m', '%.4g evals/s' % d['value'], '%.3f ms' % d['ms_per_step'])"
done
done
