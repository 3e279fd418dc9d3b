#!/bin/bash
# parity of both engines + a quick A/B bench at a quarter of the workload:  bash profiles/run_ab.sh <tag>
set -e
TAG=${1:-ab}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread -m gpu > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for e in ${ENGINES:-asm}; do
  MGP_ENGINE=$e timeout -k 10 200 python -u bench.py --states ${QS:-262144} --steps 5 --warmup 2 --keccak 0 --no-cpu > gpurun_out/${TAG}_bench_$e.json 2> gpurun_out/${TAG}_bench_$e.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_bench_$e.json')); print('$e', '%.4g evals/s' % d['value'], '%.3f ms' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'], d['results'])"
done
