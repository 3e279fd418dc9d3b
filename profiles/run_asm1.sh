#!/bin/bash
# first GPU run of the hand-written gfx950 interpreter: parity (both engines), then a short A/B bench
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 100 --timeout-method thread -m gpu > gpurun_out/asm1_tests.log 2>&1 || { tail -40 gpurun_out/asm1_tests.log; exit 1; }
tail -3 gpurun_out/asm1_tests.log
for e in asm hip; do
  MGP_ENGINE=$e timeout -k 10 200 python -u bench.py --states 262144 --steps 5 --warmup 2 --keccak 0 --no-cpu > gpurun_out/asm1_bench_$e.json 2> gpurun_out/asm1_bench_$e.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/asm1_bench_$e.json')); print('$e', d['value'], d['ms_per_step'], d['roofline']['frac'], d['results'])"
done
