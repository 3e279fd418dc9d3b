#!/bin/bash
# Round-2 check: division tests (single-digit path), the GPU suite, the default bench,
# then the Keccak fast-path A/B (8 waves/SIMD, two hashes per lane).  bash profiles/run_r2z.sh <tag>
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${1:-r2z}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "division" -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_div.log 2>&1 || { tail -30 gpurun_out/${TAG}_div.log; exit 1; }
tail -3 gpurun_out/${TAG}_div.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
ARGS="--states 65536 --steps 2 --warmup 1 --no-cpu --refute-sample 0 --frontend 0 --guided-sample 0"
for v in w8 x2 base; do
  case $v in
    base) E="MGP_KECCAK_BASE=1";;
    w8) E="MGP_KECCAK_W8=1";;
    x2) E="MGP_KECCAK_X2=1";;
  esac
  env $E timeout -k 10 300 python3 -u bench.py $ARGS > gpurun_out/${TAG}_kab_$v.json 2> gpurun_out/${TAG}_kab_$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_kab_$v.json'))['keccak'];print('$v', d['value'], d['verified']['mismatches'])"
done
