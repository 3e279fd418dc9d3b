#!/bin/bash
# Keccak fast-path A/B on the box: default kernel, 8 waves/SIMD variant, two hashes per lane,
# each on the bench's keccak leg (2^30 hashes, digests verified), short eval leg.
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--states 65536 --steps 2 --warmup 1 --no-cpu --refute-sample 0 --frontend 0 --guided-sample 0"
for v in base w8 x2 base; do
  case $v in
    base) E="";;
    w8) E="MGP_KECCAK_W8=1";;
    x2) E="MGP_KECCAK_X2=1";;
  esac
  env $E timeout -k 10 300 python3 -u bench.py $ARGS > gpurun_out/kab_$v.json 2> gpurun_out/kab_$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/kab_$v.json'))['keccak'];print('$v', d['value'], d['verified']['mismatches'])"
done
