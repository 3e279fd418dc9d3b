#!/bin/bash
# Eval step vs LDS floor per wave (caps waves/CU at 160 KiB / floor): bash profiles/run_occ_bench.sh <tag> <floors...>
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
for pad in "$@"; do
  MGP_LDS_MIN_BYTES=$pad timeout -k 10 120 python -u bench.py --steps 10 --keccak 0 --no-cpu --refute-sample 0 --frontend 0 --guided-sample 0 \
    > gpurun_out/${TAG}_occ_$pad.json 2> gpurun_out/${TAG}_occ_$pad.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_occ_$pad.json')); print('floor', $pad, 'ms/step', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4))"
done
