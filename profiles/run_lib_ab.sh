#!/bin/bash
# Eval-step A/B of two builds of libmgp on one box, interleaved:
#   bash profiles/run_lib_ab.sh <tag> <rounds>   (A = mythril_amd/libmgp.so, B = mythril_amd/libmgp_ab.so)
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; N=${2:-3}
for r in $(seq 1 $N); do
  for v in A B; do
    lib=mythril_amd/libmgp.so; [ $v = B ] && lib=mythril_amd/libmgp_ab.so
    MGP_LIB_PATH=$PWD/$lib timeout -k 10 120 python -u bench.py --steps 10 --keccak 0 --no-cpu --refute-sample 0 --frontend 0 --guided-sample 0 \
      > gpurun_out/${TAG}_${v}$r.json 2> gpurun_out/${TAG}_${v}$r.err
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_${v}$r.json')); print('$v', $r, 'ms/step', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4))"
  done
done
