#!/bin/bash
# A/B of two builds x LDS floors on one box: bash profiles/run_lib_ab2.sh <tag> "<A floors>" "<B floors>"
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
for r in 1 2; do
for v in A B; do
  lib=mythril_amd/libmgp.so; fl="$2"; [ $v = B ] && { lib=mythril_amd/libmgp_ab.so; fl="$3"; }
  for pad in $fl; do
    MGP_LDS_MIN_BYTES=$pad MGP_LIB_PATH=$PWD/$lib timeout -k 10 120 python -u bench.py --steps 10 --keccak 0 --no-cpu --refute-sample 0 --frontend 0 --guided-sample 0 \
      > gpurun_out/${TAG}_${v}_$pad.json 2> gpurun_out/${TAG}_${v}_$pad.err
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_${v}_$pad.json')); print('$v', 'floor', $pad, 'ms/step', round(d['ms_per_step'],3))"
  done
done
done
