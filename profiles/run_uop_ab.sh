#!/bin/bash
# Per-handler cost table (profiles/uop_costs.py) for libmgp.so (A) and libmgp_ab.so (B) on one box
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
for v in A B; do
  lib=mythril_amd/libmgp.so; [ $v = B ] && lib=mythril_amd/libmgp_ab.so
  echo "== $v"
  MGP_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u profiles/uop_costs.py --engine asm > gpurun_out/${TAG}_uop_$v.txt 2>&1
  grep "SIMD-cycles" gpurun_out/${TAG}_uop_$v.txt
done
