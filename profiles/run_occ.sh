#!/bin/bash
# per-uop cost vs occupancy (LDS padding limits the waves per SIMD): bash profiles/run_occ.sh
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for pad in 0 13312 20480 40960; do
  echo "== LDS per wave >= $pad"
  MGP_LDS_MIN_BYTES=$pad timeout -k 10 200 python -u profiles/uop_costs.py --engine asm > gpurun_out/occ_$pad.txt 2>&1
  grep "SIMD-cycles" gpurun_out/occ_$pad.txt | head -9
done
