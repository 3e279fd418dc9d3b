#!/bin/bash
# Keccak line of bench.py for several builds of libmgp on one box (interleaved rounds):
#   bash profiles/run_keccak_variants.sh <tag> <rounds> <lib>...
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; N=$2; shift 2
for r in $(seq 1 $N); do
  for lib in "$@"; do
    MGP_LIB_PATH=$PWD/mythril_amd/$lib timeout -k 10 150 python -u bench.py --steps 2 --states 65536 --no-cpu \
      --refute-sample 0 --frontend 0 --guided-sample 0 > gpurun_out/${TAG}_${lib}_$r.json 2> gpurun_out/${TAG}_${lib}_$r.err
    python3 -c "import json; k=json.load(open('gpurun_out/${TAG}_${lib}_$r.json'))['keccak']; print('$lib', $r, '%.4g hashes/s' % k['value'], 'verified', k['verified']['mismatches'], 'frac', round(k['roofline']['frac'], 3))"
  done
done
