#!/bin/bash
# Eval-step comparison of several builds of libmgp on one box, interleaved rounds:
#   bash profiles/run_libs.sh <tag> <rounds> <lib names under mythril_amd/ ...>
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; N=$2; shift 2
# EXTRA_ENV, e.g. "MGP_SYNTH_ABLATE=nodiv", is exported for every run
for r in $(seq 1 $N); do
  for lib in "$@"; do
    env ${EXTRA_ENV:-} MGP_LIB_PATH=$PWD/mythril_amd/$lib timeout -k 10 120 python -u bench.py --steps 10 --keccak 0 --no-cpu --refute-sample 0 --frontend 0 --guided-sample 0 \
      > gpurun_out/${TAG}_${lib}_$r.json 2> gpurun_out/${TAG}_${lib}_$r.err
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_${lib}_$r.json')); print('$lib', $r, 'ms/step', round(d['ms_per_step'],3))"
  done
done
