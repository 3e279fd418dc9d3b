#!/bin/bash
# Eval-step comparison of (library, environment) variants on one box, interleaved rounds:
#   bash profiles/run_variants.sh <tag> <rounds> "<lib>[:VAR=val,VAR=val]" ...
# (lib = a build of libmgp under mythril_amd/; the variables are exported for that run only)
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; N=$2; shift 2
for r in $(seq 1 $N); do
  i=0
  for spec in "$@"; do
    i=$((i + 1))
    lib=${spec%%:*}; envs=""
    [ "$spec" != "$lib" ] && envs=$(echo "${spec#*:}" | tr ',' ' ')
    env $envs ${EXTRA_ENV:-} MGP_LIB_PATH=$PWD/mythril_amd/$lib timeout -k 10 120 python -u bench.py --steps 10 --keccak 0 --no-cpu \
      --refute-sample 0 --frontend 0 --guided-sample 0 ${BENCH_ARGS:-} > gpurun_out/${TAG}_v${i}_$r.json 2> gpurun_out/${TAG}_v${i}_$r.err
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_v${i}_$r.json')); print('$spec', $r, 'ms/step', round(d['ms_per_step'],3))"
  done
done
