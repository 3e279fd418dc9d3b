#!/bin/bash
# eval step by workload ablation (DIV / MUL replaced by ADD in the synthetic DAGs), full size:
#   bash profiles/run_abl2.sh <tag>
set -e
TAG=${1:-abl}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in none nodiv nomul nodivmul; do
  MGP_SYNTH_ABLATE=$m timeout -k 10 120 python -u bench.py --steps 10 --keccak 0 --no-cpu --refute-sample 0 --frontend 0 --guided-sample 0 > gpurun_out/${TAG}_$m.json 2> gpurun_out/${TAG}_$m.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_$m.json')); print('$m', '%.4g evals/s' % d['value'], '%.3f ms' % d['ms_per_step'])"
done
