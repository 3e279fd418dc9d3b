#!/bin/bash
# bench time by workload ablation (DIV / MUL replaced by ADD in the synthetic DAGs):
#   bash profiles/run_abl.sh <tag>
set -e
TAG=${1:-abl}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in none nodiv nomul nodivmul; do
  MGP_SYNTH_ABLATE=$m timeout -k 10 200 python -u bench.py --states ${QS:-262144} --steps 5 --warmup 2 --keccak 0 --no-cpu > gpurun_out/${TAG}_$m.json 2> gpurun_out/${TAG}_$m.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_$m.json')); print('$m', '%.4g evals/s' % d['value'], '%.3f ms' % d['ms_per_step'])"
done
