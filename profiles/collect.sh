#!/bin/bash
# Collect the rocprofv3 evidence for one round on the GPU box:
#   bash profiles/collect.sh <tag>      (outputs under gpurun_out/prof_<tag>/)
# 1. kernel trace + per-kernel stats of a short bench run at the full workload
#    (same kernels, same launch shapes as the timed run)
# 2. separate PMC passes (never combined with tracing domains; <= 8 SQ / 4 TCC counters each)
# Summarise with: python3 profiles/analyze.py gpurun_out/prof_<tag> > profiles/<tag>_summary.md
set -euo pipefail
TAG=${1:-r1}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
ARGS="--states ${PROF_STATES:-1048576} --steps 3 --warmup 1 --keccak 67108864 --keccak-chunk 67108864 --no-cpu --refute-sample 0 --frontend 0 --suite 0 --suite-open-sweep 0 --div-split 0 --guided-sample 0"
echo "[collect] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py $ARGS > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"
pass() {  # name counters...
  local name=$1; shift
  echo "[collect] pmc $name: $*"
  timeout -s KILL 200 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
      python3 bench.py $ARGS > "$OUT/$name.json" 2> "$OUT/$name.err"
}
pass pmc_sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU
pass pmc_wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH GRBM_GUI_ACTIVE
pass pmc_fetch FETCH_SIZE
pass pmc_write WRITE_SIZE
echo "[collect] done"
