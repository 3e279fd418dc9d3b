#!/bin/bash
# instruction-cache / issue-stall counters of the interpreter (separate PMC passes)
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${1:-ic}
mkdir -p $OUT
ARGS="--states 262144 --steps 2 --warmup 1 --keccak 0 --no-cpu"
p() { local n=$1; shift; echo "[pmc] $n: $*"; timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$n -o run --output-format csv -- python3 bench.py $ARGS > $OUT/$n.json 2> $OUT/$n.err; }
p ic SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE
p act SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC
p ins SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_IFETCH SQ_BUSY_CYCLES
echo done
