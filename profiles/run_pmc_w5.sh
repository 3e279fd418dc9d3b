#!/bin/bash
# Cache / stall counters of the interpreter with and without the 5-wave descriptor
# (MGP_W5_MAX_SLOTS=4 vs -1), separate PMC passes:  bash profiles/run_pmc_w5.sh <tag>
# (measured on commit a4ff032, which had the 96-VGPR descriptor and the knob; the 10-position
# register bank that followed needs all 128 VGPRs, so later trees ignore MGP_W5_MAX_SLOTS)
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${1:-w5}
mkdir -p $OUT
ARGS="--states 262144 --steps 2 --warmup 1 --keccak 0 --no-cpu --refute-sample 0 --frontend 0 --guided-sample 0"
p() { local n=$1; shift; echo "[pmc] $n: $*"; timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$n -o run --output-format csv -- python3 bench.py $ARGS > $OUT/$n.json 2> $OUT/$n.err; }
for w in 4 -1; do
  export MGP_W5_MAX_SLOTS=$w
  p ic_$w SQC_ICACHE_HITS SQC_ICACHE_MISSES
  p dc_$w SQC_DCACHE_HITS SQC_DCACHE_MISSES
  p act_$w SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAVES
done
python3 - $OUT <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
for sub in sorted(os.listdir(d)):
    fs = glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        continue
    agg = defaultdict(float)
    for f in fs:
        for r in csv.DictReader(open(f)):
            if "mgp_eval_gfx950" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(sub, {k: "%.4g" % v for k, v in sorted(agg.items())})
PY
