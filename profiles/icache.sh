#!/bin/bash
# Instruction-fetch counters of the interpreter (diagnostic): lists the box's counters,
# keeps the SQ/SQC instruction-cache ones that exist, and runs one PMC pass of a short
# bench (outputs under gpurun_out/icache_<tag>/).
set -euo pipefail
TAG=${1:-a}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/icache_${TAG}
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
WANT="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_VALU SQ_WAVES SQ_WAIT_INST_ANY"
HAVE=""
for c in $WANT; do
  if grep -qw "$c" "$OUT/avail.txt"; then HAVE="$HAVE $c"; fi
done
echo "[icache] counters:$HAVE"
ARGS="--states ${PROF_STATES:-262144} --steps 2 --warmup 1 --keccak 0 --no-cpu --refute-sample 0 --frontend 0"
timeout -s KILL 150 rocprofv3 --pmc $HAVE -d "$OUT/pmc" -o run --output-format csv -- \
    python3 bench.py $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 - "$OUT" <<'PY'
import csv, sys, os, glob
from collections import defaultdict
d = sys.argv[1]
agg = defaultdict(float)
for f in glob.glob(os.path.join(d, "pmc", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "mgp_eval_gfx950" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
w = agg.get("SQ_WAVES", 1.0)
print({k: (v, round(v / w, 2)) for k, v in sorted(agg.items())}, "waves", w)
PY
