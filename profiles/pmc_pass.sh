#!/bin/bash
# One PMC pass of a short eval-only bench (diagnostic A/B):
#   COUNTERS="SQ_WAVES ..." bash profiles/pmc_pass.sh <tag>   -> gpurun_out/pmc_<tag>/
# Prints the per-wave value of every counter over the mgp_eval_gfx950 dispatches.
set -euo pipefail
TAG=${1:-a}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
ARGS="--states ${PROF_STATES:-262144} --steps 2 --warmup 1 --keccak 0 --no-cpu --refute-sample 0 --frontend 0 --suite 0 --suite-open-sweep 0 --div-split 0 --guided-sample 0"
timeout -s KILL 150 rocprofv3 --pmc $COUNTERS -d "$OUT/pmc" -o run --output-format csv -- \
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
print({k: round(v / w, 2) for k, v in sorted(agg.items())}, "waves", w)
PY
