#!/bin/bash
# quick A/B: parity subset + short bench + one SQ counter pass (outputs under gpurun_out/quick_<tag>/)
set -euo pipefail
TAG=${1:-q}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/quick_${TAG}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
tail -2 "$OUT/tests.log"
timeout -k 10 300 python -u bench.py --states ${QS:-262144} --steps 5 --warmup 2 --keccak 0 --no-cpu > "$OUT/bench.json" 2> "$OUT/bench.err"
grep "kernel" "$OUT/bench.err" || true
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
   -d "$OUT/pmc_sq" -o run --output-format csv -- python3 bench.py --states ${QS:-262144} --steps 2 --warmup 1 --keccak 0 --no-cpu > /dev/null 2> "$OUT/pmc.err"
python3 - "$OUT" <<'PY'
import csv, sys, os
from collections import defaultdict
d = sys.argv[1]
agg = defaultdict(float)
for r in csv.DictReader(open(os.path.join(d, "pmc_sq", "run_counter_collection.csv"))):
    if "mgp_eval_kernel" in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
w = agg["SQ_WAVES"]
print({k: round(v / w, 1) for k, v in agg.items()}, "waves", w)
PY
