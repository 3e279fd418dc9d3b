# Front-end GPU check: the front-end / determinism GPU tests, then the bench's front-end section
# on a small eval batch (no Keccak, CPU baseline, suite or sweeps).
set -e
mkdir -p gpurun_out
tag=${1:-fe2}
timeout -k 10 300 python -u -m pytest tests/test_gpu_front.py tests/test_gpu_determinism.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 300 python -u bench.py --states 65536 --steps 2 --warmup 1 --keccak 0 --no-cpu --refute-sample 0 --suite 0 --suite-open-sweep 0 --div-split 0 --guided-sample 0 --detail gpurun_out/${tag}_detail.json > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python - <<PY
import json
d = json.load(open("gpurun_out/${tag}_detail.json"))["frontend"]
print("default", round(d["seconds"]*1e3,1), d["calls_seconds"], {k: round(v,1) if isinstance(v,float) else v for k,v in d["stages_ms"].items() if not isinstance(v, dict)})
for k, v in d.get("min_groups", {}).items():
    print("min_groups", k, round(v["seconds"]*1e3,1), v["calls_seconds"], v["same_answers"])
print("cand_cap_x4", round(d["cand_cap_x4"]["seconds"]*1e3,1), "pipelines2", round(d["pipelines2"]["seconds"]*1e3,1))
print("latency", [(r["states"], round(r["ms_per_call"],2)) for r in d["latency"]])
PY
