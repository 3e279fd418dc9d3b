# One GPU call: the front-end section of the bench alone (mixed 1 024-state corpus).
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --keccak 0 --suite 0 --no-cpu --div-split 0 --refute-sample 0 --guided-sample 0 > gpurun_out/fe_r4d.json 2> gpurun_out/fe_r4d.err || { echo "bench failed"; tail -20 gpurun_out/fe_r4d.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/fe_r4d.json").read().strip().splitlines()[-1])
f = d["frontend"]
print("states/s", round(f["states_per_s"]), "s", round(f["seconds"], 3), "undecided", f["undecided"])
print("stages", json.dumps(f["stages_ms"]))
print("lat2", {k: round(v[0]["ms_per_call"], 2) for k, v in f["latency_2_by_contract"].items()})
for k in ("first_round_only", "core_async", "cand_cap_x4", "cand_cap_default"):
    print(k, round(f[k]["states_per_s"]))
PY
