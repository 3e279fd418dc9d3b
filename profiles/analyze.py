#!/usr/bin/env python3
"""Summarise a profiles/collect.sh run: per-kernel trace stats + PMC counters.

    python profiles/analyze.py gpurun_out/prof_<tag> > profiles/<tag>_summary.md
"""
import csv
import json
import os
import sys
from collections import defaultdict


KECCAK64 = ("mgp_keccak64_gfx950", "mgp_keccak64_kernel")  # hand-allocated asm / compiler-allocated HIP


def short(name):
    return name.split("(")[0].replace("void ", "").split("<")[0]


def main(d):
    out = []
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    out.append(f"# rocprofv3 summary: {d}\n")
    out.append("## kernel trace (--kernel-trace --stats)\n")
    out.append("| kernel | calls | total ms | avg us | % |")
    out.append("|---|---|---|---|---|")
    with open(stats) as f:
        for r in csv.DictReader(f):
            out.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.3f} | "
                       f"{float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
    # per-dispatch durations of the eval kernel grouped into steps
    tr = os.path.join(d, "trace", "run_kernel_trace.csv")
    evals, kcalls = [], []
    with open(tr) as f:
        for r in csv.DictReader(f):
            if short(r["Kernel_Name"]) in KECCAK64:
                kcalls.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            if short(r["Kernel_Name"]) in ("mgp_eval_kernel", "mgp_eval_gfx950", "mgp_finalize_kernel"):
                evals.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    evals.sort()
    steps, cur = [], []
    for s, e, n in evals:
        cur.append((s, e))
        if n == "mgp_finalize_kernel":
            steps.append((cur[0][0], cur[-1][1], sum(b - a for a, b in cur)))
            cur = []
    if steps:
        out.append("\n## eval step (all bucket launches + finalize)\n")
        out.append("| step | wall us (first start -> last end) | sum of kernel durations us |")
        out.append("|---|---|---|")
        for i, (a, b, busy) in enumerate(steps):
            out.append(f"| {i} | {(b - a)/1e3:.1f} | {busy/1e3:.1f} |")
    # counters
    agg = defaultdict(lambda: defaultdict(float))
    meta = {}
    for sub in sorted(os.listdir(d)):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        with open(p) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                meta[k] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"])
    out.append("\n## PMC counters (summed over dispatches; separate passes)\n")
    traffic = {}
    n_steps = max(1, sum(1 for e in evals if e[2] == "mgp_finalize_kernel"))
    for k in ("mgp_eval_gfx950", "mgp_eval_kernel") + KECCAK64 + ("mgp_valu_probe_kernel",):
        if k not in agg:
            continue
        c = agg[k]
        v, sg, lds, scr = meta[k]
        # rocprofv3's VGPR_Count decodes the descriptor's granulated count with a granule of 4;
        # gfx950 allocates arch VGPRs in granules of 8, so the field reads half the allocation
        # (mgp_eval_gfx950 declares .amdhsa_next_free_vgpr 128 and reads as 64)
        out.append(f"### {k}  (VGPR {2 * int(float(v))} allocated = rocprof VGPR_Count {v} x 2, SGPR {sg}, "
                   f"LDS {lds} B, scratch {scr})\n")
        out.append("| counter | value |")
        out.append("|---|---|")
        for n in sorted(c):
            out.append(f"| {n} | {c[n]:.4g} |")
        der = {}
        if c.get("SQ_WAVES"):
            der["VALU insts / wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
            der["SALU insts / wave"] = c.get("SQ_INSTS_SALU", 0) / c["SQ_WAVES"]
            der["LDS insts / wave"] = c.get("SQ_INSTS_LDS", 0) / c["SQ_WAVES"]
            der["SMEM insts / wave"] = c.get("SQ_INSTS_SMEM", 0) / c["SQ_WAVES"]
        if c.get("SQ_WAVE_CYCLES"):
            der["VALU active / wave-cycles"] = c.get("SQ_ACTIVE_INST_VALU", 0) / c["SQ_WAVE_CYCLES"]
            tot = c.get("SQ_WAIT_ANY", 0) + c.get("SQ_WAIT_INST_ANY", 0) + c.get("SQ_ACTIVE_INST_ANY", 0)
            if tot:
                der["wait_any share"] = c.get("SQ_WAIT_ANY", 0) / tot
                der["wait_inst_any share"] = c.get("SQ_WAIT_INST_ANY", 0) / tot
                der["active_inst_any share"] = c.get("SQ_ACTIVE_INST_ANY", 0) / tot
        if "FETCH_SIZE" in c:
            der["FETCH_SIZE KB (raw, all dispatches)"] = c["FETCH_SIZE"]
        if k in ("mgp_eval_gfx950", "mgp_eval_kernel") and "FETCH_SIZE" in c:
            # per eval step (all bucket dispatches of one step); FETCH_SIZE doubled for 16-B/lane
            # streaming reads (MI355X_MICROARCH.md, HBM section), WRITE_SIZE read as-is
            fetch = 2 * c["FETCH_SIZE"] * 1024 / n_steps
            write = c.get("WRITE_SIZE", 0) * 1024 / n_steps
            der["HBM bytes per eval step (2 x FETCH_SIZE + WRITE_SIZE)"] = fetch + write
            traffic[k] = {"fetch_bytes_per_step": fetch, "write_bytes_per_step": write,
                          "hbm_bytes_per_launch": fetch + write, "steps_in_profile": n_steps}
            if c.get("SQ_INSTS_VALU"):
                # issued VALU wave-instructions per step (x 64 lanes = lane-ops, overhead included)
                traffic[k]["valu_wave_insts_per_step"] = c["SQ_INSTS_VALU"] / n_steps
                traffic[k]["salu_insts_per_step"] = c.get("SQ_INSTS_SALU", 0) / n_steps
                # against the INT32 VALU spec peak (256 CU x 4 SIMD-32 x 2.4 GHz = 78.6 Tops/s),
                # over the traced run's average eval launch time
                try:
                    bl = json.load(open(os.path.join(d, "bench_trace.json")))
                    launch_s = bl["roofline"]["launch_ms"] * 1e-3
                    issued = c["SQ_INSTS_VALU"] / n_steps * 64 / launch_s / 1e12
                    der["issued VALU lane-ops/s (Tops/s, over the launch time)"] = issued
                    der["issued VALU / 78.64 Tops/s spec peak"] = issued / 78.6432
                    der["nominal ops/s (Tops/s, bench roofline.achieved)"] = bl["roofline"]["achieved"]
                    der["nominal / 78.64 Tops/s spec peak"] = bl["roofline"]["achieved"] / 78.6432
                except (OSError, ValueError, KeyError):
                    pass
        if k in KECCAK64 and c.get("SQ_WAVES"):
            # one preimage per lane: per-hash figures are per-wave counts / 64
            ncalls = sum(1 for _ in kcalls)
            traffic[k] = {"valu_lane_ops_per_hash": c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"],
                          "hbm_bytes_per_hash": (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024
                          / (64 * c["SQ_WAVES"]) if "FETCH_SIZE" in c else None,
                          "dispatches": ncalls}
            der["VALU lane-ops / hash"] = traffic[k]["valu_lane_ops_per_hash"]
            if traffic[k]["hbm_bytes_per_hash"] is not None:
                der["HBM bytes / hash (2 x FETCH_SIZE + WRITE_SIZE)"] = traffic[k]["hbm_bytes_per_hash"]
        if der:
            out.append("\nderived:\n")
            for n, val in der.items():
                out.append(f"- {n}: {val:.4g}")
        out.append("")
    print("\n".join(out))
    # machine-readable traffic figure for bench.py's roofline.traffic (same workload shape only)
    bj = os.path.join(d, "bench_trace.json")
    keccak_done = False
    for k, t in traffic.items():
        if k in KECCAK64:
            # the bench's default engine (the hand-allocated kernel) when the run had both
            if keccak_done or (k != KECCAK64[0] and KECCAK64[0] in traffic):
                continue
            keccak_done = True
            t.update({"kernel": k, "source": f"profiles/{os.path.basename(os.path.normpath(d)).replace('prof_', '')}"
                      f"_summary.md (rocprofv3 run {d})"})
            with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "keccak_pmc.json"), "w") as f:
                json.dump(t, f, indent=1)
            continue
        try:
            cfg = json.load(open(bj))["config"]
            tag = os.path.basename(os.path.normpath(d)).replace("prof_", "")
            t.update({"kernel": k, "states": cfg["states_per_gpu"], "cand": cfg["candidates"],
                      "source": f"profiles/{tag}_summary.md (rocprofv3 run {d})"})
            with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "eval_pmc.json"), "w") as f:
                json.dump(t, f, indent=1)
        except (OSError, ValueError, KeyError):
            pass


if __name__ == "__main__":
    main(sys.argv[1])
