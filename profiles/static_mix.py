#!/usr/bin/env python3
"""Static instruction mix per executed uop (CPU only, diagnostic).

Walks each handler of the generated kernel along its fall-through path (forward
branches into out-of-line blocks are not taken, conditional skips inside a handler
are taken when they jump forward within it — i.e. the common path), classifies
the instructions, and weights them by the bench workload's uop mix
(profiles/uop_mix.py) to estimate SALU / VALU / LDS instructions per wave.
    python profiles/static_mix.py [kernel.s]
"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def classify(op):
    if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return "VALU"
    if op.startswith("v_"):
        return "VALU"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "VMEM"
    if op.startswith(("s_load", "s_buffer_load")):
        return "SMEM"
    if op.startswith(("s_setpc", "s_branch", "s_cbranch", "s_swappc")):
        return "BR"
    if op.startswith(("s_waitcnt", "s_nop")):
        return "WAIT"
    if op.startswith("s_"):
        return "SALU"
    return None


# SIMD-cycles of VALU issue per wave64 instruction at 4 waves/SIMD (profiles/valu_mix_r1.json,
# profiles/contention_r2.json); f64 ops and cndmask are assumed, not measured
_QUARTER = ("v_alignbit", "v_alignbyte", "v_perm", "v_lshl_or", "v_lshl_add", "v_mad_u64", "v_fma_f64",
            "v_cvt_f64", "v_cvt_u32_f64", "v_rcp_f64")
_CARRY = ("v_add_co", "v_addc_co", "v_sub_co", "v_subb_co", "v_subrev_co", "v_subbrev_co")


def valu_cost(op):
    if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return 8.7
    if op.startswith(_CARRY):
        return 4.5
    if op.startswith(_QUARTER):
        return 4.0
    return 2.0 if op.startswith("v_") else 0.0


def handler_paths(lines):
    """handler name -> Counter of instruction classes along the fall-through path."""
    out = {}
    cur = None
    for l in lines:
        m = re.match(r"^mgp_h_(\w+):", l)
        if m:
            cur = m.group(1)
            out[cur] = collections.Counter()
            done = False
            continue
        if cur is None or done:
            continue
        t = l.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        c = classify(op)
        if c:
            out[cur][c] += 1
        out[cur]["COST"] += valu_cost(op)
        if op.startswith("s_setpc") or op == "s_endpgm":
            done = True
    return out


def main():
    s = sys.argv[1] if len(sys.argv) > 1 else "/tmp/_mix.s"
    if len(sys.argv) == 1:
        subprocess.run([sys.executable, os.path.join(ROOT, "mythril_amd/csrc/gen_eval_asm.py"), s, "/tmp/_mix.h"],
                       check=True)
    paths = handler_paths(open(s).read().splitlines())
    from mythril_amd import _native as N
    from oracle import uop_ref as R
    b = N.synth_generate(0x4D595448, 0, 2048, 64, 256)
    words, po, status = N.lower(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
    names = R._names()
    tot = collections.Counter()
    per = collections.Counter()
    n = 0
    for st in range(2048):
        u0 = R.uop_offset(words, int(po[st]))
        for k in range(int(words[u0])):
            w0 = int(words[u0 + 4 + 4 * k])
            f, o = names[w0 & 0xFFFF], names[w0 >> 16]
            hs = [f, o] if f.startswith("F_") else [f]
            for h in hs:
                tot.update(paths[h])
                per[h] += 1
        n += 1
    print("per wave (fall-through paths; DIV digits not counted):")
    for k in ("VALU", "SALU", "BR", "WAIT", "LDS", "VMEM", "SMEM"):
        print(f"  {k:5s} {tot[k] / n:8.1f}")
    print(f"  VALU SIMD-cycle estimate {tot['COST'] / n:8.1f}")
    print("\ntop handlers by estimated VALU SIMD-cycles per wave:")
    cc = {h: per[h] * paths[h]["COST"] / n for h in per}
    for h, c in sorted(cc.items(), key=lambda x: -x[1])[:30]:
        print(f"  {h:18s} x{per[h] / n:5.2f}  cost {paths[h]['COST']:6.1f} -> {c:6.1f}")
    print("\ntop handlers by SALU+VALU contribution per wave:")
    contrib = {h: per[h] * (paths[h]["SALU"] + paths[h]["VALU"] + paths[h]["BR"]) / n for h in per}
    for h, c in sorted(contrib.items(), key=lambda x: -x[1])[:25]:
        p = paths[h]
        print(f"  {h:18s} x{per[h] / n:5.2f}  VALU {p['VALU']:3d} SALU {p['SALU']:3d} BR {p['BR']} LDS {p['LDS']}  -> {c:6.1f}")


if __name__ == "__main__":
    main()
