#!/usr/bin/env python3
"""Per-handler cost table of the evaluation kernel (GPU, diagnostic).

For each op class, S identical states run a chain  t_i = op(t_{i-1}, x1)
of K uops over 256 candidates; the time per uop (minus a K=0 baseline)
is converted to SIMD-cycles per wave-uop:
    cycles = dt * clock * (256 CUs * 4 SIMDs) / (waves * K)
i.e. the SIMD time one wave's uop costs when the chip is full.  The ideal for a
VALU-bound handler is 2 cycles per VALU instruction (wave64 on a SIMD-32).

    python profiles/uop_costs.py [--engine asm|hip] [--states 65536] [--k 32]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import _native as N  # noqa: E402
from oracle import bvsem as S  # noqa: E402

CLOCK = 2.4e9
SIMDS = 256 * 4


def chain(op, k, width=256, bkind="var", store_every=0):
    """x0, x1 vars; t = x0; t = op(t, x1) k times; root = (t == x0) | (x1 == t)."""
    nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0]]
    consts = []
    if bkind == "const":
        consts = [0x1234567 if op not in (S.SHL, S.LSHR, S.ASHR) else 37]
        nl.append([S.CONST, 256, -1, -1, -1, 0, 0])
        b = 2
    else:
        b = 1
    t = 0
    if op == "FIB":   # t_i = t_{i-1} + t_{i-2}: B from an LDS slot, every result stored
        prev = 1
        for i in range(k):
            nl.append([S.ADD, 256, t, prev, -1, 0, 0])
            prev, t = t, len(nl) - 1
        nl.append([S.EQ, 1, t, 0, -1, 0, 0])
        nl.append([S.EQ, 1, 1, t, -1, 0, 0])
        nl.append([S.BOR, 1, len(nl) - 2, len(nl) - 1, -1, 0, 0])
        return nl, consts
    if op == "BAND":  # Bool chain: c = (x0 < x1); b_i = b_{i-1} & c  (SALU-only uops)
        nl.append([S.ULT, 1, 0, 1, -1, 0, 0])
        c = b = len(nl) - 1
        for i in range(k):
            nl.append([S.BOR if i % 2 else S.BAND, 1, b, c, -1, 0, 0])
            b = len(nl) - 1
        nl.append([S.EQ, 1, 0, 1, -1, 0, 0])
        nl.append([S.BOR, 1, b, len(nl) - 1, -1, 0, 0])
        return nl, consts
    if op == "MIX4":  # four cheap ops in rotation (handler switching on every uop)
        for i in range(k):
            nl.append([(S.ADD, S.XOR, S.SUB, S.OR)[i % 4], 256, t, b, -1, 0, 0])
            t = len(nl) - 1
        nl.append([S.EQ, 1, t, 0, -1, 0, 0])
        nl.append([S.EQ, 1, 1, t, -1, 0, 0])
        nl.append([S.BOR, 1, len(nl) - 2, len(nl) - 1, -1, 0, 0])
        return nl, consts
    for i in range(k):
        if op in (S.EQ, S.ULT, S.SLT):
            c = len(nl)
            nl.append([op, 1, t, b, -1, 0, 0])
            nl.append([S.ITE, 256, c, t, b, 0, 0])
        elif op == S.ITE:
            c = len(nl)
            nl.append([S.ULT, 1, b, 0, -1, 0, 0])
            nl.append([S.ITE, 256, c, t, b, 0, 0])
        elif op == S.EXTRACT:
            nl.append([S.EXTRACT, 128, t, -1, -1, 191, 64])
            nl.append([S.ZEXT, 256, len(nl) - 1, -1, -1, 0, 0])
        else:
            nl.append([op, 256, t, b, -1, 0, 0])
        t = len(nl) - 1
    nl.append([S.EQ, 1, t, 0, -1, 0, 0])
    nl.append([S.EQ, 1, 1, t, -1, 0, 0])
    nl.append([S.BOR, 1, len(nl) - 2, len(nl) - 1, -1, 0, 0])
    return nl, consts


def run(nl, consts, n_states, n_cand, torch, dev, stream, sh):
    from tests._util import pack_states

    nodes, noff, cs, coff = pack_states([(nl, consts)] * n_states)
    words, po, status = N.lower(nodes, noff, cs, coff)
    assert (status == 0).all()
    hdr = N.program_headers(words, po)
    n_vars = 2
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    d_words = torch.from_numpy(words.view(np.int32)).to(dev)
    d_po = torch.from_numpy(po.view(np.int64)).to(dev)
    d_cands = torch.empty(n_states * n_vars * 2 * n_cand * 4, dtype=torch.int32, device=dev)
    N.fill_candidates_dev(vp(d_words), vp(d_po), n_states, 0, 7, vp(d_cands), n_cand, n_vars, sh)
    n_chunks = (n_cand + 63) // 64
    d_first = torch.empty(n_states, dtype=torch.int32, device=dev)
    d_wit = torch.empty(n_states * n_vars * 8, dtype=torch.int32, device=dev)
    d_scratch = torch.empty(n_states * n_chunks, dtype=torch.int32, device=dev)
    slots = int(hdr[:, 2].max())

    def step():
        N.eval_batch_dev(vp(d_words), vp(d_po), n_states, vp(d_cands), n_cand, n_vars, slots, vp(d_first),
                         vp(d_wit), vp(d_scratch), sh)

    for _ in range(2):
        step()
    torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(5):
        step()
    b.record(stream)
    torch.cuda.synchronize(dev)
    return a.elapsed_time(b) / 5 * 1e-3, int(hdr[0, 0]), slots


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engine", default=None)
    ap.add_argument("--states", type=int, default=65536)
    ap.add_argument("--k", type=int, default=32)
    args = ap.parse_args()
    import torch

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)
    eng = N.set_eval_engine(args.engine)
    n_cand = 256
    waves = args.states * (n_cand // 64)
    base_t, _, _ = run(*chain(S.ADD, 0), args.states, n_cand, torch, dev, stream, sh)
    rows = []
    cases = [("MIX4 var", "MIX4", "var"), ("FIB slot+st", "FIB", "var"), ("BAND/BOR", "BAND", "var"), ("ADD var", S.ADD, "var"), ("ADD const", S.ADD, "const"), ("SUB var", S.SUB, "var"),
             ("XOR var", S.XOR, "var"), ("MUL var", S.MUL, "var"), ("UDIV var", S.UDIV, "var"),
             ("UREM var", S.UREM, "var"), ("SDIV var", S.SDIV, "var"),
             ("SHL var", S.SHL, "var"), ("LSHR const", S.LSHR, "const"),
             ("EXTRACT", S.EXTRACT, "var"), ("EQ+ITE var", S.EQ, "var"), ("ULT+ITE var", S.ULT, "var"),
             ("ITE(ULT) var", S.ITE, "var")]
    for name, op, bk in cases:
        nl, consts = chain(op, args.k, bkind=bk)
        t, n_ins, slots = run(nl, consts, args.states, n_cand, torch, dev, stream, sh)
        per_chain = args.k * (2 if op in (S.EQ, S.ULT, S.SLT, S.ITE) else 1)
        cyc = (t - base_t) * CLOCK * SIMDS / (waves * per_chain)
        rows.append({"case": name, "ms": t * 1e3, "v1_ins": n_ins, "slots": slots,
                     "simd_cycles_per_uop": cyc})
        print(f"{name:14s} {t * 1e3:8.3f} ms  ins {n_ins:4d} slots {slots:2d}  {cyc:8.1f} SIMD-cycles/uop",
              flush=True)
    print(json.dumps({"engine": eng, "states": args.states, "k": args.k, "baseline_ms": base_t * 1e3,
                      "rows": rows}))


if __name__ == "__main__":
    main()
