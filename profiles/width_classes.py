"""Static operand widths of the synthetic bench's ops (width-class handlers).

For every op in a state's root cone, an upper bound on the significant bits of its operands
from the DAG alone (VAR / UF 256, CONST its bit length, ADD max + 1, MUL sum, AND min, OR / XOR
max, UDIV a, UREM min, ITE max of branches, EXTRACT / CONCAT their width, ZEXT its operand,
everything else its width), as limbs (1..8) of the wider operand.  A translator could pick a
k-limb handler only where this bound is below 8 limbs.

    python3 profiles/width_classes.py [n_states]
"""
import collections
import re
import sys
import os

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mythril_amd import _native as N  # noqa: E402

OPS = {}
for line in open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "include", "mgp_ir.h")):
    m = re.match(r"\s*MGP_OP_(\w+)\s*=\s*(\d+)", line)
    if m:
        OPS[int(m.group(2))] = m.group(1)
ARITH = ("ADD", "SUB", "MUL", "UDIV", "UREM", "SDIV", "SREM", "AND", "OR", "XOR", "NOT", "SHL", "LSHR", "ASHR",
         "EQ", "ULT", "ULE", "SLT", "ITE")


def bitlen(v):
    for i in range(7, -1, -1):
        if v[i]:
            return 32 * i + int(v[i]).bit_length()
    return 0


def main(n_states=3000):
    b = N.synth_generate(1234, 0, n_states, 64, 256)
    nodes, off, consts, coff = b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"]
    by = collections.Counter()
    tot = collections.Counter()
    for s in range(n_states):
        nd = nodes[int(off[s]):int(off[s + 1])]
        cs = consts[int(coff[s]):int(coff[s + 1])]
        n = len(nd)
        live = np.zeros(n, bool)
        live[n - 1] = True
        for i in range(n - 1, -1, -1):
            if live[i]:
                for f in ("a", "b", "c"):
                    j = int(nd[i][f])
                    if j >= 0:
                        live[j] = True
        bits = [256] * n
        for i in range(n):
            x = nd[i]
            op, w = OPS.get(int(x["op"]), "?"), int(x["width"])
            A = bits[int(x["a"])] if x["a"] >= 0 else 0
            B = bits[int(x["b"])] if x["b"] >= 0 else 0
            C = bits[int(x["c"])] if x["c"] >= 0 else 0
            r = {"VAR": w, "CONST": bitlen(cs[int(x["p0"])]) if op == "CONST" else 0, "ADD": min(w, max(A, B) + 1),
                 "MUL": min(w, A + B), "UDIV": A, "UREM": min(A, B), "AND": min(A, B), "OR": max(A, B),
                 "XOR": max(A, B), "ITE": max(B, C), "EXTRACT": w, "CONCAT": w, "ZEXT": A}.get(op, w if w else 1)
            bits[i] = r
            if live[i] and op in ARITH:
                tot[op] += 1
                by[(op, min(8, max(1, (max(A, B) + 31) // 32)))] += 1
    all_ops = sum(tot.values())
    full = sum(by[(op, 8)] for op in tot)
    print(f"{n_states} synthetic states, {all_ops} ops in root cones: {full / all_ops:.3f} have an 8-limb operand")
    for op in sorted(tot):
        print(f"  {op:5s} {tot[op]:6d}  8 limbs {by[(op, 8)] / tot[op]:.3f}  "
              + " ".join(f"{k}:{by[(op, k)]}" for k in range(1, 8) if by[(op, k)]))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3000)
