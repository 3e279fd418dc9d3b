#!/usr/bin/env python3
"""Uop mix of the bench workload (CPU only, diagnostic).

Lowers a sample of bench.py's synthetic states and counts the executed uops by
(first handler, op handler) — uop programs are straight-line, so the static count
is the per-wave dynamic count.   python profiles/uop_mix.py [--states 4096]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import _native as N  # noqa: E402
from oracle import uop_ref as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--states", type=int, default=4096)
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    b = N.synth_generate(20240601, 0, args.states, args.nodes, 256)
    words, po, status = N.lower(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
    names = R._names()
    pairs, firsts, ops = collections.Counter(), collections.Counter(), collections.Counter()
    total = 0
    for s in range(args.states):
        if status[s]:
            continue
        u0 = R.uop_offset(words, int(po[s]))
        n = int(words[u0])
        for k in range(n):
            w0 = int(words[u0 + 4 + 4 * k])
            f, o = names[w0 & 0xFFFF], names[w0 >> 16]
            if not f.startswith("F_"):
                o = f
                f = "-"
            pairs[(f, o)] += 1
            firsts[f] += 1
            ops[o] += 1
            total += 1
    print(f"{args.states} states, {total / args.states:.1f} uops/state")
    for title, c in (("op", ops), ("first", firsts), ("pair", pairs)):
        print(f"\n## by {title}")
        for k, v in c.most_common(args.top):
            print(f"{v / args.states:8.2f} /state  {100 * v / total:5.1f}%  {k}")


if __name__ == "__main__":
    main()
