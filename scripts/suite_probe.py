"""Run the 13-contract suite (corpus.suite) through the product Prefilter on cuda:0 and
write the accounting plus the labels of undecided / contradicted queries (for study).

usage: python scripts/suite_probe.py OUT.json [contract ...]"""
import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import corpus  # noqa: E402
from mythril_amd import solver as SV  # noqa: E402


def main():
    out = sys.argv[1]
    only = set(sys.argv[2:]) or None
    t = time.perf_counter()
    qs = corpus.suite(contracts=only)
    gen = time.perf_counter() - t
    pf = SV.Prefilter(0)
    pf.check_states([list(q[3]) for q in qs[:64]])
    SV.unsat_cores().reset()
    pf._N.program_cache_clear()
    t = time.perf_counter()
    answers, wits = corpus.answer(pf, qs)
    dt = time.perf_counter() - t
    acc = corpus.account(qs, answers)
    und = collections.Counter()
    bad = []
    for q, a, w in zip(qs, answers, wits):
        if a == "undecided":
            und[(q[1], q[2].split("@")[0].split(":T")[0].split(":F")[0], q[4])] += 1
        if (q[4] == "unsat" and a == "sat") or (q[4] == "sat" and a == "unsat"):
            bad.append((q[1], q[2], q[4], a, {k: hex(v) for k, v in (w or {}).items()} if len(bad) < 8 else None))
    rep = dict(acc, generate_s=gen, seconds=dt, queries=len(qs),
               undecided=[[list(k), v] for k, v in und.most_common()], contradictions=bad)
    json.dump(rep, open(out, "w"), indent=1)
    print(json.dumps({"all": acc["all"], "held_out": acc["held_out"], "seconds": dt}))


if __name__ == "__main__":
    main()
