#!/usr/bin/env python3
"""Kernel statistics (the --stats table) from a rocprofv3 SQLite output (rocpd schema).

    python3 profiles/db_stats.py <prof_results.db> [round-tag]

This rocprofv3 writes its kernel trace to a rocpd SQLite database unless
--output-format csv is given; this reads the dispatch table and prints a markdown
table: calls, total ms, average us and share per kernel, plus the per-step wall time of
the eval kernel's bucket launches when their start times cluster into steps.
"""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    tag = sys.argv[2] if len(sys.argv) > 2 else ""
    c = sqlite3.connect(db)
    names = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    vgpr = {r[0]: (r[1], r[2], r[3]) for r in c.execute(
        "select id, arch_vgpr_count, accum_vgpr_count, sgpr_count from rocpd_info_kernel_symbol")}
    rows = list(c.execute("select kernel_id, start, end from rocpd_kernel_dispatch order by start"))
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for k, s, e in rows:
        tot[k] += (e - s) / 1e6
        cnt[k] += 1
    all_ms = sum(tot.values())
    print(f"# rocprofv3 kernel trace{(' — ' + tag) if tag else ''}\n")
    print("| kernel | calls | total ms | avg us | % | arch VGPR / AGPR / SGPR |")
    print("|---|---|---|---|---|---|")
    for k in sorted(tot, key=lambda k: -tot[k]):
        name = names.get(k, str(k)).split("(")[0]
        v = vgpr.get(k, ("", "", ""))
        print(f"| {name} | {cnt[k]} | {tot[k]:.3f} | {1e3 * tot[k] / cnt[k]:.1f} | {100 * tot[k] / all_ms:.1f} | "
              f"{v[0]} / {v[1]} / {v[2]} |")
    # eval steps: consecutive mgp_eval_gfx950 launches closer than 2 ms belong to one step
    ev = [(s, e) for k, s, e in rows if names.get(k, "").startswith("mgp_eval_gfx950")]
    steps, cur = [], []
    for s, e in ev:
        if cur and s - cur[-1][1] > 2e6:
            steps.append(cur)
            cur = []
        cur.append((s, e))
    if cur:
        steps.append(cur)
    if steps:
        print("\n| eval step | launches | wall us (first start -> last end) | sum of durations us |")
        print("|---|---|---|---|")
        for i, st in enumerate(steps):
            print(f"| {i} | {len(st)} | {(st[-1][1] - st[0][0]) / 1e3:.1f} | {sum(e - s for s, e in st) / 1e3:.1f} |")


if __name__ == "__main__":
    main()
