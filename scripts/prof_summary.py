#!/usr/bin/env python3
"""Summarise a rocprofv3 run_results.db (kernel-trace) into a per-kernel table.

    python scripts/prof_summary.py gpurun_out/prof_hip/run_results.db [--top 40] [--md out.md]
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--md", default=None)
    ap.add_argument("--width", type=int, default=90)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = defaultdict(lambda: [0, 0.0])
    tot = 0.0
    for name, s, e in rows:
        d = (e - s) / 1e6  # ns -> ms
        agg[name][0] += 1
        agg[name][1] += d
        tot += d
    items = sorted(agg.items(), key=lambda kv: -kv[1][1])
    lines = [f"total GPU kernel time: {tot:.2f} ms over {len(rows)} dispatches, {len(agg)} distinct kernels", "",
             "| % | total ms | calls | avg us | kernel |", "|---:|---:|---:|---:|---|"]
    for name, (n, ms) in items[: a.top]:
        nm = name if len(name) <= a.width else name[: a.width] + "..."
        lines.append(f"| {100 * ms / tot:.1f} | {ms:.2f} | {n} | {1000 * ms / n:.1f} | `{nm}` |")
    out = "\n".join(lines)
    print(out)
    if a.md:
        open(a.md, "w").write(out + "\n")


if __name__ == "__main__":
    main()
