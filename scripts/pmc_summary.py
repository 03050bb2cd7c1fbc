#!/usr/bin/env python3
"""Aggregate a rocprofv3 ``--pmc ... --output-format csv`` run per kernel name:
MFMA utilisation (SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE/8 x 1024 SIMDs), wave-cycle
split (active / wait-inst / wait-any) and per-kernel totals.  Usage: pmc_summary.py DIR [--md OUT]"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    agg = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r.get("Kernel_Name", "?")
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                calls[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    rows = []
    for k, c in agg.items():
        act = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        util = mf / (act * 1024) if act else 0.0
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        rows.append((act, k, len(calls[k]), util, c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                     c.get("SQ_WAIT_INST_ANY", 0) / wc, c.get("SQ_WAIT_ANY", 0) / wc,
                     c.get("SQ_INSTS_MFMA", 0), c.get("SQ_INSTS_VALU", 0)))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows) or 1.0
    tot_mf = sum(agg[r[1]].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for r in rows)
    out = [f"chip-wide MFMA busy over all kernels: {tot_mf / (tot * 1024) * 100:.1f}% of kernel-active cycles",
           "", "| % active | calls | MFMA util | active | wait-inst | wait-any | MFMA:VALU | kernel |",
           "|---:|---:|---:|---:|---:|---:|---:|---|"]
    for act, k, n, util, a, wi, wa, nm, nv in rows[:40]:
        ratio = f"1:{nv / nm:.1f}" if nm else "-"
        out.append(f"| {act / tot * 100:.1f} | {n} | {util * 100:.1f}% | {a * 100:.0f}% | {wi * 100:.0f}% | "
                   f"{wa * 100:.0f}% | {ratio} | `{k[:90]}` |")
    text = "\n".join(out)
    print(text)
    if "--md" in sys.argv:
        open(sys.argv[sys.argv.index("--md") + 1], "w").write(text + "\n")


if __name__ == "__main__":
    main()
