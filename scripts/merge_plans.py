#!/usr/bin/env python3
"""Merge plan / family override files (the ARB_CONV_PLANS / ARB_CONV_FAMILY format written by
scripts/split_plan.py) into the pinned tables csrc/conv_plans.inc / csrc/conv_family.inc.

A plan entry {M, N, K, cfg, split} replaces the table's entry for (M, N, K); a family entry
{M, N, K, split, ratio, cfg} replaces the one for (M, N, K, split, ratio).  A changed split moves
output bytes (bump NUMERICS_VERSION and re-pin the goldens); a changed cfg at the same split does not.

    python scripts/merge_plans.py --plans scripts/r5/k2plans/k2w4800_plans.txt \
        --family scripts/r5/k2plans/k2w4800_family.txt
"""
import argparse
import os
import re

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "arbius_amd", "ops", "csrc")
ENTRY = re.compile(r"^\s*\{([-\d,\s]+)\},")


def read(path):
    return [tuple(int(v) for v in m.group(1).split(",")) for m in map(ENTRY.match, open(path)) if m]


def merge(table, updates, nkey):
    lines = open(table).read().split("\n")
    head = [ln for ln in lines if not ENTRY.match(ln) and ln.strip() != "};" and ln.strip()]
    entries = {e[:nkey]: e for e in read(table)}
    changed = sum(1 for u in updates if entries.get(u[:nkey]) != u)
    for u in updates:
        entries[u[:nkey]] = u
    body = ["    {" + ", ".join(str(v) for v in e) + "}," for _, e in sorted(entries.items())]
    open(table, "w").write("\n".join(head + body + ["};", ""]))
    return changed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plans")
    ap.add_argument("--family")
    a = ap.parse_args()
    if a.plans:
        print("conv_plans.inc:", merge(os.path.join(CSRC, "conv_plans.inc"), read(a.plans), 3), "entries changed")
    if a.family:
        print("conv_family.inc:", merge(os.path.join(CSRC, "conv_family.inc"), read(a.family), 5), "entries changed")


if __name__ == "__main__":
    main()
