#!/usr/bin/env python3
"""Pick a split-K per canonical plan from a split_study.py run, trading the solo latency against the
lock-step group throughput, and write the plan / family override files for an A/B
(ARB_CONV_PLANS / ARB_CONV_FAMILY) or for merging into csrc/conv_plans.inc / conv_family.inc.

Per shape and split S the study holds the best solo time (batch 2, one stream) and the best group
time (batch 8 under the deployed concurrency, per call of the aggregate).  The cost of a choice is

    calls x (solo_us / solo_step_us + group_us / 4 / group_step_us)

(relative change of the solo step and of the per-task group step; a batch-8 launch serves 4 tasks).
A plan key (canonical M, N, K; shared by every launch of that GEMM shape) keeps its current split
and families unless another choice lowers that cost by --gain.

    python scripts/split_plan.py gpurun_out/split/k2.jsonl --out gpurun_out/split/k2
"""
import argparse
import collections
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("study")
    ap.add_argument("--out", required=True, help="prefix: <out>_plans.txt, <out>_family.txt")
    ap.add_argument("--solo-step-us", type=float, default=10000.0, help="solo UNet step (K2: ~10 ms)")
    ap.add_argument("--group-step-us", type=float, default=4800.0, help="group step per task (K2 4x4: ~4.8 ms)")
    ap.add_argument("--keep-splits", action="store_true", help="families only (bitwise neutral)")
    ap.add_argument("--gain", type=float, default=1.03, help="required cost ratio to move off the current split")
    a = ap.parse_args()
    rows = [json.loads(line) for line in open(a.study)]
    # launches that share a canonical plan key (e.g. a 3x3 conv with and without the nearest-2x
    # input) share its split: choose per key
    keys = collections.defaultdict(list)
    for r in rows:
        keys[(r["GM"], r["MNK"][1], r["MNK"][2])].append(r)
    plans, fams = [], []
    tot = {"solo_dep": 0.0, "solo_new": 0.0, "grp_dep": 0.0, "grp_new": 0.0}
    hdr = f"{'S':>3} {'solo us':>9} {'group us':>9}"
    print(f"{'M x N x K':>24} {'calls':>5} {hdr} -> {hdr}")

    for r in rows:   # a one-sided study (--only solo / group): the other side keeps its deployed choice
        for side in ("solo", "group"):
            if side + "_best" not in r:
                r[side + "_dep_us"] = 0.0
                r[side + "_best"] = {str(r["split"]): (0.0, r[side + "_cfg"])}

    def times(r, s):
        """(solo us, solo cfg, group us, group cfg) of launch r at split s (the deployed choice if faster)."""
        sb, gb = r["solo_best"][str(s)], r["group_best"][str(s)]
        if s == r["split"] and r["solo_dep_us"] <= sb[0]:
            sb = (r["solo_dep_us"], r["solo_cfg"])
        if s == r["split"] and r["group_dep_us"] <= gb[0]:
            gb = (r["group_dep_us"], r["group_cfg"])
        return sb[0], sb[1], gb[0], gb[1]

    for (GM, N, K), rs in keys.items():
        S0 = rs[0]["split"]
        splits = set.intersection(*[set(map(int, r["solo_best"])) & set(map(int, r["group_best"])) for r in rs])

        def cost(s):
            c = 0.0
            for r in rs:
                su, _, gu, _ = times(r, s)
                c += r["calls"] * (su / a.solo_step_us + gu / 4 / a.group_step_us)
            return c

        c0 = sum(r["calls"] * (r["solo_dep_us"] / a.solo_step_us + r["group_dep_us"] / 4 / a.group_step_us)
                 for r in rs)
        if a.keep_splits:
            splits = splits & {S0}
        best = min(splits | {S0}, key=cost) if S0 in splits else S0
        if cost(best) * a.gain >= c0:
            best = None
        for r in rs:
            M = r["MNK"][0]
            n = r["calls"]
            cur = (r["solo_dep_us"], r["group_dep_us"])
            su, scfg, gu, gcfg = times(r, best) if best is not None else (cur[0], r["solo_cfg"], cur[1],
                                                                           r["group_cfg"])
            tot["solo_dep"] += n * cur[0]
            tot["grp_dep"] += n * cur[1] / 4
            tot["solo_new"] += n * su
            tot["grp_new"] += n * gu / 4
            s = S0 if best is None else best
            mark = "" if best is None else (" * split" if best != S0 else " * family")
            print(f"{M:>8} x{N:>6} x{K:>6} {n:>5} {S0:>3} {cur[0]:>9.1f} {cur[1]:>9.1f} -> {s:>3} {su:>9.1f} "
                  f"{gu:>9.1f}{mark}")
            if best is not None and scfg != r["solo_cfg"] or best not in (None, S0):
                fams.append(f"{{{M}, {N}, {K}, {best}, {GM // M}, {scfg}}},")
        if best is not None:
            gcfg = times(rs[0], best)[3]
            gratio = rs[0].get("group_ratio", 1)
            if gratio == 1:     # the canonical group itself: its plan entry carries the cfg
                plans.append(f"{{{GM}, {N}, {K}, {gcfg}, {best}}},")
            fams.append(f"{{{GM}, {N}, {K}, {best}, {gratio}, {gcfg}}},")
            if best == S0 and gcfg == rs[0]["group_cfg"]:
                if gratio == 1:
                    plans.pop()
                fams.pop()
    for side, k0, k1 in (("solo  us/step", "solo_dep", "solo_new"), ("group us/task-step", "grp_dep", "grp_new")):
        if tot[k0] > 0:
            print("%s: %.0f -> %.0f (%+.1f %%)" % (side, tot[k0], tot[k1], 100 * (tot[k1] / tot[k0] - 1)))
    fams = list(dict.fromkeys(fams))
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    open(a.out + "_plans.txt", "w").write("\n".join(plans) + "\n")
    open(a.out + "_family.txt", "w").write("\n".join(fams) + "\n")
    print(f"{len(plans)} re-planned shapes -> {a.out}_plans.txt / {a.out}_family.txt")


if __name__ == "__main__":
    main()
