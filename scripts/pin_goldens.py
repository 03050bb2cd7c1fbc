#!/usr/bin/env python3
"""Compute the golden CIDs of ``arbius_amd.numerics.golden_cases`` (and the boot self-test CIDs of
``config/selftest.json``) on this GPU and write them as JSON.  Run on an MI355X after a deliberate
numerics change, together with a ``NUMERICS_VERSION`` bump.  ``--apply`` writes the result into
``tests/golden_cids.json`` and the self-test values into ``arbius_amd/config/selftest.json``;
``--apply-from FILE`` does the same on a host without a GPU from a JSON written on the box.

    python scripts/pin_goldens.py --out gpurun_out/golden_cids.json --selftest --apply
    python scripts/pin_goldens.py --apply-from gpurun_out/<tag>/golden_cids.json
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def apply(out: dict) -> None:
    """Write a pin result into the tracked golden table and the boot self-test table."""
    gold = {k: out[k] for k in ("numerics_version", "key", "cases")}
    with open(os.path.join(ROOT, "tests", "golden_cids.json"), "w") as f:
        json.dump(gold, f, indent=1)
        f.write("\n")
    if "selftest" in out:
        path = os.path.join(ROOT, "arbius_amd", "config", "selftest.json")
        table = json.load(open(path))
        for name, cid in out["selftest"].items():
            table[name]["expected"][out["key"]] = cid
        table["numerics_version"] = out["numerics_version"]
        with open(path, "w") as f:
            json.dump(table, f, indent=1)
            f.write("\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--selftest", action="store_true", help="also the boot self-test tasks (K2 100 steps)")
    ap.add_argument("--apply", action="store_true", help="write the result into the tracked tables")
    ap.add_argument("--apply-from", help="apply a result JSON written earlier (no GPU needed)")
    a = ap.parse_args()
    if a.apply_from:
        apply(json.load(open(a.apply_from)))
        return
    if not a.out:
        ap.error("--out is required")
    import torch

    from arbius_amd.node.pool import hardware_id
    from arbius_amd.numerics import NUMERICS_VERSION, golden_cases
    dev = torch.device("cuda", 0)
    key = f"{hardware_id(dev)}/random-init-seed0"
    out = {"numerics_version": NUMERICS_VERSION, "key": key, "cases": {}, "seconds": {}}
    for name, fn in golden_cases(dev):
        t0 = time.perf_counter()
        out["cases"][name] = fn()
        out["seconds"][name] = round(time.perf_counter() - t0, 2)
        print(name, out["cases"][name], flush=True)
    if a.selftest:
        from arbius_amd.numerics import selftest_cids
        out["selftest"] = selftest_cids(dev)
        print("selftest", out["selftest"], flush=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    if a.apply:
        apply(out)


if __name__ == "__main__":
    main()
