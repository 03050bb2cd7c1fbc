#!/usr/bin/env python3
"""Compute the golden CIDs of ``arbius_amd.numerics.golden_cases`` (and the boot self-test CIDs of
``config/selftest.json``) on this GPU and write them as JSON.  Run on an MI355X after a deliberate
numerics change, together with a ``NUMERICS_VERSION`` bump; copy the output to
``tests/golden_cids.json`` and the self-test values into ``arbius_amd/config/selftest.json``.

    python scripts/pin_goldens.py --out gpurun_out/golden_cids.json [--selftest]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--selftest", action="store_true", help="also the boot self-test tasks (K2 100 steps)")
    a = ap.parse_args()
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


if __name__ == "__main__":
    main()
