#!/usr/bin/env python3
"""Every tile family at the pinned split on the zeroscope UNet3D's short-K GEMMs (M = 2F x HW rows at
576x320x24): time (median of 5, isolated) and bitwise equality with the pinned plan.  A family that is
equal and faster can replace the plan's with no change to any output byte.

    python scripts/zs_shortk.py [--json out.jsonl]
"""
import argparse
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd.ops import _lib  # noqa: E402

SHAPES = [(138240, 320, 2560, "geglu"), (138240, 320, 320, "gemm"), (138240, 320, 960, "gemm"),
          (34560, 640, 640, "gemm"), (34560, 640, 5120, "geglu"), (34560, 640, 1920, "gemm"),
          (65536, 320, 320, "gemm"), (65536, 320, 2560, "geglu")]


def bench(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    out = open(a.json, "w") if a.json else None
    for M, K, N, kind in SHAPES:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
        b = torch.randn(N, device="cuda").bfloat16()
        if kind == "geglu":
            wi, bi = _lib.interleave_geglu(w), _lib.interleave_geglu(b)
            f = lambda c, s: _lib.gemm_geglu(x, wi, bi, c, s)  # noqa: E731
        else:
            f = lambda c, s: _lib.gemm(x, w, b, None, c, s)  # noqa: E731
        ref = f(-1, -1)
        plan = _lib.conv_plan(1, 1, M, K, N, 1, 0, 0, 1)
        res = {}
        for cfg in range(48):
            try:
                y = f(cfg, plan[1])
                torch.cuda.synchronize()
            except Exception:
                continue
            if not torch.equal(y, ref):
                res[cfg] = None
                continue
            res[cfg] = statistics.median(bench(lambda: f(cfg, plan[1])) for _ in range(3))
        t_plan = statistics.median(bench(lambda: f(-1, -1)) for _ in range(3))
        ok = {c: t for c, t in res.items() if t is not None}
        best = min(ok, key=ok.get) if ok else None
        row = {"M": M, "K": K, "N": N, "kind": kind, "plan": [plan[0], plan[1], _lib.cfg_name(plan[0])],
               "plan_us": round(t_plan, 1), "best": [best, _lib.cfg_name(best) if best is not None else None,
                                                     round(ok[best], 1) if best is not None else None],
               "tflops_plan": round(2.0 * M * N * K / t_plan / 1e6, 1),
               "differs": [c for c, t in res.items() if t is None],
               "all_us": {_lib.cfg_name(c): round(t, 1) for c, t in sorted(ok.items(), key=lambda kv: kv[1])[:8]}}
        print(json.dumps(row), flush=True)
        if out:
            out.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()
