#!/usr/bin/env python3
"""Every tile family at the pinned split on the SD1.5 UNet's GEMMs at the shipped lock-step group of 8
(batch 16, plans of the canonical batch 8): time (median, isolated) and bitwise equality with the
shipped choice (config/family tables).  An equal, faster family is a candidate for conv_family.inc
(then A/B in the 3-stream mix: profiles/r6/family_ab.jsonl).

    python scripts/sd_family_sweep.py [--json out.jsonl]
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

PB = (16, 8)
SHAPES = [(16384, 640, 5120, "geglu"), (4096, 1280, 1280, "gemm"), (16384, 640, 640, "gemm"),
          (4096, 5120, 1280, "gemm"), (65536, 1280, 320, "gemm"), (16384, 640, 1920, "gemm"),
          (16384, 2560, 640, "gemm"), (65536, 320, 960, "gemm")]


def bench(fn, reps=10):
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
            f = lambda c, s, pb=None: _lib.gemm_geglu(x, wi, bi, c, s, plan_batch=pb)  # noqa: E731
        else:
            f = lambda c, s, pb=None: _lib.gemm(x, w, b, None, c, s, plan_batch=pb)  # noqa: E731
        ref = f(-1, -1, PB)
        cfg0, split = _lib.gemm_choice(M, N, K, PB)
        res = {}
        for cfg in range(48):
            try:
                y = f(cfg, split)
                torch.cuda.synchronize()
            except Exception:
                continue
            eq = torch.equal(y, ref)
            res[cfg] = statistics.median(bench(lambda: f(cfg, split)) for _ in range(3)) if eq else None
        t0 = statistics.median(bench(lambda: f(-1, -1, PB)) for _ in range(3))
        ok = {c: t for c, t in res.items() if t is not None}
        best = min(ok, key=ok.get)
        row = {"M": M, "K": K, "N": N, "kind": kind, "shipped": [cfg0, split, _lib.cfg_name(cfg0)],
               "shipped_us": round(t0, 1), "best": [best, _lib.cfg_name(best), round(ok[best], 1)],
               "gain": round(t0 / ok[best] - 1, 3),
               "top": {_lib.cfg_name(c): round(t, 1) for c, t in sorted(ok.items(), key=lambda kv: kv[1])[:6]}}
        print(json.dumps(row), flush=True)
        if out:
            out.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()
