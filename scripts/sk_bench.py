#!/usr/bin/env python3
"""Short-K GEMMs of the SD1.5 UNet at lock-step batch 8 (M = 8 x tokens): the planned tile family vs
the W-stationary kernel (cfg 46 / 47, csrc/conv_sk.inc), isolated, interleaved rounds in one process
(median of 5).  TFLOP/s and HBM-side GB/s (activation in + output out, weights excluded).

    python scripts/sk_bench.py [--json out.jsonl]
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

# (M, K, N, kind): q/k/v-out projections, fused QKV, proj_in/out, GEGLU up-projection
SHAPES = [(32768, 320, 320, "gemm"), (32768, 320, 960, "gemm"), (8192, 640, 640, "gemm"), (8192, 640, 1920, "gemm"),
          (32768, 320, 2560, "geglu"), (8192, 640, 5120, "geglu")]


def bench(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3      # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = []
    for M, K, N, kind in SHAPES:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
        b = torch.randn(N, device="cuda").bfloat16()
        pcfg, psplit = _lib.gemm_choice(M, N, K, (8, 8))
        cands = {"plan": (pcfg, psplit), "sk46": (46, 1), "sk47": (47, 1)}
        if K != 320:
            cands.pop("sk46")
        if psplit != 1:
            cands = {"plan": cands["plan"]}
        if kind == "geglu":
            wi, bi = _lib.interleave_geglu(w), _lib.interleave_geglu(b)
            run = {k: (lambda c=c: _lib.gemm_geglu(x, wi, bi, c[0], c[1])) for k, c in cands.items()}
            outb = M * N // 2 * 2
        else:
            run = {k: (lambda c=c: _lib.gemm(x, w, b, None, c[0], c[1])) for k, c in cands.items()}
            outb = M * N * 2
        ref = run["plan"]()
        for k, f in run.items():
            assert torch.equal(f(), ref), (M, K, N, k)
        ts = {k: [] for k in run}
        for _ in range(5):
            for k, f in run.items():
                ts[k].append(bench(f))
        row = {"M": M, "K": K, "N": N, "kind": kind, "plan": _lib.cfg_name(pcfg) + f"/s{psplit}"}
        flop = 2.0 * M * N * K
        for k, v in ts.items():
            us = statistics.median(v)
            row[k + "_us"] = round(us, 1)
            row[k + "_tflops"] = round(flop / us / 1e6, 1)
            row[k + "_gbs"] = round((M * K * 2 + outb) / us / 1e3, 0)
        print(json.dumps(row), flush=True)
        rows.append(row)
    if a.json:
        with open(a.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
