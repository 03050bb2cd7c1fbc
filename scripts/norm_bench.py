#!/usr/bin/env python3
"""Bandwidth of the non-MMA normalisation kernels at the SD1.5 batch-8 shapes (GroupNorm table =
stats + table, GN table apply, LayerNorm): median us per call and effective GB/s over the bytes each
kernel must move.  Run twice with ARB_GN_APPLY2=0 / ARB_LN_PACKED=0 for the A/B."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd.ops import _lib  # noqa: E402


def timeit(fn, iters=50, reps=5):
    """GPU time per call: `iters` calls captured in one hipGraph, replayed (the eager loop is
    launch-bound at ~10 us per call for these small kernels)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1000 / iters)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda")
    rows = []
    for (B, H, W, C) in [(8, 64, 64, 320), (8, 32, 32, 640), (8, 16, 16, 1280), (8, 8, 8, 1280),
                         (8, 64, 64, 640), (1, 512, 512, 128), (1, 128, 128, 512)]:
        x = torch.randn(B, H, W, C, device=dev).bfloat16()
        g = torch.randn(C, device=dev).bfloat16()
        b = torch.randn(C, device=dev).bfloat16()
        nbytes = x.numel() * 2
        t_tab = timeit(lambda: _lib.group_norm_table(x, g, b, 32, 1e-5), iters=50)
        table = _lib.group_norm_table(x, g, b, 32, 1e-5)
        t_app = timeit(lambda: _lib.norm_table_apply(x, table, True), iters=50)
        rows.append({"op": "gn_table", "shape": [B, H, W, C], "us": round(t_tab, 2),
                     "GBps": round(nbytes / t_tab / 1e3, 1)})
        rows.append({"op": "gn_apply", "shape": [B, H, W, C], "us": round(t_app, 2),
                     "GBps": round(2 * nbytes / t_app / 1e3, 1)})
    for (M, C) in [(32768, 320), (8192, 640), (2048, 1280), (512, 1280), (154, 768)]:
        x = torch.randn(M, C, device=dev).bfloat16()
        g = torch.randn(C, device=dev).bfloat16()
        b = torch.randn(C, device=dev).bfloat16()
        t = timeit(lambda: _lib.layer_norm(x, g, b, 1e-5), iters=50)
        rows.append({"op": "layer_norm", "shape": [M, C], "us": round(t, 2),
                     "GBps": round(2 * x.numel() * 2 / t / 1e3, 1)})
    tag = os.environ.get("TAG", "")
    for r in rows:
        r["tag"] = tag
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
