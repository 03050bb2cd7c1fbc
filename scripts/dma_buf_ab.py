#!/usr/bin/env python3
"""Same-process A/B of buffer-resource LDS-DMA addressing (arb_set_stag2_buf: conv_glds_kernel and
conv_stag2_kernel) on the planned kernels of hot conv / GEMM shapes of SD1.5, Kandinsky2 and
zeroscope: interleaved hipGraph-replay rounds, bitwise check of every output.

    python scripts/dma_buf_ab.py [--rounds 5]
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
import scripts.autotune_conv as at  # noqa: E402

# conv: (B, H, W, Cin, Cout, k); gemm: (M, K, N)
CONVS = [(8, 64, 64, 320, 320, 3), (8, 32, 32, 640, 640, 3), (8, 16, 16, 1280, 1280, 3), (8, 96, 96, 384, 384, 3),
         (8, 48, 48, 768, 768, 3), (8, 24, 24, 1152, 1152, 3), (48, 40, 72, 320, 320, 3), (48, 20, 36, 640, 640, 3),
         (1, 128, 128, 512, 512, 3), (8, 64, 64, 960, 320, 3)]
GEMMS = [(32768, 320, 320), (8192, 640, 640), (2048, 1280, 1280), (32768, 1280, 320), (138240, 320, 320),
         (18432, 768, 2304)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    setbuf = _lib._fn("arb_set_stag2_buf")
    torch.manual_seed(0)
    cases = []
    for (B, H, W, C, Co, k) in CONVS:
        x = torch.randn(B, H, W, C, device=dev).bfloat16()
        w = (torch.randn(Co, k, k, C, device=dev) / math.sqrt(k * k * C)).bfloat16()
        b = torch.randn(Co, device=dev).bfloat16()
        cfg, sp = _lib.conv_plan(B, H, W, C, Co, k, 1, 0, 1)
        cases.append((f"conv {B}x{H}x{W}x{C}->{Co} k{k}", 2.0 * B * H * W * Co * k * k * C, cfg, sp,
                      (lambda x=x, w=w, b=b: _lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1))))
    for (M, K, N) in GEMMS:
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
        b = torch.randn(N, device=dev).bfloat16()
        cfg, sp = _lib.conv_plan(1, 1, M, K, N, 1, 0, 0, 1)
        cases.append((f"gemm {M}x{N}x{K}", 2.0 * M * N * K, cfg, sp, (lambda x=x, w=w, b=b: _lib.gemm(x, w, b))))
    ok = True
    for name, fl, cfg, sp, run in cases:
        ys = {}
        for v in (0, 1):
            setbuf(v)
            ys[v] = [run() for _ in range(3)]
        same = all(torch.equal(ys[0][0], y) for y in ys[0] + ys[1])
        ok &= same
        ts = {0: [], 1: []}
        for _ in range(a.rounds):
            for v in (0, 1):
                setbuf(v)
                ts[v].append(at.graph_time(run, reps=10, rounds=3))
        setbuf(1)
        m0, m1 = statistics.median(ts[0]), statistics.median(ts[1])
        print(json.dumps({"case": name, "cfg": cfg, "split": sp, "bitwise": same, "global_us": round(m0, 1),
                          "buf_us": round(m1, 1), "global_tf": round(fl / m0 / 1e6), "buf_tf": round(fl / m1 / 1e6),
                          "gain": round(m0 / m1 - 1, 3)}), flush=True)
    assert ok, "buffer-resource DMA changed output bytes"


if __name__ == "__main__":
    main()
