#!/usr/bin/env python3
"""Focused A/B timings (hipGraph replay, interleaved rounds in one process) of
kernel variants on the hot SD1.5 shapes: conv tile configs x split-K and the
attention kernel.  Used for ablations; prints one JSON line per measurement.

    python scripts/kernel_ab.py [conv|attn|all]
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd.ops import _lib  # noqa: E402
from scripts.autotune_conv import graph_time  # noqa: E402


def conv_ab():
    dev = torch.device("cuda")
    shapes = [(2, 16, 16, 1280, 1280), (2, 64, 64, 320, 320), (2, 32, 32, 640, 640), (1, 128, 128, 512, 512)]
    for (B, H, W, C, Co) in shapes:
        x = torch.randn(B, H, W, C, device=dev).bfloat16()
        w = (torch.randn(Co, 3, 3, C, device=dev) / math.sqrt(9 * C)).bfloat16()
        b = torch.randn(Co, device=dev).bfloat16()
        fl = 2.0 * B * H * W * Co * 9 * C
        res = {}
        for cfg in (0, 3, 5, 10, 13, 15):
            for sp in (1, 2, 4, 8):
                t = graph_time(lambda: _lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1, cfg, sp))
                res[f"{cfg}/{sp}"] = round(t, 1)
        best = min(res, key=res.get)
        print(json.dumps({"conv": [B, H, W, C, Co], "us": res, "best": best,
                          "best_tflops": round(fl / res[best] / 1e6, 1)}), flush=True)


def attn_ab():
    dev = torch.device("cuda")
    for (B, N, Nk, H, D) in [(2, 4096, 4096, 8, 40), (2, 1024, 1024, 8, 80), (2, 256, 256, 8, 160)]:
        qkv = torch.randn(B, N, 3, H, D, device=dev).bfloat16()
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        t = graph_time(lambda: _lib.flash_attention(q, k, v, 1 / math.sqrt(D), False))
        fl = 4.0 * B * H * N * Nk * D
        print(json.dumps({"attn": [B, N, Nk, H, D], "us": round(t, 1), "tflops": round(fl / t / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("conv", "all"):
        conv_ab()
    if what in ("attn", "all"):
        attn_ab()
