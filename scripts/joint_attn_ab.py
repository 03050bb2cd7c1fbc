#!/usr/bin/env python3
"""Kandinsky2 joint attention: the K/V prefix segment read in place (non-LDS-DMA kernel) vs
concatenating [context | spatial] K/V first and running the LDS-DMA kernel (bitwise equal: the keys
are the same sequence), hipGraph-replay timing including the concatenation.

    python scripts/joint_attn_ab.py
"""
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd.ops import _lib  # noqa: E402
from scripts.autotune_conv import graph_time  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for (B, N, Np, H, D) in [(8, 2304, 81, 12, 64), (8, 576, 81, 18, 64), (8, 144, 81, 24, 64), (2, 2304, 81, 12, 64)]:
        qkv = torch.randn(B, N, 3, H, D, device=dev).bfloat16()
        ckv = torch.randn(B, Np, 2, H, D, device=dev).bfloat16()
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        kp, vp = ckv[:, :, 0], ckv[:, :, 1]
        sc = 1 / math.sqrt(D)

        def pre():
            return _lib.flash_attention(q, k, v, sc, False, (kp, vp))

        def cat():
            return _lib.flash_attention(q, torch.cat([kp, k], 1), torch.cat([vp, v], 1), sc, False)
        same = torch.equal(pre(), cat())
        tp = statistics.median(graph_time(pre) for _ in range(3))
        tc = statistics.median(graph_time(cat) for _ in range(3))
        print(json.dumps({"shape": [B, N, Np, H, D], "bitwise": same, "prefix_us": round(tp, 1),
                          "cat_glds_us": round(tc, 1), "gain": round(tp / tc - 1, 3)}), flush=True)


if __name__ == "__main__":
    main()
