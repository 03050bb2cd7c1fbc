#!/usr/bin/env python3
"""Temporal attention (csrc/temporal_attention.hip) on the UNet3D shapes - zeroscope 576x320x24 levels
0 / 1 (B 2 CFG rows x 24 frames x 2880 / 720 pixels x 5 / 10 heads x 64) and a 48-frame clip - strided
out of a fused QKV tensor as the model calls it.  Prints time, effective HBM rate (q, k, v read + o
written once) and a hash of the output: equal hashes across kernel libraries (``ARBIUS_KERNEL_LIB``)
= equal bytes.

    python scripts/temporal_bench.py [--json out.jsonl]
"""
import argparse
import hashlib
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd import ops  # noqa: E402

SHAPES = [(2, 24, 2880, 5, 64), (2, 24, 720, 10, 64), (2, 48, 2880, 5, 64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    out = []
    for B, F, P, H, D in SHAPES:
        torch.manual_seed(0)
        qkv = torch.randn(B, F, P, 3, H, D, device="cuda").bfloat16()
        q, k, v = qkv[:, :, :, 0], qkv[:, :, :, 1], qkv[:, :, :, 2]
        o = ops.temporal_attention(q, k, v)
        ts = []
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                ops.temporal_attention(q, k, v)
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) / 10)
        ms = statistics.median(ts)
        byts = 4 * B * F * P * H * D * 2
        row = {"B": B, "F": F, "P": P, "H": H, "D": D, "us": round(ms * 1e3, 1),
               "hbm_tbs": round(byts / ms / 1e9, 2),
               "out_sha": hashlib.sha256(o.cpu().view(torch.int16).numpy().tobytes()).hexdigest()[:16]}
        print(json.dumps(row), flush=True)
        out.append(row)
    if a.json:
        with open(a.json, "w") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
