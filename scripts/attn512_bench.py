#!/usr/bin/env python3
"""d = 512 single-head attention: blockwise HIP kernel (csrc/attention512.hip) vs the round-4
GEMM -> row softmax -> GEMM path, on the template shapes (VAE 512^2 / 1024^2, MoVQ 96^2, zeroscope
VAE per frame).  One process, interleaved rounds, median of 3 (cdna_hip_programming.md rule 24).

    python scripts/attn512_bench.py [--json out.jsonl]
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

SHAPES = [(1, 4096), (1, 16384), (1, 9216), (24, 2880)]


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    out = []
    for B, N in SHAPES:
        q, k, v = (torch.randn(B, N, 1, 512, device="cuda").bfloat16() for _ in range(3))
        sc = 1 / math.sqrt(512)
        flop = 4.0 * B * N * N * 512
        res = {"blockwise": [], "gemm": []}
        for _ in range(3):
            _lib._A512 = True
            res["blockwise"].append(timeit(lambda: _lib._large_head_attention(q, k, v, sc)))
            _lib._A512 = False
            res["gemm"].append(timeit(lambda: _lib._large_head_attention(q, k, v, sc)))
        _lib._A512 = True
        row = {"B": B, "N": N}
        for name, ts in res.items():
            ms = statistics.median(ts)
            row[name + "_us"] = round(ms * 1e3, 1)
            row[name + "_tflops"] = round(flop / ms / 1e9, 1)
        print(json.dumps(row), flush=True)
        out.append(row)
    if a.json:
        with open(a.json, "w") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
