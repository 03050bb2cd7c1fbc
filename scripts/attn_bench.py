#!/usr/bin/env python3
"""Flash attention microbench on the template shapes - SD level-0 self-attention at the 3 x 8 group
(batch 16) and solo (batch 2), SD cross-attention, SD level 1 (d 80), zeroscope spatial d 64, K2 d 64 -
with the ILP softmax on and off (``arb_set_attn_ilp``; bitwise-equal forms).  One process, interleaved
rounds, median of 5.  ``out_sha`` hashes the default-form output of a spiked input (a late lazy
rescale): equal hashes across kernel libraries (``ARBIUS_KERNEL_LIB``) = equal bytes.

    python scripts/attn_bench.py [--json out.jsonl]
"""
import argparse
import hashlib
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd.ops import _lib  # noqa: E402

# (B, N, Nk, H, D): B counts CFG rows
SHAPES = [(16, 4096, 4096, 8, 40), (2, 4096, 4096, 8, 40), (16, 4096, 77, 8, 40), (16, 1024, 1024, 8, 80),
          (48, 2880, 2880, 5, 64), (8, 2304, 2304, 10, 64), (16, 64, 64, 8, 40)]


def timeit(fn, reps=10):
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
    try:
        ilp = _lib._fn("arb_set_attn_ilp")
    except Exception:  # noqa: BLE001 - an older library (ARBIUS_KERNEL_LIB A/B): one form only
        ilp = None
    out = []
    for B, N, Nk, H, D in SHAPES:
        torch.manual_seed(0)
        q = torch.randn(B, N, H, D, device="cuda").bfloat16()
        k = torch.randn(B, Nk, H, D, device="cuda").bfloat16()
        v = torch.randn(B, Nk, H, D, device="cuda").bfloat16()
        sc = 1 / math.sqrt(D)
        flop = 4.0 * B * H * N * Nk * D
        ks = k.clone()
        ks[B // 2, Nk // 2:] *= 8.0
        spiked = _lib.flash_attention(q, ks, v, sc, False)
        row = {"B": B, "N": N, "Nk": Nk, "H": H, "D": D,
               "out_sha": hashlib.sha256(spiked.cpu().view(torch.int16).numpy().tobytes()).hexdigest()[:16]}
        forms = {"ilp": 1, "per_tile": 0} if ilp else {"default": None}
        res = {f: [] for f in forms}
        for _ in range(5):
            for f, on in forms.items():
                if ilp:
                    ilp(on)
                res[f].append(timeit(lambda: _lib.flash_attention(q, k, v, sc, False)))
        if ilp:
            ilp(1)
            ilp(0)
            ref = _lib.flash_attention(q, ks, v, sc, False)
            ilp(1)
            row["ilp_bitwise"] = bool(torch.equal(ref, spiked))
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
