#!/usr/bin/env python3
"""Same-process A/B of the K-half staggered conv tiles' DMA prefetch distance (conv_stag2_kernel
PD 3 vs 4, arb_set_stag2_pd) and of buffer-resource DMA addressing on top of PD 4
(arb_set_stag2_buf): interleaved hipGraph-replay timing rounds on the hot stag2 shapes of
SD1.5 / Kandinsky2 at the lock-step batch, plus a bitwise check of every output (same MFMA order).

    python scripts/stag2_pd_ab.py [--rounds 5] [--conc 1]
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

# (B, H, W, Cin, Cout, k, cfg, split): planned stag2 shapes (layer_prof tables) + one split-K case
SHAPES = [
    (8, 48, 48, 768, 768, 3, 43, 1), (8, 96, 96, 768, 768, 3, 43, 1), (8, 24, 24, 1152, 1152, 3, 44, 1),
    (8, 12, 12, 1536, 1536, 3, 43, 4), (8, 16, 16, 1280, 1280, 3, 43, 2), (8, 32, 32, 640, 640, 3, 43, 1),
    (8, 64, 64, 320, 320, 3, 42, 1), (8, 24, 24, 2304, 1152, 3, 44, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--conc", type=int, default=1)
    a = ap.parse_args()
    at.CONC = a.conc
    dev = torch.device("cuda")
    setpd0, setbuf = _lib._fn("arb_set_stag2_pd"), _lib._fn("arb_set_stag2_buf")

    def setpd(v):            # 3, 4 or 5 (= 4 with buffer-resource DMA)
        setpd0(min(v, 4))
        setbuf(1 if v == 5 else 0)
    torch.manual_seed(0)
    out = []
    for (B, H, W, C, Co, k, cfg, sp) in SHAPES:
        x = torch.randn(B, H, W, C, device=dev).bfloat16()
        w = (torch.randn(Co, k, k, C, device=dev) / math.sqrt(k * k * C)).bfloat16()
        b = torch.randn(Co, device=dev).bfloat16()

        def run():
            return _lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1, cfg, sp)
        ys, ts = {}, {3: [], 4: [], 5: []}
        for pd in (3, 4, 5):
            setpd(pd)
            ys[pd] = [run() for _ in range(3)]
        same = all(torch.equal(ys[3][0], y) for y in ys[3] + ys[4] + ys[5])
        for _ in range(a.rounds):
            for pd in (3, 4, 5):
                setpd(pd)
                ts[pd].append(at.graph_time(run, reps=10, rounds=3))
        setpd(5)
        fl = 2.0 * B * H * W * Co * k * k * C
        m3, m4, m5 = statistics.median(ts[3]), statistics.median(ts[4]), statistics.median(ts[5])
        rec = {"shape": [B, H, W, C, Co, k], "cfg": cfg, "split": sp, "bitwise": same, "pd3_us": round(m3, 1),
               "pd4_us": round(m4, 1), "pd4buf_us": round(m5, 1), "pd3_tf": round(fl / m3 / 1e6),
               "pd4_tf": round(fl / m4 / 1e6), "pd4buf_tf": round(fl / m5 / 1e6), "gain": round(m3 / m4 - 1, 3),
               "gain_buf": round(m4 / m5 - 1, 3)}
        out.append(rec)
        print(json.dumps(rec), flush=True)
    assert all(r["bitwise"] for r in out), "PD 4 changed output bytes"


if __name__ == "__main__":
    main()
