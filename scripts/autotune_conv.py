#!/usr/bin/env python3
"""Offline autotuner for the implicit-GEMM conv/GEMM kernel (csrc/conv.hip).

Enumerates every conv and residual-GEMM shape of the SD1.5 UNet (batch 2, 512^2)
and VAE decoder (batch 1) by running the models on the meta device, times every
(tile cfg, split-K) candidate on the GPU with hipGraph-captured launches (so CPU
launch cost is excluded), and writes the winners as a pinned table
(``csrc/conv_plans.inc``).  The table is keyed by the GEMM dims (M, N, K): the
plan stays a pure function of the shape, identical on every GPU (determinism).

    python scripts/autotune_conv.py OUT_DIR
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd import ops  # noqa: E402
from arbius_amd.ops import _lib  # noqa: E402

NCFG = 20  # 0-9: LDS-DMA multi-stage, 10-19: register-staged
SPLITS = (1, 2, 3, 4, 6, 8)


def collect_shapes(res=512):
    from arbius_amd.models.unet2d import UNet2DCondition, UNetConfig
    from arbius_amd.models.vae import VAEDecoder
    convs, gemms = set(), set()
    orig_conv, orig_lin = ops.conv2d, ops.linear

    def conv(x, w, b=None, stride=1, padding=1, upsample=False, residual=None, temb=None):
        if x.shape[-1] % 64 == 0 and w.shape[0] % 8 == 0:
            B, H, W, C = x.shape
            convs.add((B, H, W, C, w.shape[0], w.shape[1], padding, int(bool(upsample)), stride))
        return orig_conv(x, w, b, stride, padding, upsample, residual, temb)

    def lin(x, w, b=None, residual=None):
        if residual is not None and x.shape[-1] % 64 == 0:
            gemms.add((x.numel() // x.shape[-1], x.shape[-1], w.shape[0]))
        return orig_lin(x, w, b, residual)

    ops.conv2d, ops.linear = conv, lin
    try:
        with torch.device("meta"):
            u = UNet2DCondition(UNetConfig())
            u(torch.zeros(2, res // 8, res // 8, 4), torch.tensor([500.0]), torch.zeros(2, 77, 768))
            d = VAEDecoder()
            d(torch.zeros(1, res // 8, res // 8, 4))
    finally:
        ops.conv2d, ops.linear = orig_conv, orig_lin
    return sorted(convs), sorted(gemms)


def graph_time(fn, reps=10, rounds=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1000 / reps)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    out_dir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    os.makedirs(out_dir, exist_ok=True)
    dev = torch.device("cuda")
    convs, gemms = collect_shapes()
    results, pinned = [], {}
    for (B, H, W, C, Co, k, pad, up, st) in convs:
        x = torch.randn(B, H, W, C, device=dev).bfloat16()
        w = (torch.randn(Co, k, k, C, device=dev) / math.sqrt(k * k * C)).bfloat16()
        b = torch.randn(Co, device=dev).bfloat16()
        Hl, Wl = (2 * H, 2 * W) if up else (H, W)
        Ho, Wo = (Hl + 2 * pad - k) // st + 1, (Wl + 2 * pad - k) // st + 1
        M, K = B * Ho * Wo, k * k * C
        auto = _lib.conv_plan(B, H, W, C, Co, k, pad, up, st)
        best = None
        for cfg in range(NCFG):
            for sp in SPLITS:
                if sp > 1 and sp > (K // 64) // 2:
                    continue
                try:
                    t = graph_time(lambda: _lib.conv2d_nhwc(x, w, b, pad, up, None, None, st, cfg, sp))
                except Exception as e:  # noqa: BLE001
                    print("skip", cfg, sp, e, flush=True)
                    continue
                if best is None or t < best[0]:
                    best = (t, cfg, sp)
        t_auto = graph_time(lambda: _lib.conv2d_nhwc(x, w, b, pad, up, None, None, st))
        fl = 2.0 * M * Co * K
        rec = {"kind": "conv", "shape": [B, H, W, C, Co, k, pad, up, st], "MNK": [M, Co, K], "best_us": round(best[0], 2),
               "best_cfg": best[1], "best_split": best[2], "best_tflops": round(fl / best[0] / 1e6, 1),
               "auto_cfg": auto, "auto_us": round(t_auto, 2)}
        results.append(rec)
        pinned[(M, Co, K)] = (best[1], best[2])
        print(json.dumps(rec), flush=True)
    for (M, K, N) in gemms:
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
        b = torch.randn(N, device=dev).bfloat16()
        r = torch.randn(M, N, device=dev).bfloat16()
        best = None
        for cfg in range(NCFG):
            for sp in SPLITS:
                if sp > 1 and sp > (K // 64) // 2:
                    continue
                try:
                    t = graph_time(lambda: _lib.gemm(x, w, b, r, cfg, sp))
                except Exception as e:  # noqa: BLE001
                    continue
                if best is None or t < best[0]:
                    best = (t, cfg, sp)
        t_blas = graph_time(lambda: torch.addmm(r, x, w.t()).add_(b))
        fl = 2.0 * M * N * K
        rec = {"kind": "gemm_res", "MNK": [M, N, K], "best_us": round(best[0], 2), "best_cfg": best[1],
               "best_split": best[2], "best_tflops": round(fl / best[0] / 1e6, 1), "hipblaslt_addmm_add_us": round(t_blas, 2)}
        results.append(rec)
        if (M, N, K) not in pinned:
            pinned[(M, N, K)] = (best[1], best[2])
        print(json.dumps(rec), flush=True)
    json.dump(results, open(os.path.join(out_dir, "autotune_conv.json"), "w"), indent=1)
    lines = ["// Generated by scripts/autotune_conv.py on MI355X: (M, N, K) -> (tile cfg, split-K).",
             "// Shapes not listed fall back to the cost model in conv.hip.",
             "static const PinnedPlan kPinnedPlans[] = {"]
    for (M, N, K), (c, sp) in sorted(pinned.items()):
        lines.append(f"    {{{M}, {N}, {K}, {c}, {sp}}},")
    lines.append("};")
    open(os.path.join(out_dir, "conv_plans.inc"), "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
