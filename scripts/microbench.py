#!/usr/bin/env python3
"""Per-op A/B microbenchmark on one MI355X: our HIP kernels vs the PyTorch/ROCm
library path for the SD1.5 512^2 shapes.  Interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24); random data (rule 25)."""
import json
import math
import sys
import os

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd.ops import _lib, ref  # noqa: E402


def timeit(fn, iters=20, rounds=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best.append(s.elapsed_time(e) / iters * 1000)
    best.sort()
    return best[len(best) // 2]


def main():
    dev = torch.device("cuda")
    out = []
    # ---- conv 3x3
    for (B, H, W, Ci, Co) in [(2, 64, 64, 320, 320), (2, 32, 32, 640, 640), (2, 16, 16, 1280, 1280),
                              (2, 8, 8, 1280, 1280), (2, 64, 64, 640, 320), (1, 128, 128, 512, 512),
                              (1, 256, 256, 256, 256), (1, 512, 512, 128, 128)]:
        x = torch.randn(B, H, W, Ci, device=dev).bfloat16()
        w = (torch.randn(Co, 3, 3, Ci, device=dev) / math.sqrt(9 * Ci)).bfloat16()
        b = torch.randn(Co, device=dev).bfloat16()
        xc = x.permute(0, 3, 1, 2)
        wc = w.permute(0, 3, 1, 2)
        t_ours = timeit(lambda: _lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1))
        t_miopen = timeit(lambda: F.conv2d(xc, wc, b, padding=1))
        fl = 2.0 * B * H * W * Co * 9 * Ci
        out.append({"op": "conv3x3", "shape": [B, H, W, Ci, Co], "ours_us": round(t_ours, 1),
                    "miopen_us": round(t_miopen, 1), "ours_tflops": round(fl / t_ours / 1e6, 1),
                    "miopen_tflops": round(fl / t_miopen / 1e6, 1)})
        print(json.dumps(out[-1]), flush=True)
    # ---- GEMM (linear)
    for (M, K, N) in [(8192, 320, 960), (8192, 320, 2560), (8192, 1280, 320), (8192, 320, 320),
                      (2048, 640, 5120), (2048, 2560, 640), (512, 1280, 10240), (512, 5120, 1280)]:
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
        b = torch.randn(N, device=dev).bfloat16()
        r = torch.randn(M, N, device=dev).bfloat16()
        t_ours = timeit(lambda: _lib.gemm(x, w, b, r))
        t_blas = timeit(lambda: torch.addmm(r, x, w.t()).add_(b))
        t_blas_nores = timeit(lambda: F.linear(x, w, b))
        fl = 2.0 * M * N * K
        out.append({"op": "gemm", "shape": [M, K, N], "ours_bias_res_us": round(t_ours, 1),
                    "hipblaslt_addmm_add_us": round(t_blas, 1), "hipblaslt_linear_us": round(t_blas_nores, 1),
                    "ours_tflops": round(fl / t_ours / 1e6, 1), "linear_tflops": round(fl / t_blas_nores / 1e6, 1)})
        print(json.dumps(out[-1]), flush=True)
    # ---- attention
    for (B, N, Nk, H, D) in [(2, 4096, 4096, 8, 40), (2, 1024, 1024, 8, 80), (2, 256, 256, 8, 160),
                             (2, 4096, 77, 8, 40), (2, 1024, 77, 8, 80)]:
        q = torch.randn(B, N, H, D, device=dev).bfloat16()
        k = torch.randn(B, Nk, H, D, device=dev).bfloat16()
        v = torch.randn(B, Nk, H, D, device=dev).bfloat16()
        t_ours = timeit(lambda: _lib.flash_attention(q, k, v, 1 / math.sqrt(D), False))
        qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
        t_sdpa = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt))
        fl = 4.0 * B * H * N * Nk * D
        out.append({"op": "attention", "shape": [B, N, Nk, H, D], "ours_us": round(t_ours, 1),
                    "sdpa_us": round(t_sdpa, 1), "ours_tflops": round(fl / t_ours / 1e6, 1),
                    "sdpa_tflops": round(fl / t_sdpa / 1e6, 1)})
        print(json.dumps(out[-1]), flush=True)
    # in-model layouts: strided views of a fused QKV activation, and sharper score distributions
    for (B, N, H, D, amp) in [(2, 4096, 8, 40, 1.0), (2, 4096, 8, 40, 4.0), (8, 4096, 8, 40, 1.0)]:
        qkv = (torch.randn(B, N, 3, H, D, device=dev) * amp).bfloat16()
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        t_ours = timeit(lambda: _lib.flash_attention(q, k, v, 1 / math.sqrt(D), False))
        fl = 4.0 * B * H * N * N * D
        out.append({"op": "attention_fused_qkv", "shape": [B, N, N, H, D], "amp": amp,
                    "ours_us": round(t_ours, 1), "ours_tflops": round(fl / t_ours / 1e6, 1)})
        print(json.dumps(out[-1]), flush=True)
    # ---- group norm
    for (B, HW, C) in [(2, 4096, 320), (2, 1024, 640), (2, 256, 1280), (2, 4096, 640), (2, 1024, 2560),
                       (1, 262144, 128), (1, 65536, 256)]:
        x = torch.randn(B, HW, C, device=dev).bfloat16()
        g = torch.ones(C, device=dev).bfloat16()
        bb = torch.zeros(C, device=dev).bfloat16()
        t_ours = timeit(lambda: _lib.group_norm_nhwc(x, g, bb, 32, 1e-5, True))
        xc = x.permute(0, 2, 1)
        t_torch = timeit(lambda: F.silu(F.group_norm(xc, 32, g, bb, 1e-5)))
        gbps = 2 * x.numel() * 2 / t_ours / 1e3
        out.append({"op": "groupnorm_silu", "shape": [B, HW, C], "ours_us": round(t_ours, 1),
                    "torch_us": round(t_torch, 1), "ours_GBps": round(gbps, 1)})
        print(json.dumps(out[-1]), flush=True)
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
