#!/usr/bin/env python3
"""Count the matmul FLOPs of one SD1.5 UNet evaluation (batch 2 = CFG, 512^2) on the meta device:
convs, linears (incl. hipBLASLt ones) and attention (QK^T + PV).  Used to turn measured step
times into achieved TFLOP/s (README, profiles/)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd import ops  # noqa: E402

FL = {"conv": 0.0, "linear": 0.0, "attention": 0.0}


def main(res=512):
    oc, ol, oa = ops.conv2d, ops.linear, ops.attention

    def conv(x, w, b=None, stride=1, padding=1, upsample=False, residual=None, temb=None, norm=None):
        y = oc(x, w, b, stride, padding, upsample, residual, temb, norm)
        FL["conv"] += 2.0 * y.numel() * w.shape[1] * w.shape[2] * w.shape[3]
        return y

    def lin(x, w, b=None, residual=None):
        FL["linear"] += 2.0 * (x.numel() // x.shape[-1]) * x.shape[-1] * w.shape[0]
        return ol(x, w, b, residual)

    def att(q, k, v, *a, **kw):
        B, Nq, H, D = q.shape
        FL["attention"] += 4.0 * B * H * Nq * k.shape[1] * D
        return oa(q, k, v, *a, **kw)

    ops.conv2d, ops.linear, ops.attention = conv, lin, att
    from arbius_amd.models.unet2d import UNet2DCondition, UNetConfig
    with torch.device("meta"):
        UNet2DCondition(UNetConfig())(torch.zeros(2, res // 8, res // 8, 4), torch.tensor([500.0]),
                                      torch.zeros(2, 77, 768))
    tot = sum(FL.values())
    print({k: round(v / 1e9, 1) for k, v in FL.items()}, "total GFLOP per UNet eval:", round(tot / 1e9, 1))
    return tot


if __name__ == "__main__":
    main()
