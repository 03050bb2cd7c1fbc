"""SD-family KL-VAE decoder (latent 4ch /8 -> RGB), channels-last, inference only.

Implied compute of the anythingv3 container's VAE decode:
conv_in 4->512, mid {ResBlock, single-head attention d=512 over 64x64 tokens,
ResBlock}, 4 up levels (512,512,256,128) x 3 ResBlocks with nearest-x2
upsample fused into the next conv, GroupNorm+SiLU, conv_out 128->3.
The heavy part is the full-resolution 128/256-channel convs at 256^2-512^2.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import torch.nn as nn

from .. import ops
from .layers import Conv2d, GroupNorm, Linear
from .unet2d import ResBlock


@dataclass
class VAEConfig:
    latent_channels: int = 4
    out_channels: int = 3
    block_channels: Tuple[int, ...] = (128, 256, 512, 512)
    layers_per_block: int = 2
    groups: int = 32
    eps: float = 1e-6
    scaling_factor: float = 0.18215

    @staticmethod
    def tiny():
        return VAEConfig(block_channels=(16, 32, 32, 32), groups=8)


class VAEAttention(nn.Module):
    """Single-head spatial self-attention of the VAE mid-block."""

    def __init__(self, c, groups, eps):
        super().__init__()
        self.norm = GroupNorm(groups, c, eps)
        self.to_qkv = Linear(c, 3 * c)
        self.to_out = Linear(c, c)

    def forward(self, x):
        B, H, W, C = x.shape
        qkv = self.to_qkv.forward_norm(x.view(B, H * W, C), self.norm.table(x)).view(B, H * W, 3, 1, C)
        o = ops.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2])
        return self.to_out(o.reshape(B, H * W, C), residual=x.view(B, H * W, C)).view(B, H, W, C)


class VAEDecoder(nn.Module):
    def __init__(self, cfg: VAEConfig = None):
        super().__init__()
        cfg = cfg or VAEConfig()
        self.cfg = cfg
        ch = list(reversed(cfg.block_channels))
        self.post_quant = Conv2d(cfg.latent_channels, cfg.latent_channels, 1)
        self.conv_in = Conv2d(cfg.latent_channels, ch[0], 3)
        self.mid_res1 = ResBlock(ch[0], ch[0], 0, cfg.groups, cfg.eps)
        self.mid_attn = VAEAttention(ch[0], cfg.groups, cfg.eps)
        self.mid_res2 = ResBlock(ch[0], ch[0], 0, cfg.groups, cfg.eps)
        self.up = nn.ModuleList()
        cur = ch[0]
        for lvl, c in enumerate(ch):
            blk = nn.Module()
            blk.resnets = nn.ModuleList()
            for _ in range(cfg.layers_per_block + 1):
                blk.resnets.append(ResBlock(cur, c, 0, cfg.groups, cfg.eps))
                cur = c
            blk.upsample = Conv2d(c, c, 3) if lvl < len(ch) - 1 else None
            self.up.append(blk)
        self.norm_out = GroupNorm(cfg.groups, cur, cfg.eps, silu=True)
        self.conv_out = Conv2d(cur, cfg.out_channels, 3)

    def forward(self, z):
        """z [B, h, w, 4] (already divided by scaling_factor) -> image [B, 8h, 8w, 3] in ~[-1, 1]."""
        h = self.conv_in(self.post_quant(z, ))
        h = self.mid_res1(h)
        h = self.mid_attn(h)
        h = self.mid_res2(h)
        for blk in self.up:
            for rb in blk.resnets:
                h = rb(h)
            if blk.upsample is not None:
                h = blk.upsample(h, upsample=True)
        return self.conv_out(h, norm=self.norm_out.table(h))
