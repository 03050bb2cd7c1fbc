"""MoVQ decoder (Kandinsky 2.1 image decoder), channels-last, inference only
(SURVEY.md §2.6(b) [EXT]).

Every normalisation is a SpatialNorm conditioned on the latent ``zq``:

    SpatialNorm(f, zq) = GN(f) * conv_y(up(zq)) + conv_b(up(zq))

``conv_y``/``conv_b`` are 1x1 convs and ``up`` is nearest upsampling; the two
commute, so the modulation maps are computed ONCE at latent resolution per
layer and expanded by an index gather inside ``ops.spatial_norm`` (one fused
HIP kernel: GN apply * y + b [+ SiLU]) - never materialised at full res.

Layout (taming VQGAN decoder, ch 128, ch_mult (1,2,2,4), 2+1 ResBlocks per
level, attention at the latent resolution): conv_in 4->512, mid {Res, Attn,
Res}, up levels 512@h, 256@2h, 256@4h, 128@8h, SpatialNorm+SiLU, conv_out.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import torch
import torch.nn as nn

from .. import ops
from .layers import Conv2d, Linear


@dataclass
class MoVQConfig:
    z_channels: int = 4
    out_channels: int = 3
    ch: int = 128
    ch_mult: Tuple[int, ...] = (1, 2, 2, 4)
    num_res_blocks: int = 2
    attn_levels: Tuple[int, ...] = (3,)     # level index with attention (latent resolution)
    groups: int = 32
    eps: float = 1e-6

    @staticmethod
    def kandinsky21():
        return MoVQConfig()

    @staticmethod
    def tiny():
        return MoVQConfig(ch=16, ch_mult=(1, 2, 2, 4), num_res_blocks=1, groups=8)


class SpatialNorm(nn.Module):
    def __init__(self, c, zc, groups, eps, silu):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(c), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(c), requires_grad=False)
        self.yb = Conv2d(zc, 2 * c, 1)          # conv_y and conv_b stacked along Cout
        self.groups, self.eps, self.silu, self.c = groups, eps, silu, c

    def reset(self, gen):
        self.weight.data.fill_(1.0)
        self.bias.data.zero_()

    def forward(self, f, zq):
        yb = self.yb(zq)                        # [B, h, w, 2C] at latent resolution
        return ops.spatial_norm(f, yb, self.weight, self.bias, self.groups, self.eps, self.silu)


class MoVQResBlock(nn.Module):
    def __init__(self, cin, cout, zc, groups, eps):
        super().__init__()
        self.norm1 = SpatialNorm(cin, zc, groups, eps, silu=True)
        self.conv1 = Conv2d(cin, cout, 3)
        self.norm2 = SpatialNorm(cout, zc, groups, eps, silu=True)
        self.conv2 = Conv2d(cout, cout, 3)
        self.skip = Conv2d(cin, cout, 1) if cin != cout else None

    def forward(self, x, zq):
        h = self.conv1(self.norm1(x, zq))
        skip = self.skip(x) if self.skip is not None else x
        return self.conv2(self.norm2(h, zq), residual=skip)


class MoVQAttention(nn.Module):
    def __init__(self, c, zc, groups, eps):
        super().__init__()
        self.norm = SpatialNorm(c, zc, groups, eps, silu=False)
        self.qkv = Linear(c, 3 * c)
        self.out = Linear(c, c)

    def forward(self, x, zq):
        B, H, W, C = x.shape
        qkv = self.qkv(self.norm(x, zq).view(B, H * W, C)).view(B, H * W, 3, 1, C)
        o = ops.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2])
        return self.out(o.reshape(B, H * W, C), residual=x.view(B, H * W, C)).view(B, H, W, C)


class MoVQDecoder(nn.Module):
    def __init__(self, cfg: MoVQConfig = None):
        super().__init__()
        cfg = cfg or MoVQConfig()
        self.cfg = cfg
        zc, g, e = cfg.z_channels, cfg.groups, cfg.eps
        cin = cfg.ch * cfg.ch_mult[-1]
        self.post_quant = Conv2d(zc, zc, 1)
        self.conv_in = Conv2d(zc, cin, 3)
        self.mid1 = MoVQResBlock(cin, cin, zc, g, e)
        self.mid_attn = MoVQAttention(cin, zc, g, e)
        self.mid2 = MoVQResBlock(cin, cin, zc, g, e)
        self.up = nn.ModuleList()
        nlev = len(cfg.ch_mult)
        for lvl in reversed(range(nlev)):
            blk = nn.Module()
            cout = cfg.ch * cfg.ch_mult[lvl]
            blk.res = nn.ModuleList()
            blk.attn = nn.ModuleList()
            for _ in range(cfg.num_res_blocks + 1):
                blk.res.append(MoVQResBlock(cin, cout, zc, g, e))
                cin = cout
                if lvl in cfg.attn_levels:
                    blk.attn.append(MoVQAttention(cin, zc, g, e))
            blk.upsample = Conv2d(cin, cin, 3) if lvl != 0 else None
            self.up.append(blk)
        self.norm_out = SpatialNorm(cin, zc, g, e, silu=True)
        self.conv_out = Conv2d(cin, cfg.out_channels, 3)

    def forward(self, z):
        """z [B, h, w, 4] latent -> image [B, 8h, 8w, 3] in ~[-1, 1]."""
        zq = z
        h = self.conv_in(self.post_quant(z))
        h = self.mid1(h, zq)
        h = self.mid_attn(h, zq)
        h = self.mid2(h, zq)
        for blk in self.up:
            for i, rb in enumerate(blk.res):
                h = rb(h, zq)
                if len(blk.attn):
                    h = blk.attn[i](h, zq)
            if blk.upsample is not None:
                h = blk.upsample(h, upsample=True)
        return self.conv_out(self.norm_out(h, zq))
