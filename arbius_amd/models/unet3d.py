"""Text-to-video UNet3D (zeroscopev2xl / damo, ModelScope t2v lineage),
channels-last, inference only.  [EXT] architecture per SURVEY.md §2.6(c):

  SD-style spatial blocks (ResBlock2D, Transformer2D with cross-attention to
  1024-d OpenCLIP tokens) interleaved with
  * TemporalConv: 4 x {GroupNorm+SiLU -> Conv3d (3,1,1)} + identity, and
  * TemporalTransformer: GN -> proj_in -> {self-attn over frames, second
    self-attn over frames, GEGLU FF} -> proj_out + residual,
  plus ``transformer_in`` (8 heads) right after conv_in.

MI355X layout: the video batch is ONE frame-major channels-last tensor
[B*F, H, W, C] (frames folded into the batch for every spatial op).  The
temporal ops never permute it:
  * the (3,1,1) Conv3d is the implicit-GEMM conv kernel with a 3x1 tap over the
    same memory viewed as [B, F, H*W, C] (an F x HW image);
  * temporal GroupNorm is the NHWC GroupNorm over [B, F*H*W, C];
  * temporal attention reads q/k/v as strided [B, F, HW, heads, 64] views of
    the fused-QKV GEMM output with the dedicated short-sequence MFMA kernel
    (one wave per (video, pixel, head) problem, csrc/temporal_attention.hip).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple

import torch
import torch.nn as nn

from .. import ops
from .layers import Conv2d, GroupNorm, LayerNorm, Linear, timestep_embedding
from .unet2d import Downsample, FeedForward, ResBlock, Transformer2D, Upsample


@dataclass
class UNet3DConfig:
    in_channels: int = 4
    out_channels: int = 4
    block_channels: Tuple[int, ...] = (320, 640, 1280, 1280)
    attn_levels: Tuple[bool, ...] = (True, True, True, False)
    layers_per_block: int = 2
    head_dim: int = 64
    in_heads: int = 8               # transformer_in
    cross_dim: int = 1024
    groups: int = 32
    eps: float = 1e-5
    time_dim: int = 320

    @staticmethod
    def zeroscope():
        return UNet3DConfig()

    @staticmethod
    def tiny():
        return UNet3DConfig(block_channels=(64, 64, 128, 128), layers_per_block=1, head_dim=32, in_heads=2,
                            cross_dim=32, groups=8, time_dim=64)


class TemporalConv(nn.Module):
    """identity + conv4(conv3(conv2(conv1(x)))) with conv_i = GN+SiLU -> Conv3d(3,1,1)."""

    def __init__(self, c, groups, eps):
        super().__init__()
        self.norms = nn.ModuleList([GroupNorm(groups, c, eps, silu=True) for _ in range(4)])
        self.convs = nn.ModuleList([Conv2d(c, c, 3, padding=1) for _ in range(4)])
        for cv in self.convs:      # (3,1,1) taps: weight [Cout, 3, 1, Cin]
            cv.weight = nn.Parameter(torch.empty(c, 3, 1, c), requires_grad=False)
            cv.k = 3

    def forward(self, x, frames: int):
        BF, H, W, C = x.shape
        v = x.view(BF // frames, frames, H * W, C)
        h = v
        for i in range(4):   # GN (per video) + SiLU fused into each (3,1,1) conv's prologue
            h = self.convs[i](h, residual=v if i == 3 else None, norm=self.norms[i].table(h))
        return h.view(BF, H, W, C)


class TemporalTransformer(nn.Module):
    def __init__(self, c, heads, head_dim, groups):
        super().__init__()
        inner = heads * head_dim
        self.heads, self.hd = heads, head_dim
        self.norm = GroupNorm(groups, c, 1e-6)
        self.proj_in = Linear(c, inner)
        self.norm1 = LayerNorm(inner)
        self.qkv1 = Linear(inner, 3 * inner, bias=False)
        self.out1 = Linear(inner, inner)
        self.norm2 = LayerNorm(inner)
        self.qkv2 = Linear(inner, 3 * inner, bias=False)
        self.out2 = Linear(inner, inner)
        self.norm3 = LayerNorm(inner)
        self.ff = FeedForward(inner)
        self.proj_out = Linear(inner, c)

    def _attn(self, h, ln, qkv_l, out_l, B, F, P):
        qkv = ln.linear(h, qkv_l).view(B, F, P, 3, self.heads, self.hd)     # LayerNorm folded into QKV
        o = ops.temporal_attention(qkv[:, :, :, 0], qkv[:, :, :, 1], qkv[:, :, :, 2])
        return o.view(B * F * P, -1)

    def forward(self, x, frames: int):
        BF, H, W, C = x.shape
        B, P = BF // frames, H * W
        h = self.proj_in.forward_norm(x.view(B, frames * P, C), self.norm.table(x.view(B, frames * P, C)))
        h = h.view(BF * P, -1)
        h = self.out1(self._attn(h, self.norm1, self.qkv1, self.out1, B, frames, P), residual=h)
        h = self.out2(self._attn(h, self.norm2, self.qkv2, self.out2, B, frames, P), residual=h)
        h = self.ff(h, residual=h, ln=self.norm3)
        return self.proj_out(h, residual=x.view(BF * P, C)).view(BF, H, W, C)


class UNet3DCondition(nn.Module):
    def __init__(self, cfg: UNet3DConfig = None):
        super().__init__()
        cfg = cfg or UNet3DConfig()
        self.cfg = cfg
        ch = cfg.block_channels
        tdim = cfg.time_dim * 4
        g, e, hd = cfg.groups, cfg.eps, cfg.head_dim
        self.conv_in = Conv2d(cfg.in_channels, ch[0], 3)
        self.time_lin1 = Linear(cfg.time_dim, tdim)
        self.time_lin2 = Linear(tdim, tdim)
        self.transformer_in = TemporalTransformer(ch[0], cfg.in_heads, hd, g)

        def layer(cin, cout, attn):
            m = nn.Module()
            m.res = ResBlock(cin, cout, tdim, g, e)
            m.tconv = TemporalConv(cout, g, e)
            m.attn = Transformer2D(cout, cfg.cross_dim, cout // hd, g) if attn else None
            m.tattn = TemporalTransformer(cout, cout // hd, hd, g) if attn else None
            return m

        self.down = nn.ModuleList()
        skip_ch = [ch[0]]
        cur = ch[0]
        for lvl, c in enumerate(ch):
            blk = nn.Module()
            blk.layers = nn.ModuleList()
            for _ in range(cfg.layers_per_block):
                blk.layers.append(layer(cur, c, cfg.attn_levels[lvl]))
                cur = c
                skip_ch.append(c)
            blk.downsample = Downsample(c) if lvl < len(ch) - 1 else None
            if blk.downsample is not None:
                skip_ch.append(c)
            self.down.append(blk)
        self.mid_in = layer(cur, cur, False)
        self.mid_attn = Transformer2D(cur, cfg.cross_dim, cur // hd, g)
        self.mid_tattn = TemporalTransformer(cur, cur // hd, hd, g)
        self.mid_out = layer(cur, cur, False)
        self.up = nn.ModuleList()
        rch, rattn = list(reversed(ch)), list(reversed(cfg.attn_levels))
        for lvl, c in enumerate(rch):
            blk = nn.Module()
            blk.layers = nn.ModuleList()
            for _ in range(cfg.layers_per_block + 1):
                blk.layers.append(layer(cur + skip_ch.pop(), c, rattn[lvl]))
                cur = c
            blk.upsample = Upsample(c) if lvl < len(rch) - 1 else None
            self.up.append(blk)
        self.norm_out = GroupNorm(g, ch[0], e, silu=True)
        self.conv_out = Conv2d(ch[0], cfg.out_channels, 3)

    def _resblocks(self) -> List[ResBlock]:
        return [m for m in self.modules() if isinstance(m, ResBlock)]

    def time_embed(self, t, batch, frames, dtype):
        t = t.reshape(-1).to(self.conv_in.weight.device)
        if t.numel() == 1:
            t = t.expand(batch)
        emb = timestep_embedding(t, self.cfg.time_dim).to(dtype)
        emb = ops.silu(self.time_lin2(ops.silu(self.time_lin1(emb))))
        rbs = self._resblocks()
        w = torch.cat([r.temb_proj.weight for r in rbs], 0)
        b = torch.cat([r.temb_proj.bias for r in rbs], 0)
        allp = ops.linear(emb, w, b).repeat_interleave(frames, dim=0)   # one GEMM, per-frame rows
        return dict(zip(rbs, torch.split(allp, [r.cout for r in rbs], dim=1)))

    def _layer(self, m, h, temb, ctx, frames):
        h = m.res(h, temb[m.res])
        h = m.tconv(h, frames)
        if m.attn is not None:
            h = m.attn(h, ctx)
            h = m.tattn(h, frames)
        return h

    def forward(self, x, t, ctx, frames: int):
        """x [B*F, h, w, 4] frame-major latent; t [1] timestep; ctx [B, 77, cross_dim]."""
        BF = x.shape[0]
        B = BF // frames
        temb = self.time_embed(t, B, frames, x.dtype)
        ctx_f = ctx.repeat_interleave(frames, dim=0)
        h = self.conv_in(x)
        h = self.transformer_in(h, frames)
        skips = [h]
        for blk in self.down:
            for m in blk.layers:
                h = self._layer(m, h, temb, ctx_f, frames)
                skips.append(h)
            if blk.downsample is not None:
                h = blk.downsample(h)
                skips.append(h)
        h = self._layer(self.mid_in, h, temb, ctx_f, frames)
        h = self.mid_attn(h, ctx_f)
        h = self.mid_tattn(h, frames)
        h = self._layer(self.mid_out, h, temb, ctx_f, frames)
        for blk in self.up:
            for m in blk.layers:
                h = self._layer(m, ops.cat_channels(h, skips.pop()), temb, ctx_f, frames)
            if blk.upsample is not None:
                h = blk.upsample(h)
        return self.conv_out(h, norm=self.norm_out.table(h))
