"""GLIDE / guided-diffusion style UNet (the Kandinsky 2.1 latent decoder UNet),
channels-last, inference only.  [EXT] architecture per SURVEY.md §2.6(b):

* ResBlocks with scale-shift norm: h = GN(h) * (1 + scale) + shift, scale/shift
  from the (time + image) embedding; resblock up/down-sampling;
* attention blocks whose K/V concatenate the projected TEXT tokens to the spatial
  tokens (one joint softmax over HW + 77 keys) - the ``encoder_kv`` attention;
* the CLIP image embedding conditions through the time embedding and as extra
  context tokens; output channels = 2 x latent (eps + learned variance).

Everything heavy runs on the shared HIP kernels (implicit-GEMM conv, GroupNorm,
flash attention).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import torch
import torch.nn as nn

from .. import ops
from .layers import Conv2d, GroupNorm, LayerNorm, Linear, timestep_embedding


@dataclass
class GlideUNetConfig:
    in_channels: int = 4
    out_channels: int = 8
    model_channels: int = 384
    channel_mult: Tuple[int, ...] = (1, 2, 3, 4)
    num_res_blocks: int = 3
    attention_ds: Tuple[int, ...] = (2, 4, 8)   # downsample factors with attention
    head_channels: int = 64
    text_dim: int = 1024                        # XLM-R token width (full states)
    pooled_dim: int = 768                       # M-CLIP pooled text embedding
    encoder_channels: int = 768                 # context width (model_dim) after projection
    image_embed_dim: int = 768                  # CLIP image embedding
    image_tokens: int = 10                      # image embedding -> extra context tokens
    groups: int = 32

    @staticmethod
    def kandinsky21():
        return GlideUNetConfig()

    @staticmethod
    def tiny():
        return GlideUNetConfig(model_channels=32, channel_mult=(1, 2), num_res_blocks=1, attention_ds=(2,),
                               head_channels=16, text_dim=32, pooled_dim=32, encoder_channels=32,
                               image_embed_dim=32, image_tokens=2, groups=8)


class SSResBlock(nn.Module):
    def __init__(self, cin, cout, emb_dim, groups, up=False, down=False):
        super().__init__()
        self.norm1 = GroupNorm(groups, cin, 1e-5, silu=True)
        self.conv1 = Conv2d(cin, cout, 3)
        self.emb = Linear(emb_dim, 2 * cout)
        self.norm2 = GroupNorm(groups, cout, 1e-5, silu=False)
        self.conv2 = Conv2d(cout, cout, 3)
        self.skip = Conv2d(cin, cout, 1) if cin != cout else None
        self.up, self.down = up, down
        self.cout = cout

    def forward(self, x, emb_act):
        if self.down:                                   # avg-pool does not commute with SiLU:
            h, x = ops.pool2(x, self.norm1.table(x))    # pool(GN+SiLU(x)) and pool(x), one pass
            h = self.conv1(h)
        else:                                           # GN+SiLU (and nearest-up) fused into conv1
            h = self.conv1(x, upsample=self.up, norm=self.norm1.table(x))
            if self.up:
                x = ops.upsample2(x)
        ss = self.emb(emb_act)                          # [B, 2C] = [scale | shift]
        # scale-shift norm + SiLU folded into one per-(b, c) affine table: conv2's prologue
        norm = self.norm2.table(h, mod=ss, one_plus=1.0, silu=True)
        skip = self.skip(x) if self.skip is not None else ops.materialize(x)
        return self.conv2(h, residual=skip, norm=norm)


class JointAttention(nn.Module):
    """Self-attention over spatial tokens with the context tokens appended to K/V."""

    def __init__(self, c, ctx_dim, head_channels, groups):
        super().__init__()
        self.heads = max(1, c // head_channels)
        self.norm = GroupNorm(groups, c, 1e-5)
        self.qkv = Linear(c, 3 * c)
        self.ctx_kv = Linear(ctx_dim, 2 * c)
        self.out = Linear(c, c)

    def forward(self, x, ctx):
        B, H, W, C = x.shape
        N, Hh = H * W, self.heads
        qkv = self.qkv.forward_norm(x.view(B, N, C), self.norm.table(x)).view(B, N, 3, Hh, C // Hh)
        ckv = self.ctx_kv(ctx).view(B, ctx.shape[1], 2, Hh, C // Hh)
        # joint softmax over [context tokens | spatial tokens]: the context K/V are a prefix
        # segment read in place by the flash kernel (encoder_kv attention, no concat copy)
        o = ops.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], kv_prefix=(ckv[:, :, 0], ckv[:, :, 1]))
        return self.out(o.reshape(B, N, C), residual=x.view(B, N, C)).view(B, H, W, C)


class GlideUNet(nn.Module):
    def __init__(self, cfg: GlideUNetConfig = None):
        super().__init__()
        cfg = cfg or GlideUNetConfig()
        self.cfg = cfg
        mc = cfg.model_channels
        ed = 4 * mc
        self.time1 = Linear(mc, ed)
        self.time2 = Linear(ed, ed)
        self.img_emb = Linear(cfg.image_embed_dim, ed)
        self.img_tokens = Linear(cfg.image_embed_dim, cfg.image_tokens * cfg.encoder_channels)
        self.text_proj = Linear(cfg.text_dim, cfg.encoder_channels)
        self.text_pool = Linear(cfg.pooled_dim, ed)
        self.text_norm = LayerNorm(ed)                  # diffusers add_embedding.text_norm (ln_model_n)
        self.conv_in = Conv2d(cfg.in_channels, mc, 3)
        self.down = nn.ModuleList()
        chans = [mc]
        ch, ds = mc, 1
        for lvl, mult in enumerate(cfg.channel_mult):
            for _ in range(cfg.num_res_blocks):
                blk = nn.Module()
                blk.res = SSResBlock(ch, mult * mc, ed, cfg.groups)
                ch = mult * mc
                blk.attn = JointAttention(ch, cfg.encoder_channels, cfg.head_channels, cfg.groups) \
                    if ds in cfg.attention_ds else None
                self.down.append(blk)
                chans.append(ch)
            if lvl != len(cfg.channel_mult) - 1:
                blk = nn.Module()
                blk.res = SSResBlock(ch, ch, ed, cfg.groups, down=True)
                blk.attn = None
                self.down.append(blk)
                chans.append(ch)
                ds *= 2
        self.mid1 = SSResBlock(ch, ch, ed, cfg.groups)
        self.mid_attn = JointAttention(ch, cfg.encoder_channels, cfg.head_channels, cfg.groups)
        self.mid2 = SSResBlock(ch, ch, ed, cfg.groups)
        self.up = nn.ModuleList()
        for lvl, mult in list(enumerate(cfg.channel_mult))[::-1]:
            for i in range(cfg.num_res_blocks + 1):
                blk = nn.Module()
                blk.res = SSResBlock(ch + chans.pop(), mult * mc, ed, cfg.groups)
                ch = mult * mc
                blk.attn = JointAttention(ch, cfg.encoder_channels, cfg.head_channels, cfg.groups) \
                    if ds in cfg.attention_ds else None
                blk.upsample = SSResBlock(ch, ch, ed, cfg.groups, up=True) \
                    if (lvl and i == cfg.num_res_blocks) else None
                self.up.append(blk)
            if lvl:
                ds //= 2
        self.norm_out = GroupNorm(cfg.groups, ch, 1e-5, silu=True)
        self.conv_out = Conv2d(ch, cfg.out_channels, 3)

    def forward(self, x, t, text_tokens, text_pooled, image_embed):
        """x [B,h,w,4]; t [B] or scalar; text_tokens [B,77,text_dim]; text_pooled [B,pooled_dim];
        image_embed [B,768].  Context = [image tokens | projected text tokens]."""
        B = x.shape[0]
        if not torch.is_tensor(t):
            t = torch.tensor([float(t)], device=x.device)
        t = t.reshape(-1).to(x.device)
        if t.numel() == 1:
            t = t.expand(B)
        emb = timestep_embedding(t, self.cfg.model_channels).to(x.dtype)
        emb = self.time2(ops.silu(self.time1(emb)))
        # time + (image_proj(image) + LN(text_proj(pooled text)))  (diffusers TextImageTimeEmbedding)
        emb = emb + (self.img_emb(image_embed) + self.text_norm(self.text_pool(text_pooled)))
        emb_act = ops.silu(emb)
        itok = self.img_tokens(image_embed).view(B, self.cfg.image_tokens, self.cfg.encoder_channels)
        ctx = torch.cat([itok, self.text_proj(text_tokens)], dim=1)
        h = self.conv_in(x)
        hs = [h]
        for blk in self.down:
            h = blk.res(h, emb_act)
            if blk.attn is not None:
                h = blk.attn(h, ctx)
            hs.append(h)
        h = self.mid1(h, emb_act)
        h = self.mid_attn(h, ctx)
        h = self.mid2(h, emb_act)
        for blk in self.up:
            h = blk.res(ops.cat_channels(h, hs.pop()), emb_act)
            if blk.attn is not None:
                h = blk.attn(h, ctx)
            if blk.upsample is not None:
                h = blk.upsample(h, emb_act)
        return self.conv_out(h, norm=self.norm_out.table(h))
