"""Kandinsky 2.1 diffusion prior: text -> CLIP image embedding
(SURVEY.md §2.6(b) [EXT]; DALL-E 2 style causal transformer).

Token sequence (one per CFG branch):
    [ CLIP text states (real tokens only) | pooled text | time | x_t | query ]
with learned positional embeddings indexed by the ORIGINAL positions (text
positions 0..76, then 77..80), causal attention, final LN and an output
projection of the query token -> predicted x_0 in the normalised CLIP space.

Padding: the reference masks the padding keys of the text.  Here every sequence
is laid out as [its n real text tokens | pooled | time | x_t | query | pads] and
padded to a fixed 81 tokens: under causal attention no real token ever sees a
trailing pad, so the pads need no mask, and every sequence of a lock-step group
(any mix of prompt lengths, cond and uncond rows) runs in ONE batch with static
shapes; the query token n+3 of each row is read.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn

from .. import ops
from .layers import LayerNorm, Linear, timestep_embedding


@dataclass
class PriorConfig:
    width: int = 2048
    layers: int = 20
    heads: int = 32
    clip_dim: int = 768
    text_ctx: int = 77

    @staticmethod
    def kandinsky21():
        return PriorConfig()

    @staticmethod
    def tiny():
        return PriorConfig(width=64, layers=2, heads=2, clip_dim=32)


class PriorBlock(nn.Module):
    def __init__(self, cfg: PriorConfig):
        super().__init__()
        w = cfg.width
        self.heads = cfg.heads
        self.ln1 = LayerNorm(w)
        self.qkv = Linear(w, 3 * w)
        self.out = Linear(w, w)
        self.ln2 = LayerNorm(w)
        self.fc1 = Linear(w, 4 * w)
        self.fc2 = Linear(4 * w, w)

    def forward(self, x):
        B, N, C = x.shape
        H = self.heads
        qkv = self.ln1.linear(x, self.qkv).view(B, N, 3, H, C // H)   # LayerNorm folded into QKV
        o = ops.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], causal=True)
        x = self.out(o.reshape(B, N, C), residual=x)
        return self.fc2(self.ln2.linear(x, self.fc1, act="gelu"), residual=x)     # GELU in the GEMM epilogue


class PriorTransformer(nn.Module):
    def __init__(self, cfg: PriorConfig = None):
        super().__init__()
        cfg = cfg or PriorConfig()
        self.cfg = cfg
        w, d = cfg.width, cfg.clip_dim
        self.text_enc_proj = Linear(d, w)
        self.text_emb_proj = Linear(d, w)
        self.img_proj = Linear(d, w)
        self.time1 = Linear(w, w)
        self.time2 = Linear(w, w)
        self.pos = nn.Parameter(torch.zeros(cfg.text_ctx + 4, w), requires_grad=False)
        self.query = nn.Parameter(torch.zeros(w), requires_grad=False)
        self.blocks = nn.ModuleList([PriorBlock(cfg) for _ in range(cfg.layers)])
        self.final_ln = LayerNorm(w)
        self.out_proj = Linear(w, d)
        # CLIP image-embedding normalisation statistics (checkpoint buffers)
        self.clip_mean = nn.Parameter(torch.zeros(d), requires_grad=False)
        self.clip_std = nn.Parameter(torch.ones(d), requires_grad=False)

    def reset(self, gen):
        self.pos.data.normal_(0, 0.01, generator=gen)
        self.query.data.normal_(0, 0.01, generator=gen)

    def layout(self, ns, device):
        """Gather map of the padded sequences: token j of row b comes from source slot idx[b, j] of
        [text 0..76 | pooled, time, x_t, query | zero], and the query sits at n_b + 3."""
        ctx = self.cfg.text_ctx
        L = ctx + 4
        j = torch.arange(L, device=device)[None]
        n = torch.tensor([int(v) for v in ns], device=device)[:, None]
        idx = torch.where(j < n, j, torch.where(j < n + 4, ctx + (j - n), torch.full_like(j, L)))
        return idx, (n[:, 0] + 3)

    def forward(self, x_t, t, text_states, text_pooled, ns, layout=None, tt=None):
        """x_t [B,d] (normalised), t scalar, text_states [B,77,d], text_pooled [B,d], ns[b] = real
        text tokens of row b -> predicted x_0 [B,d].  ``layout``: a cached ``self.layout(ns)``;
        ``tt``: the timestep as a device tensor [1] fp32 instead of ``t`` (hipGraph replay)."""
        w = self.cfg.width
        B = x_t.shape[0]
        idx, q = layout if layout is not None else self.layout(ns, x_t.device)
        if tt is None:
            tt = torch.tensor([float(t)], device=x_t.device)
        temb = self.time2(ops.silu(self.time1(timestep_embedding(tt, w).to(x_t.dtype))))
        src = torch.cat([self.text_enc_proj(text_states), self.text_emb_proj(text_pooled)[:, None],
                         temb[:, None].expand(B, 1, w), self.img_proj(x_t)[:, None],
                         self.query.to(x_t.dtype)[None, None].expand(B, 1, w),
                         torch.zeros(B, 1, w, dtype=x_t.dtype, device=x_t.device)], dim=1)
        pos = torch.cat([self.pos, torch.zeros(1, w, dtype=self.pos.dtype, device=self.pos.device)]).to(x_t.dtype)
        g = idx[:, :, None].expand(B, idx.shape[1], w)
        h = torch.gather(src, 1, g) + pos[idx]
        for blk in self.blocks:
            h = blk(h)
        last = h[torch.arange(B, device=h.device), q][:, None]
        return self.out_proj(self.final_ln(last))[:, 0]
