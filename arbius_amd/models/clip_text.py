"""CLIP text transformer (ViT-L/14 text tower for SD1.5; also the OpenCLIP
ViT-H text tower for zeroscope/damo and the Kandinsky prior encoder).

Causal pre-LN transformer, quick-GELU (OpenAI) or GELU (OpenCLIP) MLP; the
attention is the shared HIP flash kernel with ``causal=True``.  Runs once per
task ([2, 77, 768]).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn

from .. import ops
from .layers import Embedding, LayerNorm, Linear


@dataclass
class CLIPTextConfig:
    vocab: int = 49408
    max_len: int = 77
    width: int = 768
    layers: int = 12
    heads: int = 12
    mlp: int = 3072
    quick_gelu: bool = True
    # SD2/zeroscope use the penultimate layer; SD1.5 uses the last (+final LN)
    skip_last: int = 0

    @staticmethod
    def vit_l14():
        return CLIPTextConfig()

    @staticmethod
    def vit_h14():
        return CLIPTextConfig(width=1024, layers=24, heads=16, mlp=4096, quick_gelu=False, skip_last=1)

    @staticmethod
    def tiny(width=32):
        return CLIPTextConfig(width=width, layers=2, heads=2, mlp=4 * width)


class CLIPLayer(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.heads = cfg.heads
        self.ln1 = LayerNorm(cfg.width)
        self.qkv = Linear(cfg.width, 3 * cfg.width)
        self.out = Linear(cfg.width, cfg.width)
        self.ln2 = LayerNorm(cfg.width)
        self.fc1 = Linear(cfg.width, cfg.mlp)
        self.fc2 = Linear(cfg.mlp, cfg.width)
        self.quick = cfg.quick_gelu

    def forward(self, x):
        B, N, C = x.shape
        H = self.heads
        qkv = self.ln1.linear(x, self.qkv).view(B, N, 3, H, C // H)   # LayerNorm folded into QKV
        o = ops.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], causal=True)
        x = self.out(o.reshape(B, N, C), residual=x)
        h = self.ln2.linear(x, self.fc1, act="quick_gelu" if self.quick else "gelu")   # LN + act in the GEMM
        return self.fc2(h, residual=x)


class CLIPTextEncoder(nn.Module):
    def __init__(self, cfg: CLIPTextConfig = None):
        super().__init__()
        cfg = cfg or CLIPTextConfig()
        self.cfg = cfg
        self.tok = Embedding(cfg.vocab, cfg.width)
        self.pos = Embedding(cfg.max_len, cfg.width)
        self.layers = nn.ModuleList([CLIPLayer(cfg) for _ in range(cfg.layers)])
        self.final_ln = LayerNorm(cfg.width)

    def forward(self, ids):
        """ids [B, 77] int64 -> hidden [B, 77, width] (and pooled EOS features)."""
        x = self.tok(ids) + self.pos.weight[: ids.shape[1]][None]
        n = len(self.layers) - self.cfg.skip_last
        for layer in self.layers[:n]:
            x = layer(x)
        x = self.final_ln(x)
        eos = ids.argmax(dim=-1)  # EOS has the largest id in the CLIP vocab
        pooled = x[torch.arange(x.shape[0], device=x.device), eos]
        return x, pooled
