"""XLM-RoBERTa text tower + M-CLIP pooling head (the Kandinsky 2.1 multilingual
text encoder, SURVEY.md §2.6(b) [EXT]).

Post-LN BERT layout: embeddings (word + position[offset 2] + type) -> LN ->
L x {x = LN(x + Attn(x)); x = LN(x + FFN_gelu(x))}.  M-CLIP returns the full
token states ``[77, 1024]`` (decoder context) and a masked-mean pooled vector
projected 1024 -> 768.

Padding: instead of an additive key mask, each sequence runs with its keys
and values sliced to its real length (queries at pad positions still attend
to the real tokens, exactly as a masked softmax does), so the shared flash
kernel needs no mask support and pad keys cost nothing.
"""
from __future__ import annotations

import hashlib
import re
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from .. import ops
from .layers import Embedding, LayerNorm, Linear


@dataclass
class XLMRConfig:
    vocab: int = 250002
    width: int = 1024
    layers: int = 24
    heads: int = 16
    mlp: int = 4096
    max_pos: int = 514
    max_len: int = 77
    proj_dim: int = 768           # M-CLIP LinearTransformation
    eps: float = 1e-5

    @staticmethod
    def large():
        return XLMRConfig()

    @staticmethod
    def tiny():
        return XLMRConfig(vocab=1000, width=32, layers=2, heads=2, mlp=64, max_pos=100, proj_dim=32)


class XLMRTokenizer:
    """sentencepiece tokenizer when ``sentencepiece.bpe.model`` is available
    locally; otherwise a deterministic hashed-word fallback with the same id
    layout (<s>=0, <pad>=1, </s>=2, 77 positions)."""
    BOS, PAD, EOS = 0, 1, 2
    _WORD = re.compile(r"\w+|[^\w\s]+")

    def __init__(self, vocab: int, max_len: int = 77, model_dir: Optional[str] = None):
        self.vocab, self.max_len = vocab, max_len
        self._sp = None
        self.source = "hashed-words"
        from .tokenizer import find_file
        f = find_file(model_dir, "sentencepiece.bpe.model",
                      ("", "xlmr_tokenizer", "tokenizer_xlmr", "mclip_tokenizer", "tokenizer", "text_encoder"))
        if f is not None:
            import sentencepiece as spm
            self._sp = spm.SentencePieceProcessor(model_file=str(f))
            self.source = str(f.parent)

    def __call__(self, text: str) -> Tuple[List[int], int]:
        if self._sp is not None:
            ids = [i + 1 for i in self._sp.encode(text)]   # fairseq offset
        else:
            ids = []
            for w in self._WORD.findall(text.lower()):
                h = int.from_bytes(hashlib.blake2b(w.encode(), digest_size=8).digest(), "little")
                ids.append(4 + h % (self.vocab - 4))
        ids = [self.BOS] + ids[: self.max_len - 2] + [self.EOS]
        n = len(ids)
        return ids + [self.PAD] * (self.max_len - n), n


class XLMRLayer(nn.Module):
    def __init__(self, cfg: XLMRConfig):
        super().__init__()
        self.heads = cfg.heads
        self.qkv = Linear(cfg.width, 3 * cfg.width)
        self.out = Linear(cfg.width, cfg.width)
        self.ln1 = LayerNorm(cfg.width, cfg.eps)
        self.fc1 = Linear(cfg.width, cfg.mlp)
        self.fc2 = Linear(cfg.mlp, cfg.width)
        self.ln2 = LayerNorm(cfg.width, cfg.eps)

    def forward(self, x, ns: List[int]):
        """x [B, 77, C]; ns[b] = real tokens of sequence b (its keys / values are sliced to them;
        sequences of equal length share one attention launch)."""
        B, N, C = x.shape
        H = self.heads
        qkv = self.qkv(x).view(B, N, 3, H, C // H)
        if len(set(ns)) == 1:
            o = ops.attention(qkv[:, :, 0], qkv[:, :ns[0], 1], qkv[:, :ns[0], 2])
        else:
            o = torch.empty(B, N, H, C // H, dtype=x.dtype, device=x.device)
            for n in sorted(set(ns)):
                rows = [b for b in range(B) if ns[b] == n]
                i0, i1 = rows[0], rows[-1] + 1
                if rows == list(range(i0, i1)):          # contiguous run: views, no gather
                    o[i0:i1] = ops.attention(qkv[i0:i1, :, 0], qkv[i0:i1, :n, 1], qkv[i0:i1, :n, 2])
                else:
                    for b in rows:
                        o[b:b + 1] = ops.attention(qkv[b:b + 1, :, 0], qkv[b:b + 1, :n, 1], qkv[b:b + 1, :n, 2])
        x = self.ln1(self.out(o.reshape(B, N, C), residual=x))
        h = self.fc1(x, act="gelu")                                 # GELU in the GEMM epilogue
        return self.ln2(self.fc2(h, residual=x))


class MCLIPText(nn.Module):
    def __init__(self, cfg: XLMRConfig = None):
        super().__init__()
        cfg = cfg or XLMRConfig()
        self.cfg = cfg
        self.tok = Embedding(cfg.vocab, cfg.width)
        self.pos = Embedding(cfg.max_pos, cfg.width)
        self.tok_type = Embedding(1, cfg.width)
        self.ln = LayerNorm(cfg.width, cfg.eps)
        self.layers = nn.ModuleList([XLMRLayer(cfg) for _ in range(cfg.layers)])
        self.proj = Linear(cfg.width, cfg.proj_dim)

    def forward(self, ids: torch.Tensor, ns):
        """ids [B, 77], ns = real length of each sequence (an int: every row) -> (full [B,77,W],
        pooled [B,proj]).  Row-wise arithmetic only (GEMM plans under ``ops.plan_batch``), so a
        sequence's outputs do not depend on the other rows of the batch."""
        B, L = ids.shape
        ns = [int(ns)] * B if isinstance(ns, int) else [int(n) for n in ns]
        pos = torch.arange(L, device=ids.device)[None].expand(B, L)
        lim = torch.tensor(ns, device=ids.device)[:, None]
        pos = torch.where(pos < lim, pos + 2, torch.ones_like(pos))   # pad positions use padding_idx
        x = self.tok(ids) + self.pos(pos) + self.tok_type.weight[0]
        x = self.ln(x)
        for layer in self.layers:
            x = layer(x, ns)
        pooled = torch.stack([x[b, :n].float().mean(dim=0) for b, n in enumerate(ns)]).to(x.dtype)
        return x, self.proj(pooled)
