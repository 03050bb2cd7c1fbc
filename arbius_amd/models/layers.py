"""Channels-last building blocks shared by every model family.

All spatial activations are ``[B, H, W, C]`` and all token activations
``[B, N, C]``; every heavy op goes through ``arbius_amd.ops`` (HIP kernels on
GPU, PyTorch reference on CPU).  Parameters are plain tensors registered on
``nn.Module`` so weights can be RCCL-broadcast / loaded from safetensors
without any framework glue.

Random init is deterministic per module path (``init_weights(seed)``): the
benchmark runs random-init weights of the real architectures (BASELINE.json).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import ops


class Linear(nn.Module):
    def __init__(self, cin, cout, bias=True):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(cout, cin), requires_grad=False)
        self.bias = nn.Parameter(torch.empty(cout), requires_grad=False) if bias else None
        self.cin, self.cout = cin, cout

    def reset(self, gen):
        bound = 1.0 / math.sqrt(self.cin)
        self.weight.data.uniform_(-bound, bound, generator=gen)
        if self.bias is not None:
            self.bias.data.uniform_(-bound, bound, generator=gen)

    def forward(self, x, residual=None, act=None):
        return ops.linear(x, self.weight, self.bias, residual=residual, act=act)

    def forward_norm(self, x, norm):
        """x [B, ..., Cin] with a GroupNorm(+SiLU) prologue from ``norm = (table, silu)`` (table per
        batch row b): run as a 1x1 implicit-GEMM conv over the [B, 1, N, Cin] view."""
        B, C = x.shape[0], x.shape[-1]
        y = ops.conv2d(x.reshape(B, 1, -1, C), self.weight.view(self.cout, 1, 1, self.cin), self.bias,
                       padding=0, norm=norm)
        return y.view(*x.shape[:-1], self.cout)


class Conv2d(nn.Module):
    """kxk conv, stride 1 or 2, channels-last; weight [Cout, k, k, Cin]."""

    def __init__(self, cin, cout, k=3, stride=1, padding=None, bias=True):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(cout, k, k, cin), requires_grad=False)
        self.bias = nn.Parameter(torch.empty(cout), requires_grad=False) if bias else None
        self.cin, self.cout, self.k, self.stride = cin, cout, k, stride
        self.padding = k // 2 if padding is None else padding

    def reset(self, gen):
        bound = 1.0 / math.sqrt(self.cin * self.k * self.k)
        self.weight.data.uniform_(-bound, bound, generator=gen)
        if self.bias is not None:
            self.bias.data.uniform_(-bound, bound, generator=gen)

    def forward(self, x, upsample=False, residual=None, temb=None, norm=None):
        """``norm = (table, silu)``: GroupNorm(+SiLU) prologue fused into the conv."""
        return ops.conv2d(x, self.weight, self.bias, stride=self.stride, padding=self.padding,
                          upsample=upsample, residual=residual, temb=temb, norm=norm)


class GroupNorm(nn.Module):
    def __init__(self, groups, channels, eps=1e-5, silu=False):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(channels), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(channels), requires_grad=False)
        self.groups, self.eps, self.silu = groups, eps, silu

    def reset(self, gen):
        self.weight.data.fill_(1.0)
        self.bias.data.zero_()

    def forward(self, x, silu=None):
        return ops.group_norm(x, self.weight, self.bias, self.groups, self.eps,
                              self.silu if silu is None else silu)

    def table(self, x, mod=None, one_plus=0.0, silu=None):
        """This GroupNorm of ``x`` for a consumer (``ops.NormSpec``): a fused operand prologue from
        the (lazily computed) affine table, or one stats + table-apply pass in front of it."""
        return ops.NormSpec(x, self.weight, self.bias, self.groups, self.eps, mod, one_plus,
                            self.silu if silu is None else silu)


class LayerNorm(nn.Module):
    def __init__(self, channels, eps=1e-5):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(channels), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(channels), requires_grad=False)
        self.eps = eps

    def reset(self, gen):
        self.weight.data.fill_(1.0)
        self.bias.data.zero_()

    def forward(self, x):
        return ops.layer_norm(x, self.weight, self.bias, self.eps)

    def linear(self, x, lin: "Linear", residual=None, act=None):
        """act(lin(self(x))) with this LayerNorm (and the activation) folded into the GEMM (ops.ln_linear)."""
        return ops.ln_linear(x, self.weight, self.bias, self.eps, lin.weight, lin.bias, residual=residual, act=act)

    def linear_geglu(self, x, lin: "Linear"):
        """GEGLU projection of self(x) with this LayerNorm folded in (ops.ln_linear_geglu)."""
        return ops.ln_linear_geglu(x, self.weight, self.bias, self.eps, lin.weight, lin.bias)


class Embedding(nn.Module):
    def __init__(self, n, dim):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(n, dim), requires_grad=False)

    def reset(self, gen):
        self.weight.data.normal_(0.0, 0.02, generator=gen)

    def forward(self, idx):
        return self.weight[idx]


def init_weights(module: nn.Module, seed: int = 0) -> nn.Module:
    """Deterministic random init of every leaf with a ``reset(gen)``, in
    module-registration order, from one CPU generator."""
    gen = torch.Generator(device="cpu").manual_seed(seed)
    for m in module.modules():
        if hasattr(m, "reset") and m is not module:
            m.reset(gen)
    return module


def timestep_embedding(t, dim, flip_sin_to_cos=True, freq_shift=0.0, max_period=10000):
    """Sinusoidal timestep features (diffusers ``get_timestep_embedding`` semantics)."""
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(half, dtype=torch.float32, device=t.device)
    exponent = exponent / (half - freq_shift)
    emb = t.float()[:, None] * torch.exp(exponent)[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


def fuse_qkv(layers):
    """Concatenate the weights of several bias-free Linear layers into one GEMM."""
    return torch.cat([l.weight for l in layers], dim=0)
