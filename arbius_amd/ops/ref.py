"""Plain-PyTorch reference implementations of every fused op.

These are the numerics oracle for the HIP kernels in ``csrc/`` (tests compare
the kernels against these in fp32) and the execution path for CPU tensors
(the CPU plumbing config: anythingv3 64x64 2-step DDIM).

Tensor conventions (shared with the HIP kernels):
  * activations are channels-last: images ``[B, H, W, C]``, tokens ``[B, N, C]``
  * conv weights are ``[Cout, kh, kw, Cin]`` (OHWI) so a 3x3 conv is an
    implicit GEMM over K = kh*kw*Cin with contiguous Cin.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def conv2d_nhwc(x, w, b=None, stride=1, padding=1, upsample=False):
    """x [B,H,W,Cin], w [Cout,kh,kw,Cin] -> [B,Ho,Wo,Cout].

    ``upsample=True`` applies a nearest x2 upsample to ``x`` first (the fused
    Upsample2D + conv of the UNet / VAE decoders)."""
    xc = x.permute(0, 3, 1, 2)
    if upsample:
        xc = F.interpolate(xc, scale_factor=2.0, mode="nearest")
    pad = (padding, 0) if w.shape[1] != w.shape[2] else padding   # (3,1) temporal kernel
    y = F.conv2d(xc, w.permute(0, 3, 1, 2), b, stride=stride, padding=pad)
    return y.permute(0, 2, 3, 1).contiguous()


def group_norm_nhwc(x, gamma, beta, groups, eps, silu=False, residual=None):
    """GroupNorm over a channels-last tensor [B, *spatial, C] (+ optional SiLU)."""
    B, C = x.shape[0], x.shape[-1]
    xf = x.float().reshape(B, -1, groups, C // groups)
    mean = xf.mean(dim=(1, 3), keepdim=True)
    var = xf.var(dim=(1, 3), unbiased=False, keepdim=True)
    y = (xf - mean) * torch.rsqrt(var + eps)
    y = y.reshape(x.shape) * gamma.float() + beta.float()
    if silu:
        y = F.silu(y)
    if residual is not None:
        y = y + residual.float()
    return y.to(x.dtype)


def group_norm_mod_nhwc(x, gamma, beta, groups, eps, silu, mod, one_plus):
    """GN(x) * (mod[..., :C] + one_plus) + mod[..., C:] with ``mod`` [B, mh, mw, 2C]
    nearest-upsampled to x's grid (+ SiLU)."""
    B, H, W, C = x.shape
    xf = x.float().reshape(B, -1, groups, C // groups)
    mean = xf.mean(dim=(1, 3), keepdim=True)
    var = xf.var(dim=(1, 3), unbiased=False, keepdim=True)
    y = ((xf - mean) * torch.rsqrt(var + eps)).reshape(x.shape) * gamma.float() + beta.float()
    m = mod.float()
    m = m.repeat_interleave(H // m.shape[1], dim=1).repeat_interleave(W // m.shape[2], dim=2)
    y = y * (m[..., :C] + one_plus) + m[..., C:]
    if silu:
        y = F.silu(y)
    return y.to(x.dtype)


def group_norm_table(x, gamma, beta, groups, eps, mod=None, one_plus=0.0):
    """Reference of the GroupNorm affine table [B, C, 2] (scale, shift)."""
    B, C = x.shape[0], x.shape[-1]
    xf = x.float().reshape(B, -1, groups, C // groups)
    mean = xf.mean(dim=(1, 3))
    var = xf.var(dim=(1, 3), unbiased=False)
    rstd = torch.rsqrt(var + eps)
    cg = C // groups
    sc = rstd.repeat_interleave(cg, dim=1) * gamma.float()[None]
    sf = beta.float()[None] - mean.repeat_interleave(cg, dim=1) * sc
    if mod is not None:
        m = mod[:, :C].float() + one_plus
        sc, sf = sc * m, sf * m + mod[:, C:].float()
    return torch.stack([sc, sf], dim=-1).contiguous()


def layer_norm(x, gamma, beta, eps):
    return F.layer_norm(x.float(), (x.shape[-1],), gamma.float(), beta.float(), eps).to(x.dtype)


def attention(q, k, v, scale=None, causal=False):
    """Token-major multi-head attention.

    q [B, Nq, H, D], k/v [B, Nk, H, D] (any strides) -> out [B, Nq, H, D]."""
    D = q.shape[-1]
    if scale is None:
        scale = 1.0 / math.sqrt(D)
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        n_q, n_k = s.shape[-2], s.shape[-1]
        mask = torch.ones(n_q, n_k, dtype=torch.bool, device=s.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, vf)
    return o.transpose(1, 2).to(q.dtype)


def geglu(h):
    """h [..., 2F] -> a * gelu(gate) with (a, gate) = split(h)."""
    a, gate = h.float().chunk(2, dim=-1)
    return (a * F.gelu(gate)).to(h.dtype)


def silu(x):
    return F.silu(x.float()).to(x.dtype)


def cfg_combine(eps, scale):
    """eps [2B, ...] = cat(uncond, cond) -> uncond + scale*(cond-uncond), fp32."""
    u, c = eps.float().chunk(2)
    return u + scale * (c - u)


def temporal_attention(q, k, v, scale=None):
    """Attention along the frame axis: q/k/v [B, F, P, H, D] -> [B, F, P, H, D]."""
    B, Fr, P, H, D = q.shape
    qs, ks, vs = (t.permute(0, 2, 1, 3, 4).reshape(B * P, Fr, H, D) for t in (q, k, v))
    o = attention(qs, ks, vs, scale)
    return o.reshape(B, P, Fr, H, D).permute(0, 2, 1, 3, 4).contiguous()


def convgru_gates1(ih, h, cat_buf, cx):
    C = h.shape[1]
    r, z = torch.sigmoid(ih[:, :C].float()), torch.sigmoid(ih[:, C:].float())
    cat_buf[:, cx:cx + C] = (r * h.float()).to(cat_buf.dtype)
    return z.to(h.dtype)


def convgru_gates2(c, h, z):
    zf = z.float()
    return ((1 - zf) * h.float() + zf * torch.tanh(c.float())).to(h.dtype)


def sampler_step(tasks):
    """fp32 torch form of csrc/sampler.hip (same formula, same order of terms; CPU / A-B path)."""
    for a in tasks:
        x = a["x"]
        u, c = a["u"].float(), a["c"].float()
        uu, cc = u[..., :4].reshape(x.shape), c[..., :4].reshape(x.shape)
        e = uu + a["g"] * (cc - uu)
        he = a["he"]
        E = he[0] * e
        for coef, key in zip(he[1:], ("h1", "h2", "h3")):
            if a.get(key) is not None:
                E = E + coef * a[key]
        x0 = a["px"] * x + a["pe"] * E
        if a["clamp"] is not None:
            x0 = x0.clamp(-a["clamp"], a["clamp"])
        out = a["ox"] * a["xsrc"] + a["oe"] * E + a["ox0"] * x0
        if a["read_p"]:
            out = out + a["od"] * (x0 - a["p"])
        if a.get("noise") is not None:
            if a["learned"] is not None:
                lb, plv = a["learned"]
                f = (c[..., 4:].reshape(x.shape) + 1.0) * 0.5
                std = torch.exp(0.5 * (f * lb + (1.0 - f) * plv))
            else:
                std = a["std"]
            out = out + std * a["noise"]
        if a.get("hs") is not None:
            a["hs"].copy_(e)
        if a["store_x0"]:
            a["p"].copy_(x0)
        if a["store_cur"]:
            a["cur"].copy_(x)
        x.copy_(out)
        for key in ("xin0", "xin1"):
            if a.get(key) is not None:
                a[key].copy_((out * a["in_scale"]).reshape(a[key].shape).to(a[key].dtype))
