"""ctypes binding of ``libarbius_kernels.so`` (the gfx950 HIP kernels in csrc/).

Kernels are launched on PyTorch's current HIP stream, output buffers come from
the PyTorch caching allocator, so everything here is hipGraph-capture safe.
Shape/stride checks happen on the host BEFORE a launch (a bad launch on the
shared GPU box can fault the whole node).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

_HERE = Path(__file__).resolve().parent
# ARBIUS_KERNEL_LIB: an alternative in-tree build (A/B runs of a kernel change)
_LIB_PATH = _HERE / os.environ.get("ARBIUS_KERNEL_LIB", "libarbius_kernels.so")
_lib = None
_SYMBOLS = {}

c_void_p, c_int, c_long, c_float, c_size_t = (ctypes.c_void_p, ctypes.c_int, ctypes.c_long,
                                              ctypes.c_float, ctypes.c_size_t)

_SIGS = {
    "arb_group_norm_workspace": (c_size_t, [c_int, c_int, c_int, c_int]),
    "arb_group_norm_nhwc": (c_int, [c_void_p] * 5 + [c_int] * 4 + [c_float, c_int, c_void_p]),
    "arb_group_norm_mod_nhwc": (c_int, [c_void_p] * 6 + [c_int] * 5 + [c_float, c_int, c_int, c_int, c_float,
                                                                        c_void_p]),
    "arb_layer_norm": (c_int, [c_void_p] * 4 + [c_int, c_int, c_float, c_long, c_void_p]),
    "arb_flash_attention": (c_int, [c_void_p] * 5 + [c_int] * 5 + [c_float, c_int] + [c_void_p] * 3
                            + [c_int, c_void_p]),
    "arb_geglu": (c_int, [c_void_p, c_void_p, c_long, c_int, c_void_p]),
    "arb_silu": (c_int, [c_void_p, c_void_p, c_long, c_void_p]),
    "arb_norm_table_apply": (c_int, [c_void_p] * 3 + [c_int, c_long, c_int, c_int, c_void_p]),
    "arb_norm_pool2": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "arb_upsample2": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "arb_conv2d_nhwc": (c_int, [c_void_p] * 8 + [c_int] * 12 + [c_void_p]),
    "arb_set_gn_table_lds": (None, [c_int]),
    "arb_set_gn_tail": (None, [c_int]),
    "arb_set_attn_prescale": (None, [c_int]),
    "arb_set_stag2_pd": (None, [c_int]),
    "arb_set_stag2_buf": (None, [c_int]),
    "arb_set_attn_pp": (None, [c_int]),
    "arb_set_attn_ilp": (None, [c_int]),
    "arb_set_attn_glds": (None, [c_int]),
    "arb_conv2d_nhwc_tld": (c_int, [c_void_p] * 4 + [c_int] + [c_void_p] * 4 + [c_int] * 12 + [c_void_p]),
    "arb_conv2d_nhwc_f16": (c_int, [c_void_p] * 7 + [c_int] * 11 + [c_void_p]),
    "arb_group_norm_table": (c_int, [c_void_p] * 4 + [c_float] + [c_void_p] * 2 + [c_int] * 4 + [c_float, c_void_p]),
    "arb_conv2d_workspace": (c_size_t, [c_int] * 11),
    "arb_conv2d_plan": (c_int, [c_int] * 9 + [c_void_p]),
    "arb_conv_family": (c_int, [c_int] * 6),
    "arb_gemm_bias_res": (c_int, [c_void_p] * 6 + [c_int] * 5 + [c_void_p]),
    "arb_gemm_geglu": (c_int, [c_void_p] * 5 + [c_int] * 5 + [c_void_p]),
    "arb_temporal_attention": (c_int, [c_void_p] * 5 + [c_int] * 5 + [c_float, c_void_p]),
    "arb_convgru_gates": (c_int, [c_int] + [c_void_p] * 4 + [c_long, c_int, c_int, c_int, c_void_p]),
    "arb_sampler_step": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p]),
    "arb_dwconv_f16": (c_int, [c_void_p] * 4 + [c_int] * 8 + [c_void_p]),
    "arb_softmax_rows": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p]),
    "arb_group_norm_slice_ok": (c_int, [c_int] * 3),
    "arb_group_norm_slice": (c_int, [c_void_p] * 2 + [c_int] + [c_void_p] * 4 + [c_float] + [c_int] * 4
                             + [c_float, c_int, c_void_p]),
    "arb_group_norm_table_cat": (c_int, [c_void_p] * 2 + [c_int] + [c_void_p] * 3 + [c_float] + [c_void_p] * 2
                                 + [c_int] * 4 + [c_float, c_void_p]),
    "arb_norm_table_apply_cat": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_long, c_int, c_int,
                                         c_void_p]),
    "arb_conv2d_nhwc_cat": (c_int, [c_void_p, c_void_p, c_int] + [c_void_p] * 6 + [c_int] * 11 + [c_void_p]),
    "arb_row_stats": (c_int, [c_void_p, c_void_p, c_int, c_int, c_float, c_long, c_void_p]),
    "arb_conv2d_ex": (c_int, [c_void_p] * 7 + [c_int] * 13 + [c_void_p]),
    "arb_rvm_resize_u8": (c_int, [c_void_p, c_void_p] + [c_int] * 5 + [c_void_p]),
    "arb_rvm_stem": (c_int, [c_void_p] * 3 + [c_int] * 3 + [c_void_p]),
    "arb_rvm_pool3": (c_int, [c_void_p] * 4 + [c_int] * 3 + [c_void_p]),
    "arb_rvm_upcat": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p] + [c_int] * 4
                      + [c_void_p]),
    "arb_rvm_pack": (c_int, [c_void_p, c_int, c_void_p, c_long, c_int, c_int, c_void_p, c_int, c_long, c_void_p]),
    "arb_rvm_gru_out": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p, c_int,
                                c_void_p, c_long, c_int, c_long, c_int, c_void_p]),
    "arb_rvm_dgf": (c_int, [c_void_p] * 7 + [c_int] * 6 + [c_float] * 3 + [c_void_p]),
    "arb_rvm_args_sizes": (c_size_t, [c_int]),
    "arb_rvm_chan_mean": (c_int, [c_void_p, c_void_p, c_int, c_long, c_int, c_void_p]),
    "arb_rvm_gate": (c_int, [c_void_p, c_void_p, c_int, c_long, c_int, c_int, c_void_p]),
    "arb_gemm_ln": (c_int, [c_void_p] * 8 + [c_int] * 7 + [c_void_p]),
    "arb_gemm_act": (c_int, [c_void_p] * 6 + [c_int] * 6 + [c_void_p]),
    "arb_image_u8": (c_int, [c_void_p, c_void_p, c_long, c_int, c_void_p]),
    "arb_rgb_to_yuv420": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "arb_attention512": (c_int, [c_void_p] * 5 + [c_int] * 4 + [c_float, c_void_p, c_void_p]),
    "arb_attention512_workspace": (c_long, [c_int] * 4),
    "arb_h264_intra_workspace": (c_size_t, [c_int] * 3),
    "arb_h264_intra_encode": (c_int, [c_void_p] * 3 + [c_int] * 4 + [c_void_p, c_void_p, ctypes.c_longlong, c_void_p,
                                                                    c_void_p]),
    "arb_h264_intra_host": (c_int, [c_void_p] * 3 + [c_int] * 4 + [c_void_p, ctypes.c_longlong, c_void_p, c_void_p]),
    "arb_set_h264_sync": (None, [c_int]),
}


def lib():
    """Load the kernel library; raises (loudly) if it is missing or stale."""
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            if os.environ.get("ARBIUS_AUTOBUILD", "1") == "1":
                from .build import build
                build()
            if not _LIB_PATH.exists():
                raise RuntimeError(
                    f"{_LIB_PATH} missing: build it with `python -m arbius_amd.ops.build` "
                    "(GPU tensors never fall back to eager PyTorch)")
        L = ctypes.CDLL(str(_LIB_PATH))
        for name, (res, args) in _SIGS.items():
            try:
                fn = getattr(L, name)
            except AttributeError:
                continue
            fn.restype = res
            fn.argtypes = args
            _SYMBOLS[name] = fn
        _lib = L
    return _lib


def loaded() -> bool:
    return _lib is not None


# ---- shape audit (ops/audit.py): every launch symbol becomes a recording stub and HIP streams are
# not touched, so the models run on the META device through the real host-side validation and plan
# selection of this module (no GPU, no data).  Host-only queries still call the library.
_AUDIT = None
_HOST_SYMBOLS = ("arb_conv2d_plan", "arb_conv_family", "arb_conv2d_workspace", "arb_group_norm_workspace",
                 "arb_group_norm_slice_ok",
                 "arb_rvm_args_sizes", "arb_attention512_workspace", "arb_h264_intra_workspace",
                 "arb_h264_intra_host")


def auditing() -> bool:
    return _AUDIT is not None


def audit_note(kind, **info):
    """Record one planned launch (conv / GEMM shape, tile config, split-K) while auditing."""
    if _AUDIT is not None:
        _AUDIT.append(dict(kind=kind, **info))


def has(op: str) -> bool:
    try:
        lib()
    except Exception:
        return False
    return ("arb_" + op) in _SYMBOLS


def _fn(name):
    lib()
    try:
        fn = _SYMBOLS[name]
    except KeyError:
        raise RuntimeError(f"kernel symbol {name} not in {_LIB_PATH} (rebuild)") from None
    if _AUDIT is not None and name not in _HOST_SYMBOLS:
        return lambda *a: (_AUDIT.append(dict(kind="launch", symbol=name)), 0)[1]
    return fn


def _stream():
    if _AUDIT is not None:
        return ctypes.c_void_p(0)
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


# ARBIUS_EXPERIMENT_SKIP (numerics.NUMERICS_ENV_KNOBS; never when mining): op classes whose kernels
# are NOT launched (the output stays uninitialised) - ablation runs that measure what each class
# costs inside the deployed concurrent-stream mix.  Classes: shortk (GEMM / 1x1 conv, K <= 640),
# geglu, gemmbig (GEMM / 1x1 conv, K > 640), conv3 (3x3 / temporal convs), attn, attn512, lnorm
# (LayerNorm + row stats), gnstats / gnapply (ops/__init__.py).
_SKIP = frozenset(filter(None, os.environ.get("ARBIUS_EXPERIMENT_SKIP", "").split(",")))


def _skip(cls: str) -> bool:
    return cls in _SKIP


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: HIP launch failed (rc={rc})")


def _bf16(*ts):
    for t in ts:
        if t is not None and t.dtype != torch.bfloat16:
            raise TypeError(f"HIP kernels take bf16 tensors, got {t.dtype}")


# --------------------------------------------------------------------------- norms
def group_norm_nhwc(x, gamma, beta, groups, eps, silu):
    _bf16(x, gamma, beta)
    x = x.contiguous()
    B, C = x.shape[0], x.shape[-1]
    HW = x.numel() // (B * C)
    if C % 8 or C // 8 > 512 or C % groups or groups > 256:
        raise ValueError(f"group_norm: unsupported C={C} G={groups}")
    ws_bytes = _fn("arb_group_norm_workspace")(B, HW, C, groups)
    ws = torch.empty(max(16, ws_bytes), dtype=torch.uint8, device=x.device)
    y = torch.empty_like(x)
    _check(_fn("arb_group_norm_nhwc")(_p(x), _p(y), _p(gamma), _p(beta), _p(ws), B, HW, C, groups,
                                      float(eps), int(bool(silu)), _stream()), "group_norm")
    return y


def group_norm_mod_nhwc(x, gamma, beta, groups, eps, silu, mod, one_plus):
    """GroupNorm whose output is modulated by ``mod`` [B, mh, mw, 2C] (nearest-upsampled):
    out = GN(x) * (mod[..., :C] + one_plus) + mod[..., C:]  (+ SiLU)."""
    _bf16(x, gamma, beta, mod)
    x = x.contiguous()
    mod = mod.contiguous()
    B, H, W, C = x.shape
    mh, mw = mod.shape[1], mod.shape[2]
    if C % 8 or C // 8 > 512 or C % groups or groups > 256 or mod.shape[-1] != 2 * C or H % mh or W % mw:
        raise ValueError(f"group_norm_mod: unsupported x={tuple(x.shape)} mod={tuple(mod.shape)} G={groups}")
    ws_bytes = _fn("arb_group_norm_workspace")(B, H * W, C, groups)
    ws = torch.empty(max(16, ws_bytes), dtype=torch.uint8, device=x.device)
    y = torch.empty_like(x)
    _check(_fn("arb_group_norm_mod_nhwc")(_p(x), _p(y), _p(gamma), _p(beta), _p(ws), _p(mod), B, H, W, C, groups,
                                          float(eps), int(bool(silu)), mh, mw, float(one_plus), _stream()),
           "group_norm_mod")
    return y


def layer_norm(x, gamma, beta, eps, plan_rows=None):
    """plan_rows: the row count the kernel variant is chosen for (the canonical batch's rows under
    ops.plan_batch, so a lock-step group picks its solo tasks' variant); default: the actual rows."""
    _bf16(x, gamma, beta)
    x = x.contiguous()
    C = x.shape[-1]
    if C % 8 or C > 2048:
        raise ValueError(f"layer_norm: unsupported C={C}")
    M = x.numel() // C
    y = torch.empty_like(x)
    if _skip("lnorm"):
        return y
    _check(_fn("arb_layer_norm")(_p(x), _p(y), _p(gamma), _p(beta), M, C, float(eps),
                                 int(M if plan_rows is None else plan_rows), _stream()), "layer_norm")
    return y


# --------------------------------------------------------------------------- attention
def flash_attention(q, k, v, scale, causal, kv_prefix=None):
    """q [B,Nq,H,D], k/v [B,Nk,H,D] (last dim contiguous, strides multiple of 8).
    ``kv_prefix = (kp, vp)`` [B,Np,H,D]: extra keys/values ahead of k/v (joint attention)."""
    _bf16(q, k, v)
    B, Nq, H, D = q.shape
    Nk = k.shape[1]
    if D > 160:
        if _skip("attn512"):
            return torch.empty_like(q)
        if kv_prefix is not None:
            k, v = torch.cat([kv_prefix[0], k], 1), torch.cat([kv_prefix[1], v], 1)
        return _large_head_attention(q, k, v, scale)
    Np, kp, vp, pst = 0, None, None, None
    if kv_prefix is not None:
        kp, vp = kv_prefix
        _bf16(kp, vp)
        Np = kp.shape[1]
        if kp.stride(2) != k.stride(2) or vp.stride(2) != v.stride(2) or causal:
            raise ValueError("flash_attention: prefix K/V must share the head stride (and no causal mask)")
        for t in (kp, vp):
            if t.stride(-1) != 1 or any(s % 8 for s in t.stride()[:3]) or t.data_ptr() % 16:
                raise ValueError("flash_attention: prefix last dim contiguous, strides/base 16B aligned")
        pst = (ctypes.c_long * 4)(kp.stride(0), kp.stride(1), vp.stride(0), vp.stride(1))
    for t in (q, k, v):
        if t.stride(-1) != 1 or any(s % 8 for s in t.stride()[:3]) or t.data_ptr() % 16:
            raise ValueError("flash_attention: last dim must be contiguous, strides/base 16B aligned")
    if D % 8:
        raise ValueError(f"flash_attention: D={D} not a multiple of 8")
    o = torch.empty(B, Nq, H, D, dtype=q.dtype, device=q.device)
    if _skip("attn"):
        return o
    strides = (ctypes.c_long * 12)(q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
                                   v.stride(0), v.stride(1), v.stride(2), o.stride(0), o.stride(1), o.stride(2))
    _check(_fn("arb_flash_attention")(_p(q), _p(k), _p(v), _p(o), strides, B, H, Nq, Nk + Np, D, float(scale),
                                      int(bool(causal)), _p(kp), _p(vp), pst, Np, _stream()), "flash_attention")
    return o


def temporal_attention(q, k, v, scale):
    """Attention over the frame axis: q/k/v [B, F, P, H, D] views (any strides, last dim
    contiguous) -> o [B, F, P, H, D] contiguous.  One wave per (b, p, h) problem."""
    _bf16(q, k, v)
    B, F, P, H, D = q.shape
    for t in (q, k, v):
        if t.stride(-1) != 1 or any(s % 8 for s in t.stride()[:4]) or t.data_ptr() % 16:
            raise ValueError("temporal_attention: last dim must be contiguous, strides/base 16B aligned")
    if F > 96 or D not in (32, 64, 128):
        raise ValueError(f"temporal_attention: unsupported F={F} D={D}")
    o = torch.empty(B, F, P, H, D, dtype=q.dtype, device=q.device)
    st = []
    for t in (q, k, v, o):
        st += [t.stride(0), t.stride(1), t.stride(2), t.stride(3)]
    strides = (ctypes.c_long * 16)(*st)
    _check(_fn("arb_temporal_attention")(_p(q), _p(k), _p(v), _p(o), strides, B, F, P, H, D, float(scale),
                                         _stream()), "temporal_attention")
    return o


def softmax_rows(s, scale, valid=None):
    """P = softmax(scale * S) over the first `valid` columns of the last dim (default all; the rest
    written 0) (csrc/elementwise.hip), S bf16 [..., N], N % 8 == 0."""
    _bf16(s)
    s = s.contiguous()
    N = s.shape[-1]
    p = torch.empty_like(s)
    _check(_fn("arb_softmax_rows")(_p(s), _p(p), s.numel() // N, N, N if valid is None else int(valid),
                                   float(scale), _stream()), "softmax_rows")
    return p


def attention512(q, k, v, scale):
    """Blockwise (O(N) memory) attention at head dim 512 (csrc/attention512.hip): the single-head
    VAE / MoVQ mid-block attention.  q/k/v [B, N, H, 512], last dim contiguous."""
    _bf16(q, k, v)
    B, Nq, H, D = q.shape
    Nk = k.shape[1]
    if D != 512 or k.shape[-1] != 512 or v.shape[-1] != 512 or tuple(k.shape) != tuple(v.shape):
        raise ValueError(f"attention512: q {tuple(q.shape)} k {tuple(k.shape)} v {tuple(v.shape)}")
    for t in (q, k, v):
        if t.stride(-1) != 1 or any(s % 8 for s in t.stride()[:3]) or t.data_ptr() % 16:
            raise ValueError("attention512: last dim must be contiguous, strides/base 16B aligned")
    o = torch.empty(B, Nq, H, D, dtype=q.dtype, device=q.device)
    if _skip("attn512"):
        return o
    wsb = _fn("arb_attention512_workspace")(B, H, Nq, Nk)
    ws = torch.empty(wsb, dtype=torch.uint8, device=q.device) if wsb else None
    strides = (ctypes.c_long * 12)(q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
                                   v.stride(0), v.stride(1), v.stride(2), o.stride(0), o.stride(1), o.stride(2))
    _check(_fn("arb_attention512")(_p(q), _p(k), _p(v), _p(o), strides, B, H, Nq, Nk, float(scale), _p(ws),
                                   _stream()), "attention512")
    return o


# ARB_ATTN512=0: the round-4 GEMM -> row softmax -> GEMM path for d = 512 (A/B; other bytes)
_A512 = os.environ.get("ARB_ATTN512", "1") != "0"


def _large_head_attention(q, k, v, scale):
    """Head dims > 160: d = 512 (the single-head VAE / MoVQ mid-block attention, once per task) on the
    blockwise kernel (``attention512``).  Other large heads (none in the templates): S = Q K^T on the
    implicit-GEMM kernel, the HIP row softmax, O = P V on the implicit-GEMM kernel (per batch and
    head; V^T made contiguous once).  Key counts off the 64-tile are zero-padded: the padded score
    columns are excluded by the softmax (written 0), so P V never sees them."""
    B, Nq, H, D = q.shape
    Nk = k.shape[1]
    if D == 512 and k.shape[-1] == 512 and _A512:
        return attention512(q, k, v, scale)
    if D % 64:
        from . import _library
        _library("attention", f"head dim {D} (the GEMM path needs D % 64 == 0)")
        qf, kf, vf = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
        s = torch.matmul(qf, kf.transpose(-1, -2)).float() * scale
        return torch.matmul(torch.softmax(s, dim=-1).to(q.dtype), vf).transpose(1, 2).contiguous()
    Np = -(-Nk // 64) * 64
    if Np != Nk:
        k = torch.nn.functional.pad(k, (0, 0, 0, 0, 0, Np - Nk))
        v = torch.nn.functional.pad(v, (0, 0, 0, 0, 0, Np - Nk))
    # each (b, h) output is the GEMM's own [Nq, D] tensor: no strided write into a preallocated output
    # (a contiguous-to-contiguous copy_ is a memcpy - inside a captured hipGraph a memcpy node, which
    # serialised the other task streams' graphs: profiles/graph_serialisation_r4.md)
    outs = []
    for b in range(B):
        for h in range(H):
            s = gemm(q[b, :, h], k[b, :, h].contiguous())                     # [Nq, Np] = q k^T
            outs.append(gemm(softmax_rows(s, scale, Nk), v[b, :, h].t().contiguous()))
    if B * H == 1:
        return outs[0].view(1, Nq, 1, D)
    return torch.stack(outs).view(B, H, Nq, D).transpose(1, 2).contiguous()


# --------------------------------------------------------------------------- ConvGRU (fp16)
def _cl_fp16(*ts):
    for t in ts:
        if t.dtype != torch.float16 or not t.is_contiguous(memory_format=torch.channels_last):
            raise TypeError("convgru kernels take fp16 channels_last NCHW tensors")


_DW_ACT = {None: 0, "relu": 1, "hs": 2}


def dwconv_f16(x, wt, bias, k, stride, dil, act=None):
    """Depthwise k x k conv + bias + activation (csrc/depthwise.hip).  x: fp16 channels_last NCHW
    [B, C, H, W] (NHWC memory); wt [k*k, C] fp16 (taps-major); padding dil * (k // 2).  Returns a
    channels_last NCHW tensor."""
    if x.dtype != torch.float16 or wt.dtype != torch.float16 or (bias is not None and bias.dtype != torch.float16):
        raise TypeError("dwconv_f16: fp16 tensors only")
    B, C, H, W = x.shape
    if not x.is_contiguous(memory_format=torch.channels_last) or C % 8 or tuple(wt.shape) != (k * k, C):
        raise ValueError(f"dwconv_f16: unsupported x {tuple(x.shape)} / wt {tuple(wt.shape)}")
    pad = dil * (k // 2)
    Ho = (H + 2 * pad - dil * (k - 1) - 1) // stride + 1
    Wo = (W + 2 * pad - dil * (k - 1) - 1) // stride + 1
    y = torch.empty(B, Ho, Wo, C, dtype=x.dtype, device=x.device)
    _check(_fn("arb_dwconv_f16")(_p(x), _p(wt.contiguous()), _p(bias), _p(y), B, H, W, C, k, stride, dil,
                                 _DW_ACT[act], _stream()), "dwconv_f16")
    return y.permute(0, 3, 1, 2)


def convgru_gates1(ih, h, cat_buf, cx):
    """ih [N,2C,H,W] -> z [N,C,H,W]; writes sigmoid(r)*h into cat_buf[:, cx:cx+C] (in place)."""
    _cl_fp16(ih, h, cat_buf)
    N, C2, H, W = ih.shape
    C = C2 // 2
    z = torch.empty_like(h, memory_format=torch.channels_last)
    _check(_fn("arb_convgru_gates")(1, _p(ih), _p(h), _p(z), _p(cat_buf), N * H * W, C, cat_buf.shape[1], cx,
                                    _stream()), "convgru_gates1")
    return z


def convgru_gates2(c, h, z):
    """h' = (1 - z) * h + z * tanh(c)."""
    _cl_fp16(c, h, z)
    N, C, H, W = c.shape
    out = torch.empty_like(h, memory_format=torch.channels_last)
    _check(_fn("arb_convgru_gates")(2, _p(c), _p(h), _p(z), _p(out), N * H * W, C, 0, 0, _stream()),
           "convgru_gates2")
    return out


# --------------------------------------------------------------------------- elementwise
def geglu(h):
    _bf16(h)
    h = h.contiguous()
    F2 = h.shape[-1]
    F = F2 // 2
    M = h.numel() // F2
    out = torch.empty(*h.shape[:-1], F, dtype=h.dtype, device=h.device)
    _check(_fn("arb_geglu")(_p(h), _p(out), M, F, _stream()), "geglu")
    return out


def silu(x):
    _bf16(x)
    x = x.contiguous()
    if x.numel() % 8:
        from . import _library, ref
        _library("silu", f"{x.numel()} elements")
        return ref.silu(x)
    y = torch.empty_like(x)
    _check(_fn("arb_silu")(_p(x), _p(y), x.numel(), _stream()), "silu")
    return y


def _cat_parts(x, x2):
    """(x, x2) of a channel concat read in place: both contiguous, same leading dims, C1 % 64 == 0."""
    _bf16(x, x2)
    x, x2 = x.contiguous(), x2.contiguous()
    if x.shape[:-1] != x2.shape[:-1] or x.shape[-1] % 64 or x2.shape[-1] % 8:
        raise ValueError(f"channel concat: bad parts {tuple(x.shape)} | {tuple(x2.shape)}")
    return x, x2


def norm_pool2(x, table=None, silu=False, raw=True):
    """2x2 average pool of x [B, H, W, C] (``raw``) and of its GroupNorm-table transform (``table``
    [B, C, 2] fp32, +SiLU, rounded to bf16 before pooling) in one pass (csrc/elementwise.hip).
    Returns (pooled normalised or None, pooled x or None)."""
    _bf16(x)
    x = x.contiguous()
    B, H, W, C = x.shape
    if C % 8 or H % 2 or W % 2 or (table is not None and (tuple(table.shape) != (B, C, 2)
                                                         or table.dtype != torch.float32)):
        raise ValueError(f"norm_pool2: unsupported x {tuple(x.shape)}")
    yn = torch.empty(B, H // 2, W // 2, C, dtype=x.dtype, device=x.device) if table is not None else None
    yx = torch.empty(B, H // 2, W // 2, C, dtype=x.dtype, device=x.device) if raw else None
    _check(_fn("arb_norm_pool2")(_p(x), _p(None if table is None else table.contiguous()), int(bool(silu)), _p(yn),
                                 _p(yx), B, H, W, C, _stream()), "norm_pool2")
    return yn, yx


def upsample2(x):
    """Nearest 2x up-sampling of a channels-last bf16 tensor [B, H, W, C] -> [B, 2H, 2W, C]."""
    _bf16(x)
    x = x.contiguous()
    B, H, W, C = x.shape
    if C % 8:
        raise ValueError(f"upsample2: C % 8 != 0 ({tuple(x.shape)})")
    y = torch.empty(B, 2 * H, 2 * W, C, dtype=x.dtype, device=x.device)
    _check(_fn("arb_upsample2")(_p(x), _p(y), B, H, W, C, _stream()), "upsample2")
    return y


def norm_table_apply(x, table, silu=False, x2=None):
    """x [B, *, C] * table[b, c].scale + .shift (+SiLU) - the unfused GroupNorm-table prologue.
    ``x2``: the channels [C1, C) of a concat [x | x2] read in place (the output is the concat)."""
    if x2 is not None:
        x, x2 = _cat_parts(x, x2)
        B, C1, C = x.shape[0], x.shape[-1], x.shape[-1] + x2.shape[-1]
        if tuple(table.shape) != (B, C, 2) or table.dtype != torch.float32:
            raise ValueError(f"norm_table_apply: bad table {tuple(table.shape)}")
        y = torch.empty(*x.shape[:-1], C, dtype=x.dtype, device=x.device)
        _check(_fn("arb_norm_table_apply_cat")(_p(x), _p(x2), C1, _p(y), _p(table.contiguous()), B,
                                               x.numel() // (B * C1), C, int(bool(silu)), _stream()),
               "norm_table_apply_cat")
        return y
    _bf16(x)
    x = x.contiguous()
    B, C = x.shape[0], x.shape[-1]
    if C % 8 or tuple(table.shape) != (B, C, 2) or table.dtype != torch.float32:
        raise ValueError(f"norm_table_apply: bad shapes x={tuple(x.shape)} table={tuple(table.shape)}")
    table = table.contiguous()
    y = torch.empty_like(x)
    _check(_fn("arb_norm_table_apply")(_p(x), _p(y), _p(table), B, x.numel() // (B * C), C, int(bool(silu)),
                                       _stream()), "norm_table_apply")
    return y


def conv_plan(B, H, W, Cin, Cout, k, pad, upsample, stride):
    out = (ctypes.c_int * 2)()
    _fn("arb_conv2d_plan")(B, H, W, Cin, Cout, k, pad, int(bool(upsample)), stride, out)
    return out[0], out[1]


def conv_choice(B, H, W, Cin, Cout, kcode, pad, upsample, stride, plan_b):
    """(cfg, split) a planned conv launch runs: the canonical batch's plan at its split-K on the tile
    family tuned for the actual shape (what ``conv2d_nhwc`` does; -1, -1 = the library's own plan)."""
    if not plan_b:
        return -1, -1
    kh, kw = (3, 1) if kcode == 31 else (kcode, kcode)
    Hl, Wl = (2 * H, 2 * W) if upsample else (H, W)
    Ho = (Hl + 2 * pad - kh) // stride + 1
    Wo = (Wl + 2 * (0 if kcode == 31 else pad) - kw) // stride + 1
    cfg, split = conv_plan(plan_b, H, W, Cin, Cout, kcode, pad, upsample, stride)
    ratio = plan_b // B if plan_b % B == 0 else 0
    return _fn("arb_conv_family")(B * Ho * Wo, Cout, kh * kw * Cin, split, ratio, cfg), split


def gemm_choice(M, N, K, plan_batch):
    """(cfg, split) of a planned GEMM launch of M rows (see ``gemm``)."""
    if not (plan_batch and plan_batch[1]):
        return -1, -1
    cfg, split = conv_plan(1, 1, M * plan_batch[1] // plan_batch[0], K, N, 1, 0, 0, 1)
    return _fn("arb_conv_family")(M, N, K, split, plan_batch[1] // plan_batch[0], cfg), split


# tile configs by id (csrc/conv.hip conv_run): kernel template the launch runs
_CFG4 = ["128x128", "64x128", "128x64", "64x64", "160x64", "160x128", "320x32", "256x64", "128x256", "64x256"]
_CFG_NAMES = {20: "glds<256,256>", 21: "glds<320,128>", 22: "glds<256,128>", 23: "glds<320,192>",
              24: "persist<128,128>", 25: "persist<256,128>", 26: "persist<160,128>", 27: "persist<128,64>",
              28: "glds3<128,256>", 29: "glds3<256,128>", 30: "glds3<192,192>", 31: "glds3<320,64>",
              32: "xreg<160,8,2>", 33: "xreg<128,8,2>", 34: "xreg<160,8,1>", 35: "xreg<256,8,1>",
              36: "stag<256,128>", 37: "stag<128,256>", 38: "stag<192,192>", 39: "stag<320,64>",
              40: "stag<160,256>", 41: "stag<160,128>", 42: "stag2<320,128>", 43: "stag2<256,256>",
              44: "stag2<256,192>", 45: "stag2<192,192>",
              46: "sk<160>", 47: "sk<80>"}


def cfg_name(cfg: int) -> str:
    if cfg < 0:
        return "?"
    if cfg < 10:
        return "glds4w<%s>" % _CFG4[cfg]
    if cfg < 20:
        return "igemm<%s>" % _CFG4[cfg - 10]
    return _CFG_NAMES.get(cfg, f"cfg{cfg}")


def group_norm_slice_ok(x, groups, x2=None) -> bool:
    """Whether ``group_norm_slice`` serves this GroupNorm: a function of (rows per image, C, G) only."""
    C = x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
    HW = x.numel() // (x.shape[0] * x.shape[-1])
    return bool(_fn("arb_group_norm_slice_ok")(HW, C, groups))


def group_norm_slice(x, gamma, beta, groups, eps, mod=None, one_plus=0.0, silu=False, x2=None):
    """GroupNorm (+ scale-shift ``mod`` [B, 2C])(+SiLU) of x [B, *, C] - or of the channel concat
    [x | x2] read in place - applied, in one launch per (group, image) slice (csrc/groupnorm.hip
    ``gn_slice_kernel``; small slices only, see ``group_norm_slice_ok``).  Returns the bf16 output."""
    _bf16(x, gamma, beta, mod)
    C1 = 0
    if x2 is not None:
        x, x2 = _cat_parts(x, x2)
        C1 = x.shape[-1]
    x = x.contiguous()
    B, C = x.shape[0], x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
    HW = x.numel() // (B * x.shape[-1])
    if mod is not None:
        mod = mod.contiguous()
        if tuple(mod.shape) != (B, 2 * C):
            raise ValueError("group_norm_slice: mod must be [B, 2C]")
    y = torch.empty(*x.shape[:-1], C, dtype=x.dtype, device=x.device)
    audit_note("group_norm_slice", M=B * HW, N=C, K=groups)
    if _skip("gnstats"):
        return y
    _check(_fn("arb_group_norm_slice")(_p(x), _p(x2), C1, _p(y), _p(gamma), _p(beta), _p(mod), float(one_plus), B,
                                       HW, C, groups, float(eps), int(bool(silu)), _stream()), "group_norm_slice")
    return y


def group_norm_table(x, gamma, beta, groups, eps, mod=None, one_plus=0.0, x2=None):
    """GroupNorm of x [B, *, C] as a per-(batch, channel) affine table [B, C, 2] fp32
    (scale, shift) for a consumer prologue; ``mod`` [B, 2C] folds a scale-shift modulation.
    ``x2``: GroupNorm of the channel concat [x | x2], read in place (same bytes)."""
    _bf16(x, gamma, beta, mod)
    C1 = 0
    if x2 is not None:
        x, x2 = _cat_parts(x, x2)
        C1 = x.shape[-1]
    x = x.contiguous()
    B, C = x.shape[0], x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
    HW = x.numel() // (B * x.shape[-1])
    if C % 8 or C // 8 > 512 or C % groups or groups > 256:
        raise ValueError(f"group_norm_table: unsupported C={C} G={groups}")
    if mod is not None:
        mod = mod.contiguous()
        if tuple(mod.shape) != (B, 2 * C):
            raise ValueError("group_norm_table: mod must be [B, 2C]")
    ws = torch.empty(max(16, _fn("arb_group_norm_workspace")(B, HW, C, groups)), dtype=torch.uint8, device=x.device)
    table = torch.empty(B, C, 2, dtype=torch.float32, device=x.device)
    if x2 is not None:
        _check(_fn("arb_group_norm_table_cat")(_p(x), _p(x2), C1, _p(gamma), _p(beta), _p(mod), float(one_plus),
                                               _p(ws), _p(table), B, HW, C, groups, float(eps), _stream()),
               "group_norm_table_cat")
        return table
    _check(_fn("arb_group_norm_table")(_p(x), _p(gamma), _p(beta), _p(mod), float(one_plus), _p(ws), _p(table), B,
                                       HW, C, groups, float(eps), _stream()), "group_norm_table")
    return table


def conv2d_nhwc(x, w, b, padding, upsample, residual, temb=None, stride=1, cfg=-1, split=-1, norm=None,
                norm_silu=False, plan_b=None, x2=None):
    """Implicit-GEMM conv (csrc/conv.hip).  x [B,H,W,Cin], w [Cout,k,k,Cin] -> [B,Ho,Wo,Cout].
    Fused epilogue: + bias[n] + temb[b, n] + residual[m, n]; optional GroupNorm(+SiLU)
    prologue from a ``group_norm_table`` (the normalised x never hits HBM).  fp16 tensors run the
    fp16 twin of the kernel (mfma f16; no norm prologue).  ``x2``: the input is the channel concat
    [x | x2] read in place (bf16, no norm prologue; bytes equal the concatenated-input conv)."""
    x1 = None
    if x2 is not None:
        if norm is not None:
            raise ValueError("conv2d: no norm prologue on a concat input")
        x1, x2 = _cat_parts(x, x2)
        x = x1
    f16 = x.dtype == torch.float16
    if f16:
        for t in (w, b, residual, temb):
            if t is not None and t.dtype != torch.float16:
                raise TypeError("conv2d fp16: every operand must be fp16")
        if norm is not None:
            raise ValueError("conv2d fp16: no norm prologue")
    else:
        _bf16(x, w, b, residual, temb)
    if x1 is None:
        x = x.contiguous()
    w = w.contiguous()
    B, H, W, Cin = x.shape
    if x1 is not None:
        Cin += x2.shape[-1]
    Cout, kh, kw, Cin2 = w.shape
    temporal = (kh, kw) == (3, 1)      # (3,1,1) Conv3d over a [B, F, HW, C] view
    if Cin != Cin2 or not (kh == kw and kh in (1, 3) or temporal) or Cin % 64 or Cout % 8 or stride not in (1, 2):
        raise ValueError(f"conv2d: unsupported shape x={tuple(x.shape)} w={tuple(w.shape)} stride={stride}")
    Hl, Wl = (2 * H, 2 * W) if upsample else (H, W)
    padw = 0 if temporal else padding
    Ho = (Hl + 2 * padding - kh) // stride + 1
    Wo = (Wl + 2 * padw - kw) // stride + 1
    y = torch.empty(B, Ho, Wo, Cout, dtype=x.dtype, device=x.device)
    if residual is not None:
        residual = residual.contiguous()
        if tuple(residual.shape) != tuple(y.shape):
            raise ValueError(f"conv2d residual {tuple(residual.shape)} != out {tuple(y.shape)}")
    temb_ld = 0
    if temb is not None:
        if tuple(temb.shape) != (B, Cout):
            raise ValueError("conv2d temb must be [B, Cout]")
        # a column slice of the batched ResBlock time projection is read in place at its row stride
        if (not f16 and x1 is None and temb.stride(-1) == 1 and temb.stride(0) % 8 == 0
                and temb.stride(0) >= Cout and temb.data_ptr() % 16 == 0):
            temb_ld = temb.stride(0) if B > 1 else Cout
        else:
            temb = temb.contiguous()
    if b is not None and b.numel() != Cout:
        raise ValueError("conv2d bias size")
    if norm is not None:
        if norm.dtype != torch.float32 or tuple(norm.shape) != (B, Cin, 2) or not norm.is_contiguous():
            raise ValueError("conv2d norm table must be contiguous fp32 [B, Cin, 2]")
    kcode = 31 if temporal else kh
    if plan_b and cfg < 0:   # batch-invariant: the canonical batch's plan at its split-K, on the tile
        # family tuned for the actual shape (bitwise-neutral)
        cfg, split = conv_choice(B, H, W, Cin, Cout, kcode, padding, upsample, stride, plan_b)
    args = (B, H, W, Cin, Cout, kcode, padding, int(bool(upsample)), stride, int(cfg), int(split))
    audit_note("conv", M=B * Ho * Wo, N=Cout, K=kh * kw * Cin, cfg=int(cfg), split=int(split), plan_b=plan_b,
               batch=B, shape=(B, H, W, Cin, Cout, kcode, padding, int(bool(upsample)), stride), dtype=str(x.dtype))
    if _skip("conv3" if kh > 1 else "shortk" if Cin <= 640 else "gemmbig"):
        return y
    ws_bytes = _fn("arb_conv2d_workspace")(*args)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device) if ws_bytes else None
    if f16:
        _check(_fn("arb_conv2d_nhwc_f16")(_p(x), _p(w), _p(b), _p(temb), _p(residual), _p(y), _p(ws), *args,
                                          _stream()), "conv2d_f16")
        return y
    if x1 is not None:
        _check(_fn("arb_conv2d_nhwc_cat")(_p(x1), _p(x2), x1.shape[-1], _p(w), _p(b), _p(temb), _p(residual), _p(y),
                                          _p(ws), *args, _stream()), "conv2d_cat")
        return y
    if temb_ld:
        _check(_fn("arb_conv2d_nhwc_tld")(_p(x), _p(w), _p(b), _p(temb), temb_ld, _p(residual), _p(y), _p(ws), _p(norm),
                                          *args, int(bool(norm_silu)), _stream()), "conv2d")
        return y
    _check(_fn("arb_conv2d_nhwc")(_p(x), _p(w), _p(b), _p(temb), _p(residual), _p(y), _p(ws), _p(norm), *args,
                                  int(bool(norm_silu)), _stream()), "conv2d")
    return y


ACTS = {None: 0, "gelu": 3, "quick_gelu": 4}


def gemm(x, w, b=None, residual=None, cfg=-1, split=-1, plan_batch=None, act=None):
    """out = x @ w^T (+ b + residual) on the implicit-GEMM kernel. x [...,K], w [N,K].
    plan_batch = (batch, canonical batch): plan for M * canonical / batch rows (batch-invariant).
    ``act``: "gelu" / "quick_gelu" applied in the epilogue (conv.hip act_f)."""
    _bf16(x, w, b, residual)
    K = x.shape[-1]
    N = w.shape[0]
    x2 = x.reshape(-1, K).contiguous()
    M = x2.shape[0]
    if K % 64 or N % 8 or w.shape[1] != K:
        raise ValueError(f"gemm: unsupported K={K} N={N}")
    if plan_batch and plan_batch[1] and cfg < 0:
        cfg, split = gemm_choice(M, N, K, plan_batch)
    audit_note("gemm", M=M, N=N, K=K, cfg=int(cfg), split=int(split), plan_b=plan_batch and plan_batch[1],
               batch=plan_batch and plan_batch[0], dtype=str(x.dtype))
    y = torch.empty(M, N, dtype=x.dtype, device=x.device)
    if _skip("shortk" if K <= 640 else "gemmbig"):
        return y.reshape(*x.shape[:-1], N)
    r2 = residual.reshape(M, N).contiguous() if residual is not None else None
    ws_bytes = _fn("arb_conv2d_workspace")(1, 1, M, K, N, 1, 0, 0, 1, int(cfg), int(split))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device) if ws_bytes else None
    if act is not None:
        _check(_fn("arb_gemm_act")(_p(x2), _p(w.contiguous()), _p(b), _p(r2), _p(y), _p(ws), M, N, K, int(cfg),
                                   int(split), ACTS[act], _stream()), "gemm_act")
        return y.reshape(*x.shape[:-1], N)
    _check(_fn("arb_gemm_bias_res")(_p(x2), _p(w.contiguous()), _p(b), _p(r2), _p(y), _p(ws), M, N, K, int(cfg),
                                    int(split), _stream()), "gemm")
    return y.reshape(*x.shape[:-1], N)


def gemm_geglu(x, w_il, b_il=None, cfg=-1, split=-1, plan_batch=None):
    """value * gelu(gate) of x @ w^T + b in the GEMM epilogue.  ``w_il`` / ``b_il``: the projection's
    rows interleaved in blocks of 16 as [value 8 | gate 8] (``interleave_geglu``); out [..., N/2].
    Bitwise equal to ``geglu(gemm(x, w, b))`` (both halves rounded to bf16 before the product)."""
    _bf16(x, w_il, b_il)
    K = x.shape[-1]
    N = w_il.shape[0]
    x2 = x.reshape(-1, K).contiguous()
    M = x2.shape[0]
    if K % 64 or N % 16 or w_il.shape[1] != K:
        raise ValueError(f"gemm_geglu: unsupported K={K} N={N}")
    if plan_batch and plan_batch[1] and cfg < 0:
        cfg, split = gemm_choice(M, N, K, plan_batch)
    audit_note("gemm", M=M, N=N, K=K, cfg=int(cfg), split=int(split), plan_b=plan_batch and plan_batch[1],
               batch=plan_batch and plan_batch[0], dtype=str(x.dtype))
    y = torch.empty(M, N // 2, dtype=x.dtype, device=x.device)
    if _skip("geglu"):
        return y.reshape(*x.shape[:-1], N // 2)
    ws_bytes = _fn("arb_conv2d_workspace")(1, 1, M, K, N, 1, 0, 0, 1, int(cfg), int(split))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device) if ws_bytes else None
    _check(_fn("arb_gemm_geglu")(_p(x2), _p(w_il.contiguous()), _p(b_il), _p(y), _p(ws), M, N, K, int(cfg),
                                 int(split), _stream()), "gemm_geglu")
    return y.reshape(*x.shape[:-1], N // 2)


def row_stats(x, eps, plan_rows=None):
    """(mean, rstd) per row of x [..., C] (csrc/norm.hip, the LayerNorm kernel's arithmetic) -> fp32
    [M, 2] - the statistics of a LayerNorm folded into the following GEMM."""
    _bf16(x)
    x = x.contiguous()
    C = x.shape[-1]
    if C % 8 or C > 2048:
        raise ValueError(f"row_stats: unsupported C={C}")
    M = x.numel() // C
    rs = torch.empty(M, 2, dtype=torch.float32, device=x.device)
    if _skip("lnorm"):
        return rs
    _check(_fn("arb_row_stats")(_p(x), _p(rs), M, C, float(eps), int(M if plan_rows is None else plan_rows),
                                _stream()), "row_stats")
    return rs


def gemm_ln(x, w, b, wsum, rs, residual=None, geglu=False, cfg=-1, split=-1, plan_batch=None, act=None):
    """LayerNorm folded into a GEMM: x is the LN INPUT, ``w`` / ``b`` / ``wsum`` from ``ops.ln_fold``,
    ``rs`` = ``row_stats(x)``.  out = rstd (x w^T - mean wsum) + b (+ residual | GEGLU, out N/2)."""
    _bf16(x, w, b, residual)
    K = x.shape[-1]
    N = w.shape[0]
    x2 = x.reshape(-1, K).contiguous()
    M = x2.shape[0]
    if K % 64 or N % (16 if geglu else 8) or w.shape[1] != K or tuple(rs.shape) != (M, 2) or wsum.numel() != N:
        raise ValueError(f"gemm_ln: unsupported M={M} K={K} N={N}")
    if rs.dtype != torch.float32 or wsum.dtype != torch.float32 or not rs.is_contiguous() or not wsum.is_contiguous():
        raise ValueError("gemm_ln: row stats / wsum must be contiguous fp32")
    if plan_batch and plan_batch[1] and cfg < 0:
        cfg, split = gemm_choice(M, N, K, plan_batch)
    audit_note("gemm", M=M, N=N, K=K, cfg=int(cfg), split=int(split), plan_b=plan_batch and plan_batch[1],
               batch=plan_batch and plan_batch[0], dtype=str(x.dtype))
    y = torch.empty(M, N // 2 if geglu else N, dtype=x.dtype, device=x.device)
    if _skip("geglu" if geglu else "shortk" if K <= 640 else "gemmbig"):
        return y.reshape(*x.shape[:-1], y.shape[-1])
    r2 = residual.reshape(M, N).contiguous() if residual is not None else None
    ws_bytes = _fn("arb_conv2d_workspace")(1, 1, M, K, N, 1, 0, 0, 1, int(cfg), int(split))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device) if ws_bytes else None
    _check(_fn("arb_gemm_ln")(_p(x2), _p(w.contiguous()), _p(b), _p(r2), _p(y), _p(ws), _p(rs), _p(wsum), M, N, K,
                              int(cfg), int(split), int(bool(geglu)), ACTS[act], _stream()), "gemm_ln")
    return y.reshape(*x.shape[:-1], y.shape[-1])


def interleave_geglu(t):
    """[value F | gate F] rows (dim 0) -> blocks of 16 rows [value 8 | gate 8] (F % 8 == 0)."""
    F_ = t.shape[0] // 2
    v, g = t[:F_].reshape(F_ // 8, 8, *t.shape[1:]), t[F_:].reshape(F_ // 8, 8, *t.shape[1:])
    return torch.stack([v, g], dim=1).reshape(t.shape).contiguous()


# --------------------------------------------------------------------------- fused CFG + sampler step
class _SampTask(ctypes.Structure):
    """Mirror of ``SampTask`` in csrc/sampler.hip (13 pointers, 16 floats, flags)."""
    _fields_ = ([(n, c_void_p) for n in ("u", "c", "x", "xsrc", "p", "cur", "hs", "h1", "h2", "h3", "noise",
                                         "xin0", "xin1")]
                + [(n, c_float) for n in ("g", "he0", "he1", "he2", "he3", "px", "pe", "clampv", "ox", "oe",
                                          "ox0", "od", "stdv", "logb", "plv", "in_scale")]
                + [("flags", c_int), ("_pad", c_int)])


def sampler_step(tasks):
    """The fused CFG + sampler update of a lock-step group (dicts from
    ``models.schedulers.TaskSampler.task_args``): one launch per 8 tasks (the kernel's per-launch task
    table; every task's arithmetic is its own, so the chunking moves no byte).  Shapes / dtypes /
    contiguity are checked here."""
    if not tasks:
        raise ValueError("sampler_step: no tasks")
    if len(tasks) > 8:
        for i in range(0, len(tasks), 8):
            sampler_step(tasks[i:i + 8])
        return
    x0 = tasks[0]["x"]
    n_pix = x0.numel() // 4
    cout = tasks[0]["u"].shape[-1]
    arr = (_SampTask * len(tasks))()
    for k, a in enumerate(tasks):
        x = a["x"]
        if x.dtype != torch.float32 or not x.is_contiguous() or x.numel() != n_pix * 4 or x.shape[-1] != 4:
            raise ValueError("sampler_step: x must be contiguous fp32 [..., 4] of the group's size")
        for key in ("u", "c"):
            t = a[key]
            if t.dtype != torch.bfloat16 or not t.is_contiguous() or t.numel() != n_pix * cout or t.shape[-1] != cout:
                raise ValueError(f"sampler_step: {key} must be contiguous bf16 [..., {cout}] matching x")
        for key in ("xsrc", "p", "cur", "hs", "h1", "h2", "h3", "noise"):
            t = a.get(key)
            if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != n_pix * 4):
                raise ValueError(f"sampler_step: {key} must be contiguous fp32 like x")
        for key in ("xin0", "xin1"):
            t = a.get(key)
            if t is not None and (t.dtype != torch.bfloat16 or not t.is_contiguous() or t.numel() != n_pix * 4):
                raise ValueError(f"sampler_step: {key} must be contiguous bf16 like x")
        r = arr[k]
        for key in ("u", "c", "x", "xsrc", "p", "cur", "hs", "h1", "h2", "h3", "noise", "xin0", "xin1"):
            t = a.get(key)
            setattr(r, key, t.data_ptr() if t is not None else None)
        he = a["he"]
        r.g, r.he0, r.he1, r.he2, r.he3 = a["g"], he[0], he[1], he[2], he[3]
        r.px, r.pe, r.clampv = a["px"], a["pe"], a["clamp"] or 0.0
        r.ox, r.oe, r.ox0, r.od, r.stdv = a["ox"], a["oe"], a["ox0"], a["od"], a["std"]
        lb, plv = a["learned"] if a["learned"] is not None else (0.0, 0.0)
        r.logb, r.plv, r.in_scale = lb, plv, a["in_scale"]
        if a["learned"] is not None and cout != 8:
            raise ValueError("sampler_step: learned variance needs the var channels (cout 8)")
        r.flags = (int(bool(a["store_x0"])) | int(bool(a["store_cur"])) << 1 | int(a["learned"] is not None) << 2
                   | int(a["clamp"] is not None) << 3 | int(bool(a["read_p"])) << 4)
    _check(_fn("arb_sampler_step")(ctypes.cast(arr, c_void_p), len(tasks), n_pix, cout, _stream()), "sampler_step")


# --------------------------------------------------------------------------- general conv entry
def conv_ex(x, w_pad, b, k, stride=1, pad=None, act=0, residual=None, cfg=-1, split=-1):
    """Implicit-GEMM conv on NHWC ``x`` [B,H,W,Cx] with Cx % 8 == 0 (NOT necessarily % 64: the kernel
    reads zeros for the channels up to the next multiple of 64 - no padded copy of x).  ``w_pad``
    [Cout, k, k, Cpad] zero-padded (Cpad = Cx rounded up to 64), Cout % 8 == 0; act 0/1/2 = none /
    ReLU / hardswish fused into the epilogue (after bias and residual).  bf16 or fp16."""
    f16 = x.dtype == torch.float16
    if not f16:
        _bf16(x, w_pad, b, residual)
    for t in (w_pad, b, residual):
        if t is not None and t.dtype != x.dtype:
            raise TypeError("conv_ex: operands must share the activation dtype")
    x = x.contiguous()
    B, H, W, Cx = x.shape
    Cout, kh, kw, Cp = w_pad.shape
    pad = k // 2 if pad is None else pad
    if Cx % 8 or Cp != -(-Cx // 64) * 64 or Cout % 8 or kh != k or kw != k or k not in (1, 3) or stride not in (1, 2):
        raise ValueError(f"conv_ex: unsupported x={tuple(x.shape)} w={tuple(w_pad.shape)}")
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    y = torch.empty(B, Ho, Wo, Cout, dtype=x.dtype, device=x.device)
    if residual is not None:
        residual = residual.contiguous()
        if tuple(residual.shape) != tuple(y.shape):
            raise ValueError("conv_ex: residual shape")
    if b is not None and b.numel() != Cout:
        raise ValueError("conv_ex: bias size")
    ws_bytes = _fn("arb_conv2d_workspace")(B, H, W, Cp, Cout, k, pad, 0, stride, int(cfg), int(split))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device) if ws_bytes else None
    _check(_fn("arb_conv2d_ex")(_p(x), _p(w_pad.contiguous()), _p(b), None, _p(residual), _p(y), _p(ws), B, H, W, Cx,
                                Cout, k, pad, 0, stride, int(cfg), int(split), int(act), int(f16), _stream()),
           "conv_ex")
    return y


# --------------------------------------------------------------------------- RVM fused passes
def _f16(*ts):
    for t in ts:
        if t is not None and (t.dtype != torch.float16 or not t.is_contiguous()):
            raise TypeError("RVM kernels take contiguous fp16 tensors")


def rvm_resize_u8(frames, h, w):
    """uint8 [T,H,W,3] -> fp16 [T,h,w,3] = bilinear(frames / 255) (align_corners=False, size given)."""
    if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[-1] != 3 or not frames.is_contiguous():
        raise TypeError("rvm_resize_u8: contiguous uint8 [T,H,W,3]")
    T, H, W, _ = frames.shape
    out = torch.empty(T, h, w, 3, dtype=torch.float16, device=frames.device)
    _check(_fn("arb_rvm_resize_u8")(_p(frames), _p(out), T, H, W, h, w, _stream()), "rvm_resize_u8")
    return out


def rvm_stem(small, args_blob):
    """3x3 s2 conv 3 -> 16 on the normalised source + bias + hardswish -> fp16 [T, ceil(h/2), ceil(w/2), 16]."""
    _f16(small)
    T, h, w, _ = small.shape
    out = torch.empty(T, (h + 1) // 2, (w + 1) // 2, 16, dtype=torch.float16, device=small.device)
    _check(_fn("arb_rvm_stem")(_p(small), _p(out), ctypes.c_char_p(args_blob), T, h, w, _stream()), "rvm_stem")
    return out


def rvm_pool3(s0):
    _f16(s0)
    T, h, w, _ = s0.shape
    dims = []
    for _ in range(3):
        h, w = (h + 1) // 2, (w + 1) // 2
        dims.append((h, w))
    s1, s2, s3 = (torch.empty(T, hh, ww, 3, dtype=torch.float16, device=s0.device) for hh, ww in dims)
    _check(_fn("arb_rvm_pool3")(_p(s0), _p(s1), _p(s2), _p(s3), T, s0.shape[1], s0.shape[2], _stream()), "rvm_pool3")
    return s1, s2, s3


def rvm_upcat(x, f, s, Cd):
    """[up2x(x)[:H,:W] | f | s | zeros] -> fp16 [T,H,W,Cd]; (H, W) = s's spatial size; f may be None."""
    _f16(x, f, s)
    T, H, W, cs = s.shape
    cf = f.shape[-1] if f is not None else 0
    out = torch.empty(T, H, W, Cd, dtype=torch.float16, device=s.device)
    _check(_fn("arb_rvm_upcat")(_p(x), x.shape[1], x.shape[2], x.shape[3], _p(f), cf, _p(s), cs, _p(out), T, H, W, Cd,
                                _stream()), "rvm_upcat")
    return out


def rvm_pack(buf, a, aoff, CA, b, CB):
    """buf [P, bs] rows <- [a[:, aoff:aoff+CA] | b (or zeros)]; a [P, as] rows."""
    _f16(buf, b)
    P = buf.numel() // buf.shape[-1]
    _check(_fn("arb_rvm_pack")(_p(buf), buf.shape[-1], _p(a), a.stride(-2) if a.dim() > 1 else a.shape[-1], aoff, CA,
                               _p(b), CB, P, _stream()), "rvm_pack")


def rvm_gru_out(cc, h, z, out, oc, buf=None, nx=None, noff=0):
    """h <- (1 - z) h + z tanh(cc[..., :C]) in place; out[p, oc:oc+C] <- h'; buf <- [nx[p, noff:+C] | h']."""
    C = h.shape[-1]
    P = h.numel() // C
    _check(_fn("arb_rvm_gru_out")(_p(cc), cc.shape[-1], _p(h), _p(z), _p(out), out.shape[-1], oc, _p(buf),
                                  buf.shape[-1] if buf is not None else 0, _p(nx),
                                  nx.shape[-1] if nx is not None else 0, noff, P, C, _stream()), "rvm_gru_out")


def rvm_dgf(hid, small, args_dev, frames, mode, green):
    """Projection head + deep guided filter + composite -> uint8 [T,H,W,3] at the frames' resolution."""
    _f16(hid, small)
    T, h, w, _ = small.shape
    H, W = frames.shape[1], frames.shape[2]
    xy = torch.empty(T * h * w * 8, dtype=torch.float32, device=hid.device)
    ab = torch.empty_like(xy)
    out = torch.empty(T, H, W, 3, dtype=torch.uint8, device=hid.device)
    _check(_fn("arb_rvm_dgf")(_p(hid), _p(small), _p(args_dev), _p(xy), _p(ab), _p(frames), _p(out), T, H, W, h, w,
                              int(mode), float(green[0]), float(green[1]), float(green[2]), _stream()), "rvm_dgf")
    return out


def rvm_chan_mean(x):
    """fp16 [T, H, W, C] -> fp16 [T, 1, 1, C] spatial mean (fp32 accumulation, fixed order)."""
    _f16(x)
    if not x.is_contiguous() or x.shape[-1] % 8:
        raise ValueError("rvm_chan_mean: contiguous [T, H, W, C], C % 8 == 0")
    T, C = x.shape[0], x.shape[-1]
    out = torch.empty(T, 1, 1, C, dtype=torch.float16, device=x.device)
    _check(_fn("arb_rvm_chan_mean")(_p(x), _p(out), T, x.numel() // (T * C), C, _stream()), "rvm_chan_mean")
    return out


def rvm_gate(x, w, mode):
    """x [T, H, W, C] *= (hardsigmoid if mode == 0 else sigmoid)(w [T, 1, 1, C]) in place; returns x."""
    _f16(x, w)
    if not (x.is_contiguous() and w.is_contiguous()) or x.shape[-1] % 8 or w.numel() != x.shape[0] * x.shape[-1]:
        raise ValueError("rvm_gate: contiguous x [T, H, W, C] and w [T, 1, 1, C], C % 8 == 0")
    T, C = x.shape[0], x.shape[-1]
    _check(_fn("arb_rvm_gate")(_p(x), _p(w), T, x.numel() // (T * C), C, int(mode), _stream()), "rvm_gate")
    return x


def rvm_args_size(which: int) -> int:
    return int(_fn("arb_rvm_args_sizes")(which))


def image_u8(x, mode: int):
    """Decoded bf16 image [..., 3] -> uint8 (csrc/elementwise.hip image_u8_kernel): mode 0 the KL-VAE's
    round(clamp(x / 2 + 0.5, 0, 1) * 255), mode 1 the MoVQ's round(clamp((x + 1) * 127.5, 0, 255))."""
    _bf16(x)
    x = x.contiguous()
    y = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    _check(_fn("arb_image_u8")(_p(x), _p(y), x.numel(), int(mode), _stream()), "image_u8")
    return y


def rgb_to_yuv420(x, out=None):
    """uint8 RGB frames [T, H, W, 3] -> macroblock-padded BT.601 4:2:0 planes (y [T, H16, W16], cb, cr
    [T, H16 / 2, W16 / 2]) (csrc/elementwise.hip rgb_to_yuv420_kernel; the H.264 encoder's input, same
    samples as native rgb_to_420).  ``out``: optional (y, cb, cr) destination tensors."""
    if x.dtype != torch.uint8 or x.dim() != 4 or x.shape[-1] != 3:
        raise ValueError("rgb_to_yuv420: uint8 [T, H, W, 3]")
    x = x.contiguous()
    T, H, W, _ = x.shape
    H16, W16 = (H + 15) // 16 * 16, (W + 15) // 16 * 16
    if out is None:
        out = (torch.empty(T, H16, W16, dtype=torch.uint8, device=x.device),
               torch.empty(T, H16 // 2, W16 // 2, dtype=torch.uint8, device=x.device),
               torch.empty(T, H16 // 2, W16 // 2, dtype=torch.uint8, device=x.device))
    y, cb, cr = out
    if (tuple(y.shape) != (T, H16, W16) or tuple(cb.shape) != (T, H16 // 2, W16 // 2)
            or tuple(cr.shape) != tuple(cb.shape) or not all(t.is_contiguous() for t in out)):
        raise ValueError("rgb_to_yuv420: bad destination planes")
    _check(_fn("arb_rgb_to_yuv420")(_p(x), _p(y), _p(cb), _p(cr), T, H, W, _stream()), "rgb_to_yuv420")
    return y, cb, cr


def _h264_planes(y, cb, cr):
    if y.dim() != 3 or y.dtype != torch.uint8:
        raise ValueError("h264_intra: y uint8 [F, H16, W16]")
    F, H16, W16 = y.shape
    if F < 1 or H16 % 16 or W16 % 16 or H16 < 16 or W16 < 16:
        raise ValueError("h264_intra: planes must be macroblock-padded (multiples of 16)")
    for c in (cb, cr):
        if c.dtype != torch.uint8 or tuple(c.shape) != (F, H16 // 2, W16 // 2):
            raise ValueError("h264_intra: cb / cr uint8 [F, H16 / 2, W16 / 2]")
    if not all(t.is_contiguous() for t in (y, cb, cr)):
        raise ValueError("h264_intra: planes must be contiguous")
    return int(F), int(H16), int(W16)


def h264_intra_capacity(F: int, H16: int, W16: int) -> int:
    """Output bytes reserved for F pictures: 2 bytes per 4:2:0 sample (a picture past it is re-encoded
    on the host)."""
    return F * (H16 * W16 * 3 + 64)


def h264_intra_encode(y, cb, cr, qp: int, return_ws: bool = False):
    """avc-intra slices of F pictures on the GPU (csrc/h264_intra.hip): macroblock-padded 4:2:0 planes
    (device uint8) -> (out, meta) device tensors; picture f's RBSP is out[meta[f]:] with
    meta[2 + F + f] bits before the stop bit, meta[F + 1] != 0 on an error (the caller falls back
    to the native encoder).  Queued on the current stream; nothing is synchronised here."""
    F, H16, W16 = _h264_planes(y, cb, cr)
    if not 0 <= int(qp) <= 51:
        raise ValueError("h264_intra: qp in [0, 51]")
    ws = torch.empty(int(_fn("arb_h264_intra_workspace")(F, W16, H16)), dtype=torch.uint8, device=y.device)
    cap = h264_intra_capacity(F, H16, W16)
    out = torch.empty(cap, dtype=torch.uint8, device=y.device)
    meta = torch.empty(2 * F + 2, dtype=torch.int64, device=y.device)
    _check(_fn("arb_h264_intra_encode")(_p(y), _p(cb), _p(cr), F, W16, H16, int(qp), _p(ws), _p(out), cap, _p(meta),
                                        _stream()), "h264_intra_encode")
    return (out, meta, ws) if return_ws else (out, meta)


def h264_intra_host(y, cb, cr, qp: int, return_ws: bool = False):
    """The GPU encoder's per-macroblock functions run on the CPU (numpy planes) -> (out, meta) numpy
    arrays in the layout of ``h264_intra_encode`` (tests on machines without a GPU)."""
    import numpy as np
    yt, cbt, crt = (torch.from_numpy(np.ascontiguousarray(a)) for a in (y, cb, cr))
    F, H16, W16 = _h264_planes(yt, cbt, crt)
    cap = h264_intra_capacity(F, H16, W16)
    out = np.zeros(cap, np.uint8)
    meta = np.zeros(2 * F + 2, np.int64)
    ws = np.zeros(int(_fn("arb_h264_intra_workspace")(F, W16, H16)), np.uint8) if return_ws else None
    rc = _fn("arb_h264_intra_host")(yt.data_ptr(), cbt.data_ptr(), crt.data_ptr(), F, W16, H16, int(qp),
                                    out.ctypes.data, cap, meta.ctypes.data, None if ws is None else ws.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"h264_intra_host failed ({rc})")
    return (out, meta, ws) if return_ws else (out, meta)

