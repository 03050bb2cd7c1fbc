"""Numerics of the gfx950 HIP kernels vs the fp32 PyTorch reference (ops/ref.py)."""
import math

import pytest
import torch

from arbius_amd import ops
from arbius_amd.ops import _lib, ref

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("B,H,W,C,G,silu", [(2, 64, 64, 320, 32, True), (2, 32, 32, 640, 32, False),
                                            (2, 8, 8, 1280, 32, True), (1, 128, 128, 256, 32, True),
                                            (2, 16, 16, 1280, 32, False), (1, 7, 9, 64, 8, True),
                                            (2, 16, 16, 2560, 32, True), (2, 32, 32, 1920, 32, True),
                                            (2, 64, 64, 960, 32, False), (2, 8, 8, 2048, 32, True)])
def test_group_norm(cuda, B, H, W, C, G, silu):
    torch.manual_seed(0)
    x = (torch.randn(B, H, W, C, device=cuda) * 3 + 5).bfloat16()
    g = (torch.rand(C, device=cuda) + 0.5).bfloat16()
    b = torch.randn(C, device=cuda).bfloat16()
    y = _lib.group_norm_nhwc(x, g, b, G, 1e-5, silu)
    r = ref.group_norm_nhwc(x.float(), g.float(), b.float(), G, 1e-5, silu)
    assert _rel(y, r) < 1e-2
    y2 = _lib.group_norm_nhwc(x, g, b, G, 1e-5, silu)
    assert torch.equal(y, y2), "group norm must be bitwise deterministic"


@pytest.mark.parametrize("M,C", [(8192, 320), (2048, 640), (154, 768), (512, 1280), (77, 1024), (4099, 320),
                                 (77, 384), (33, 2048), (65, 256), (19, 960)])
def test_layer_norm(cuda, M, C):
    """Packed-row LayerNorm (every (lanes/row, vectors/lane) geometry the UNets and text towers use,
    ragged row counts) and the fallback wave-per-row kernel (C = 960) against fp32; row_stats is the
    same per-row arithmetic."""
    x = (torch.randn(M, C, device=cuda) * 3 + 1).bfloat16()
    g = torch.randn(C, device=cuda).bfloat16()
    b = torch.randn(C, device=cuda).bfloat16()
    y = _lib.layer_norm(x, g, b, 1e-5)
    assert _rel(y, ref.layer_norm(x.float(), g.float(), b.float(), 1e-5)) < 1e-2
    assert torch.equal(y, _lib.layer_norm(x, g, b, 1e-5))
    rs = _lib.row_stats(x, 1e-5)
    xf = x.float()
    assert torch.allclose(rs[:, 0], xf.mean(1), atol=1e-3, rtol=1e-3)
    assert torch.allclose(rs[:, 1], torch.rsqrt(xf.var(1, unbiased=False) + 1e-5), rtol=2e-3)


@pytest.mark.parametrize("B,Nq,Nk,H,D,causal", [
    (2, 4096, 4096, 8, 40, False), (2, 1024, 1024, 8, 80, False), (2, 256, 256, 8, 160, False),
    (2, 64, 64, 8, 160, False), (2, 4096, 77, 8, 40, False), (2, 1024, 77, 8, 80, False),
    (2, 77, 77, 12, 64, True), (3, 100, 37, 4, 64, False), (5, 24, 24, 5, 64, False),
    (1, 300, 300, 2, 128, True), (2, 200, 130, 3, 32, False), (1, 129, 65, 1, 96, False),
    (1, 200, 100, 3, 72, False), (2, 150, 150, 2, 24, True), (1, 64, 64, 1, 8, False),
    (8, 4096, 4096, 8, 40, False), (4, 8192, 300, 8, 64, False)])   # last two: 4 q-tiles per wave
def test_flash_attention(cuda, B, Nq, Nk, H, D, causal):
    torch.manual_seed(1)
    # fused-QKV-like strided views
    qkv = torch.randn(B, Nq, 3, H, D, device=cuda).bfloat16()
    q = qkv[:, :, 0]
    kv = torch.randn(B, Nk, 2, H, D, device=cuda).bfloat16()
    k, v = kv[:, :, 0], kv[:, :, 1]
    if causal:
        k, v = qkv[:, :, 1], qkv[:, :, 2]
    scale = 1 / math.sqrt(D)
    o = _lib.flash_attention(q, k, v, scale, causal)
    r = ref.attention(q.float(), k.float(), v.float(), scale, causal)
    assert o.shape == r.shape
    assert _rel(o, r) < 2e-2, _rel(o, r)
    o2 = _lib.flash_attention(q, k, v, scale, causal)
    assert torch.equal(o, o2)


def test_flash_attention_rescale_spike(cuda):
    """Force the online-softmax rescale branch: a huge score in a LATE kv block."""
    B, N, H, D = 1, 512, 2, 64
    q = torch.randn(B, N, H, D, device=cuda) * 0.1
    k = torch.randn(B, N, H, D, device=cuda) * 0.1
    v = torch.randn(B, N, H, D, device=cuda)
    k[:, 400] = q[:, 3] * 40  # query 3 spikes at key 400 (7th kv block)
    q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
    o = _lib.flash_attention(q, k, v, 1 / 8, False)
    r = ref.attention(q.float(), k.float(), v.float(), 1 / 8)
    assert _rel(o, r) < 2e-2


def test_geglu_silu(cuda):
    h = torch.randn(1000, 2 * 1280, device=cuda).bfloat16()
    assert _rel(_lib.geglu(h), ref.geglu(h.float())) < 1e-2
    x = torch.randn(4096, 320, device=cuda).bfloat16()
    assert _rel(_lib.silu(x), ref.silu(x.float())) < 1e-2


@pytest.mark.parametrize("B,H,W,Cin,Cout,k,up,stride,temb,res", [
    (2, 64, 64, 320, 320, 3, False, 1, True, False), (2, 32, 32, 640, 640, 3, False, 1, False, True),
    (2, 8, 8, 1280, 1280, 3, False, 1, True, True), (2, 16, 16, 2560, 1280, 1, False, 1, False, False),
    (2, 32, 32, 320, 320, 3, True, 1, False, False), (2, 64, 64, 320, 320, 3, False, 2, False, False),
    (1, 64, 64, 512, 512, 3, False, 1, False, True), (1, 9, 13, 128, 24, 3, False, 1, True, True),
    (3, 5, 7, 64, 72, 3, True, 2, False, False), (2, 16, 16, 960, 640, 1, False, 1, False, True)])
def test_conv2d(cuda, B, H, W, Cin, Cout, k, up, stride, temb, res):
    torch.manual_seed(2)
    x = torch.randn(B, H, W, Cin, device=cuda).bfloat16()
    w = (torch.randn(Cout, k, k, Cin, device=cuda) / math.sqrt(k * k * Cin)).bfloat16()
    b = torch.randn(Cout, device=cuda).bfloat16()
    pad = k // 2
    Hl, Wl = (2 * H, 2 * W) if up else (H, W)
    Ho, Wo = (Hl + 2 * pad - k) // stride + 1, (Wl + 2 * pad - k) // stride + 1
    t = torch.randn(B, Cout, device=cuda).bfloat16() if temb else None
    r = torch.randn(B, Ho, Wo, Cout, device=cuda).bfloat16() if res else None
    y = _lib.conv2d_nhwc(x, w, b, pad, up, r, t, stride)
    ref_y = ref.conv2d_nhwc(x.float(), w.float(), b.float(), stride, pad, up)
    if temb:
        ref_y = ref_y + t.float()[:, None, None, :]
    if res:
        ref_y = ref_y + r.float()
    assert y.shape == ref_y.shape
    assert _rel(y, ref_y) < 1e-2, _rel(y, ref_y)
    assert torch.equal(y, _lib.conv2d_nhwc(x, w, b, pad, up, r, t, stride))


@pytest.mark.parametrize("M,K,N", [(8192, 320, 320), (8192, 1280, 320), (2048, 2560, 640), (128, 5120, 1280),
                                   (77, 768, 640), (100, 64, 24)])
def test_gemm(cuda, M, K, N):
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    r = torch.randn(M, N, device=cuda).bfloat16()
    y = _lib.gemm(x, w, b, r)
    assert _rel(y, x.float() @ w.float().t() + b.float() + r.float()) < 1e-2


@pytest.mark.parametrize("cfg", list(range(20)) + list(range(20, 28)) + list(range(32, 46)))
@pytest.mark.parametrize("split", [1, 3])
def test_conv2d_all_tile_configs(cuda, cfg, split):
    """Every tile config of both kernel variants (LDS-DMA ring / register staged) and split-K."""
    torch.manual_seed(3)
    B, H, W, Cin, Cout = 2, 12, 10, 128, 160
    x = torch.randn(B, H, W, Cin, device=cuda).bfloat16()
    w = (torch.randn(Cout, 3, 3, Cin, device=cuda) / math.sqrt(9 * Cin)).bfloat16()
    b = torch.randn(Cout, device=cuda).bfloat16()
    r = torch.randn(B, H, W, Cout, device=cuda).bfloat16()
    y = _lib.conv2d_nhwc(x, w, b, 1, False, r, None, 1, cfg, split)
    ref_y = ref.conv2d_nhwc(x.float(), w.float(), b.float(), 1, 1, False) + r.float()
    assert _rel(y, ref_y) < 1e-2, (cfg, split, _rel(y, ref_y))


@pytest.mark.parametrize("B,H,W,C,Co,k", [(8, 64, 64, 320, 320, 3), (2, 16, 16, 640, 1280, 1), (1, 9, 13, 128, 72, 3)])
def test_conv_tile_families_bitwise_equal(cuda, B, H, W, C, Co, k):
    """Every tile family (register-staged, LDS-DMA ring, 8-wave, 3-stage 8-wave) reduces each output
    in the same MFMA order at split 1, so they are bitwise interchangeable - what lets the planner
    remap a norm-prologue or two-source call onto the register-staged kernel without changing bytes."""
    torch.manual_seed(12)
    x = torch.randn(B, H, W, C, device=cuda).bfloat16()
    w = (torch.randn(Co, k, k, C, device=cuda) / math.sqrt(k * k * C)).bfloat16()
    b = torch.randn(Co, device=cuda).bfloat16()
    pad = k // 2
    ref_y = _lib.conv2d_nhwc(x, w, b, pad, False, None, None, 1, 10, 1)
    for cfg in (0, 3, 5, 6, 13, 15, 16, 20, 21, 22, 28, 29, 31, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45):
        y = _lib.conv2d_nhwc(x, w, b, pad, False, None, None, 1, cfg, 1)
        assert torch.equal(y, ref_y), cfg


@pytest.mark.parametrize("split", [2, 3])
@pytest.mark.parametrize("B,H,W,C,Co,k", [(2, 32, 32, 640, 640, 3), (2, 8, 8, 1280, 1280, 3),
                                          (2, 16, 16, 640, 1280, 1)])
def test_conv_tile_families_bitwise_equal_at_split(cuda, split, B, H, W, C, Co, k):
    """At a fixed split-K every family walks the same K range per slab in the same MFMA order and
    the slabs are summed in slab order, so families stay bitwise interchangeable - what lets a solo
    task run the canonical (batch-8) split on a tile family tuned for its own shape
    (ops/csrc/conv_family.inc, scripts/tune_family.py)."""
    torch.manual_seed(13)
    x = torch.randn(B, H, W, C, device=cuda).bfloat16()
    w = (torch.randn(Co, k, k, C, device=cuda) / math.sqrt(k * k * C)).bfloat16()
    b = torch.randn(Co, device=cuda).bfloat16()
    r = torch.randn(B, H, W, Co, device=cuda).bfloat16()
    pad = k // 2
    ref_y = _lib.conv2d_nhwc(x, w, b, pad, False, r, None, 1, 15, split)
    for cfg in (0, 3, 4, 5, 10, 13, 14, 16, 20, 21, 22, 28, 29, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42,
                43, 44, 45):
        y = _lib.conv2d_nhwc(x, w, b, pad, False, r, None, 1, cfg, split)
        assert torch.equal(y, ref_y), cfg


@pytest.mark.parametrize("cfg", [24, 25, 26, 27])
@pytest.mark.parametrize("res", [False, True])
def test_gemm_persistent_many_tiles(cuda, cfg, res):
    """Persistent short-K kernel: > 256 tiles, so blocks walk several tiles through one DMA ring
    (bias rides the ring; residual read in the epilogue).  Bitwise equal to the one-tile kernels."""
    torch.manual_seed(6)
    M, K, N = 8200, 320, 648
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    r = torch.randn(M, N, device=cuda).bfloat16() if res else None
    y = _lib.gemm(x, w, b, r, cfg, 1)
    ref_y = x.float() @ w.float().t() + b.float() + (r.float() if res else 0)
    assert _rel(y, ref_y) < 1e-2
    assert torch.equal(y, _lib.gemm(x, w, b, r, 15, 1))


@pytest.mark.parametrize("M,K,N,cfg,split", [
    (8200, 320, 2560, -1, -1), (8200, 320, 2560, 15, 1), (8200, 320, 2560, 25, 1), (8200, 320, 2560, 21, 1),
    (8200, 320, 2560, 0, 1), (512, 1280, 10240, 13, 3), (512, 1280, 10240, 22, 2), (300, 640, 5120, 3, 1),
    (8200, 320, 2560, 32, 1), (300, 640, 5120, 35, 1), (8200, 320, 2560, 46, 1), (8192, 640, 5120, 47, 1),
    (300, 640, 5120, 47, 1), (1000, 320, 2576, 47, 1)])
def test_gemm_geglu_bitwise_equals_unfused(cuda, M, K, N, cfg, split):
    """GEGLU in the GEMM epilogue (interleaved value/gate rows) == geglu(gemm(x, w, b)) bitwise,
    for register / LDS-DMA / 8-wave tiles, split-K (reduce kernel) and the persistent remap."""
    torch.manual_seed(7)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    want = _lib.geglu(_lib.gemm(x, w, b, None, cfg, split))
    got = _lib.gemm_geglu(x, _lib.interleave_geglu(w), _lib.interleave_geglu(b), cfg, split)
    assert got.shape == (M, N // 2)
    assert torch.equal(got, want)
    r = ref.geglu(x.float() @ w.float().t() + b.float())
    assert _rel(got, r) < 2e-2


@pytest.mark.parametrize("cfg", [32, 33, 34, 35])
@pytest.mark.parametrize("B,H,W,Cin,Cout,k,up,stride,res,temb", [
    (8, 64, 64, 320, 320, 3, False, 1, True, False), (8, 64, 64, 640, 320, 3, False, 1, False, True),
    (2, 37, 29, 320, 640, 1, False, 1, True, True), (2, 37, 29, 128, 1280, 3, False, 1, False, False),
    (2, 16, 16, 320, 320, 3, True, 1, False, False), (3, 33, 35, 192, 200, 3, False, 2, True, False)])
def test_conv2d_xreg_tiles_bitwise_equal_register_staged(cuda, cfg, B, H, W, Cin, Cout, k, up, stride, res, temb):
    """X-in-registers tiles (activation fragments straight to VGPRs, weights through the LDS-DMA
    ring): partial M / N tiles, upsample, stride 2, bias + temb + residual epilogue.  Same per-output
    MFMA order as the register-staged kernel, so bitwise equal to it; and close to fp32."""
    torch.manual_seed(21)
    x = torch.randn(B, H, W, Cin, device=cuda).bfloat16()
    w = (torch.randn(Cout, k, k, Cin, device=cuda) / math.sqrt(k * k * Cin)).bfloat16()
    b = torch.randn(Cout, device=cuda).bfloat16()
    pad = k // 2
    Ho = ((2 * H if up else H) + 2 * pad - k) // stride + 1
    Wo = ((2 * W if up else W) + 2 * pad - k) // stride + 1
    r = torch.randn(B, Ho, Wo, Cout, device=cuda).bfloat16() if res else None
    t = torch.randn(B, Cout, device=cuda).bfloat16() if temb else None
    y = _lib.conv2d_nhwc(x, w, b, pad, up, r, t, stride, cfg, 1)
    ref_y = ref.conv2d_nhwc(x.float(), w.float(), b.float(), stride, pad, up)
    if res:
        ref_y = ref_y + r.float()
    if temb:
        ref_y = ref_y + t.float()[:, None, None, :]
    assert _rel(y, ref_y) < 1e-2
    assert torch.equal(y, _lib.conv2d_nhwc(x, w, b, pad, up, r, t, stride, 15, 1))
    assert torch.equal(y, _lib.conv2d_nhwc(x, w, b, pad, up, r, t, stride, cfg, 1))   # run to run


@pytest.mark.parametrize("cfg", [20, 21, 22, 23])
@pytest.mark.parametrize("Cout,k", [(320, 3), (640, 1), (1280, 3)])
def test_conv2d_big_tiles_match_register_staged(cuda, cfg, Cout, k):
    """8-wave LDS-DMA tiles (partial M and N edge tiles) against the 4-wave register-staged
    kernel: same per-element K order (32-wide MFMA steps in K-tile order), so bitwise equal."""
    torch.manual_seed(5)
    B, H, W, Cin = 2, 37, 29, 320
    x = torch.randn(B, H, W, Cin, device=cuda).bfloat16()
    w = (torch.randn(Cout, k, k, Cin, device=cuda) / math.sqrt(k * k * Cin)).bfloat16()
    b = torch.randn(Cout, device=cuda).bfloat16()
    pad = k // 2
    y = _lib.conv2d_nhwc(x, w, b, pad, False, None, None, 1, cfg, 1)
    ref_y = ref.conv2d_nhwc(x.float(), w.float(), b.float(), 1, pad, False)
    assert _rel(y, ref_y) < 1e-2
    y_reg = _lib.conv2d_nhwc(x, w, b, pad, False, None, None, 1, 15, 1)
    assert torch.equal(y, y_reg)


@pytest.mark.parametrize("B,H,W,C,G,mh,mw,one_plus,silu", [
    (1, 96, 96, 512, 32, 96, 96, 0.0, True), (1, 192, 192, 256, 32, 96, 96, 0.0, True),
    (1, 768, 768, 128, 32, 96, 96, 0.0, False), (2, 48, 48, 768, 32, 1, 1, 1.0, True),
    (2, 12, 12, 3072, 32, 1, 1, 1.0, True), (2, 9, 15, 64, 8, 3, 5, 0.0, True)])
def test_group_norm_modulated(cuda, B, H, W, C, G, mh, mw, one_plus, silu):
    """SpatialNorm (MoVQ) / scale-shift norm (GLIDE) fused apply vs fp32 reference."""
    torch.manual_seed(2)
    x = (torch.randn(B, H, W, C, device=cuda) * 2 + 1).bfloat16()
    g = (torch.rand(C, device=cuda) + 0.5).bfloat16()
    b = torch.randn(C, device=cuda).bfloat16()
    mod = torch.randn(B, mh, mw, 2 * C, device=cuda).bfloat16()
    y = _lib.group_norm_mod_nhwc(x, g, b, G, 1e-6, silu, mod, one_plus)
    r = ref.group_norm_mod_nhwc(x.float(), g.float(), b.float(), G, 1e-6, silu, mod.float(), one_plus)
    assert _rel(y, r) < 1e-2
    assert torch.equal(y, _lib.group_norm_mod_nhwc(x, g, b, G, 1e-6, silu, mod, one_plus))


@pytest.mark.parametrize("B,F,P,H,D", [(2, 24, 2880, 5, 64), (2, 16, 64, 2, 64), (1, 1, 10, 1, 64),
                                       (2, 33, 17, 3, 64), (1, 96, 9, 2, 64), (2, 24, 40, 4, 32),
                                       (1, 24, 30, 2, 128), (1, 70, 5, 1, 128)])
def test_temporal_attention(cuda, B, F, P, H, D):
    """Frame-axis attention on strided views of a fused-QKV frame-major activation."""
    torch.manual_seed(3)
    qkv = torch.randn(B, F, P, 3, H, D, device=cuda).bfloat16()
    q, k, v = qkv[:, :, :, 0], qkv[:, :, :, 1], qkv[:, :, :, 2]
    o = _lib.temporal_attention(q, k, v, 1 / math.sqrt(D))
    r = ref.temporal_attention(q.float(), k.float(), v.float(), 1 / math.sqrt(D))
    assert _rel(o, r) < 2e-2
    assert torch.equal(o, _lib.temporal_attention(q, k, v, 1 / math.sqrt(D)))


@pytest.mark.parametrize("B,F,P,C,Co", [(2, 24, 2880, 320, 320), (1, 16, 64, 128, 64), (2, 5, 33, 64, 128)])
def test_temporal_conv3x1(cuda, B, F, P, C, Co):
    """(3,1,1) Conv3d over [B, F, HW, C] as a 3x1 implicit-GEMM conv (+ fused residual)."""
    torch.manual_seed(4)
    x = torch.randn(B, F, P, C, device=cuda).bfloat16()
    w = (torch.randn(Co, 3, 1, C, device=cuda) / math.sqrt(3 * C)).bfloat16()
    b = torch.randn(Co, device=cuda).bfloat16()
    res = torch.randn(B, F, P, Co, device=cuda).bfloat16()
    y = _lib.conv2d_nhwc(x, w, b, 1, False, res)
    r = ref.conv2d_nhwc(x.float(), w.float(), b.float(), 1, 1) + res.float()
    assert y.shape == r.shape and _rel(y, r) < 1e-2


@pytest.mark.parametrize("N,C,H,W", [(1, 64, 18, 32), (2, 20, 36, 64), (1, 16, 144, 256), (3, 40, 9, 16)])
def test_convgru_gates(cuda, N, C, H, W):
    """RVM ConvGRU fused gates (fp16 channels-last) vs fp32 reference."""
    torch.manual_seed(5)
    cl = torch.channels_last
    ih = torch.randn(N, 2 * C, H, W, device=cuda).half().contiguous(memory_format=cl)
    h = torch.rand(N, C, H, W, device=cuda).half().contiguous(memory_format=cl)
    buf = torch.randn(N, 2 * C, H, W, device=cuda).half().contiguous(memory_format=cl)
    buf_r = buf.clone()
    z = _lib.convgru_gates1(ih, h, buf, C)
    zr = ref.convgru_gates1(ih, h, buf_r, C)
    assert _rel(z, zr) < 2e-3 and _rel(buf, buf_r) < 2e-3
    c = torch.randn(N, C, H, W, device=cuda).half().contiguous(memory_format=cl)
    hn = _lib.convgru_gates2(c, h, z)
    assert _rel(hn, ref.convgru_gates2(c, h, z)) < 2e-3


@pytest.mark.parametrize("B,H,W,C1,C2,Co", [(8, 64, 64, 320, 320, 320), (8, 32, 32, 640, 320, 640),
                                             (8, 16, 16, 1280, 640, 1280), (2, 8, 8, 1280, 1280, 1280),
                                             (2, 24, 24, 1536, 1152, 1536)])
def test_skip_concat_read_in_place_is_bitwise(cuda, B, H, W, C1, C2, Co):
    """UNet up-path [h | skip] read in place (ops.CatPair): GroupNorm table, table-apply, the 1x1
    shortcut conv and a whole ResBlock are bitwise equal to the materialised-concat path."""
    from arbius_amd.models.layers import init_weights
    from arbius_amd.models.unet2d import ResBlock
    torch.manual_seed(11)
    a = torch.randn(B, H, W, C1, device=cuda).bfloat16()
    b = (torch.randn(B, H, W, C2, device=cuda) * 2).bfloat16()
    cat = torch.cat([a, b], -1)
    pair = ops.cat_channels(a, b)
    assert isinstance(pair, ops.CatPair)
    g = (torch.rand(C1 + C2, device=cuda) + 0.5).bfloat16()
    bt = torch.randn(C1 + C2, device=cuda).bfloat16()
    t1, t2 = ops.group_norm_table(pair, g, bt, 32, 1e-5), ops.group_norm_table(cat, g, bt, 32, 1e-5)
    assert torch.equal(t1, t2)
    assert torch.equal(_lib.norm_table_apply(a, t1, True, x2=b), _lib.norm_table_apply(cat, t2, True))
    w = (torch.randn(Co, 1, 1, C1 + C2, device=cuda) / math.sqrt(C1 + C2)).bfloat16()
    bias = torch.randn(Co, device=cuda).bfloat16()
    for pb in (None, 2):
        with ops.plan_batch(pb) if pb else torch.no_grad():
            assert torch.equal(ops.conv2d(pair, w, bias, padding=0), ops.conv2d(cat, w, bias, padding=0))
    rb = init_weights(ResBlock(C1 + C2, Co, 4 * 64, 32, 1e-5), 3).to(cuda, torch.bfloat16)
    temb = torch.randn(B, Co, device=cuda).bfloat16()
    with torch.no_grad():
        assert torch.equal(rb(pair, temb), rb(cat, temb))


@pytest.mark.parametrize("B,N,D", [(1, 4096, 512), (2, 2880, 512), (1, 1024, 512), (1, 100, 512)])
def test_large_head_attention(cuda, B, N, D):
    """d = 512 single-head attention (VAE / MoVQ mid block): GEMM -> HIP row softmax -> GEMM."""
    torch.manual_seed(10)
    qkv = torch.randn(B, N, 3, 1, D, device=cuda).bfloat16()
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    scale = 1 / math.sqrt(D)
    o = ops.attention(q, k, v)
    r = ref.attention(q.float(), k.float(), v.float(), scale, False)
    assert o.shape == r.shape and _rel(o, r) < 2e-2
    assert torch.equal(o, ops.attention(q, k, v))


@pytest.mark.parametrize("B,C,H,W,k,stride,dil,act", [
    (2, 72, 64, 64, 3, 2, 1, "relu"), (3, 120, 32, 30, 5, 1, 1, None), (2, 960, 16, 16, 5, 1, 2, "hs"),
    (1, 200, 17, 13, 3, 1, 1, "hs"), (4, 16, 135, 240, 3, 1, 1, "relu"), (2, 672, 33, 31, 5, 2, 1, "hs")])
def test_depthwise_conv_f16(cuda, B, C, H, W, k, stride, dil, act):
    """RVM MobileNetV3 depthwise conv + bias + act (csrc/depthwise.hip) vs fp32 torch, bitwise re-run."""
    import torch.nn.functional as F
    torch.manual_seed(8)
    cl = torch.channels_last
    x = torch.randn(B, C, H, W, device=cuda).half().contiguous(memory_format=cl)
    w = (torch.randn(C, 1, k, k, device=cuda) / k).half()
    b = torch.randn(C, device=cuda).half()
    y = ops.depthwise_conv(x, w, b, stride, dil, act)
    r = F.conv2d(x.float(), w.float(), b.float(), stride=stride, padding=dil * (k // 2), dilation=dil, groups=C)
    r = F.relu(r) if act == "relu" else (F.hardswish(r) if act == "hs" else r)
    assert y.shape == r.shape and y.is_contiguous(memory_format=cl)
    assert _rel(y, r) < 2e-3
    assert torch.equal(y, ops.depthwise_conv(x, w, b, stride, dil, act))


@pytest.mark.parametrize("B,H,W,Cin,Cout,k", [(2, 64, 64, 4, 320, 3), (2, 64, 64, 320, 4, 3), (1, 96, 96, 4, 1024, 1),
                                              (1, 128, 128, 128, 3, 3), (1, 96, 96, 4, 512, 3)])
def test_small_channel_conv_padded_onto_mfma(cuda, B, H, W, Cin, Cout, k):
    """conv_in / conv_out / SpatialNorm maps run on the HIP kernel via channel padding."""
    from arbius_amd import ops
    torch.manual_seed(6)
    x = torch.randn(B, H, W, Cin, device=cuda).bfloat16()
    w = (torch.randn(Cout, k, k, Cin, device=cuda) / math.sqrt(k * k * Cin)).bfloat16()
    b = torch.randn(Cout, device=cuda).bfloat16()
    y = ops.conv2d(x, w, b, padding=k // 2)
    r = ref.conv2d_nhwc(x.float(), w.float(), b.float(), 1, k // 2)
    assert y.shape == r.shape and y.is_contiguous() and _rel(y, r) < 1e-2


@pytest.mark.parametrize("H,W,C,G", [(8, 8, 1280, 32), (16, 16, 1280, 32), (32, 32, 640, 32), (5, 7, 320, 32),
                                     (8, 8, 2560, 32), (64, 64, 320, 32), (3, 3, 96, 8), (24, 24, 1152, 32)])
def test_group_norm_table_paths_accurate_and_batch_invariant(cuda, H, W, C, G):
    """Every GN-table path (single-launch small-image kernel, stats + table slabs) against fp32,
    and image 0 of a batch of 8 bitwise equal to the same image alone (lock-step groups)."""
    torch.manual_seed(13)
    x = (torch.randn(8, H, W, C, device=cuda) * 3 + 1).bfloat16()
    g = (torch.rand(C, device=cuda) + 0.5).bfloat16()
    bt = torch.randn(C, device=cuda).bfloat16()
    t8 = _lib.group_norm_table(x, g, bt, G, 1e-5)
    rt = ref.group_norm_table(x.float(), g.float(), bt.float(), G, 1e-5)
    assert _rel(t8, rt) < 1e-4
    t1 = _lib.group_norm_table(x[:1].contiguous(), g, bt, G, 1e-5)
    assert torch.equal(t8[:1], t1)
    assert torch.equal(t8, _lib.group_norm_table(x, g, bt, G, 1e-5))


@pytest.mark.parametrize("B,H,W,C,Co,k,silu,up,mod", [
    (2, 64, 64, 320, 320, 3, True, False, False), (2, 32, 32, 640, 1280, 3, True, False, False),
    (2, 16, 16, 2560, 1280, 3, True, False, False), (1, 48, 48, 384, 384, 3, True, True, False),
    (2, 24, 24, 768, 768, 3, True, False, True), (2, 1, 4096, 320, 320, 1, False, False, False),
    (2, 24, 2880, 320, 320, 31, True, False, False)])
def test_conv_groupnorm_prologue(cuda, B, H, W, C, Co, k, silu, up, mod):
    """GroupNorm(+SiLU, +scale-shift) fused into the conv operand load == GN then conv."""
    from arbius_amd import ops
    torch.manual_seed(7)
    x = (torch.randn(B, H, W, C, device=cuda) * 2 + 0.5).bfloat16()
    kh, kw = (3, 1) if k == 31 else (k, k)
    w = (torch.randn(Co, kh, kw, C, device=cuda) / math.sqrt(kh * kw * C)).bfloat16()
    b = torch.randn(Co, device=cuda).bfloat16()
    g = (torch.rand(C, device=cuda) + 0.5).bfloat16()
    bt = torch.randn(C, device=cuda).bfloat16()
    m = torch.randn(B, 2 * C, device=cuda).bfloat16() if mod else None
    table = _lib.group_norm_table(x, g, bt, 32, 1e-5, m, 1.0)
    rt = ref.group_norm_table(x.float(), g.float(), bt.float(), 32, 1e-5, None if m is None else m.float(), 1.0)
    assert _rel(table, rt) < 1e-4
    pad = 0 if k == 1 else 1
    y = _lib.conv2d_nhwc(x, w, b, pad, up, None, None, 1, norm=table, norm_silu=silu)
    xn = ops.apply_norm_table(x.float(), rt, silu)
    r = ref.conv2d_nhwc(xn, w.float(), b.float(), 1, pad, up)
    assert _rel(y, r) < 1.5e-2
    assert torch.equal(y, _lib.conv2d_nhwc(x, w, b, pad, up, None, None, 1, norm=table, norm_silu=silu))


@pytest.mark.parametrize("B,Nq,Np,H,D", [(2, 2304, 87, 12, 64), (2, 576, 87, 18, 64), (1, 100, 5, 2, 64),
                                         (2, 144, 64, 4, 40)])
def test_flash_attention_kv_prefix(cuda, B, Nq, Np, H, D):
    """Joint attention: prefix K/V segment read in place == attention over the concatenation."""
    torch.manual_seed(8)
    qkv = torch.randn(B, Nq, 3, H, D, device=cuda).bfloat16()
    ckv = torch.randn(B, Np, 2, H, D, device=cuda).bfloat16()
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    kp, vp = ckv[:, :, 0], ckv[:, :, 1]
    o = _lib.flash_attention(q, k, v, 1 / math.sqrt(D), False, (kp, vp))
    r = ref.attention(q.float(), torch.cat([kp, k], 1).float(), torch.cat([vp, v], 1).float(), 1 / math.sqrt(D))
    assert _rel(o, r) < 2e-2
    oc = _lib.flash_attention(q, torch.cat([kp, k], 1), torch.cat([vp, v], 1), 1 / math.sqrt(D), False)
    assert torch.equal(o, oc), "prefix segment must be bitwise identical to the concatenated keys"
    fn = _lib._fn("arb_set_attn_glds")      # register-staged K/V (the round-5 prefix path) == LDS-DMA
    try:
        fn(0)
        o_reg = _lib.flash_attention(q, k, v, 1 / math.sqrt(D), False, (kp, vp))
    finally:
        fn(1)
    assert torch.equal(o, o_reg)


@pytest.mark.parametrize("cfg", [0, 3, 5])
def test_splitk_inlaunch_reduce_bitwise_equals_reduce_kernel(cuda, cfg):
    """In-launch split-K reduction (register-staged kernels) sums slabs in the same order as the
    separate reduce kernel (LDS-DMA kernels): identical bits."""
    torch.manual_seed(9)
    x = torch.randn(2, 16, 16, 640, device=cuda).bfloat16()
    w = (torch.randn(1280, 3, 3, 640, device=cuda) / 76).bfloat16()
    b = torch.randn(1280, device=cuda).bfloat16()
    r = torch.randn(2, 16, 16, 1280, device=cuda).bfloat16()
    a = _lib.conv2d_nhwc(x, w, b, 1, False, r, None, 1, cfg + 10, 4)
    g = _lib.conv2d_nhwc(x, w, b, 1, False, r, None, 1, cfg, 4)
    assert torch.equal(a, g)
    assert torch.equal(a, _lib.conv2d_nhwc(x, w, b, 1, False, r, None, 1, cfg + 10, 4))


@pytest.mark.parametrize("B,H,W,C,silu", [(2, 16, 16, 320, True), (1, 8, 24, 1280, False), (3, 5, 7, 64, True),
                                          (2, 9, 13, 2560, True), (1, 64, 64, 4096, False)])
def test_norm_table_apply(cuda, B, H, W, C, silu):
    """Unfused GroupNorm-table prologue kernel == fp32 x*scale+shift(+SiLU)."""
    from arbius_amd import ops
    torch.manual_seed(11)
    x = torch.randn(B, H, W, C, device=cuda).bfloat16()
    table = torch.randn(B, C, 2, device=cuda)
    y = _lib.norm_table_apply(x, table, silu)
    r = ops.apply_norm_table(x.float(), table, silu)
    assert _rel(y, r) < 1e-2


@pytest.mark.parametrize("B,H,W,C,silu", [(8, 96, 96, 384, True), (2, 48, 48, 768, True), (1, 24, 24, 1152, False),
                                         (3, 6, 10, 64, True)])
def test_norm_pool2(cuda, B, H, W, C, silu):
    """GLIDE down-sampling: one pass == fp32 avg-pool of x and of bf16(GN-table transform(x)),
    bitwise equal to the unfused CPU-order arithmetic on the same bf16 intermediates."""
    torch.manual_seed(14)
    x = (torch.randn(B, H, W, C, device=cuda) * 2 + 0.3).bfloat16()
    table = torch.randn(B, C, 2, device=cuda)
    yn, yx = _lib.norm_pool2(x, table, silu)
    pool = torch.nn.functional.avg_pool2d
    rx = pool(x.float().permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
    xn = ops.apply_norm_table(x.float(), table, silu).bfloat16().float()
    rn = pool(xn.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
    assert _rel(yx, rx) < 5e-3 and _rel(yn, rn) < 5e-3
    yn2, yx2 = ops.pool2(x.cpu(), (table.cpu(), silu))          # CPU path: same formula, fp32
    assert _rel(yx, yx2.to(cuda)) < 5e-3 and _rel(yn, yn2.to(cuda)) < 1e-2
    assert torch.equal(yx, _lib.norm_pool2(x, None, False)[1])


@pytest.mark.parametrize("B,H,W,C", [(8, 48, 48, 768), (2, 12, 12, 1536), (1, 3, 5, 8)])
def test_upsample2(cuda, B, H, W, C):
    x = torch.randn(B, H, W, C, device=cuda).bfloat16()
    assert torch.equal(ops.upsample2(x), x.repeat_interleave(2, dim=1).repeat_interleave(2, dim=2))


@pytest.mark.parametrize("B,H,W,Cin,Cout,k,stride", [(12, 72, 128, 64, 128, 3, 1), (12, 36, 64, 80, 40, 1, 1),
                                                     (4, 144, 256, 16, 24, 3, 2), (2, 18, 32, 960, 128, 1, 1),
                                                     (1, 9, 16, 64, 64, 3, 1)])
def test_conv2d_fp16(cuda, B, H, W, Cin, Cout, k, stride):
    """fp16 twin of the implicit-GEMM kernel (robust video matting), incl. zero-padded channel
    counts (ops.conv2d pads Cin to a multiple of 64) == fp32 reference conv."""
    from arbius_amd import ops
    torch.manual_seed(12)
    x = torch.randn(B, H, W, Cin, device=cuda).half()
    w = (torch.randn(Cout, k, k, Cin, device=cuda) / math.sqrt(k * k * Cin)).half()
    b = torch.randn(Cout, device=cuda).half()
    y = ops.conv2d(x, w, b, stride=stride, padding=k // 2)
    r = ref.conv2d_nhwc(x.float(), w.float(), b.float(), stride, k // 2, False)
    assert y.dtype == torch.float16 and tuple(y.shape) == tuple(r.shape)
    assert _rel(y, r) < 5e-3
    assert torch.equal(y, ops.conv2d(x, w, b, stride=stride, padding=k // 2))


@pytest.mark.parametrize("name", ["DDIM", "K_EULER", "K_EULER_ANCESTRAL", "DPMSolverMultistep", "PNDM", "KLMS",
                                  "p_sampler"])
def test_fused_sampler_hip_vs_fp32_reference(cuda, name):
    """csrc/sampler.hip (one launch per step for a lock-step group of 3) vs ops.ref.sampler_step
    (fp32 torch): final latents and every step's bf16 UNet input; bitwise run-to-run."""
    from arbius_amd.models import schedulers as S

    def run(ref_ops):
        g = torch.Generator().manual_seed(11)
        cout = 8 if name == "p_sampler" else 4
        tasks = []
        for k in range(3):
            sched = (S.GaussianDiffusion(6, clamp=2.0) if name == "p_sampler" else S.make_scheduler(name, 7))
            x = torch.randn(1, 16, 24, 4, generator=g) * sched.init_noise_sigma
            tasks.append(S.TaskSampler(sched, x, torch.Generator().manual_seed(100 + k), cuda))
        xin = torch.empty(6, 16, 24, 4, dtype=torch.bfloat16, device=cuda)

        def rows(k, out):
            return (None if out is None else out[2 * k], None if out is None else out[2 * k + 1],
                    xin[2 * k], xin[2 * k + 1])

        samp = S.GroupSampler(tasks, [7.5, 3.0, 12.0], xin, rows)
        ops.set_reference_ops(ref_ops)
        try:
            samp.write_input(0)
            ins = []
            for i in range(len(tasks[0].plans)):
                out = (torch.randn(6, 16, 24, cout, generator=g) * 0.5).to(cuda, torch.bfloat16)
                samp.step(i, out)
                ins.append(xin.float().clone())
        finally:
            ops.set_reference_ops(False)
        return [t.x.clone() for t in tasks], ins

    a, ai = run(False)
    b, bi = run(True)
    a2, _ = run(False)
    for x, y, z in zip(a, b, a2):
        assert torch.equal(x, z), "fused sampler must be bitwise deterministic"
        assert torch.allclose(x, y, rtol=1e-4, atol=1e-4 * max(1.0, y.abs().max().item())), (x - y).abs().max()
    for x, y in zip(ai[:-1], bi[:-1]):
        assert (x - y).abs().max() <= 0.02 * max(1.0, y.abs().max().item())   # one bf16 ulp at most


@pytest.mark.parametrize("M,K,N,geglu,res", [(8 * 4096, 320, 960, False, False), (8 * 1024, 640, 640, False, False),
                                             (8 * 256, 1280, 10240, True, False), (2 * 77, 768, 3072, False, False),
                                             (300, 320, 2560, True, False), (1000, 1280, 1280, False, True)])
@pytest.mark.parametrize("cfg,split", [(-1, -1), (10, 1), (12, 3), (24, 1), (5, 2), (32, 1), (46, 1), (47, 1)])
def test_gemm_with_folded_layer_norm(cuda, M, K, N, geglu, res, cfg, split):
    """LayerNorm folded into the GEMM epilogue (row stats + gamma-scaled weights + wsum) against the
    fp32 reference LN -> linear (-> GEGLU), on every epilogue path: planned, register-staged,
    split-K reduce, persistent, LDS-DMA + split, X-in-registers."""
    from arbius_amd import ops
    torch.manual_seed(7)
    x = (torch.randn(M, K, device=cuda) * 3 + 1.5).bfloat16()        # offset mean: the fold must cancel it
    g = (torch.rand(K, device=cuda) + 0.5).bfloat16()
    be = (torch.randn(K, device=cuda) * 0.2).bfloat16()
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    r = torch.randn(M, N, device=cuda).bfloat16() if res else None
    wf, bf, wsum = ops.ln_fold(g, be, w, b, geglu=geglu)
    rs = _lib.row_stats(x, 1e-5)
    y = _lib.gemm_ln(x, wf, bf, wsum, rs, r, geglu=geglu, cfg=cfg, split=split)
    h = ref.layer_norm(x.float(), g.float(), be.float(), 1e-5) @ w.float().t() + b.float()
    if geglu:
        h = ref.geglu(h)
    if res:
        h = h + r.float()
    assert _rel(y, h) < 1.5e-2, _rel(y, h)
    assert torch.equal(y, _lib.gemm_ln(x, wf, bf, wsum, rs, r, geglu=geglu, cfg=cfg, split=split))   # bitwise rerun


@pytest.mark.parametrize("C,T,heads", [(320, 1024, 5), (640, 256, 10), (1280, 64, 20), (768, 77, 12)])
def test_transformer_block_batch_invariant(cuda, C, T, heads):
    """A lock-step group (batch 8) reproduces each CFG pair's solo (batch 2) bytes through a whole
    transformer block under ops.plan_batch(2): every size-dependent kernel choice (LayerNorm variant,
    LN fold into the GEMM, GEMM plan, attention tiling) is made for the canonical batch, never the
    launch's own row count (a choice by rows made a group's LN differ from solo)."""
    from arbius_amd.models.layers import init_weights
    from arbius_amd.models.unet2d import BasicTransformerBlock
    torch.manual_seed(12)
    blk = init_weights(BasicTransformerBlock(C, 768, heads), 5).to(cuda, torch.bfloat16)
    h = (torch.randn(8, T, C, device=cuda) * 2 + 0.5).bfloat16()
    ctx = torch.randn(8, 77, 768, device=cuda).bfloat16()
    xs = (torch.randn(8, T, C, device=cuda) + 1).bfloat16()
    g = (torch.rand(C, device=cuda) + 0.5).bfloat16()
    be = torch.randn(C, device=cuda).bfloat16()
    with torch.no_grad(), ops.plan_batch(2):
        full = blk(h, ctx)
        ln_full = ops.layer_norm(xs, g, be, 1e-5)
        for j in range(4):
            sl = slice(2 * j, 2 * j + 2)
            assert torch.equal(blk(h[sl].contiguous(), ctx[sl].contiguous()), full[sl]), f"pair {j}"
            assert torch.equal(ops.layer_norm(xs[sl].contiguous(), g, be, 1e-5), ln_full[sl])


@pytest.mark.parametrize("cfg,split", [(-1, -1), (10, 1), (21, 1), (34, 1), (36, 2), (24, 1), (15, 3)])
def test_conv_temb_column_slice_read_in_place(cuda, cfg, split):
    """The ResBlock time embedding is a column slice of ONE batched projection [B, sum(Cout)]; the
    conv epilogue reads it at its row stride (no contiguous copy) with bytes equal to the copied
    operand, on every epilogue path (LDS-staged, split-K reduce, persistent)."""
    torch.manual_seed(14)
    B, H, W, C, Co = 4, 16, 16, 128, 192
    x = torch.randn(B, H, W, C, device=cuda).bfloat16()
    w = (torch.randn(Co, 3, 3, C, device=cuda) / math.sqrt(9 * C)).bfloat16()
    b = torch.randn(Co, device=cuda).bfloat16()
    allp = torch.randn(B, 64 + Co + 320, device=cuda).bfloat16()
    temb = allp[:, 64:64 + Co]
    assert not temb.is_contiguous()
    y = _lib.conv2d_nhwc(x, w, b, 1, False, None, temb, 1, cfg, split)
    assert torch.equal(y, _lib.conv2d_nhwc(x, w, b, 1, False, None, temb.contiguous(), 1, cfg, split))
    ref_y = ref.conv2d_nhwc(x.float(), w.float(), b.float(), 1, 1, False) + temb.float()[:, None, None, :]
    assert _rel(y, ref_y) < 1e-2


@pytest.mark.parametrize("B,HW,C,G,mod", [(8, 4096, 320, 32, False), (8, 1024, 640, 32, False),
                                          (8, 256, 1280, 32, True), (2, 64, 2560, 32, False),
                                          (16, 9216, 384, 32, True), (1, 16384, 128, 32, False),
                                          (4, 2880, 960, 32, False), (2, 144, 1536, 32, True)])
def test_group_norm_table_wave_kernel_bitwise_equals_lds_tree(cuda, B, HW, C, G, mod):
    """The one-wave GroupNorm table kernel reproduces the 256-thread LDS tree's Chan combine exactly
    (same leaves, same pairings): tables bitwise equal, so the faster kernel moves no output byte."""
    torch.manual_seed(15)
    x = (torch.randn(B, HW, C, device=cuda) * 2 + 0.7).bfloat16()
    g = (torch.rand(C, device=cuda) + 0.5).bfloat16()
    bt = torch.randn(C, device=cuda).bfloat16()
    m = torch.randn(B, 2 * C, device=cuda).bfloat16() if mod else None
    fn = _lib._fn("arb_set_gn_table_lds")
    try:
        fn(1)
        t_lds = _lib.group_norm_table(x, g, bt, G, 1e-5, m, 1.0 if mod else 0.0)
        fn(0)
        t_wave = _lib.group_norm_table(x, g, bt, G, 1e-5, m, 1.0 if mod else 0.0)
    finally:
        fn(0)
    assert torch.equal(t_lds, t_wave)
    r = ref.group_norm_table(x.float(), g.float(), bt.float(), G, 1e-5, m.float() if mod else None,
                             1.0 if mod else 0.0)
    assert _rel(t_wave, r) < 1e-4


@pytest.mark.parametrize("B,HW,C,G,mod,cat", [(2, 576, 1152, 32, True, False), (2, 144, 1536, 32, False, False),
                                              (8, 144, 3072, 32, False, True), (2, 2304, 384, 32, True, False),
                                              (8, 256, 1280, 32, False, False), (8, 64, 2560, 32, False, True),
                                              (3, 100, 64, 4, False, False), (1, 48, 512, 8, True, False),
                                              (8, 4096, 320, 32, False, False), (2, 9216, 384, 32, True, False),
                                              (8, 1024, 1280, 32, False, True)])
def test_group_norm_fused_tail_bitwise_equals_two_launches(cuda, B, HW, C, G, mod, cat):
    """Statistics + table in one launch (the image's last stats block builds the table after a ticket)
    == the stats kernel followed by the one-wave table kernel, bit for bit - also when the input is a
    skip concat read in place - and every ticket is re-armed (a second call gives the same table)."""
    torch.manual_seed(16)
    x = (torch.randn(B, HW, C, device=cuda) * 2 + 0.7).bfloat16()
    g = (torch.rand(C, device=cuda) + 0.5).bfloat16()
    bt = torch.randn(C, device=cuda).bfloat16()
    m = torch.randn(B, 2 * C, device=cuda).bfloat16() if mod else None
    op = 1.0 if mod else 0.0
    x2 = None
    if cat:
        x, x2 = x[..., :C // 2].contiguous(), x[..., C // 2:].contiguous()
    fn = _lib._fn("arb_set_gn_tail")
    try:
        fn(0)
        t_two = _lib.group_norm_table(x, g, bt, G, 1e-5, m, op, x2=x2)
        fn(1)
        t_one = _lib.group_norm_table(x, g, bt, G, 1e-5, m, op, x2=x2)
        t_again = _lib.group_norm_table(x, g, bt, G, 1e-5, m, op, x2=x2)
    finally:
        fn(0)
    assert torch.equal(t_one, t_two)
    assert torch.equal(t_again, t_two)
    xf = x.float() if x2 is None else torch.cat([x, x2], -1).float()
    r = ref.group_norm_table(xf, g.float(), bt.float(), G, 1e-5, m.float() if mod else None, op)
    assert _rel(t_one, r) < 1e-4


@pytest.mark.parametrize("B,HW,C,G,mod,silu,cat", [(2, 576, 1152, 32, True, True, False),
                                                   (2, 144, 1536, 32, False, True, False),
                                                   (8, 144, 2048, 32, False, True, True),
                                                   (8, 256, 1280, 32, False, False, False),
                                                   (2, 1024, 640, 32, True, True, False),
                                                   (8, 64, 1920, 32, False, True, True),
                                                   (3, 100, 64, 4, False, True, False)])
def test_group_norm_slice_one_launch(cuda, B, HW, C, G, mod, silu, cat):
    """Small-slice GroupNorm (+scale-shift)(+SiLU) in one launch == the fp32 reference, also with the skip
    concat read in place; each (group, image) slice is one block, so an image's bytes do not depend on
    the batch it shares a launch with (lock-step groups == solo), and reruns are bitwise equal."""
    from arbius_amd import ops
    torch.manual_seed(17)
    x = (torch.randn(B, HW, C, device=cuda) * 2 + 0.7).bfloat16()
    g = (torch.rand(C, device=cuda) + 0.5).bfloat16()
    bt = torch.randn(C, device=cuda).bfloat16()
    m = (torch.randn(B, 2 * C, device=cuda) * 0.3).bfloat16() if mod else None
    op = 1.0 if mod else 0.0
    xa, xb = (x[..., :C // 2].contiguous(), x[..., C // 2:].contiguous()) if cat else (x, None)
    assert _lib.group_norm_slice_ok(xa, G, xb)
    y = _lib.group_norm_slice(xa, g, bt, G, 1e-5, m, op, silu, x2=xb)
    assert torch.equal(y, _lib.group_norm_slice(xa, g, bt, G, 1e-5, m, op, silu, x2=xb))
    rt = ref.group_norm_table(x.float(), g.float(), bt.float(), G, 1e-5, None if m is None else m.float(), op)
    r = ops.apply_norm_table(x.float(), rt, silu)
    assert _rel(y, r) < 1e-2
    if B > 1:   # image 1 alone == image 1 inside the batch
        m1 = None if m is None else m[1:2].contiguous()
        y1 = _lib.group_norm_slice(xa[1:2].contiguous(), g, bt, G, 1e-5, m1, op, silu,
                                   x2=None if xb is None else xb[1:2].contiguous())
        assert torch.equal(y1[0], y[1])


@pytest.mark.parametrize("F", [97, 200])
def test_temporal_attention_long_clips_via_flash(cuda, F):
    """damo accepts up to 500 frames: beyond the register-resident kernel's 96 the op gathers the
    (video, pixel) problems into the flash kernel - strided views of a fused QKV activation."""
    B, P, H, D = 2, 12, 2, 64
    qkv = torch.randn(B * F, P, 3 * H * D, device=cuda).to(torch.bfloat16)
    v5 = qkv.view(B, F, P, 3, H, D)
    q, k, v = v5[:, :, :, 0], v5[:, :, :, 1], v5[:, :, :, 2]
    o = ops.temporal_attention(q, k, v)
    r = ref.temporal_attention(q.float(), k.float(), v.float(), 1 / math.sqrt(D))
    assert o.shape == (B, F, P, H, D) and _rel(o, r) < 2e-2
    assert torch.equal(o, ops.temporal_attention(q, k, v))


@pytest.mark.parametrize("B,N,Nk,H,D,causal", [(8, 4096, 4096, 8, 40, False), (2, 4096, 4096, 8, 40, False),
                                               (8, 1024, 1024, 8, 80, False), (2, 77, 77, 12, 64, True),
                                               (2, 2304, 2304, 10, 64, False), (4, 300, 333, 5, 64, False),
                                               (16, 64, 64, 2, 40, False), (2, 130, 130, 3, 40, True)])
def test_flash_attention_pipelined_ring_bitwise(cuda, B, N, Nk, H, D, causal):
    """The software-pipelined K / V ring (PV of tile j-1 under QK + softmax of tile j) applies the
    same *alpha / +PV sequence to O as the plain loop: outputs bitwise equal."""
    torch.manual_seed(21)
    q = torch.randn(B, N, H, D, device=cuda).bfloat16()
    k = torch.randn(B, Nk, H, D, device=cuda).bfloat16() * 1.5
    v = torch.randn(B, Nk, H, D, device=cuda).bfloat16()
    fn = _lib._fn("arb_set_attn_pp")
    try:
        fn(0)
        plain = _lib.flash_attention(q, k, v, 1 / math.sqrt(D), causal)
        fn(1)
        piped = _lib.flash_attention(q, k, v, 1 / math.sqrt(D), causal)
    finally:
        fn(0)
    assert torch.equal(plain, piped)
    r = ref.attention(q.float(), k.float(), v.float(), 1 / math.sqrt(D), causal)
    assert _rel(piped, r) < 2e-2


@pytest.mark.parametrize("B,N,Nk,H,D,causal", [(16, 4096, 4096, 8, 40, False), (2, 4096, 4096, 8, 40, False),
                                               (8, 1024, 1024, 10, 64, False), (3, 2880, 2880, 5, 64, False),
                                               (4, 2000, 2000, 8, 40, True), (8, 1500, 700, 4, 64, False),
                                               (32, 1100, 1100, 8, 32, False), (16, 4096, 77, 8, 40, False),
                                               (48, 700, 77, 8, 24, False), (2, 130, 130, 3, 40, True),
                                               (4, 300, 333, 5, 64, False), (1, 64, 64, 1, 8, False)])
def test_flash_attention_ilp_softmax_bitwise(cuda, B, N, Nk, H, D, causal):
    """The ILP softmax (all query tiles of a key tile at once: max3 tree, gfx950 lane swaps, wave-uniform
    lazy-rescale branch with per-lane selects) == the per-query-tile softmax, bit for bit - including
    late rescales (a spiked second half of the keys), partial and causal tiles."""
    torch.manual_seed(23)
    q = torch.randn(B, N, H, D, device=cuda).bfloat16()
    k = torch.randn(B, Nk, H, D, device=cuda).bfloat16() * 1.5
    v = torch.randn(B, Nk, H, D, device=cuda).bfloat16()
    k[B // 2, Nk // 2:] *= 8.0           # a late rescale in one batch entry
    fn = _lib._fn("arb_set_attn_ilp")
    try:
        fn(0)
        plain = _lib.flash_attention(q, k, v, 1 / math.sqrt(D), causal)
        fn(1)
        ilp = _lib.flash_attention(q, k, v, 1 / math.sqrt(D), causal)
        ilp2 = _lib.flash_attention(q, k, v, 1 / math.sqrt(D), causal)
    finally:
        fn(1)
    assert torch.equal(plain, ilp) and torch.equal(ilp, ilp2)
    r = ref.attention(q.float(), k.float(), v.float(), 1 / math.sqrt(D), causal)
    assert _rel(ilp, r) < 2e-2


@pytest.mark.parametrize("B,N,Nk,H,D,causal", [(8, 4096, 4096, 8, 40, False), (8, 1024, 1024, 8, 80, False),
                                               (2, 77, 77, 12, 64, True), (2, 256, 256, 8, 160, False),
                                               (4, 300, 333, 5, 64, False), (2, 130, 130, 3, 40, True)])
def test_flash_attention_prescaled_q(cuda, B, N, Nk, H, D, causal):
    """Prescaled-Q softmax (S^T chains start from -m_run, exp2 straight off the accumulators; the
    default) against the raw-score form and the fp32 reference; deterministic on re-run."""
    torch.manual_seed(22)
    q = torch.randn(B, N, H, D, device=cuda).bfloat16()
    k = torch.randn(B, Nk, H, D, device=cuda).bfloat16()
    v = torch.randn(B, Nk, H, D, device=cuda).bfloat16()
    fn = _lib._fn("arb_set_attn_prescale")
    try:
        fn(0)
        raw = ops.attention(q, k, v, causal=causal)
        fn(1)
        ps = ops.attention(q, k, v, causal=causal)
    finally:
        fn(1)
    r = ref.attention(q.float(), k.float(), v.float(), 1 / math.sqrt(D), causal)
    assert _rel(ps, r) < 2e-2 and _rel(raw, r) < 2e-2 and _rel(ps, raw) < 1e-2
    assert torch.equal(ps, ops.attention(q, k, v, causal=causal))


@pytest.mark.parametrize("B,H,W,C,Co,cfg,split", [(8, 48, 48, 768, 768, 43, 1), (8, 24, 24, 1152, 1152, 44, 1),
                                                  (8, 12, 12, 1536, 1536, 43, 4), (2, 64, 64, 320, 320, 42, 1),
                                                  (1, 7, 9, 256, 192, 44, 1), (2, 16, 16, 1280, 1280, 43, 3)])
def test_stag2_prefetch_distance_bitwise(cuda, B, H, W, C, Co, cfg, split):
    """K-half staggered tiles with the DMA issued 4 halves ahead (lgkmcnt-retired slot reads), and that
    form with buffer-resource DMA addressing, == 3 halves ahead, bit for bit, over repeated launches
    (a WAR race would show as a flipped tile, a missing zero fill as garbage at the borders)."""
    torch.manual_seed(23)
    x = torch.randn(B, H, W, C, device=cuda).bfloat16()
    w = (torch.randn(Co, 3, 3, C, device=cuda) / math.sqrt(9 * C)).bfloat16()
    b = torch.randn(Co, device=cuda).bfloat16()
    fn, fb = _lib._fn("arb_set_stag2_pd"), _lib._fn("arb_set_stag2_buf")
    try:
        fn(3)
        fb(0)
        ref3 = _lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1, cfg, split)
        fn(4)
        outs = [_lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1, cfg, split) for _ in range(5)]
        fb(1)   # buffer-resource DMA: padding taps / rows past N zero-filled by the range check
        outs += [_lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1, cfg, split) for _ in range(5)]
    finally:
        fn(4)
        fb(1)
    assert all(torch.equal(o, ref3) for o in outs)
    r = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b.float(),
                                   padding=1).permute(0, 2, 3, 1)
    assert _rel(ref3, r) < 1e-2


@pytest.mark.parametrize("cfg", [0, 3, 5, 9, 20, 21, 22, 23, 28, 29, 30, 31, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45])
def test_lds_dma_buffer_resource_bitwise(cuda, cfg):
    """LDS-DMA through buffer resources (range-checked zero fill for padding taps / rows past N and M)
    == the global_load_lds + zero-page form, bit for bit, on a shape with borders and ragged tiles."""
    torch.manual_seed(24)
    B, H, W, C, Co = 2, 13, 11, 192, 200
    x = torch.randn(B, H, W, C, device=cuda).bfloat16()
    w = (torch.randn(Co, 3, 3, C, device=cuda) / math.sqrt(9 * C)).bfloat16()
    b = torch.randn(Co, device=cuda).bfloat16()
    fb = _lib._fn("arb_set_stag2_buf")
    try:
        fb(0)
        ref = _lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1, cfg, 1)
        fb(1)
        got = [_lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1, cfg, 1) for _ in range(3)]
    finally:
        fb(1)
    assert all(torch.equal(g, ref) for g in got)


@pytest.mark.parametrize("B,Nq,Nk", [(1, 4096, 4096), (1, 9216, 9216), (1, 300, 777), (3, 64, 2048), (1, 16, 5000),
                                     (2, 2880, 2880)])
def test_attention512_blockwise(cuda, B, Nq, Nk):
    """Blockwise d = 512 attention (csrc/attention512.hip: key splits merged in order at 4096 / 9216
    keys, partial 32-key tiles, Nq != Nk) vs the fp32 reference; bitwise rerun."""
    torch.manual_seed(11)
    q = torch.randn(B, Nq, 1, 512, device=cuda).bfloat16()
    kv = torch.randn(B, Nk, 2, 1, 512, device=cuda).bfloat16()
    k, v = kv[:, :, 0], kv[:, :, 1]
    o = _lib.attention512(q, k, v, 1 / math.sqrt(512))
    r = ref.attention(q.float(), k.float(), v.float(), 1 / math.sqrt(512), False)
    assert _rel(o, r) < 1e-2
    assert torch.equal(o, _lib.attention512(q, k, v, 1 / math.sqrt(512)))


def test_attention512_rescale_spike(cuda):
    """One key tile far above the running max (forces the lazy rescale mid-row, and in one key split
    only): still the reference within bf16 rounding."""
    torch.manual_seed(12)
    B, N = 1, 4096
    q = torch.randn(B, N, 1, 512, device=cuda) * 0.5
    k = torch.randn(B, N, 1, 512, device=cuda) * 0.5
    k[:, 2500] = q[:, 7] * 4.0               # query 7 locks onto key 2500 (third split)
    k[:, 40] = -q[:, 9] * 4.0
    v = torch.randn(B, N, 1, 512, device=cuda)
    q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
    o = _lib.attention512(q, k, v, 1 / math.sqrt(512))
    r = ref.attention(q.float(), k.float(), v.float(), 1 / math.sqrt(512), False)
    assert _rel(o, r) < 1e-2 and _rel(o[:, 7], r[:, 7]) < 1e-2


def test_attention512_memory_is_linear(cuda):
    """16,384 tokens (anythingv3 at 1024^2): no score matrix - the call allocates only its output (the
    GEMM path's [N, N] bf16 scores alone are 512 MiB)."""
    q = torch.randn(1, 16384, 1, 512, device=cuda).bfloat16()
    k = torch.randn(1, 16384, 1, 512, device=cuda).bfloat16()
    v = torch.randn(1, 16384, 1, 512, device=cuda).bfloat16()
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    o = ops.attention(q, k, v)
    torch.cuda.synchronize()
    assert torch.cuda.max_memory_allocated() - base <= 2 * o.numel() * o.element_size()
    assert torch.isfinite(o.float()).all()


@pytest.mark.parametrize("cfg", [46, 47])
@pytest.mark.parametrize("M,K,N,res,act", [(32768, 320, 320, False, None), (8200, 320, 960, True, None),
                                           (8192, 640, 640, True, None), (4100, 640, 1920, False, None),
                                           (300, 320, 328, True, None), (1000, 640, 88, False, "gelu"),
                                           (333, 320, 1280, True, "quick_gelu"), (8192, 1280, 640, True, None)])
def test_gemm_w_stationary_bitwise_equal_tiled(cuda, cfg, M, K, N, res, act):
    """W-stationary short-K kernel (csrc/conv_sk.inc, cfg 46 / 47: resident weight panel, activation
    rows straight to VGPRs, epilogue from registers): ragged M, partial weight panels, bias +
    residual / activation epilogues, bitwise equal to the register-staged tile at split 1; shapes
    outside its range (K = 1280, K = 640 on cfg 46) take the X-in-registers tile (same bytes)."""
    torch.manual_seed(21)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    r = torch.randn(M, N, device=cuda).bfloat16() if res else None
    y = _lib.gemm(x, w, b, r, cfg, 1, act=act)
    assert torch.equal(y, _lib.gemm(x, w, b, r, 15, 1, act=act))
    assert torch.equal(y, _lib.gemm(x, w, b, r, cfg, 1, act=act))
    h = x.float() @ w.float().t() + b.float() + (r.float() if res else 0)
    if act == "gelu":
        h = torch.nn.functional.gelu(h)
    elif act == "quick_gelu":
        h = h * torch.sigmoid(1.702 * h)
    assert _rel(y, h) < 1.5e-2


@pytest.mark.parametrize("mode", [0, 1])
def test_image_u8_equals_aten_chain(cuda, mode):
    """The decode tail in one HIP pass == the PyTorch expression chain, byte for byte (incl. values
    exactly at .5 after scaling, and out-of-range inputs)."""
    torch.manual_seed(30)
    x = (torch.randn(333, 517, 3, device=cuda) * 1.3).bfloat16()
    x.view(-1)[:8] = torch.tensor([-1.0, 1.0, 0.0, 2.5, -3.0, 1 / 255, 0.5, -0.5], device=cuda).bfloat16()
    got = _lib.image_u8(x, mode)
    f = x.float()
    want = ((f / 2 + 0.5).clamp(0, 1) * 255).round() if mode == 0 else ((f + 1.0) * 127.5).clamp(0, 255).round()
    assert torch.equal(got, want.to(torch.uint8))
