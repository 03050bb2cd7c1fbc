"""Numerics of the gfx950 HIP kernels vs the fp32 PyTorch reference (ops/ref.py)."""
import math

import pytest
import torch

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


@pytest.mark.parametrize("M,C", [(8192, 320), (2048, 640), (154, 768), (512, 1280), (77, 1024)])
def test_layer_norm(cuda, M, C):
    x = torch.randn(M, C, device=cuda).bfloat16()
    g = torch.randn(C, device=cuda).bfloat16()
    b = torch.randn(C, device=cuda).bfloat16()
    y = _lib.layer_norm(x, g, b, 1e-5)
    assert _rel(y, ref.layer_norm(x.float(), g.float(), b.float(), 1e-5)) < 1e-2


@pytest.mark.parametrize("B,Nq,Nk,H,D,causal", [
    (2, 4096, 4096, 8, 40, False), (2, 1024, 1024, 8, 80, False), (2, 256, 256, 8, 160, False),
    (2, 64, 64, 8, 160, False), (2, 4096, 77, 8, 40, False), (2, 1024, 77, 8, 80, False),
    (2, 77, 77, 12, 64, True), (3, 100, 37, 4, 64, False), (5, 24, 24, 5, 64, False),
    (1, 300, 300, 2, 128, True), (2, 200, 130, 3, 32, False), (1, 129, 65, 1, 96, False)])
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
