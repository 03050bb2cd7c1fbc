"""RVM HIP fast path (csrc/rvm.hip + models/rvm_fast.py) against fp32 PyTorch oracles of the same
operations, and end to end against the PyTorch-op network (reference ops, fp32)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from arbius_amd import ops
from arbius_amd.ops import _lib

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_resize_u8_matches_interpolate(cuda):
    g = torch.Generator().manual_seed(0)
    fr = torch.randint(0, 256, (3, 181, 333, 3), generator=g, dtype=torch.uint8).to(cuda)
    for (h, w) in ((97, 178), (181, 333), (45, 89)):
        y = _lib.rvm_resize_u8(fr, h, w)
        ref = F.interpolate(fr.permute(0, 3, 1, 2).float() / 255, (h, w), mode="bilinear", align_corners=False)
        assert (y.float() - ref.permute(0, 2, 3, 1)).abs().max().item() < 2e-3


def test_pool3_and_upcat_match_torch(cuda):
    torch.manual_seed(1)
    s0 = torch.rand(2, 37, 61, 3, device=cuda).half()
    s1, s2, s3 = _lib.rvm_pool3(s0)
    r1 = F.avg_pool2d(s0.permute(0, 3, 1, 2), 2, 2, ceil_mode=True)
    r2 = F.avg_pool2d(r1, 2, 2, ceil_mode=True)
    r3 = F.avg_pool2d(r2, 2, 2, ceil_mode=True)
    for a, b in ((s1, r1), (s2, r2), (s3, r3)):
        assert a.shape == b.permute(0, 2, 3, 1).shape
        assert (a.float() - b.permute(0, 2, 3, 1).float()).abs().max().item() < 2e-3
    x = torch.randn(2, 10, 16, 40, device=cuda).half()
    f = torch.randn(2, 19, 31, 24, device=cuda).half()
    s = torch.randn(2, 19, 31, 3, device=cuda).half()
    y = _lib.rvm_upcat(x, f, s, 72)
    up = F.interpolate(x.permute(0, 3, 1, 2).float(), scale_factor=2.0, mode="bilinear", align_corners=False)
    up = up[:, :, :19, :31].permute(0, 2, 3, 1)
    ref = torch.cat([up, f.float(), s.float(), torch.zeros(2, 19, 31, 5, device=cuda)], -1)
    assert (y.float() - ref).abs().max().item() < 1e-2


@pytest.mark.parametrize("T,H,W,C", [(3, 17, 29, 96), (2, 68, 120, 16), (4, 9, 16, 960), (1, 1, 1, 40)])
def test_chan_mean_and_gates_match_torch(cuda, T, H, W, C):
    """Squeeze-excite / LR-ASPP pooling and gating kernels against fp32 torch."""
    torch.manual_seed(4)
    x = torch.randn(T, H, W, C, device=cuda).half()
    m = _lib.rvm_chan_mean(x)
    ref = x.float().mean(dim=(1, 2), keepdim=True)
    assert (m.float() - ref).abs().max().item() < 2e-3
    assert torch.equal(m, _lib.rvm_chan_mean(x))
    w = torch.randn(T, 1, 1, C, device=cuda).half() * 4
    for mode, fn in ((0, F.hardsigmoid), (1, torch.sigmoid)):
        y = _lib.rvm_gate(x.clone(), w, mode)
        r = x.float() * fn(w.float()).half().float()
        assert (y.float() - r).abs().max().item() < 1e-2


@pytest.mark.parametrize("cx,co,k,stride,act,res", [(24, 72, 1, 1, 2, False), (40, 40, 1, 1, 0, True),
                                                     (176, 80, 3, 1, 1, False), (16, 16, 3, 1, 1, False),
                                                     (960, 128, 1, 1, 1, False), (72, 24, 1, 1, 0, True),
                                                     (80, 24, 3, 1, 0, False), (16, 64, 1, 1, 2, False)])
def test_conv_ex_padded_channels_and_act(cuda, cx, co, k, stride, act, res):
    """Channels that are not a multiple of 64 read in place (zeros for the padding) + fused activation."""
    torch.manual_seed(2)
    x = torch.randn(3, 23, 41, cx, device=cuda).half()
    w = (torch.randn(co, k, k, cx, device=cuda) / math.sqrt(k * k * cx)).half()
    b = torch.randn(co, device=cuda).half()
    cp = -(-cx // 64) * 64
    wp = torch.zeros(co, k, k, cp, device=cuda).half()
    wp[..., :cx] = w
    r = torch.randn(3, 23, 41, co, device=cuda).half() if res else None
    y = _lib.conv_ex(x, wp, b, k, stride, k // 2, act, r)
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), b.float(), stride, k // 2)
    ref = ref.permute(0, 2, 3, 1)
    if res:
        ref = ref + r.float()
    ref = F.relu(ref) if act == 1 else F.hardswish(ref) if act == 2 else ref
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("H,W", [(360, 640), (240, 320), (200, 176)])
def test_fast_matting_matches_reference_network(cuda, H, W):
    """The whole fast path (stem, encoder with fused epilogues, pooled pyramid, upcat, in-place
    ConvGRU over 2 chunks, guided filter - or, for inputs <= 512 px, the full-resolution head -
    composite) against the PyTorch-op network in fp32."""
    from arbius_amd.models.rvm import RVMConfig, RVMPipeline
    cfg = RVMConfig(chunk=4)
    fast = RVMPipeline(cfg, device=cuda)
    assert fast._fast_ok(min(1.0, cfg.max_side / max(H, W)))
    rng = np.random.default_rng(3)
    yy, xx = np.mgrid[0:H, 0:W]
    base = ((xx[None] + 9 * np.arange(6)[:, None, None]) % 256).astype(np.uint8)
    clip = np.stack([base, (yy[None] % 256).astype(np.uint8).repeat(6, 0),
                     rng.integers(0, 256, base.shape, dtype=np.uint8)], axis=-1)
    got = fast(clip, "green-screen")
    again = fast(clip, "green-screen")
    assert np.array_equal(got, again)                      # bitwise rerun
    ref_pipe = RVMPipeline(cfg, device=cuda, dtype=torch.float32)
    ref_pipe.net.load_state_dict(fast.net.state_dict())
    ops.set_reference_ops(True)
    try:
        ref = ref_pipe(clip, "green-screen")
    finally:
        ops.set_reference_ops(False)
    d = np.abs(got.astype(int) - ref.astype(int))
    assert d.mean() < 1.5 and np.percentile(d, 99) <= 8, (d.mean(), np.percentile(d, 99))
    for mode in ("alpha-mask", "foreground-mask"):
        assert fast(clip, mode).shape == clip.shape


def test_long_clip_takes_the_staged_download_with_the_same_bytes(cuda, monkeypatch):
    """a clip above the pinned-result cap (or a failed pin) downloads through the reusable
    staging buffers instead of one page-locked array of the whole clip - same bytes either way."""
    from arbius_amd.models import rvm
    from arbius_amd.models.rvm import RVMConfig, RVMPipeline
    pipe = RVMPipeline(RVMConfig(chunk=4), device=cuda)
    rng = np.random.default_rng(5)
    clip = rng.integers(0, 256, (9, 240, 320, 3), dtype=np.uint8)
    pinned = pipe(clip, "green-screen")
    monkeypatch.setattr(rvm, "_PINNED_OUT_MAX", 0)
    staged = pipe(clip, "green-screen")
    assert np.array_equal(pinned, staged)


@pytest.mark.parametrize("T,H,W", [(2, 37, 53), (3, 180, 320), (1, 1080, 1920)])
def test_gpu_yuv420_equals_host_conversion(cuda, T, H, W):
    """csrc/elementwise.hip rgb_to_yuv420_kernel == native rgb_to_420 (the encoder's host conversion),
    padding rows / columns included, sample for sample."""
    from arbius_amd import native
    rng = np.random.default_rng(T * H + W)
    fr = rng.integers(0, 256, (T, H, W, 3), dtype=np.uint8)
    fr[0, :4] = 0
    fr[-1, -4:] = 255                                     # the clip range [1, 254] at both ends
    ref = native.rgb_to_yuv420_planes(fr)
    got = ops.rgb_to_yuv420(torch.from_numpy(fr).to(cuda))
    assert ops.native_loaded()
    for a, b in zip(got, ref):
        assert tuple(a.shape) == b.shape and np.array_equal(a.cpu().numpy(), b)


def test_rvm_solve_path_yuv_planes_encode_to_the_rgb_bytes(cuda, monkeypatch):
    """The solve path (RVMPipeline.matte_for_encode) encodes the GPU-converted 4:2:0 planes on the GPU
    (csrc/h264_intra.hip): the MP4 is byte-identical to encoding the RGB composite on the host, and so
    are the A/B paths - planes downloaded for the host encoder, the staged RGB download, and a clip
    the GPU encoder flags (capacity) falling back to the host encode."""
    from arbius_amd.models import rvm
    from arbius_amd.models.rvm import RVMConfig, RVMPipeline
    from arbius_amd.utils.mp4 import H264IntraClip, Yuv420Clip, encode_mp4
    pipe = RVMPipeline(RVMConfig(chunk=4), device=cuda)
    rng = np.random.default_rng(9)
    clip = rng.integers(0, 256, (9, 181, 322, 3), dtype=np.uint8)
    rgb = pipe(clip, "green-screen")
    want = encode_mp4(rgb, 24)
    enc = pipe.matte_for_encode(clip, "green-screen")
    assert isinstance(enc, H264IntraClip) and len(enc) == 9
    assert encode_mp4(enc, 24) == want
    monkeypatch.setattr(_lib, "h264_intra_capacity", lambda F, H16, W16: 64)   # flagged -> host encode
    flagged = pipe.matte_for_encode(clip, "green-screen")
    assert isinstance(flagged, Yuv420Clip) and encode_mp4(flagged, 24) == want
    monkeypatch.setattr(rvm, "_GPU_H264", False)
    planes = pipe.matte_for_encode(clip, "green-screen")
    assert isinstance(planes, Yuv420Clip) and len(planes) == 9
    assert encode_mp4(planes, 24) == want
    monkeypatch.setattr(rvm, "_PINNED_OUT_MAX", 0)        # staged download: RGB frames, same bytes
    staged = pipe.matte_for_encode(clip, "green-screen")
    assert not isinstance(staged, (Yuv420Clip, H264IntraClip)) and encode_mp4(staged, 24) == want
