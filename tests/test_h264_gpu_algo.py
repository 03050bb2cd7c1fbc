"""The GPU H.264 intra encoder's per-macroblock functions (ops/csrc/h264_intra.hip, __host__
__device__) run on the CPU through ``arb_h264_intra_host``: their slices must be the native encoder's
bytes (native/src/h264.cpp encode_idr), NAL for NAL, and ``encode_mp4`` of the result the MP4 of the
same planes.  Runs without a GPU; the device launch of the same code is tests/test_h264_gpu.py."""
import numpy as np
import pytest

from arbius_amd import native
from arbius_amd.ops import _lib

pytestmark = pytest.mark.skipif(not (native.loaded and _lib._LIB_PATH.exists()),
                                reason="native runtime / kernel library not built")


def planes(kind, F, H16, W16, seed):
    rng = np.random.default_rng(seed)
    if kind == "noise":
        return (rng.integers(1, 255, (F, H16, W16), dtype=np.uint8),
                rng.integers(1, 255, (F, H16 // 2, W16 // 2), dtype=np.uint8),
                rng.integers(1, 255, (F, H16 // 2, W16 // 2), dtype=np.uint8))
    if kind == "flat":
        v = [0, 255, 128][seed % 3]
        return (np.full((F, H16, W16), v, np.uint8), np.full((F, H16 // 2, W16 // 2), 255 - v, np.uint8),
                np.full((F, H16 // 2, W16 // 2), v, np.uint8))
    if kind == "edges":     # hard 0 / 255 steps: large residuals, level escapes, plane prediction clips
        yy, xx = np.mgrid[0:H16, 0:W16]
        y = np.stack([(((xx // (3 + t)) + (yy // 5)) % 2) * 255 for t in range(F)]).astype(np.uint8)
        yc, xc = np.mgrid[0:H16 // 2, 0:W16 // 2]
        c = np.stack([((xc // 3 + yc // 2 + t) % 2) * 254 for t in range(F)]).astype(np.uint8)
        return y, c, 254 - c
    yy, xx = np.mgrid[0:H16, 0:W16]         # smooth gradients + a little noise: every mode wins somewhere
    y = np.stack([(xx * 3 + yy * 2 + 7 * t) % 230 + 10 + rng.integers(0, 6, (H16, W16)) for t in range(F)])
    yc, xc = np.mgrid[0:H16 // 2, 0:W16 // 2]
    cb = np.stack([(xc + 2 * yc + t) % 200 + 20 for t in range(F)])
    cr = np.stack([(2 * xc + 3 * yc + 3 * t) % 180 + 30 for t in range(F)])
    return y.astype(np.uint8), cb.astype(np.uint8), cr.astype(np.uint8)


CASES = [("smooth", 2, 32, 48, 20), ("noise", 3, 64, 80, 20), ("flat", 2, 16, 16, 20), ("flat", 1, 48, 16, 20),
         ("edges", 2, 96, 64, 20), ("edges", 1, 64, 64, 0), ("noise", 1, 32, 32, 0), ("smooth", 2, 80, 112, 51),
         ("noise", 1, 16, 160, 37), ("smooth", 1, 160, 16, 8)]


@pytest.mark.parametrize("kind,F,H16,W16,qp", CASES)
def test_host_run_of_gpu_encoder_equals_native(kind, F, H16, W16, qp):
    y, cb, cr = planes(kind, F, H16, W16, F * H16 + W16 + qp)
    _, _, want = native.h264_encode_yuv420_frames(y, cb, cr, W16, H16, qp, 2)
    out, meta = _lib.h264_intra_host(y, cb, cr, qp)
    assert meta[F + 1] == 0
    got = native.h264_nals_from_rbsp(out, meta, F, 2)
    assert len(got) == len(want)
    for f, (a, b) in enumerate(zip(got, want)):
        assert a == b, f"picture {f}: {len(a)} vs {len(b)} bytes"


def test_intra_clip_mp4_equals_yuv_clip_mp4():
    from arbius_amd.utils.mp4 import INTRA_QP, H264IntraClip, Yuv420Clip, encode_mp4
    y, cb, cr = planes("smooth", 3, 48, 64, 1)
    out, meta = _lib.h264_intra_host(y, cb, cr, INTRA_QP)
    a = encode_mp4(H264IntraClip(out, meta, 60, 41, INTRA_QP), 24)
    b = encode_mp4(Yuv420Clip(y, cb, cr, 60, 41), 24)
    assert a == b


def test_capacity_flag_and_rbsp_checks():
    y, cb, cr = planes("noise", 2, 32, 32, 3)
    out, meta = _lib.h264_intra_host(y, cb, cr, 20)
    bad = meta.copy()
    bad[3] = 2                                     # an encoder error flag
    with pytest.raises(RuntimeError):
        native.h264_nals_from_rbsp(out, bad, 2, 1)
    bad = meta.copy()
    bad[2 + 2] = 8 * out.size                      # a picture past the buffer
    with pytest.raises(ValueError):
        native.h264_nals_from_rbsp(out, bad, 2, 1)
