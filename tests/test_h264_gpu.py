"""GPU H.264 intra encoder (ops/csrc/h264_intra.hip) against the native encoder
(native/src/h264.cpp encode_idr): identical NALs for every case of the host-run test, a 1080p clip
and a many-picture clip (one workgroup per picture), run to run."""
import pytest
import torch

from arbius_amd import native, ops
from test_h264_gpu_algo import CASES, planes

pytestmark = pytest.mark.gpu


def _gpu_nals(y, cb, cr, qp, cuda):
    t = [torch.from_numpy(a).to(cuda) for a in (y, cb, cr)]
    out, meta = ops.h264_intra_encode(*t, qp)
    assert ops.native_loaded()
    m = meta.cpu().numpy()
    assert m[len(y) + 1] == 0
    buf = out[:int(m[len(y)])].cpu().numpy()
    return native.h264_nals_from_rbsp(buf, m, len(y), 4)


@pytest.mark.parametrize("kind,F,H16,W16,qp", CASES + [("smooth", 2, 1088, 1920, 20), ("noise", 40, 64, 96, 20)])
def test_gpu_encoder_equals_native(cuda, kind, F, H16, W16, qp):
    y, cb, cr = planes(kind, F, H16, W16, F * H16 + W16 + qp)
    _, _, want = native.h264_encode_yuv420_frames(y, cb, cr, W16, H16, qp, 8)
    got = _gpu_nals(y, cb, cr, qp, cuda)
    assert len(got) == len(want)
    for f, (a, b) in enumerate(zip(got, want)):
        assert a == b, f"picture {f}: {len(a)} vs {len(b)} bytes"


def test_gpu_encoder_rerun_and_capacity_flag(cuda, monkeypatch):
    from arbius_amd.ops import _lib
    y, cb, cr = planes("noise", 3, 48, 64, 11)
    a = _gpu_nals(y, cb, cr, 20, cuda)
    assert _gpu_nals(y, cb, cr, 20, cuda) == a
    monkeypatch.setattr(_lib, "h264_intra_capacity", lambda F, H16, W16: 64)
    out, meta = ops.h264_intra_encode(*[torch.from_numpy(p).to(cuda) for p in (y, cb, cr)], 20)
    assert meta.cpu().numpy()[4] & 2
