"""Video families (BASELINE config #4 zeroscopev2xl, damo) and the deterministic
MP4 writer / H.264 intra codec, on CPU: bitstream/container structure, lossless PCM round
trip, CAVLC intra encoder == decoder reconstruction, decodability probe, tiny UNet3D pipeline
determinism and a node round trip with out-1.mp4.

The CAVLC codec (``native/src/h264.cpp``) is checked against itself (encoder recon == decoder
output), its VLC tables for prefix-freeness, and its rate/distortion for sanity; no third-party
H.264 decoder exists in the image, so conformance against libavcodec is parity unpinned."""
import asyncio
import json

import numpy as np
import torch

from arbius_amd.models.video import VideoConfig, VideoPipeline
from arbius_amd.utils.mp4 import _ep, encode_mp4, read_mp4_pcm, rgb_to_yuv420, sps_pps
from arbius_amd.node.pool import LocalSolverPool

from test_node_e2e import _full_cycle, make_miner, make_world


class _Reader:
    def __init__(self, data):
        self.bits = "".join(f"{b:08b}" for b in data)
        self.i = 0

    def u(self, n):
        v = int(self.bits[self.i:self.i + n], 2) if n else 0
        self.i += n
        return v

    def ue(self):
        z = 0
        while self.bits[self.i] == "0":
            z += 1
            self.i += 1
        return self.u(z + 1) - 1

    def se(self):
        k = self.ue()
        return (k + 1) // 2 if k % 2 else -(k // 2)


def test_sps_fields_and_cropping():
    sps, pps = sps_pps(1920, 1080)
    assert sps[0] == 0x67 and pps[0] == 0x68
    r = _Reader(sps[1:])
    assert (r.u(8), r.u(8), r.u(8)) == (66, 0xC0, 51)
    assert r.ue() == 0 and r.ue() == 0 and r.ue() == 2 and r.ue() == 1 and r.u(1) == 0
    assert r.ue() + 1 == 120 and r.ue() + 1 == 68          # 1920/16, 1088/16
    assert r.u(1) == 1 and r.u(1) == 1
    assert r.u(1) == 1 and [r.ue() for _ in range(4)] == [0, 0, 0, 4]   # crop 8 rows (CropUnitY = 2)
    assert r.u(1) == 0 and r.u(1) == 1                        # no VUI, stop bit


def test_emulation_prevention():
    assert _ep(b"\x00\x00\x01\x00\x00\x00\x00") == b"\x00\x00\x03\x01\x00\x00\x03\x00\x00"


def test_mp4_pcm_roundtrip_lossless_and_deterministic():
    rng = np.random.default_rng(0)
    frames = [rng.integers(0, 256, (40, 72, 3), dtype=np.uint8) for _ in range(4)]
    a, b = encode_mp4(frames, 24, codec="pcm"), encode_mp4(frames, 24, codec="pcm")
    assert a == b and a[4:8] == b"ftyp" and a[a.index(b"moov") - 4:].startswith(a[a.index(b"moov") - 4:][:4])
    fps, planes = read_mp4_pcm(a)
    assert fps == 24 and len(planes) == 4
    for f, (y, cb, cr) in zip(frames, planes):
        ey, ecb, ecr = rgb_to_yuv420(np.pad(f, ((0, 8), (0, 8), (0, 0)), mode="edge"))
        assert (y == ey).all() and (cb == ecb).all() and (cr == ecr).all()
        assert y.min() >= 1 and cb.min() >= 1      # no start-code emulation possible in PCM bytes


def test_video_tiny_deterministic():
    pipe = VideoPipeline(VideoConfig.tiny(), device="cpu")
    kw = dict(num_frames=5, width=64, height=64, num_inference_steps=2, seed=3)
    a, b = pipe("arbius test cat", **kw), pipe("arbius test cat", **kw)
    assert a.shape == (5, 64, 64, 3) and (a == b).all()
    assert not (a == pipe("arbius test cat", **{**kw, "seed": 4})).all()


def test_temporal_ops_reference_semantics():
    """TemporalConv/TemporalTransformer mix information across frames only."""
    from arbius_amd.models.layers import init_weights
    from arbius_amd.models.unet3d import TemporalConv
    tc = init_weights(torch.nn.ModuleDict({"t": TemporalConv(64, 8, 1e-5)}), 0)["t"].eval()
    x = torch.randn(2 * 4, 3, 3, 64)
    y = tc(x, frames=4)
    x2 = x.clone()
    x2[4:] += 1.0                      # perturb the second video only
    y2 = tc(x2, frames=4)
    assert torch.allclose(y[:4], y2[:4]) and not torch.allclose(y[4:], y2[4:])


def test_damo_tiny_through_node():
    e, tok, mid = make_world("damo")
    pool = LocalSolverPool("cpu", tiny=True)
    m = make_miner(e, mid, pool, model="damo")
    inp = {"prompt": "arbius test cat", "num_frames": 3, "num_inference_steps": 2, "fps": 8}
    tid = asyncio.run(_full_cycle(e, mid, m, inp))
    model = m.models[mid.lower()]
    row = json.loads(m.db.get_task_input(tid, e.tasks[tid].cid)["data"])
    sol = pool.solve_sync(model, tid, row)
    assert sol.files[0][0] == "out-1.mp4" and sol.cid == e.solutions[tid].cid


# ------------------------------------------------------------------------------------ CAVLC intra codec
def _test_picture(H=64, W=96, seed=0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W]
    y = ((xx * 2 + yy + 10 * np.sin(xx / 5.0)) % 256).astype(np.uint8)
    y[H // 3:H // 3 + 20, W // 3:W // 3 + 30] = rng.integers(0, 256, (20, 30))
    cb = ((xx[::2, ::2] + 100) % 256).astype(np.uint8)
    cr = ((yy[::2, ::2] * 3 + 50) % 256).astype(np.uint8)
    cr[:8, :8] = rng.integers(0, 256, (8, 8))
    return y, cb, cr


def test_h264_vlc_tables_prefix_free():
    from arbius_amd import native
    assert native.h264_tables_ok()


def test_h264_parameter_sets_python_equals_native():
    from arbius_amd import native
    for w, h, qp in ((1920, 1080, 20), (96, 64, 26), (100, 50, 40)):
        assert sps_pps(w, h, qp) == tuple(native.h264_parameter_sets(w, h, qp))


def test_h264_intra_recon_is_decoder_output_every_qp():
    from arbius_amd import native
    y, cb, cr = _test_picture()
    psnr, size = [], []
    for qp in (4, 10, 20, 28, 36, 44, 51):     # (below ~4 Baseline level escapes clamp |level|)
        nal, ry, rcb, rcr = native.h264_encode_yuv(y, cb, cr, qp, 1)
        assert nal[0] == 0x65
        sps, pps = native.h264_parameter_sets(96, 64, qp)
        (dy, dcb, dcr, crop), = native.h264_decode([sps, pps, nal])
        assert crop == (96, 64)
        assert (dy == ry).all() and (dcb == rcb).all() and (dcr == rcr).all()
        mse = np.mean((ry.astype(float) - y) ** 2)
        psnr.append(10 * np.log10(255 ** 2 / max(mse, 1e-6)))
        size.append(len(nal))
    assert all(a > b for a, b in zip(psnr, psnr[1:])) and psnr[0] > 50 and psnr[2] > 40
    assert all(a > b for a, b in zip(size, size[1:]))


def test_h264_multi_slice_and_pcm_decode():
    """I_PCM pictures (round-1 outputs) still decode losslessly through the native decoder."""
    from arbius_amd.utils.mp4 import decode_h264, read_mp4_nals
    rng = np.random.default_rng(5)
    frames = [rng.integers(0, 256, (40, 72, 3), dtype=np.uint8) for _ in range(3)]
    fps, nals, (W, H) = read_mp4_nals(encode_mp4(frames, 7, codec="pcm"))
    planes, crop = decode_h264(nals)
    assert fps == 7 and crop == (72, 40) and (W, H) == (72, 40)
    for f, (y, cb, cr) in zip(frames, planes):
        ey, ecb, ecr = rgb_to_yuv420(np.pad(f, ((0, 8), (0, 8), (0, 0)), mode="edge"))
        assert (y == ey).all() and (cb == ecb).all() and (cr == ecr).all()


def test_mp4_avc_ippp_roundtrip():
    """The IPPP codec (deblocked, row-band slices) through the MP4 container: sync samples listed in
    stss, probe + decode accept it, and the picture is close to the intra one."""
    from arbius_amd.utils.mp4 import GOP, read_mp4_nals
    from arbius_amd.utils.video_io import decode, probe
    yy, xx = np.mgrid[0:90, 0:160]
    frames = [np.stack([(xx + 3 * t) % 256, (yy * 2 + t) % 256, ((xx + yy) // 2) % 256], -1).astype(np.uint8)
              for t in range(GOP + 5)]
    a = encode_mp4(frames, 12, codec="avc")
    assert a == encode_mp4(frames, 12, codec="avc", threads=1)
    assert b"stss" in a and b"AVC IPPP" in a
    intra = encode_mp4(frames, 12)
    assert len(a) < 0.6 * len(intra)
    _, nals, _ = read_mp4_nals(a)
    assert {n[0] & 0x1F for n in nals[2:]} == {1, 5}
    probe(a)
    dec, fps = decode(a)
    ref, _ = decode(encode_mp4(frames, 12, codec="pcm"))
    assert fps == 12 and dec.shape == (GOP + 5, 90, 160, 3)
    assert 10 * np.log10(255 ** 2 / np.mean((dec.astype(float) - ref) ** 2)) > 36


def test_mp4_avc_intra_roundtrip_small_and_deterministic():
    from arbius_amd.utils.video_io import decode, probe
    yy, xx = np.mgrid[0:90, 0:160]
    frames = [np.stack([(xx + 3 * t) % 256, (yy * 2 + t) % 256, ((xx + yy) // 2) % 256], -1).astype(np.uint8)
              for t in range(6)]
    a = encode_mp4(frames, 12, codec="avc-intra")
    assert a == encode_mp4(frames, 12, codec="avc-intra", threads=1)   # thread count never changes bytes
    pcm = encode_mp4(frames, 12, codec="pcm")
    assert len(pcm) > 10 * len(a)
    probe(a)
    probe(pcm)
    dec, fps = decode(a)
    ref, _ = decode(pcm)                                  # lossless YCbCr -> RGB of the same frames
    assert fps == 12 and dec.shape == (6, 90, 160, 3)
    mse = np.mean((dec.astype(float) - ref) ** 2)
    assert 10 * np.log10(255 ** 2 / mse) > 38


def test_probe_rejects_streams_outside_the_decoder_subset():
    import pytest
    from arbius_amd.utils.mp4 import _Bits, _ep
    from arbius_amd.utils.video_io import UndecodableVideo, decode, probe
    sps, pps = sps_pps(64, 64)
    hdr = _Bits()
    hdr.ue(0); hdr.ue(6); hdr.ue(0); hdr.u(4, 1)          # first_mb 0, slice_type B
    hdr.trailing()
    b_slice = b"\x41" + _ep(hdr.bytes())
    stream = b"".join(b"\x00\x00\x00\x01" + n for n in (sps, pps, b_slice))
    with pytest.raises(UndecodableVideo, match="B / SP / SI"):
        probe(stream)
    with pytest.raises(UndecodableVideo):
        decode(stream)
    cabac = _Bits()
    cabac.ue(0); cabac.ue(0); cabac.u(1, 1)               # entropy_coding_mode_flag = 1
    cabac.trailing()
    idr = encode_mp4([np.zeros((64, 64, 3), np.uint8)], 1)
    from arbius_amd.utils.mp4 import read_mp4_nals
    _, nals, _ = read_mp4_nals(idr)
    bad = b"".join(b"\x00\x00\x01" + n for n in (nals[0], b"\x68" + _ep(cabac.bytes()), nals[2]))
    with pytest.raises(UndecodableVideo, match="CABAC"):
        probe(bad)
    with pytest.raises(UndecodableVideo):
        probe(b"not a video at all")
    good = b"".join(b"\x00\x00\x00\x01" + n for n in nals)   # Annex-B of our own stream
    probe(good)
    assert decode(good)[0].shape == (1, 64, 64, 3)


def test_undecodable_video_input_is_skipped_not_invalid():
    """A task whose input_video this node cannot decode is skipped at hydration (metric), never
    stored invalid (which would make the node contest a task other miners can solve)."""
    import base64
    from test_node_e2e import submit
    e, tok, mid = make_world("robust_video_matting")
    pool = LocalSolverPool("cpu", tiny=True)
    m = make_miner(e, mid, pool, model="robust_video_matting")
    src = "data:video/mp4;base64," + base64.b64encode(b"\x00\x00\x00\x01\x41garbage").decode()

    async def go():
        await m.boot()
        await m.poll_events()
        await m.drain()
        tid = submit(e, mid, {"input_video": src, "output_type": "alpha-mask"})
        await m.poll_events()
        await m.drain()
        return tid
    tid = asyncio.run(go())
    assert tid not in e.solutions
    assert m.metrics.counters.get("tasks_undecodable_input", 0) == 1
    assert not m.db.get_invalid_task(tid)


# ---- Intra_4x4 decode path, independent of the native encoder: an I_PCM macroblock with random
# samples followed by I_NxN macroblocks with zero residual (cbp 0), so every decoded sample is a
# chain of 4x4 predictions (all 9 modes, top-right substitution, predicted-mode signalling)
def _p4(top, left, tl, mode):
    """Intra_4x4 prediction (H.264 8.3.1.2) from p[-1,-1] = tl, p[0..7,-1] = top, p[-1,0..3] = left."""
    def P(x, y):
        if y == -1:
            return tl if x == -1 else top[x]
        return left[y]
    out = np.zeros((4, 4), np.int64)
    for y in range(4):
        for x in range(4):
            if mode == 0:
                v = P(x, -1)
            elif mode == 1:
                v = P(-1, y)
            elif mode == 2:
                v = None
            elif mode == 3:
                v = (P(6, -1) + 3 * P(7, -1) + 2) >> 2 if x == y == 3 else \
                    (P(x + y, -1) + 2 * P(x + y + 1, -1) + P(x + y + 2, -1) + 2) >> 2
            elif mode == 4:
                if x > y:
                    v = (P(x - y - 2, -1) + 2 * P(x - y - 1, -1) + P(x - y, -1) + 2) >> 2
                elif x < y:
                    v = (P(-1, y - x - 2) + 2 * P(-1, y - x - 1) + P(-1, y - x) + 2) >> 2
                else:
                    v = (P(0, -1) + 2 * P(-1, -1) + P(-1, 0) + 2) >> 2
            elif mode == 5:
                z = 2 * x - y
                if z in (0, 2, 4, 6):
                    v = (P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 1) >> 1
                elif z in (1, 3, 5):
                    v = (P(x - (y >> 1) - 2, -1) + 2 * P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 2) >> 2
                elif z == -1:
                    v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2
                else:
                    v = (P(-1, y - 1) + 2 * P(-1, y - 2) + P(-1, y - 3) + 2) >> 2
            elif mode == 6:
                z = 2 * y - x
                if z in (0, 2, 4, 6):
                    v = (P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 1) >> 1
                elif z in (1, 3, 5):
                    v = (P(-1, y - (x >> 1) - 2) + 2 * P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 2) >> 2
                elif z == -1:
                    v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2
                else:
                    v = (P(x - 1, -1) + 2 * P(x - 2, -1) + P(x - 3, -1) + 2) >> 2
            elif mode == 7:
                v = (P(x + (y >> 1), -1) + P(x + (y >> 1) + 1, -1) + 1) >> 1 if y % 2 == 0 else \
                    (P(x + (y >> 1), -1) + 2 * P(x + (y >> 1) + 1, -1) + P(x + (y >> 1) + 2, -1) + 2) >> 2
            else:
                z = x + 2 * y
                if z in (0, 2, 4):
                    v = (P(-1, y + (x >> 1)) + P(-1, y + (x >> 1) + 1) + 1) >> 1
                elif z in (1, 3):
                    v = (P(-1, y + (x >> 1)) + 2 * P(-1, y + (x >> 1) + 1) + P(-1, y + (x >> 1) + 2) + 2) >> 2
                elif z == 5:
                    v = (P(-1, 2) + 3 * P(-1, 3) + 2) >> 2
                else:
                    v = P(-1, 3)
            out[y, x] = v if v is not None else 0
    return out


def test_intra4x4_decode_matches_independent_prediction_chain():
    from arbius_amd.utils.mp4 import _Bits, _ep, decode_h264
    rng = np.random.default_rng(9)
    W = H = 32
    Y = np.zeros((H, W), np.int64)
    Cb = np.zeros((H // 2, W // 2), np.int64)
    Cr = np.zeros((H // 2, W // 2), np.int64)
    pcm_y = rng.integers(1, 255, (16, 16))
    pcm_c = rng.integers(1, 255, (2, 8, 8))
    blk_xy = [(0, 0), (1, 0), (0, 1), (1, 1), (2, 0), (3, 0), (2, 1), (3, 1),
              (0, 2), (1, 2), (0, 3), (1, 3), (2, 2), (3, 2), (2, 3), (3, 3)]
    modes = {}                      # (bx, by) in 4x4-block units -> mode (I_NxN macroblocks only)
    bits = _Bits()
    bits.ue(0); bits.ue(7); bits.ue(0); bits.u(4, 0); bits.ue(0); bits.u(1, 0); bits.u(1, 0)
    bits.se(0); bits.ue(1)          # slice header: qp delta 0, deblocking off
    used = set()
    for mb in range(4):
        mx, my = mb % 2, mb // 2
        if mb == 0:
            bits.ue(25)
            bits.align_zero()
            for v in pcm_y.ravel():
                bits.u(8, int(v))
            for c in range(2):
                for v in pcm_c[c].ravel():
                    bits.u(8, int(v))
            Y[:16, :16] = pcm_y
            Cb[:8, :8], Cr[:8, :8] = pcm_c
            continue
        bits.ue(0)                  # I_NxN
        for k, (lx, ly) in enumerate(blk_xy):
            bx, by = 4 * mx + lx, 4 * my + ly
            x0, y0 = 4 * bx, 4 * by
            has_l = bx > 0
            has_t = by > 0
            has_tl = has_l and has_t
            if ly == 0:
                has_tr = by > 0 and bx + 1 < 8 and (lx < 3 or mx + 1 < 2)
            elif lx == 3:
                has_tr = False
            else:
                has_tr = blk_xy.index((lx + 1, ly - 1)) < k
            ok = [m for m in range(9) if not ((m in (0, 3, 7) and not has_t) or (m in (1, 8) and not has_l)
                                               or (m in (4, 5, 6) and not has_tl))]
            m = ok[(3 * mb + k) % len(ok)]
            used.add(m)
            if has_l and has_t:
                ma, mbm = modes.get((bx - 1, by), 2), modes.get((bx, by - 1), 2)
                pred = min(ma, mbm)
            else:
                pred = 2
            if m == pred:
                bits.u(1, 1)
            else:
                bits.u(1, 0)
                bits.u(3, m if m < pred else m - 1)
            modes[(bx, by)] = m
            top = [int(Y[y0 - 1, x0 + i]) if has_t else 0 for i in range(4)]
            top += [int(Y[y0 - 1, x0 + i]) if has_tr else top[3] for i in range(4, 8)]
            left = [int(Y[y0 + i, x0 - 1]) if has_l else 0 for i in range(4)]
            tl = int(Y[y0 - 1, x0 - 1]) if has_tl else 0
            if m == 2:
                s = (sum(top[:4]) if has_t else 0) + (sum(left) if has_l else 0)
                n = 4 * (has_t + has_l)
                dc = (s + n // 2) // n if n else 128
                Y[y0:y0 + 4, x0:x0 + 4] = dc
            else:
                Y[y0:y0 + 4, x0:x0 + 4] = _p4(top, left, tl, m)
        bits.ue(0)                  # intra_chroma_pred_mode DC
        bits.ue(3)                  # coded_block_pattern me(v): codeNum 3 -> cbp 0 (no mb_qp_delta)
        for C in (Cb, Cr):          # chroma DC prediction (8.3.4, 4:2:0), no residual
            cx, cy = 8 * mx, 8 * my
            for by4 in range(2):
                for bx4 in range(2):
                    t = C[cy - 1, cx + 4 * bx4:cx + 4 * bx4 + 4].sum() if my else None
                    l_ = C[cy + 4 * by4:cy + 4 * by4 + 4, cx - 1].sum() if mx else None
                    if (bx4, by4) in ((0, 0), (1, 1)):
                        v = (t + l_ + 4) >> 3 if t is not None and l_ is not None else \
                            (l_ + 2) >> 2 if l_ is not None else (t + 2) >> 2 if t is not None else 128
                    elif (bx4, by4) == (1, 0):
                        v = (t + 2) >> 2 if t is not None else (l_ + 2) >> 2 if l_ is not None else 128
                    else:
                        v = (l_ + 2) >> 2 if l_ is not None else (t + 2) >> 2 if t is not None else 128
                    C[cy + 4 * by4:cy + 4 * by4 + 4, cx + 4 * bx4:cx + 4 * bx4 + 4] = v
    bits.trailing()
    assert used == set(range(9))
    sps, pps = sps_pps(W, H)
    nal = bytes([0x65]) + _ep(bits.bytes())
    [(y, cb, cr)], crop = decode_h264([sps, pps, nal])
    assert crop == (W, H)
    assert (y == Y).all() and (cb == Cb).all() and (cr == Cr).all()


def test_decoder_refuses_oversized_pictures():
    """A few bits per macroblock can declare huge pictures: the decoder caps picture size (4K) and
    the total decoded samples before allocating (untrusted input_video)."""
    import pytest
    from arbius_amd import native
    from arbius_amd.utils.mp4 import _Bits, _ep
    s = _Bits()
    s.u(8, 66); s.u(8, 0xC0); s.u(8, 51); s.ue(0); s.ue(0); s.ue(2); s.ue(1); s.u(1, 0)
    s.ue(299); s.ue(10)                    # 4800 x 176: wider than 4096
    s.u(1, 1); s.u(1, 1); s.u(1, 0); s.u(1, 0); s.trailing()
    with pytest.raises(ValueError, match="too large"):
        native.h264_decode([b"\x67" + _ep(s.bytes())])
