"""H.264 P slices + in-loop deblocking: the native IPPP encoder's
reconstruction is the decoder's output (production and randomised decoder-coverage streams), and
the decoder agrees with independent Python implementations of deblocking, motion compensation and
motion-vector prediction (tests/h264_ref.py) on streams built bit by bit here."""
import numpy as np
import pytest

from arbius_amd import native
from arbius_amd.utils.mp4 import _Bits, _ep, rgb_to_yuv420, sps_pps

import h264_ref as ref

pytestmark = pytest.mark.skipif(not native.loaded, reason="native runtime not built")


def _clip(F, H, W, seed=0):
    """Moving textured content (translation + a rotating blob) as 4:2:0 planes."""
    yy, xx = np.mgrid[0:H, 0:W]
    rng = np.random.default_rng(seed)
    noise = rng.integers(0, 24, (H, W))
    frames = []
    for t in range(F):
        r = np.sin((xx + 3 * t) / 7.0) * 80 + 128 + noise
        g = np.cos((yy - 2 * t) / 5.0) * 60 + 128
        b = (xx + yy + 5 * t) % 256
        cx, cy = W / 2 + 10 * np.cos(t / 3), H / 2 + 8 * np.sin(t / 3)
        blob = ((xx - cx) ** 2 + (yy - cy) ** 2) < (min(H, W) / 5) ** 2
        f = np.stack([r, g, b], -1)
        f[blob] = (240, 30, 60)
        frames.append(np.clip(f, 0, 255).astype(np.uint8))
    planes = [rgb_to_yuv420(f) for f in frames]
    return tuple(np.stack(p) for p in zip(*planes)), frames


def _encode(Y, CB, CR, qp, gop, seed=0, refs=1, rows=2):
    pics, ry, rcb, rcr = native.h264_encode_yuv_stream(Y, CB, CR, qp, gop, seed, refs, 4, rows)
    H, W = Y.shape[1:]
    sps, pps = native.h264_parameter_sets(W, H, qp, refs)
    return [sps, pps] + [n for p in pics for n in p], pics, (ry, rcb, rcr)


@pytest.mark.parametrize("seed,refs,qp", [(0, 1, 20), (0, 1, 34), (1, 1, 26), (2, 3, 26), (5, 2, 14), (9, 4, 40)])
def test_recon_is_decoder_output(seed, refs, qp):
    (Y, CB, CR), _ = _clip(9, 48, 80, seed)
    nals, pics, (ry, rcb, rcr) = _encode(Y, CB, CR, qp, 5 if seed else 6, seed, refs)
    dec = native.h264_decode(nals, 3)
    assert len(dec) == 9
    for i, (y, cb, cr, crop) in enumerate(dec):
        assert crop == (80, 48)
        assert (y == ry[i]).all() and (cb == rcb[i]).all() and (cr == rcr[i]).all(), i
    if seed:          # coverage mode really produced the syntax it is meant to cover
        types = {n[0] & 0x1F for p in pics for n in p}
        assert types == {1, 5} and any(len(p) > 1 for p in pics)


def test_ippp_is_smaller_than_intra_at_equal_quality():
    (Y, CB, CR), _ = _clip(12, 64, 96)
    intra = sum(len(native.h264_encode_yuv(Y[i], CB[i], CR[i], 24, i)[0]) for i in range(12))
    nals, _, (ry, _, _) = _encode(Y, CB, CR, 24, 12)
    inter = sum(len(n) for n in nals[2:])
    psnr = 10 * np.log10(255 ** 2 / np.mean((ry.astype(float) - Y) ** 2))
    assert inter < 0.6 * intra and psnr > 36, (inter, intra, psnr)
    # the bytes never depend on the thread count
    again = native.h264_encode_yuv_stream(Y, CB, CR, 24, 12, 0, 1, 1, 2)[0]
    assert [n for p in again for n in p] == nals[2:]


@pytest.mark.parametrize("seed", [3, 4, 11])
def test_deblocking_matches_independent_reference(seed):
    (Y, CB, CR), _ = _clip(6, 48, 64, seed)
    nals, _, _ = _encode(Y, CB, CR, 30, 3, seed, 2)
    dec = native.h264_decode(nals, 2, True)
    filtered = 0
    for y, cb, cr, crop, side in dec:
        ry_, rcb_, rcr_ = ref.deblock(side, 64, 48)
        assert (ry_ == y).all() and (rcb_ == cb).all() and (rcr_ == cr).all()
        filtered += int((side["y"].reshape(48, 64) != y).sum())
        assert {d[0] for d in side["deblock"]} <= {0, 1, 2}
    assert filtered > 100            # the filter actually changed samples


# ---- hand-built streams: I_PCM references, then P pictures of every partition shape with no
# residual and no deblocking, so every decoded sample is a motion-compensated prediction
W, H = 64, 48
MBW, MBH = W // 16, H // 16
SUB_SHAPES = {0: [(0, 0, 2, 2)], 1: [(0, 0, 2, 1), (0, 1, 2, 1)], 2: [(0, 0, 1, 2), (1, 0, 1, 2)],
              3: [(0, 0, 1, 1), (1, 0, 1, 1), (0, 1, 1, 1), (1, 1, 1, 1)]}


def _pcm(bits, rng, Y, Cb, Cr, mx, my):
    bits.align_zero()
    ys = rng.integers(0, 256, (16, 16))
    cs = rng.integers(0, 256, (2, 8, 8))
    for v in ys.ravel():
        bits.u(8, int(v))
    for c in range(2):
        for v in cs[c].ravel():
            bits.u(8, int(v))
    Y[16 * my:16 * my + 16, 16 * mx:16 * mx + 16] = ys
    Cb[8 * my:8 * my + 8, 8 * mx:8 * mx + 8] = cs[0]
    Cr[8 * my:8 * my + 8, 8 * mx:8 * mx + 8] = cs[1]


def _p_picture(rng, frame_num, refs, nref, mmco=None):
    """One P slice NAL + the expected picture.  refs: list of (Y, Cb, Cr) in RefPicList0 order."""
    bits = _Bits()
    bits.ue(0); bits.ue(5); bits.ue(0); bits.u(4, frame_num)
    if nref > 1:
        bits.u(1, 1); bits.ue(nref - 1)
    else:
        bits.u(1, 0)
    bits.u(1, 0)                                     # no list modification
    if mmco:
        bits.u(1, 1)
        for op, v in mmco:
            bits.ue(op); bits.ue(v)
        bits.ue(0)
    else:
        bits.u(1, 0)
    bits.se(0); bits.ue(1)                           # slice_qp_delta, deblocking off
    Y = np.zeros((H, W), np.int64); Cb = np.zeros((H // 2, W // 2), np.int64); Cr = np.zeros_like(Cb)
    field = ref.MotionField(MBW, MBH)
    run = 0
    kinds = []

    def te(r):
        if nref == 2:
            bits.u(1, 1 - r)
        elif nref > 2:
            bits.ue(r)

    def put(x, y, w, h, r, mv):
        py_, pcb, pcr = ref.predict_block(refs[r], 4 * x, 4 * y, 4 * w, 4 * h, mv)
        Y[4 * y:4 * y + 4 * h, 4 * x:4 * x + 4 * w] = py_
        Cb[2 * y:2 * y + 2 * h, 2 * x:2 * x + 2 * w] = pcb
        Cr[2 * y:2 * y + 2 * h, 2 * x:2 * x + 2 * w] = pcr

    for mb in range(MBW * MBH):
        mx, my = mb % MBW, mb // MBW
        bx, by = 4 * mx, 4 * my
        kind = int(rng.integers(0, 7))
        kinds.append(kind)
        dec = set()
        if kind == 0:                                 # P_Skip
            mv = field.skip_mv(mb)
            field.set(bx, by, 4, 4, (0, mv[0], mv[1]), dec)
            put(bx, by, 4, 4, 0, mv)
            run += 1
            continue
        bits.ue(run)
        run = 0
        if kind == 6:                                 # I_PCM inside the P slice
            bits.ue(5 + 25)
            _pcm(bits, rng, Y, Cb, Cr, mx, my)
            field.set(bx, by, 4, 4, "intra", dec)
            continue
        mvd = lambda: (int(rng.integers(-40, 41)), int(rng.integers(-40, 41)))
        if kind <= 3:                                 # 16x16, 16x8, 8x16
            parts = {1: [(0, 0, 4, 4, None)], 2: [(0, 0, 4, 2, "16x8_top"), (0, 2, 4, 2, "16x8_bottom")],
                     3: [(0, 0, 2, 4, "8x16_left"), (2, 0, 2, 4, "8x16_right")]}[kind]
            bits.ue(kind - 1)
            rs = [int(rng.integers(0, nref)) for _ in parts]
            for r in rs:
                te(r)
            for (x, y, w, h, shape), r in zip(parts, rs):
                d = mvd()
                bits.se(d[0]); bits.se(d[1])
                p = field.predict(mb, bx + x, by + y, w, h, r, dec, shape)
                mv = (p[0] + d[0], p[1] + d[1])
                field.set(bx + x, by + y, w, h, (r, mv[0], mv[1]), dec)
                put(bx + x, by + y, w, h, r, mv)
        else:                                         # P_8x8 (kind 4) / P_8x8ref0 (kind 5)
            bits.ue(3 if kind == 4 or nref == 1 else 4)
            subs = [int(rng.integers(0, 4)) for _ in range(4)]
            for t in subs:
                bits.ue(t)
            rs = [int(rng.integers(0, nref)) if (kind == 4 or nref == 1) else 0 for _ in range(4)]
            if kind == 4 or nref == 1:
                for r in rs:
                    te(r)
            for s, (t, r) in enumerate(zip(subs, rs)):
                sx, sy = bx + 2 * (s % 2), by + 2 * (s // 2)
                for (x, y, w, h) in SUB_SHAPES[t]:
                    d = mvd()
                    bits.se(d[0]); bits.se(d[1])
                    p = field.predict(mb, sx + x, sy + y, w, h, r, dec)
                    mv = (p[0] + d[0], p[1] + d[1])
                    field.set(sx + x, sy + y, w, h, (r, mv[0], mv[1]), dec)
                    put(sx + x, sy + y, w, h, r, mv)
        bits.ue(0)                                    # coded_block_pattern 0: no residual
    if run:
        bits.ue(run)
    bits.trailing()
    return bytes([0x41]) + _ep(bits.bytes()), (Y, Cb, Cr), kinds


def test_inter_prediction_matches_independent_reference():
    rng = np.random.default_rng(21)
    sps, pps = sps_pps(W, H, 26, max_refs=2)
    # IDR of I_PCM macroblocks
    bits = _Bits()
    bits.ue(0); bits.ue(7); bits.ue(0); bits.u(4, 0); bits.ue(0); bits.u(1, 0); bits.u(1, 0); bits.se(0); bits.ue(1)
    I = [np.zeros((H, W), np.int64), np.zeros((H // 2, W // 2), np.int64), np.zeros((H // 2, W // 2), np.int64)]
    for mb in range(MBW * MBH):
        bits.ue(25)
        _pcm(bits, rng, *I, mb % MBW, mb // MBW)
    bits.trailing()
    idr = bytes([0x65]) + _ep(bits.bytes())
    # P1 (one reference), P2 (two references, then MMCO 1 drops P1), P3 (two references: P2, IDR)
    p1, P1, k1 = _p_picture(rng, 1, [I], 1)
    p2, P2, k2 = _p_picture(rng, 2, [P1, I], 2, mmco=[(1, 0)])
    p3, P3, k3 = _p_picture(rng, 3, [P2, I], 2)
    assert set(k1 + k2 + k3) == set(range(7))
    dec = native.h264_decode([sps, pps, idr, p1, p2, p3], 1)
    assert len(dec) == 4
    assert (dec[0][0] == I[0]).all()
    for (y, cb, cr, _), (ey, ecb, ecr) in zip(dec[1:], (P1, P2, P3)):
        assert (y == ey).all() and (cb == ecb).all() and (cr == ecr).all()


def test_decoder_refuses_inter_streams_outside_the_subset():
    rng = np.random.default_rng(2)
    sps, pps = sps_pps(W, H, 26)
    bits = _Bits()
    bits.ue(0); bits.ue(7); bits.ue(0); bits.u(4, 0); bits.ue(0); bits.u(1, 0); bits.u(1, 0); bits.se(0); bits.ue(1)
    I = [np.zeros((H, W), np.int64), np.zeros((H // 2, W // 2), np.int64), np.zeros((H // 2, W // 2), np.int64)]
    for mb in range(MBW * MBH):
        bits.ue(25)
        _pcm(bits, rng, *I, mb % MBW, mb // MBW)
    bits.trailing()
    idr = bytes([0x65]) + _ep(bits.bytes())
    p1, _, _ = _p_picture(rng, 1, [I], 1)
    native.h264_decode([sps, pps, idr, p1])
    with pytest.raises(ValueError, match="gap in frame_num"):
        native.h264_decode([sps, pps, idr, _p_picture(rng, 3, [I], 1)[0]])
    with pytest.raises(ValueError, match="ref_idx|reference"):    # ref_idx 1 with one reference picture
        native.h264_decode([sps, pps, idr, _p_picture(np.random.default_rng(5), 1, [I, I], 2)[0]])
    b = _Bits()
    b.ue(0); b.ue(6); b.ue(0); b.u(4, 1); b.trailing()        # B slice
    with pytest.raises(ValueError, match="B"):
        native.h264_decode([sps, pps, idr, bytes([0x41]) + _ep(b.bytes())])
    with pytest.raises(ValueError, match="P slice"):           # P slice inside an IDR picture
        b = _Bits(); b.ue(0); b.ue(5); b.ue(0); b.u(4, 0); b.trailing()
        native.h264_decode([sps, pps, bytes([0x65]) + _ep(b.bytes())])


def test_decode_budget_bounds_total_samples(monkeypatch):
    """The total decoded size is capped before any picture is allocated (untrusted
    input_video), and the cap is an operator knob."""
    from arbius_amd.utils.mp4 import decode_h264_rgb
    (Y, CB, CR), _ = _clip(4, 48, 80)
    nals, _, _ = _encode(Y, CB, CR, 30, 2)
    assert native.h264_decode_rgb(nals, 2).shape == (4, 48, 80, 3)
    with pytest.raises(ValueError, match="too large"):
        native.h264_decode_rgb(nals, 2, 4 * 48 * 80 - 1)
    monkeypatch.setenv("ARBIUS_MAX_VIDEO_SAMPLES", str(3 * 48 * 80))
    with pytest.raises(ValueError, match="too large"):
        decode_h264_rgb(nals)
