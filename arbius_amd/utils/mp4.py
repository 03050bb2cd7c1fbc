"""Deterministic MP4 (H.264) writer / reader for the video models' ``out-1.mp4``
(templates zeroscopev2xl / damo / robust_video_matting, SURVEY.md §2.6(c,d)) and their
``input_video``.

There is no ffmpeg/libx264 in the image and a solution CID must be a pure
function of the frames, so the codec is self-contained and bit-exact:

* colour: RGB -> BT.601 limited-range YCbCr 4:2:0 in integer arithmetic
  (chroma = rounded 2x2 mean of the RGB samples, then the integer matrix);
* bitstream: H.264 Constrained Baseline CAVLC at a fixed QP (``native/src/h264.cpp``; the
  encoder's reconstruction IS every conforming decoder's output):
  - ``codec="avc-intra"`` (default, the output codec of every video template): every picture one
    IDR slice of Intra_16x16 macroblocks, deblocking off, pictures encoded in parallel;
  - ``codec="avc"``: IPPP - an IDR every ``GOP`` pictures, P pictures of P_Skip / P_L0_16x16
    (quarter-sample motion search) / Intra_16x16 macroblocks, in-loop deblocking on, slices of
    ``ROWS_PER_SLICE`` macroblock rows encoded in parallel.  1.7-2x smaller files, but its motion
    search made the RVM task host-bound (1.12 s vs ~0.2 s encode per 1080p 48-frame clip on the
    MI355X box: 6.4k vs 16k clips/h, ``profiles/bench_r3_rvm_ippp.json``), so it is opt-in;
  - ``codec="pcm"``: raw I_PCM macroblocks (round 1; a 48-frame 1080p clip was ~149 MB);
* container: ftyp + moov (faststart) + mdat, fixed zero timestamps, AVCC
  4-byte NAL lengths, avcC with the SPS/PPS.

Odd sizes are padded to whole macroblocks with edge replication and cropped back in the SPS.
"""
from __future__ import annotations

import struct
from typing import List, Sequence, Tuple

import numpy as np

PROFILE_IDC, CONSTRAINT_FLAGS, LEVEL_IDC = 66, 0xC0, 51
# fixed quantiser of the CAVLC intra stream (part of NUMERICS_VERSION: changing it changes CIDs)
INTRA_QP = 20
GOP, ROWS_PER_SLICE = 30, 4
CODECS = ("avc", "avc-intra", "pcm")


class _Bits:
    def __init__(self):
        self.bits: List[int] = []

    def u(self, n: int, v: int):
        self.bits.extend((v >> (n - 1 - i)) & 1 for i in range(n))

    def ue(self, v: int):
        v += 1
        n = v.bit_length()
        self.u(n - 1, 0)
        self.u(n, v)

    def se(self, v: int):
        self.ue(2 * v - 1 if v > 0 else -2 * v)

    def align_zero(self):
        while len(self.bits) % 8:
            self.bits.append(0)

    def trailing(self):
        self.bits.append(1)
        self.align_zero()

    def bytes(self) -> bytes:
        assert len(self.bits) % 8 == 0
        out = bytearray()
        for i in range(0, len(self.bits), 8):
            b = 0
            for bit in self.bits[i:i + 8]:
                b = (b << 1) | bit
            out.append(b)
        return bytes(out)


def _ep(rbsp: bytes) -> bytes:
    """Emulation prevention (insert 0x03 after 00 00 when the next byte is <= 3)."""
    out = bytearray()
    zeros = 0
    for b in rbsp:
        if zeros >= 2 and b <= 3:
            out.append(3)
            zeros = 0
        out.append(b)
        zeros = zeros + 1 if b == 0 else 0
    return bytes(out)


def _nal(ref_idc: int, typ: int, payload: bytes) -> bytes:
    return bytes([(ref_idc << 5) | typ]) + payload


def sps_pps(width: int, height: int, qp: int = 26, max_refs: int = 1) -> Tuple[bytes, bytes]:
    mbw, mbh = (width + 15) // 16, (height + 15) // 16
    s = _Bits()
    s.u(8, PROFILE_IDC); s.u(8, CONSTRAINT_FLAGS); s.u(8, LEVEL_IDC)
    s.ue(0)               # seq_parameter_set_id
    s.ue(0)               # log2_max_frame_num_minus4
    s.ue(2)               # pic_order_cnt_type
    s.ue(max_refs)        # max_num_ref_frames
    s.u(1, 0)             # gaps_in_frame_num_value_allowed_flag
    s.ue(mbw - 1); s.ue(mbh - 1)
    s.u(1, 1)             # frame_mbs_only_flag
    s.u(1, 1)             # direct_8x8_inference_flag
    crop_r, crop_b = (mbw * 16 - width) // 2, (mbh * 16 - height) // 2
    if crop_r or crop_b:
        s.u(1, 1); s.ue(0); s.ue(crop_r); s.ue(0); s.ue(crop_b)
    else:
        s.u(1, 0)
    s.u(1, 0)             # vui_parameters_present_flag
    s.trailing()
    p = _Bits()
    p.ue(0); p.ue(0)      # pps id, sps id
    p.u(1, 0)             # entropy_coding_mode_flag (CAVLC)
    p.u(1, 0)             # bottom_field_pic_order_in_frame_present_flag
    p.ue(0)               # num_slice_groups_minus1
    p.ue(0); p.ue(0)      # num_ref_idx_l0/l1_default_active_minus1
    p.u(1, 0); p.u(2, 0)  # weighted_pred_flag, weighted_bipred_idc
    p.se(qp - 26); p.se(0); p.se(0)   # pic_init_qp/qs_minus26, chroma_qp_index_offset
    p.u(1, 1)             # deblocking_filter_control_present_flag
    p.u(1, 0); p.u(1, 0)  # constrained_intra_pred_flag, redundant_pic_cnt_present_flag
    p.trailing()
    return _nal(3, 7, _ep(s.bytes())), _nal(3, 8, _ep(p.bytes()))


def rgb_to_yuv420(frame: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """uint8 [H, W, 3] (H, W multiples of 16) -> Y [H, W], Cb/Cr [H/2, W/2], BT.601 limited range."""
    f = frame.astype(np.int32)
    r, g, b = f[..., 0], f[..., 1], f[..., 2]
    y = ((66 * r + 129 * g + 25 * b + 128) >> 8) + 16
    H, W = r.shape
    q = f.reshape(H // 2, 2, W // 2, 2, 3).sum(axis=(1, 3))
    r2, g2, b2 = q[..., 0], q[..., 1], q[..., 2]          # 4 x mean
    cb = ((-38 * r2 - 74 * g2 + 112 * b2 + 512) >> 10) + 128
    cr = ((112 * r2 - 94 * g2 - 18 * b2 + 512) >> 10) + 128
    clip = lambda a: np.clip(a, 1, 254).astype(np.uint8)
    return clip(y), clip(cb), clip(cr)


def _pad16(frame: np.ndarray) -> np.ndarray:
    H, W = frame.shape[:2]
    ph, pw = (-H) % 16, (-W) % 16
    if ph or pw:
        frame = np.pad(frame, ((0, ph), (0, pw), (0, 0)), mode="edge")
    return frame


def encode_idr_pcm(frame: np.ndarray, idr_pic_id: int) -> bytes:
    """One RGB frame -> one IDR slice NAL of I_PCM macroblocks."""
    hdr = _Bits()
    hdr.ue(0)             # first_mb_in_slice
    hdr.ue(7)             # slice_type: I (all slices)
    hdr.ue(0)             # pic_parameter_set_id
    hdr.u(4, 0)           # frame_num
    hdr.ue(idr_pic_id & 1)
    hdr.u(1, 0); hdr.u(1, 0)   # no_output_of_prior_pics_flag, long_term_reference_flag
    hdr.se(0)             # slice_qp_delta
    hdr.ue(1)             # disable_deblocking_filter_idc
    hdr.ue(25)            # mb_type I_PCM (first macroblock)
    hdr.align_zero()      # pcm_alignment_zero_bits
    from .. import native
    f16 = _pad16(frame)
    body = native.pcm_slice_body(f16) if native.loaded else pcm_slice_body_py(f16)
    return _nal(3, 5, _ep(hdr.bytes()) + body + b"\x80")


def pcm_slice_body_py(frame: np.ndarray) -> bytes:
    """Macroblock payload of one picture (reference of ``native.pcm_slice_body``):
    MB0 samples, then ``0x0D 0x00`` (ue(25) + 7 alignment zeros) + samples per MB."""
    y, cb, cr = rgb_to_yuv420(frame)
    H, W = y.shape
    mbh, mbw = H // 16, W // 16
    n = mbh * mbw
    body = np.empty((n, 386), dtype=np.uint8)
    body[:, 0], body[:, 1] = 0x0D, 0x00
    body[:, 2:258] = y.reshape(mbh, 16, mbw, 16).transpose(0, 2, 1, 3).reshape(n, 256)
    body[:, 258:322] = cb.reshape(mbh, 8, mbw, 8).transpose(0, 2, 1, 3).reshape(n, 64)
    body[:, 322:386] = cr.reshape(mbh, 8, mbw, 8).transpose(0, 2, 1, 3).reshape(n, 64)
    return body.tobytes()[2:]


# ------------------------------------------------------------------------------------ container
def _box(typ: bytes, *parts: bytes) -> bytes:
    data = b"".join(parts)
    return struct.pack(">I", 8 + len(data)) + typ + data


def _full(typ: bytes, version: int, flags: int, *parts: bytes) -> bytes:
    return _box(typ, struct.pack(">I", (version << 24) | flags), *parts)


_MATRIX = struct.pack(">9I", 0x10000, 0, 0, 0, 0x10000, 0, 0, 0, 0x40000000)


def _moov(width, height, fps, sizes, sps, pps, mdat_offset, pcm=False, sync=None) -> bytes:
    F = len(sizes)
    dur_ms = int(round(F * 1000 / fps))
    mvhd = _full(b"mvhd", 0, 0, struct.pack(">IIII", 0, 0, 1000, dur_ms), struct.pack(">IH", 0x10000, 0x100),
                 b"\0" * 10, _MATRIX, b"\0" * 24, struct.pack(">I", 2))
    tkhd = _full(b"tkhd", 0, 3, struct.pack(">IIIII", 0, 0, 1, 0, dur_ms), b"\0" * 8,
                 struct.pack(">hhhH", 0, 0, 0, 0), _MATRIX, struct.pack(">II", width << 16, height << 16))
    mdhd = _full(b"mdhd", 0, 0, struct.pack(">IIIIHH", 0, 0, fps, F, 0x55C4, 0))
    hdlr = _full(b"hdlr", 0, 0, struct.pack(">I", 0), b"vide", b"\0" * 12, b"VideoHandler\0")
    vmhd = _full(b"vmhd", 0, 1, b"\0" * 8)
    dinf = _box(b"dinf", _full(b"dref", 0, 0, struct.pack(">I", 1), _full(b"url ", 0, 1)))
    avcc = _box(b"avcC", bytes([1, PROFILE_IDC, CONSTRAINT_FLAGS, LEVEL_IDC, 0xFF, 0xE1]),
                struct.pack(">H", len(sps)), sps, b"\x01", struct.pack(">H", len(pps)), pps)
    name = (b"\x0bI_PCM H.264" if pcm else b"\x0fAVC intra CAVLC" if sync is None else
            b"\x0eAVC IPPP CAVLC").ljust(32, b"\0")
    avc1 = _box(b"avc1", b"\0" * 6, struct.pack(">H", 1), b"\0" * 16, struct.pack(">HH", width, height),
                struct.pack(">III", 0x480000, 0x480000, 0), struct.pack(">H", 1), name,
                struct.pack(">Hh", 0x18, -1), avcc)
    stsd = _full(b"stsd", 0, 0, struct.pack(">I", 1), avc1)
    stts = _full(b"stts", 0, 0, struct.pack(">III", 1, F, 1))
    stsc = _full(b"stsc", 0, 0, struct.pack(">IIII", 1, 1, F, 1))
    stsz = _full(b"stsz", 0, 0, struct.pack(">II", 0, F), struct.pack(">%dI" % F, *sizes))
    stco = _full(b"stco", 0, 0, struct.pack(">II", 1, mdat_offset))
    # stss: the sync (IDR) samples; absent = every sample is a sync sample (intra streams)
    stss = [] if sync is None else [_full(b"stss", 0, 0, struct.pack(">I", len(sync)),
                                          struct.pack(">%dI" % len(sync), *[k + 1 for k in sync]))]
    stbl = _box(b"stbl", stsd, stts, *stss, stsc, stsz, stco)
    minf = _box(b"minf", vmhd, dinf, stbl)
    mdia = _box(b"mdia", mdhd, hdlr, minf)
    return _box(b"moov", mvhd, _box(b"trak", tkhd, mdia))


class Yuv420Clip:
    """A clip already converted to the encoder's input: macroblock-padded BT.601 4:2:0 planes
    y [F, H16, W16], cb / cr [F, H16 / 2, W16 / 2] of a ``width`` x ``height`` picture - the samples
    ``rgb_to_yuv420`` / native ``rgb_to_420`` compute from the RGB frames (the GPU converts the video
    models' output before the download: ``ops.rgb_to_yuv420``).  ``encode_mp4`` of it gives the bytes
    of ``encode_mp4`` of the RGB frames."""
    __slots__ = ("y", "cb", "cr", "width", "height", "keep")

    def __init__(self, y: np.ndarray, cb: np.ndarray, cr: np.ndarray, width: int, height: int, keep=None):
        self.y, self.cb, self.cr, self.width, self.height = y, cb, cr, int(width), int(height)
        self.keep = keep          # the pinned host block the planes view (kept alive until the encode)

    def __len__(self):
        return int(self.y.shape[0])


class H264IntraClip:
    """A clip already encoded by the GPU intra encoder (``ops.h264_intra_encode``): every picture's
    slice RBSP in ``buf`` at ``meta[f]`` with ``meta[F + 2 + f]`` bits (the native
    ``h264_nals_from_rbsp`` layout).  ``encode_mp4`` of it adds emulation prevention and muxes: the
    bytes of ``encode_mp4`` of the same 4:2:0 planes (avc-intra at ``qp``)."""
    __slots__ = ("buf", "meta", "width", "height", "qp", "keep")

    def __init__(self, buf: np.ndarray, meta: np.ndarray, width: int, height: int, qp: int, keep=None):
        self.buf, self.meta = buf, np.ascontiguousarray(meta, dtype=np.int64)
        self.width, self.height, self.qp = int(width), int(height), int(qp)
        self.keep = keep          # the pinned host block ``buf`` views

    def __len__(self):
        return (len(self.meta) - 2) // 2


def encode_mp4(frames: Sequence[np.ndarray], fps: int, codec: str = "avc-intra", threads: int = 16,
               nice: int = 0) -> bytes:
    """uint8 RGB frames [H, W, 3] (all the same size), or one uint8 array [F, H, W, 3] (passed to
    the native encoder without a copy), or a ``Yuv420Clip`` (``avc-intra`` only) -> MP4 bytes
    (deterministic).  ``nice`` > 0 runs the intra encode's threads at that lower CPU priority (a
    background tail next to GPU-feeding threads); bytes never depend on it."""
    if isinstance(frames, Yuv420Clip):
        return _encode_mp4_yuv(frames, fps, codec, threads, nice)
    if isinstance(frames, H264IntraClip):
        return _encode_mp4_slices(frames, fps, codec, threads)
    if isinstance(frames, np.ndarray) and frames.ndim == 4:
        if frames.dtype != np.uint8 or frames.shape[3] != 3:
            raise ValueError("encode_mp4: frames must be uint8 [F, H, W, 3]")
        clip = np.ascontiguousarray(frames)
        frames = list(clip)
    else:
        frames = list(frames)
        clip = None
    if not frames:
        raise ValueError("encode_mp4: no frames")
    if codec not in CODECS:
        raise ValueError(f"encode_mp4: codec must be one of {CODECS}")
    H, W = frames[0].shape[:2]
    fps = max(1, int(fps))
    for f in frames:
        if f.shape != (H, W, 3) or f.dtype != np.uint8:
            raise ValueError("encode_mp4: frames must be uint8 [H, W, 3] of one size")
    pcm = codec == "pcm"
    sync = None
    if pcm:
        sps, pps = sps_pps(W, H)
        pics = [[encode_idr_pcm(f, i)] for i, f in enumerate(frames)]
    else:
        from .. import native
        if not native.loaded:
            raise RuntimeError("encode_mp4: the native runtime (H.264 encoder) is not built; "
                               "run python -m arbius_amd.native.build")
        sps, pps = sps_pps(W, H, INTRA_QP)
        clip = np.stack(frames) if clip is None else clip
        if codec == "avc":
            _, _, pics = native.h264_encode_rgb_stream(clip, INTRA_QP, GOP, threads, ROWS_PER_SLICE)
            sync = list(range(0, len(frames), GOP))
        else:
            _, _, nals = native.h264_encode_rgb(clip, INTRA_QP, threads, nice)
            pics = [[n] for n in nals]
    return _mux(W, H, fps, sps, pps, pics, pcm, sync)


def _encode_mp4_yuv(clip: "Yuv420Clip", fps: int, codec: str, threads: int, nice: int) -> bytes:
    if codec != "avc-intra":
        raise ValueError("encode_mp4: a Yuv420Clip encodes as avc-intra only")
    if len(clip) < 1:
        raise ValueError("encode_mp4: no frames")
    from .. import native
    if not native.loaded:
        raise RuntimeError("encode_mp4: the native runtime (H.264 encoder) is not built; "
                           "run python -m arbius_amd.native.build")
    W, H = clip.width, clip.height
    sps, pps = sps_pps(W, H, INTRA_QP)
    _, _, nals = native.h264_encode_yuv420_frames(clip.y, clip.cb, clip.cr, W, H, INTRA_QP, threads, nice)
    return _mux(W, H, max(1, int(fps)), sps, pps, [[n] for n in nals], False, None)


def _encode_mp4_slices(clip: "H264IntraClip", fps: int, codec: str, threads: int) -> bytes:
    if codec != "avc-intra" or clip.qp != INTRA_QP:
        raise ValueError("encode_mp4: an H264IntraClip is avc-intra at INTRA_QP")
    from .. import native
    if not native.loaded:
        raise RuntimeError("encode_mp4: the native runtime is not built; run python -m arbius_amd.native.build")
    F = len(clip)
    if F < 1:
        raise ValueError("encode_mp4: no frames")
    nals = native.h264_nals_from_rbsp(np.ascontiguousarray(clip.buf, dtype=np.uint8).reshape(-1), clip.meta, F,
                                      max(1, min(int(threads), 4)))
    sps, pps = sps_pps(clip.width, clip.height, INTRA_QP)
    return _mux(clip.width, clip.height, max(1, int(fps)), sps, pps, [[n] for n in nals], False, None)


def _mux(W, H, fps, sps, pps, pics, pcm, sync) -> bytes:
    samples = [b"".join(struct.pack(">I", len(n)) + n for n in p) for p in pics]
    sizes = [len(s) for s in samples]
    ftyp = _box(b"ftyp", b"isom", struct.pack(">I", 512), b"isomiso2avc1mp41")
    moov_len = len(_moov(W, H, fps, sizes, sps, pps, 0, pcm, sync))
    mdat_payload = sum(sizes)
    offset = len(ftyp) + moov_len + 8
    moov = _moov(W, H, fps, sizes, sps, pps, offset, pcm, sync)
    if 8 + mdat_payload > 0xFFFFFFFF:
        raise ValueError("encode_mp4: output above 4 GiB")
    return ftyp + moov + struct.pack(">I", 8 + mdat_payload) + b"mdat" + b"".join(samples)


# ------------------------------------------------------------------------------------ readers
def _boxes(data: bytes, start: int = 0, end: int = None):
    end = len(data) if end is None else end
    i = start
    while i < end:
        size, typ = struct.unpack(">I4s", data[i:i + 8])
        yield typ, i + 8, i + size
        i += size


def read_mp4_pcm(data: bytes, with_size: bool = False):
    """Parse an MP4 written by ``encode_mp4`` back into (fps, [(Y, Cb, Cr)]) (+ (W, H))."""
    top = {t: (a, b) for t, a, b in _boxes(data)}
    ma, mb = top[b"moov"]

    def find(path, a, b):
        for t, x, y in _boxes(data, a, b):
            if t == path[0]:
                if len(path) == 1:
                    return x, y
                skip = {b"stsd": 8, b"avc1": 78, b"dref": 8}.get(path[0], 0)
                return find(path[1:], x + skip, y)
        raise KeyError(path)

    ha, hb = find([b"trak", b"mdia", b"mdhd"], ma, mb)
    fps = struct.unpack(">I", data[ha + 12:ha + 16])[0]
    sa, sb = find([b"trak", b"mdia", b"minf", b"stbl", b"stsz"], ma, mb)
    n = struct.unpack(">I", data[sa + 8:sa + 12])[0]
    sizes = struct.unpack(">%dI" % n, data[sa + 12:sa + 12 + 4 * n])
    ca, cb = find([b"trak", b"mdia", b"minf", b"stbl", b"stco"], ma, mb)
    off = struct.unpack(">I", data[ca + 8:ca + 12])[0]
    va, vb = find([b"trak", b"mdia", b"minf", b"stbl", b"stsd", b"avc1"], ma, mb)
    W, H = struct.unpack(">HH", data[va + 24:va + 28])
    W16, H16 = (W + 15) // 16 * 16, (H + 15) // 16 * 16
    mbw, mbh = W16 // 16, H16 // 16
    out = []
    for s in sizes:
        nal = data[off + 4:off + s]
        off += s
        assert nal[0] & 0x1F == 5
        nmb = mbw * mbh
        body = np.frombuffer(nal[len(nal) - 1 - (nmb * 386 - 2):len(nal) - 1], dtype=np.uint8)
        body = np.concatenate([np.zeros(2, np.uint8), body]).reshape(nmb, 386)
        y = body[:, 2:258].reshape(mbh, mbw, 16, 16).transpose(0, 2, 1, 3).reshape(H16, W16)
        cbp = body[:, 258:322].reshape(mbh, mbw, 8, 8).transpose(0, 2, 1, 3).reshape(H16 // 2, W16 // 2)
        crp = body[:, 322:386].reshape(mbh, mbw, 8, 8).transpose(0, 2, 1, 3).reshape(H16 // 2, W16 // 2)
        out.append((y, cbp, crp))
    return (fps, out, (W, H)) if with_size else (fps, out)


def read_mp4_nals(data: bytes):
    """Demux an MP4 with one avc1 track: (fps, [NAL bytes] = SPS, PPS, one slice NAL per sample
    (4-byte AVCC lengths; every NAL of a sample), (W, H)).  Raises ValueError on other layouts."""
    try:
        top = {t: (a, b) for t, a, b in _boxes(data)}
        ma, mb = top[b"moov"]

        def find(path, a, b):
            for t, x, y in _boxes(data, a, b):
                if t == path[0]:
                    if len(path) == 1:
                        return x, y
                    skip = {b"stsd": 8, b"avc1": 78, b"dref": 8}.get(path[0], 0)
                    return find(path[1:], x + skip, y)
            raise KeyError(path)

        stbl = [b"trak", b"mdia", b"minf", b"stbl"]
        ha, _ = find([b"trak", b"mdia", b"mdhd"], ma, mb)
        ver = data[ha]
        ts_off = ha + (20 if ver == 1 else 12)
        timescale = struct.unpack(">I", data[ts_off:ts_off + 4])[0]
        dur = (struct.unpack(">Q", data[ts_off + 4:ts_off + 12])[0] if ver == 1
               else struct.unpack(">I", data[ts_off + 4:ts_off + 8])[0])
        sa, _ = find(stbl + [b"stsz"], ma, mb)
        const, n = struct.unpack(">II", data[sa + 4:sa + 12])
        sizes = [const] * n if const else list(struct.unpack(">%dI" % n, data[sa + 12:sa + 12 + 4 * n]))
        # chunk offsets (stco / co64) and samples-per-chunk runs (stsc)
        try:
            ca, _ = find(stbl + [b"stco"], ma, mb)
            nc = struct.unpack(">I", data[ca + 4:ca + 8])[0]
            chunks = list(struct.unpack(">%dI" % nc, data[ca + 8:ca + 8 + 4 * nc]))
        except KeyError:
            ca, _ = find(stbl + [b"co64"], ma, mb)
            nc = struct.unpack(">I", data[ca + 4:ca + 8])[0]
            chunks = list(struct.unpack(">%dQ" % nc, data[ca + 8:ca + 8 + 8 * nc]))
        xa, _ = find(stbl + [b"stsc"], ma, mb)
        ne = struct.unpack(">I", data[xa + 4:xa + 8])[0]
        runs = [struct.unpack(">III", data[xa + 8 + 12 * i:xa + 20 + 12 * i]) for i in range(ne)]
        va, vb = find(stbl + [b"stsd", b"avc1"], ma, mb)
        W, H = struct.unpack(">HH", data[va + 24:va + 28])
        ca_, _ = find([b"avcC"], va + 78, vb)
        cfg = data[ca_:]
        nsps = cfg[5] & 0x1F
        i = 6
        ps = []
        for _ in range(nsps):
            ln = struct.unpack(">H", cfg[i:i + 2])[0]
            ps.append(bytes(cfg[i + 2:i + 2 + ln]))
            i += 2 + ln
        npps = cfg[i]
        i += 1
        for _ in range(npps):
            ln = struct.unpack(">H", cfg[i:i + 2])[0]
            ps.append(bytes(cfg[i + 2:i + 2 + ln]))
            i += 2 + ln
        nal_len = (cfg[4] & 3) + 1
        nals = list(ps)
        s = 0
        for ci, off in enumerate(chunks):
            per = next(r[1] for r in reversed(runs) if r[0] <= ci + 1)
            for _ in range(per):
                if s >= n:
                    break
                end, p = off + sizes[s], off
                while p < end:
                    ln = int.from_bytes(data[p:p + nal_len], "big")
                    nals.append(bytes(data[p + nal_len:p + nal_len + ln]))
                    p += nal_len + ln
                off = end
                s += 1
        fps = int(round(n * timescale / dur)) if dur else 24
        return max(1, fps), nals, (W, H)
    except (KeyError, struct.error, IndexError, StopIteration) as e:
        raise ValueError(f"not an MP4 with one H.264 (avc1) video track: {e!r}") from None


def annexb_nals(data: bytes) -> List[bytes]:
    """Split an Annex-B byte stream (00 00 01 / 00 00 00 01 start codes) into NAL units."""
    out, i, n = [], 0, len(data)
    starts = []
    while True:
        j = data.find(b"\x00\x00\x01", i)
        if j < 0:
            break
        starts.append(j + 3)
        i = j + 3
    for k, st in enumerate(starts):
        end = starts[k + 1] - 3 if k + 1 < len(starts) else n
        nal = data[st:end]
        while nal.endswith(b"\x00"):          # trailing_zero_8bits / next 4-byte start code
            nal = nal[:-1]
        if nal:
            out.append(bytes(nal))
    return out


def _threads() -> int:
    import os
    return max(1, min(16, os.cpu_count() or 1))


def max_video_samples() -> int:
    """Total luma samples one input video may decode to (untrusted input: a few bits per macroblock
    can declare huge videos).  Default 2^30 (~17 s of 1080p30, ~3.2 GB of RGB); operators with
    more host memory raise it with ``$ARBIUS_MAX_VIDEO_SAMPLES``."""
    import os
    return int(os.environ.get("ARBIUS_MAX_VIDEO_SAMPLES", 1 << 30))


def decode_h264_rgb(nals: Sequence[bytes]) -> np.ndarray:
    """NAL units -> uint8 RGB [F, H, W, 3] (cropped), native decoder + integer BT.601 inverse."""
    from .. import native
    if not native.loaded:
        raise RuntimeError("the native runtime (H.264 decoder) is not built")
    return native.h264_decode_rgb(list(nals), _threads(), max_video_samples())


def decode_h264(nals: Sequence[bytes]):
    """NAL units -> [(Y, Cb, Cr)] at macroblock-padded size, plus (crop_w, crop_h), through the
    native intra decoder.  ValueError for streams outside its subset (P/B slices, CABAC, ...)."""
    from .. import native
    if not native.loaded:
        raise RuntimeError("the native runtime (H.264 decoder) is not built")
    pics = native.h264_decode(list(nals), _threads(), False, max_video_samples())
    if not pics:
        raise ValueError("no pictures in the H.264 stream")
    return [(y, cb, cr) for y, cb, cr, _ in pics], pics[0][3]
