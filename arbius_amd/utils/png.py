"""Deterministic PNG encoder (no timestamps, no metadata, fixed zlib level).

Consensus requires byte-identical outputs for identical pixels (SURVEY.md
§7.3.1): every miner must produce the same ``out-1.png`` bytes and therefore
the same directory CID.  Rows use PNG filter 0 (None); the zlib level is fixed.
The IDAT stream is deflated in fixed 128 KiB segments (pigz layout: each segment
primed with the previous 32 KiB, sync-flushed, one Adler-32 over the whole input),
so the native encoder compresses them in parallel; the bytes never depend on the
thread count.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

PNG_SIG = b"\x89PNG\r\n\x1a\n"


def _chunk(tag: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


SEG = 128 * 1024


def zlib_segmented(data: bytes, level: int) -> bytes:
    """Reference of the native segmented zlib stream (native.cpp ``zlib_segmented``)."""
    n = len(data)
    nseg = max(1, -(-n // SEG))
    out = []
    for i in range(nseg):
        off = i * SEG
        dict_ = data[max(0, off - 32768):off]
        co = zlib.compressobj(level, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY, zdict=dict_) if dict_ else \
            zlib.compressobj(level, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY)
        last = i + 1 == nseg
        out.append(co.compress(data[off:off + SEG]) + co.flush(zlib.Z_FINISH if last else zlib.Z_SYNC_FLUSH))
    flevel = 0 if level == 1 else 1 if 0 <= level < 6 else 2 if level in (6, -1) else 3
    hdr = (0x78 << 8) | (flevel << 6)
    hdr |= 31 - hdr % 31
    return struct.pack(">H", hdr) + b"".join(out) + struct.pack(">I", zlib.adler32(data) & 0xFFFFFFFF)


def encode_png(img: np.ndarray, level: int = 6) -> bytes:
    """img: uint8 [H, W, 3] (RGB) or [H, W, 4] (RGBA) or [H, W] (gray).  Native C++
    encoder when built (byte-identical: same zlib, same parameters)."""
    from .. import native
    if native.loaded and isinstance(img, np.ndarray) and img.dtype == np.uint8 and img.ndim in (2, 3):
        return native.png_encode(img, level)
    return encode_png_py(img, level)


def encode_png_py(img: np.ndarray, level: int = 6) -> bytes:
    """Python reference of ``encode_png``."""
    img = np.ascontiguousarray(img)
    if img.dtype != np.uint8:
        raise TypeError("encode_png expects uint8")
    if img.ndim == 2:
        img = img[:, :, None]
    h, w, c = img.shape
    color = {1: 0, 3: 2, 4: 6}[c]
    raw = np.zeros((h, 1 + w * c), dtype=np.uint8)
    raw[:, 1:] = img.reshape(h, w * c)
    ihdr = struct.pack(">IIBBBBB", w, h, 8, color, 0, 0, 0)
    idat = zlib_segmented(raw.tobytes(), level)
    return PNG_SIG + _chunk(b"IHDR", ihdr) + _chunk(b"IDAT", idat) + _chunk(b"IEND", b"")


def decode_png(data: bytes) -> np.ndarray:
    """Decoder for the files this module writes (filter 0, 8-bit)."""
    assert data[:8] == PNG_SIG
    pos, idat = 8, b""
    w = h = c = None
    while pos < len(data):
        (ln,) = struct.unpack(">I", data[pos:pos + 4])
        tag = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + ln]
        pos += 12 + ln
        if tag == b"IHDR":
            w, h, _, color = struct.unpack(">IIBB", body[:10])
            c = {0: 1, 2: 3, 6: 4}[color]
        elif tag == b"IDAT":
            idat += body
    raw = np.frombuffer(zlib.decompress(idat), dtype=np.uint8).reshape(h, 1 + w * c)
    if (raw[:, 0] != 0).any():
        raise ValueError("only filter-0 PNGs supported")
    return raw[:, 1:].reshape(h, w, c)
