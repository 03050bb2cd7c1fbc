"""Video input for the matting template (``input_video`` is a ``file`` variable:
a URL / IPFS reference to a video, ``templates/robust_video_matting.json:6``).

Sources: local path, ``http(s)://`` URL, ``ipfs://CID`` / bare CID (fetched from
``$ARBIUS_IPFS_GATEWAY``, default the local kubo gateway), ``data:`` URI.
Containers: MP4 written by ``utils/mp4.py`` (H.264 I_PCM, decoded natively and
exactly), ``.npy`` uint8 [T, H, W, 3] (``allow_pickle=False``); anything else is
decoded by an ``ffmpeg`` binary when one is on PATH (the image ships none -
then the task fails loudly instead of guessing).
"""
from __future__ import annotations

import base64
import io
import os
import shutil
import subprocess
import tempfile
from typing import Tuple

import numpy as np


def fetch(ref: str) -> bytes:
    if ref.startswith("data:"):
        return base64.b64decode(ref.split(",", 1)[1])
    if ref.startswith(("http://", "https://")):
        import httpx
        r = httpx.get(ref, timeout=120.0, follow_redirects=True)
        r.raise_for_status()
        return r.content
    if ref.startswith("ipfs://") or (ref.startswith("Qm") and len(ref) == 46):
        import httpx
        gw = os.environ.get("ARBIUS_IPFS_GATEWAY", "http://127.0.0.1:8080")
        r = httpx.get(f"{gw.rstrip('/')}/ipfs/{ref.replace('ipfs://', '')}", timeout=120.0)
        r.raise_for_status()
        return r.content
    with open(ref, "rb") as f:
        return f.read()


def yuv420_to_rgb(y, cb, cr, H, W) -> np.ndarray:
    """BT.601 limited range -> uint8 RGB (integer arithmetic, inverse of mp4.rgb_to_yuv420)."""
    c = y[:H, :W].astype(np.int32) - 16
    d = np.repeat(np.repeat(cb, 2, 0), 2, 1)[:H, :W].astype(np.int32) - 128
    e = np.repeat(np.repeat(cr, 2, 0), 2, 1)[:H, :W].astype(np.int32) - 128
    r = (298 * c + 409 * e + 128) >> 8
    g = (298 * c - 100 * d - 208 * e + 128) >> 8
    b = (298 * c + 516 * d + 128) >> 8
    return np.clip(np.stack([r, g, b], -1), 0, 255).astype(np.uint8)


def decode(data: bytes) -> Tuple[np.ndarray, int]:
    if data[:6] == b"\x93NUMPY":
        arr = np.load(io.BytesIO(data), allow_pickle=False)
        return arr.astype(np.uint8), 24
    if data[4:8] == b"ftyp":
        try:
            from .mp4 import read_mp4_pcm
            fps, planes, (W, H) = read_mp4_pcm(data, with_size=True)
            return np.stack([yuv420_to_rgb(y, cb, cr, H, W) for y, cb, cr in planes]), fps
        except Exception:  # noqa: BLE001 - not our I_PCM layout: external decoder
            pass
    ff = shutil.which("ffmpeg")
    if ff is None:
        raise RuntimeError("input video is not an I_PCM MP4 / .npy and no ffmpeg binary is available to decode it")
    with tempfile.NamedTemporaryFile(suffix=".mp4") as f:
        f.write(data)
        f.flush()
        probe = subprocess.run([ff, "-i", f.name], capture_output=True, text=True)
        import re
        m = re.search(r"(\d+)x(\d+)[, ].*?(\d+(?:\.\d+)?) fps", probe.stderr)
        if not m:
            raise RuntimeError("ffmpeg could not probe the input video")
        W, H, fps = int(m.group(1)), int(m.group(2)), float(m.group(3))
        raw = subprocess.run([ff, "-v", "error", "-i", f.name, "-f", "rawvideo", "-pix_fmt", "rgb24", "-"],
                             capture_output=True, check=True).stdout
    return np.frombuffer(raw, np.uint8).reshape(-1, H, W, 3), int(round(fps))


def load_video(ref: str) -> Tuple[np.ndarray, int]:
    return decode(fetch(ref))
