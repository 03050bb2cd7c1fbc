"""Video input for the matting template (``input_video`` is a ``file`` variable:
a URL / IPFS reference to a video, ``templates/robust_video_matting.json:6``).

``input_video`` is UNTRUSTED task input from the chain, so ``fetch`` only accepts:

* ``ipfs://<cid>`` or a bare CID - fetched from the operator's configured gateway
  (``$ARBIUS_IPFS_GATEWAY``, default the local kubo gateway);
* ``https://`` URLs whose host resolves ONLY to public unicast addresses (no loopback,
  private, link-local / cloud-metadata, CGNAT, multicast or reserved ranges - no SSRF against
  the control RPC, the kubo API or instance metadata); optionally restricted to an allow-list
  (``$ARBIUS_VIDEO_HOSTS``, comma separated).  Redirects are followed by hand, each hop checked;
* ``data:`` URIs (self-contained).
Local paths, ``file://`` and plain ``http://`` are refused (``VideoSourceError``), and every
download is capped at ``MAX_VIDEO_BYTES``.

Containers: MP4 written by ``utils/mp4.py`` (H.264 I_PCM, decoded natively and
exactly), ``.npy`` uint8 [T, H, W, 3] (``allow_pickle=False``); anything else is
decoded by an ``ffmpeg`` binary when one is on PATH (the image ships none -
then the task fails loudly instead of guessing).
"""
from __future__ import annotations

import base64
import io
import os
import re
import shutil
import subprocess
import tempfile
from typing import Tuple

import numpy as np


MAX_VIDEO_BYTES = 512 << 20
_CID = re.compile(r"^(Qm[1-9A-HJ-NP-Za-km-z]{44}|b[a-z2-7]{20,})(/[A-Za-z0-9._\-/]*)?$")


class VideoSourceError(ValueError):
    """``input_video`` names a source this node refuses to read (local file, private address...)."""


def _public_host(host: str) -> bool:
    """True when every address ``host`` resolves to is public unicast."""
    import ipaddress
    import socket
    try:
        infos = socket.getaddrinfo(host, 443, proto=socket.IPPROTO_TCP)
    except OSError:
        return False
    if not infos:
        return False
    for info in infos:
        ip = ipaddress.ip_address(info[4][0].split("%")[0])
        if getattr(ip, "ipv4_mapped", None):
            ip = ip.ipv4_mapped
        if (ip.is_private or ip.is_loopback or ip.is_link_local or ip.is_multicast or ip.is_reserved
                or ip.is_unspecified or not ip.is_global):
            return False
    return True


def check_source(ref: str) -> str:
    """Classify an ``input_video`` reference: 'ipfs' | 'https' | 'data'; raises ``VideoSourceError``."""
    from urllib.parse import urlsplit
    if not isinstance(ref, str) or not ref:
        raise VideoSourceError("input_video must be a non-empty string")
    if ref.startswith("data:"):
        return "data"
    if ref.startswith("ipfs://") or _CID.match(ref):
        if not _CID.match(ref[len("ipfs://"):] if ref.startswith("ipfs://") else ref):
            raise VideoSourceError("malformed IPFS reference")
        return "ipfs"
    u = urlsplit(ref)
    if u.scheme != "https" or not u.hostname or u.username or u.password:
        raise VideoSourceError(f"refused input_video source {ref[:80]!r}: only ipfs:// / CID, https:// or data: URIs")
    allow = [h.strip().lower() for h in os.environ.get("ARBIUS_VIDEO_HOSTS", "").split(",") if h.strip()]
    if allow and u.hostname.lower() not in allow:
        raise VideoSourceError(f"host {u.hostname} is not in ARBIUS_VIDEO_HOSTS")
    if not _public_host(u.hostname):
        raise VideoSourceError(f"host {u.hostname} resolves to a non-public address")
    return "https"


def _get(url: str, max_redirects: int = 3) -> bytes:
    import httpx
    for _ in range(max_redirects + 1):
        with httpx.stream("GET", url, timeout=120.0, follow_redirects=False) as r:
            if r.status_code in (301, 302, 303, 307, 308):
                nxt = str(r.url.join(r.headers.get("location", "")))
                check_source(nxt)                  # every hop must pass the same policy
                url = nxt
                continue
            r.raise_for_status()
            buf = bytearray()
            for chunk in r.iter_bytes():
                buf += chunk
                if len(buf) > MAX_VIDEO_BYTES:
                    raise VideoSourceError("input video exceeds MAX_VIDEO_BYTES")
            return bytes(buf)
    raise VideoSourceError("too many redirects")


def fetch(ref: str) -> bytes:
    kind = check_source(ref)
    if kind == "data":
        data = base64.b64decode(ref.split(",", 1)[1])
    elif kind == "https":
        data = _get(ref)
    else:
        import httpx
        gw = os.environ.get("ARBIUS_IPFS_GATEWAY", "http://127.0.0.1:8080")   # operator-configured
        r = httpx.get(f"{gw.rstrip('/')}/ipfs/{ref.replace('ipfs://', '')}", timeout=120.0)
        r.raise_for_status()
        data = r.content
    if len(data) > MAX_VIDEO_BYTES:
        raise VideoSourceError("input video exceeds MAX_VIDEO_BYTES")
    return data


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
