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

Containers: MP4 (any single avc1 track) or a raw Annex-B H.264 stream, decoded by the native
decoder (``native/src/h264.cpp``: Constrained Baseline CAVLC - I and P slices, I_PCM /
Intra_16x16 / Intra_4x4, P_Skip and every P partition, multiple reference pictures, in-loop
deblocking; a superset of what ``utils/mp4.py`` writes), and ``.npy`` uint8 [T, H, W, 3]
(``allow_pickle=False``).  Anything else (B slices, CABAC / High profile, interlace) is decoded
by an ``ffmpeg`` binary when one is on PATH; the image ships none, so ``probe`` rejects such
inputs at hydration (``UndecodableVideo``: the node skips the task, it does not mark it
invalid - a miner with a full decoder may solve it).
"""
from __future__ import annotations

import base64
import io
import json
import logging
import os
import re
import shutil
import subprocess
import tempfile
from typing import List, Tuple

import numpy as np

log = logging.getLogger("arbius.video")


MAX_VIDEO_BYTES = 512 << 20
_CID = re.compile(r"^(Qm[1-9A-HJ-NP-Za-km-z]{44}|b[a-z2-7]{20,})(/[A-Za-z0-9._\-/]*)?$")


class VideoSourceError(ValueError):
    """``input_video`` names a source this node refuses to read (local file, private address...)."""


def _is_public(addr: str) -> bool:
    import ipaddress
    ip = ipaddress.ip_address(addr.split("%")[0])
    if getattr(ip, "ipv4_mapped", None):
        ip = ip.ipv4_mapped
    return not (ip.is_private or ip.is_loopback or ip.is_link_local or ip.is_multicast or ip.is_reserved
                or ip.is_unspecified or not ip.is_global)


def resolve_public(host: str, port: int = 443) -> List[str]:
    """Every address ``host`` resolves to, or [] unless ALL of them are public unicast."""
    import socket
    try:
        infos = socket.getaddrinfo(host, port, proto=socket.IPPROTO_TCP)
    except OSError:
        return []
    addrs = []
    for info in infos:
        a = info[4][0]
        if not _is_public(a):
            return []
        if a not in addrs:
            addrs.append(a)
    return addrs


def _public_host(host: str) -> bool:
    """True when every address ``host`` resolves to is public unicast."""
    return bool(resolve_public(host))


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


def _read_capped(r) -> bytes:
    buf = bytearray()
    for chunk in r.iter_bytes():
        buf += chunk
        if len(buf) > MAX_VIDEO_BYTES:
            raise VideoSourceError("input video exceeds MAX_VIDEO_BYTES")
    return bytes(buf)


def pinned_request(url: str):
    """(url to connect to, Host header, TLS server name): the host is resolved ONCE, every address
    must be public, and the connection goes to that validated address - no second resolution by the
    HTTP client, so DNS rebinding between the check and the connect cannot reach a private address.
    TLS SNI and certificate verification still use the hostname."""
    from urllib.parse import urlsplit, urlunsplit
    u = urlsplit(url)
    port = u.port or 443
    addrs = resolve_public(u.hostname, port)
    if not addrs:
        raise VideoSourceError(f"host {u.hostname} resolves to a non-public address")
    ip = addrs[0]
    netloc = (f"[{ip}]" if ":" in ip else ip) + (f":{u.port}" if u.port else "")
    host_hdr = u.hostname + (f":{u.port}" if u.port else "")
    return urlunsplit((u.scheme, netloc, u.path or "/", u.query, "")), host_hdr, u.hostname


def _get(url: str, max_redirects: int = 3) -> bytes:
    import httpx
    for _ in range(max_redirects + 1):
        target, host_hdr, sni = pinned_request(url)
        with httpx.Client(timeout=120.0, follow_redirects=False) as cl:
            req = cl.build_request("GET", target, headers={"Host": host_hdr}, extensions={"sni_hostname": sni})
            r = cl.send(req, stream=True)
            try:
                if r.status_code in (301, 302, 303, 307, 308):
                    from urllib.parse import urljoin
                    nxt = urljoin(url, r.headers.get("location", ""))
                    check_source(nxt)              # every hop must pass the same policy
                    url = nxt
                    continue
                r.raise_for_status()
                return _read_capped(r)
            finally:
                r.close()
    raise VideoSourceError("too many redirects")


# Fetched inputs are cached on disk between hydration (``probe_video``) and the solve
# (``load_video``, possibly in a GPU worker process): one download per task input.  The cache is a
# directory private to this user (mode 0700, owner checked before every use: another local user
# must not be able to plant or swap the bytes behind a task's input), by default per uid under the
# temp dir; ``$ARBIUS_VIDEO_CACHE`` (e.g. under the node's data dir) overrides it.  A cached
# ``ipfs://Qm...`` entry is also checked against its CID (kubo's default chunking) before use.
_CACHE_DIR = os.environ.get("ARBIUS_VIDEO_CACHE") or os.path.join(tempfile.gettempdir(),
                                                                  f"arbius_video_cache-{os.getuid()}")
_CACHE_KEEP = 16


def _cache_dir_ok(create: bool) -> bool:
    """The cache dir exists (or was created) as a directory owned by us with no group/other access."""
    import stat
    try:
        if create:
            os.makedirs(_CACHE_DIR, mode=0o700, exist_ok=True)
        st = os.lstat(_CACHE_DIR)
    except OSError:
        return False
    return stat.S_ISDIR(st.st_mode) and st.st_uid == os.getuid() and not (st.st_mode & 0o077)


def _cache_path(ref: str) -> str:
    import hashlib
    return os.path.join(_CACHE_DIR, hashlib.sha256(ref.encode()).hexdigest())


def _cid_matches(ref: str, data: bytes) -> bool:
    """For a bare CIDv0 reference (``Qm...`` without a path): the bytes' UnixFS file CID (kubo
    defaults) equals it.  Other references (paths, CIDv1, https) are not content-addressed here."""
    cid = ref[len("ipfs://"):] if ref.startswith("ipfs://") else ref
    if not (cid.startswith("Qm") and "/" not in cid):
        return True
    from ..ipfs.unixfs import add_file
    return add_file(data).cid_str == cid


def _cache_get(ref: str):
    """Cached bytes of ``ref``, or None.  An entry is used only with its sidecar (written by
    ``_cache_put`` after the download was checked once, ADVICE r4: no re-hash of up to 512 MB per
    task) and only when file and sidecar are ours and agree on the size."""
    if not _cache_dir_ok(False):
        return None
    p = _cache_path(ref)
    try:
        for q in (p, p + ".meta"):
            st = os.lstat(q)
            if st.st_uid != os.getuid() or not os.path.isfile(q):
                return None
        with open(p + ".meta") as f:
            meta = json.load(f)
        with open(p, "rb") as f:
            data = f.read(MAX_VIDEO_BYTES + 1)
        os.utime(p)
    except (OSError, ValueError):
        return None
    if meta.get("ref") != ref or meta.get("size") != len(data) or len(data) > MAX_VIDEO_BYTES:
        return None
    return data


def _cache_put(ref: str, data: bytes, verified: bool):
    try:
        if not _cache_dir_ok(True):
            return
        p = _cache_path(ref)
        tmp = p + f".{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, p)
        with open(tmp, "w") as f:
            json.dump({"ref": ref, "size": len(data), "verified": bool(verified)}, f)
        os.replace(tmp, p + ".meta")
        ents = sorted((os.path.getmtime(os.path.join(_CACHE_DIR, e)), e) for e in os.listdir(_CACHE_DIR)
                      if not e.endswith((".tmp", ".meta")))
        for _, e in ents[:-_CACHE_KEEP]:
            for q in (e, e + ".meta"):
                try:
                    os.unlink(os.path.join(_CACHE_DIR, q))
                except FileNotFoundError:
                    pass
    except OSError:
        pass


def fetch(ref: str) -> bytes:
    kind = check_source(ref)
    if kind == "data":
        data = base64.b64decode(ref.split(",", 1)[1])
    else:
        data = _cache_get(ref)
        if data is None:
            if kind == "https":
                data = _get(ref)
            else:
                import httpx
                gw = os.environ.get("ARBIUS_IPFS_GATEWAY", "http://127.0.0.1:8080")   # operator-configured
                with httpx.stream("GET", f"{gw.rstrip('/')}/ipfs/{ref.replace('ipfs://', '')}", timeout=120.0) as r:
                    r.raise_for_status()
                    data = _read_capped(r)                 # capped while streaming, never read whole first
            # checked ONCE, here: a bare CIDv0 must be the bytes' UnixFS CID under kubo's defaults.  A
            # file added with another chunker / layout cannot be re-derived: it is kept as unverified
            # (the operator's gateway served it) instead of being fetched again on every use.
            verified = _cid_matches(ref, data)
            if not verified:
                log.warning("input %s: bytes do not re-derive the CID under kubo's default layout "
                            "(another chunker?) - used unverified", ref[:80])
            _cache_put(ref, data, verified)
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


class UndecodableVideo(ValueError):
    """The input is not a video this node can decode (outside the native H.264 I/P subset and
    no ffmpeg): the task is skipped, never marked invalid - other miners may decode it."""


def _ue(bits: str, i: int) -> Tuple[int, int]:
    z = 0
    while i < len(bits) and bits[i] == "0":
        z += 1
        i += 1
    if i + z + 1 > len(bits):
        raise UndecodableVideo("truncated slice header")
    return int(bits[i:i + z + 1], 2) - 1, i + z + 1


def _demux(data: bytes) -> Tuple[List[bytes], int]:
    from .mp4 import annexb_nals, read_mp4_nals
    if data[4:8] == b"ftyp":
        try:
            fps, nals, _ = read_mp4_nals(data)
        except ValueError as e:
            raise UndecodableVideo(str(e)) from None
        return nals, fps
    if data.startswith(b"\x00\x00\x01") or data.startswith(b"\x00\x00\x00\x01"):
        return annexb_nals(data), 24          # raw Annex-B stream: no timing, template default
    raise UndecodableVideo("input video is neither an MP4 nor an H.264 Annex-B stream")


def probe(data: bytes) -> None:
    """Cheap decodability check (hydration): container, then every slice header's slice_type
    must be I or P (no B / SP / SI), and the first two pictures must decode through the native
    decoder (which refuses CABAC, interlace, weighted prediction, ... in their parameter sets and
    slice headers)."""
    if data[:6] == b"\x93NUMPY":
        return
    if shutil.which("ffmpeg"):
        return
    nals, _ = _demux(data)
    head_pics, pictures = [], 0
    for n in nals:
        typ = n[0] & 0x1F
        if typ in (7, 8):
            if pictures <= 2:       # parameter sets re-sent or updated between the first pictures
                head_pics.append(n)
            continue
        if typ in (1, 5):
            head = "".join(f"{b:08b}" for b in n[1:9].replace(b"\x00\x00\x03", b"\x00\x00"))
            first_mb, i = _ue(head, 0)
            slice_type, _ = _ue(head, i)
            if slice_type % 5 not in (0, 2):
                raise UndecodableVideo("input video has B / SP / SI slices: only I and P slices decode natively")
            if first_mb == 0:
                pictures += 1
            if pictures <= 2:
                head_pics.append(n)
        elif pictures == 0:
            head_pics.append(n)
    from .mp4 import decode_h264
    try:
        decode_h264(head_pics)
    except ValueError as e:
        raise UndecodableVideo(str(e)) from None


def decode(data: bytes) -> Tuple[np.ndarray, int]:
    if data[:6] == b"\x93NUMPY":
        arr = np.load(io.BytesIO(data), allow_pickle=False)
        return arr.astype(np.uint8), 24
    try:
        nals, fps = _demux(data)
        from .mp4 import decode_h264_rgb
        return decode_h264_rgb(nals), fps
    except ValueError as e:
        native_err = e
    ff = shutil.which("ffmpeg")
    if ff is None:
        raise UndecodableVideo(f"native H.264 decoder: {native_err}; no ffmpeg binary for other streams")
    with tempfile.NamedTemporaryFile(suffix=".mp4") as f:
        f.write(data)
        f.flush()
        probe_out = subprocess.run([ff, "-i", f.name], capture_output=True, text=True)
        import re
        m = re.search(r"(\d+)x(\d+)[, ].*?(\d+(?:\.\d+)?) fps", probe_out.stderr)
        if not m:
            raise UndecodableVideo("ffmpeg could not probe the input video")
        W, H, fps = int(m.group(1)), int(m.group(2)), float(m.group(3))
        raw = subprocess.run([ff, "-v", "error", "-i", f.name, "-f", "rawvideo", "-pix_fmt", "rgb24", "-"],
                             capture_output=True, check=True).stdout
    return np.frombuffer(raw, np.uint8).reshape(-1, H, W, 3), int(round(fps))


def load_video(ref: str) -> Tuple[np.ndarray, int]:
    return decode(fetch(ref))


def probe_video(ref: str) -> None:
    """Hydration-time check: the source is allowed AND decodable (raises VideoSourceError /
    UndecodableVideo).  Fetch failures propagate as their own exceptions."""
    probe(fetch(ref))
