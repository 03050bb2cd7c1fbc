"""CPU-only golden bytes of the consensus encoders.

Every image CID hashes a PNG whose IDAT stream comes out of a deflate implementation, and every
video CID hashes the H.264 / MP4 bytes of ``native/src/h264.cpp``.  The GPU goldens
(``tests/test_golden_gpu.py``) pin whole tasks on gfx950; these pin the encoders alone, on any
host: a different zlib (zlib-ng, another version) behind the native module or the Python fallback
changes the PNG hash and fails here, and ``check_mining_env`` refuses to ``start`` on it.
"""
import hashlib

import numpy as np
import pytest

from arbius_amd import native, numerics
from arbius_amd.utils.png import decode_png, encode_png, encode_png_py

PNG_SHA = "e1f023bc5065d5352499ffb2050d96ed878e73f012b5c0d5de6f458bf243b3de"          # 400x300 RGB, level 6
MP4_INTRA_SHA = "3960efd519faca24b87528a250901267e537436f28e1bbccd106fb14097972d7"    # 6 x 128x96, avc-intra
MP4_AVC_SHA = "26a0bb9685834f2c08c86edf0a40b813a4c02034f8ad737f2fa4ed05db4edb19"      # same clip, IPPP avc


def image(h, w, seed):
    """Smooth ramps with 1-2 bits of integer-hash noise (deflate has matches to choose between)."""
    y, x = np.mgrid[0:h, 0:w].astype(np.uint32)
    v = (x * 2654435761 + y * 40503 + seed * 97) & 0xFFFFFFFF
    v ^= v >> 13
    v = (v * 1103515245 + 12345) & 0xFFFFFFFF
    smooth = ((x * 3 + y * 5) // 7) & 255
    rgb = np.stack([(smooth + (v >> 30)) & 255, (smooth * 3 + (x // 17)) & 255, (y // 9 + (v >> 31)) & 255], -1)
    return rgb.astype(np.uint8)


def _sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.mark.skipif(not native.loaded, reason="native runtime not built")
def test_native_png_bytes_pinned():
    img = image(300, 400, 1)
    png = encode_png(img)
    assert _sha(png) == PNG_SHA
    assert (decode_png(png) == img).all()
    assert native.deflate_id() == numerics.DEFLATE_ID


def test_python_png_fallback_bytes_pinned():
    """The pure-Python encoder deflates through the interpreter's zlib: on a host whose zlib is not
    the pinned one this fails - and ``start`` refuses that node (next test)."""
    import zlib
    img = image(300, 400, 1)
    if f"zlib-{zlib.ZLIB_RUNTIME_VERSION}" != numerics.DEFLATE_ID:
        pytest.fail(f"host zlib {zlib.ZLIB_RUNTIME_VERSION} is not {numerics.DEFLATE_ID}: the Python PNG "
                    "fallback would emit non-consensus bytes here")
    assert _sha(encode_png_py(img)) == PNG_SHA


def test_start_refuses_a_foreign_deflate(tmp_path, monkeypatch):
    numerics.check_mining_env({}, deflate_id=numerics.DEFLATE_ID)
    with pytest.raises(SystemExit, match="deflate"):
        numerics.check_mining_env({}, deflate_id="zlib-1.3.1")
    # through the CLI: a swapped deflate stops `start` before it touches the chain
    import json
    from arbius_amd import cli
    monkeypatch.setattr(numerics, "deflate_identity", lambda: "zlib-ng-2.1.6")
    cfg = tmp_path / "MiningConfig.json"
    cfg.write_text(json.dumps({"db_path": str(tmp_path / "db.sqlite"), "mi355x": {"mock_chain": True}}))
    with pytest.raises(SystemExit, match="zlib-ng"):
        cli.main(["start", str(cfg)])


@pytest.mark.skipif(not native.loaded, reason="native runtime not built")
def test_mp4_bytes_pinned():
    from arbius_amd.utils.mp4 import encode_mp4
    clip = np.stack([image(96, 128, s) for s in range(6)])
    assert _sha(encode_mp4(clip, 24, codec="avc-intra")) == MP4_INTRA_SHA
    assert _sha(encode_mp4(clip, 24, codec="avc")) == MP4_AVC_SHA
    assert _sha(encode_mp4(clip, 24, codec="avc-intra", threads=1)) == MP4_INTRA_SHA   # thread-count free


@pytest.mark.skipif(not native.loaded, reason="native runtime not built")
def test_native_module_carries_its_own_deflate():
    """The extension links libz.a with private symbols: no dynamic libz dependency, no exported
    deflate a host library could interpose or be interposed by."""
    import subprocess
    so = native._native.__file__
    ldd = subprocess.run(["ldd", so], capture_output=True, text=True).stdout
    assert "libz.so" not in ldd
    syms = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True).stdout
    assert not any(line.split()[-1].startswith(("deflate", "inflate", "zlibVersion")) for line in syms.splitlines()
                   if line.strip())
