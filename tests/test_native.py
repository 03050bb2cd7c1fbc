"""Native C++ runtime (arbius_amd/native) == its Python references, byte for byte."""
import os

import numpy as np
import pytest

from arbius_amd import native
from arbius_amd.utils.keccak import keccak256_py
from arbius_amd.utils.mp4 import _pad16, pcm_slice_body_py
from arbius_amd.utils.png import encode_png_py

pytestmark = pytest.mark.skipif(not native.loaded, reason="native extension not built")


def test_keccak_matches_python():
    for n in (0, 1, 31, 135, 136, 137, 271, 272, 1000):
        d = os.urandom(n)
        assert native.keccak256(d) == keccak256_py(d)
    assert native.keccak256(b"").hex() == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"


@pytest.mark.parametrize("shape", [(64, 48, 3), (17, 5, 4), (9, 9), (512, 512, 3)])
def test_png_matches_python(shape):
    img = np.random.default_rng(0).integers(0, 256, shape, dtype=np.uint8)
    for level in (1, 6, 9):
        assert native.png_encode(img, level) == encode_png_py(img, level)


def test_png_segmented_zlib_stream_is_standard():
    """The IDAT stream is a segmented (pigz-layout) zlib stream: any inflater decodes it to the filtered
    rows; segments are cut at fixed 128 KiB offsets, so a 768^2 RGB image spans 14 of them and a tiny one
    is a single segment with the plain zlib framing."""
    import zlib

    from arbius_amd.utils.png import SEG, decode_png, zlib_segmented
    rng = np.random.default_rng(5)
    for n in (0, 1, SEG - 1, SEG, SEG + 1, 5 * SEG + 77):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        z = zlib_segmented(data, 6)
        assert zlib.decompress(z) == data
        assert z[:2] == zlib.compress(data, 6)[:2]            # same header bytes as zlib's own framing
    img = rng.integers(0, 256, (768, 768, 3), dtype=np.uint8)
    blob = native.png_encode(img, 6)
    assert np.array_equal(decode_png(blob).reshape(img.shape), img)


@pytest.mark.parametrize("hw", [(16, 16), (320, 576), (90, 160), (1080, 1920)])
def test_pcm_body_matches_python(hw):
    f = _pad16(np.random.default_rng(1).integers(0, 256, (*hw, 3), dtype=np.uint8))
    a = native.pcm_slice_body(f)
    assert a == pcm_slice_body_py(f)
    assert a == native.pcm_slice_body(f, threads=3)      # thread count never changes bytes


def test_native_secp256k1_matches_python_reference():
    """C++ ECDSA (constant-time ladder) == the Python reference: pubkeys, RFC 6979 signatures
    (r, s, recid) and ecrecover, on random keys / digests and edge scalars."""
    import os as _os
    import random

    from arbius_amd import native
    from arbius_amd.chain import secp256k1 as S
    if not (native.loaded and hasattr(native, "secp256k1_sign")):
        import pytest
        pytest.skip("native extension not built")
    rng = random.Random(7)
    keys = [1, 2, 3, S.N - 1, S.N - 2, 0xac0974bec39a17e36ba4a6b4d238ff944bacb478cbed5efcae784d7bf4f2ff80]
    keys += [rng.randrange(1, S.N) for _ in range(40)]
    for d in keys:
        assert S.pubkey(d) == S.py_pubkey(d)
        for h in (bytes(32), b"\xff" * 32, _os.urandom(32), rng.randbytes(32)):
            got = S.sign(h, d)
            assert got == S.py_sign(h, d)
            assert S.recover(h, *got) == S.py_recover(h, *got) == S.py_pubkey(d)
    # hardhat account 0 (miner/test/utils.test.ts:18)
    assert S.address_from_priv(keys[5]).lower() == "0xf39fd6e51aad88f6f4ce6ab8827279cfffb92266"
    assert native.secp256k1_recover(b"\x01" * 32, bytes(32), b"\x01" * 32, 0) is None   # r = 0
