#!/usr/bin/env python3
"""Build the native C++ runtime (native/src/*.cpp: keccak, PNG, H.264 codec, secp256k1) with
AddressSanitizer + UndefinedBehaviorSanitizer (or ThreadSanitizer) on the CPU and exercise every
entry point against its Python reference under the sanitizer runtime, plus corrupted H.264
input.  Host code only - no GPU.

    python scripts/sanitize_native.py [OUT_DIR]          # exit 0 = clean
    python scripts/sanitize_native.py --tsan [OUT_DIR]   # data races in the threaded codec
"""
import os
import subprocess
import sys
import sysconfig
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "arbius_amd", "native", "src")

EXERCISE = r'''
import hashlib, os, random, sys
import numpy as np
import _native as N
sys.path.insert(0, os.environ["ARB_ROOT"])
from arbius_amd.utils import keccak as K, png as P
from arbius_amd.chain import secp256k1 as S
rng = random.Random(3)
for n in (0, 1, 135, 136, 137, 1000, 4096):
    d = rng.randbytes(n)
    assert N.keccak256(d) == K.keccak256_py(d)
    assert N.sha256(d) == hashlib.sha256(d).digest()
for shape in ((1, 1, 3), (7, 13, 3), (64, 48, 3), (33, 65, 4)):
    img = np.random.default_rng(len(shape)).integers(0, 256, shape, dtype=np.uint8)
    N.png_encode(img, 6)
for (h, w) in ((16, 16), (48, 80), (32, 64)):
    fr = np.random.default_rng(h).integers(0, 256, (h, w, 3), dtype=np.uint8)
    N.pcm_slice_body(fr, 4)
for _ in range(20):
    d = rng.randrange(1, S.N)
    h = rng.randbytes(32)
    r, s, rec = N.secp256k1_sign(h, d.to_bytes(32, "big"))
    assert (int.from_bytes(r, "big"), int.from_bytes(s, "big"), rec) == S.py_sign(h, d)
    pub = N.secp256k1_recover(h, r, s, rec)
    assert pub == N.secp256k1_pubkey(d.to_bytes(32, "big"))
for bad in (bytes(32), (S.N).to_bytes(32, "big")):
    try:
        N.secp256k1_sign(b"\0" * 32, bad)
        raise SystemExit("accepted an invalid key")
    except ValueError:
        pass
# H.264 intra codec: encoder / decoder round trip, then the decoder on corrupted (untrusted) input
import numpy as np
rng = np.random.default_rng(0)
y = rng.integers(0, 256, (48, 64), dtype=np.uint8)
cb = rng.integers(0, 256, (24, 32), dtype=np.uint8)
cr = rng.integers(0, 256, (24, 32), dtype=np.uint8)
for qp in (4, 20, 51):
    nal, ry, rcb, rcr = N.h264_encode_yuv(y, cb, cr, qp, 0)
    sps, pps = N.h264_parameter_sets(64, 48, qp)
    (dy, dcb, dcr, _), = N.h264_decode([sps, pps, nal], 2)
    assert (dy == ry).all() and (dcb == rcb).all() and (dcr == rcr).all()
    for trial in range(200):
        bad = bytearray(nal)
        if trial % 2:
            bad = bad[:rng.integers(1, len(bad))]
        else:
            for _ in range(3):
                bad[rng.integers(1, len(bad))] ^= 1 << int(rng.integers(0, 8))
        try:
            N.h264_decode([sps, pps, bytes(bad)], 1)
        except ValueError:
            pass
# hand-made hostile slices: exp-golomb values with 31 leading zeros (>= 2^31) in every field that
# becomes an index (first_mb_in_slice, intra_chroma_pred_mode, slice QP delta)
def ue(v):
    x = v + 1
    return "0" * (x.bit_length() - 1) + format(x, "b")
def se(v):
    return ue(2 * v - 1 if v > 0 else -2 * v)
def nal(bits):
    bits += "1"
    bits += "0" * (-len(bits) % 8)
    return bytes([0x65]) + int(bits, 2).to_bytes(len(bits) // 8, "big")
BIG = (1 << 32) - 2
head = lambda first=0, qpd=0: ue(first) + ue(7) + ue(0) + "0000" + ue(0) + "00" + se(qpd) + ue(1)
hostile = [nal(head(first=BIG)), nal(head(first=(1 << 31) + 5)), nal(head(qpd=(1 << 31) - 1)),
           nal(head() + ue(3) + ue(BIG) + se(0)),               # I_16x16 DC, chroma mode 2^32-2
           nal(head() + ue(0) + "1" * 16 + ue((1 << 31) + 1) + ue(0))]   # I_NxN, chroma mode >= 2^31
sps, pps = N.h264_parameter_sets(64, 48, 20)
for h in hostile:
    try:
        N.h264_decode([sps, pps, h], 1)
        raise SystemExit("accepted a hostile slice")
    except ValueError:
        pass
frames = rng.integers(0, 256, (3, 40, 72, 3), dtype=np.uint8)
_, _, nals = N.h264_encode_rgb(frames, 24, 3)
assert N.h264_decode_rgb([sps_ for sps_ in N.h264_parameter_sets(72, 40, 24)] + list(nals), 2).shape == (3, 40, 72, 3)
# IPPP / coverage-mode streams (P slices, several references, slice-parallel decode, wavefront
# deblocking): round trip, then corrupted P slices
F = 6
ys = rng.integers(0, 256, (F, 48, 64), dtype=np.uint8)
cbs = rng.integers(0, 256, (F, 24, 32), dtype=np.uint8)
crs = rng.integers(0, 256, (F, 24, 32), dtype=np.uint8)
for seed, refs in ((0, 1), (3, 3)):
    pics, ry, rcb, rcr = N.h264_encode_yuv_stream(ys, cbs, crs, 26, 4, seed, refs, 4, 1)
    ps = list(N.h264_parameter_sets(64, 48, 26, refs))
    flat = [n for p in pics for n in p]
    dec = N.h264_decode(ps + flat, 4)
    assert all((d[0] == ry[i]).all() for i, d in enumerate(dec))
    N.h264_decode(ps + flat, 4, True)
    for trial in range(300):
        bad = list(flat)
        k = int(rng.integers(0, len(bad)))
        b = bytearray(bad[k])
        if trial % 3 == 0:
            b = b[:rng.integers(1, len(b))]
        else:
            for _ in range(1 + trial % 4):
                b[rng.integers(1, len(b))] ^= 1 << int(rng.integers(0, 8))
        bad[k] = bytes(b)
        try:
            N.h264_decode(ps + bad, 4)
        except ValueError:
            pass
        try:
            N.h264_decode_rgb(ps + bad, 3)
        except ValueError:
            pass
frames = rng.integers(0, 256, (5, 40, 72, 3), dtype=np.uint8)
s_, p_, pics = N.h264_encode_rgb_stream(frames, 24, 3, 4, 1)
assert N.h264_decode_rgb([s_, p_] + [n for p in pics for n in p], 4).shape == (5, 40, 72, 3)
print("sanitized native runtime: all entry points clean")
'''


def main():
    args = [a for a in sys.argv[1:] if a != "--tsan"]
    tsan = "--tsan" in sys.argv        # ThreadSanitizer build (slice-parallel decode, wavefront deblocking)
    out_dir = args[0] if args else tempfile.mkdtemp(prefix="arb_asan_")
    import pybind11
    so = os.path.join(out_dir, "_native" + sysconfig.get_config_var("EXT_SUFFIX"))
    flags = ["-O1", "-g", "-fno-omit-frame-pointer"] + (
        ["-fsanitize=thread"] if tsan else ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])
    cmd = ["g++", *flags, "-shared", "-fPIC", "-std=c++17", "-pthread", "-I", pybind11.get_include(),
           "-I", sysconfig.get_paths()["include"], os.path.join(SRC, "native.cpp"), os.path.join(SRC, "secp256k1.cpp"),
           os.path.join(SRC, "h264.cpp"),
           "-lz", "-o", so]
    subprocess.run(cmd, check=True)
    lib = lambda n: subprocess.check_output(["g++", f"-print-file-name={n}"], text=True).strip()
    preload = lib("libtsan.so") if tsan else f"{lib('libasan.so')}:{lib('libubsan.so')}"
    env = dict(os.environ, LD_PRELOAD=preload, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0",
               PYTHONPATH=out_dir, ARB_ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", EXERCISE], env=env, capture_output=True, text=True)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr[:6000] + ("\n...\n" + r.stderr[-2000:] if len(r.stderr) > 8000 else r.stderr[6000:]))
    return r.returncode


if __name__ == "__main__":
    sys.exit(main())
