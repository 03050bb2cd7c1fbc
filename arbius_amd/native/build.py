"""Build the native CPU runtime extension in-tree (``arbius_amd/native/_native*.so``).

    python -m arbius_amd.native.build

zlib is linked STATICALLY (``libz.a``) with its symbols kept private (``--exclude-libs``): the PNG
IDAT bytes are consensus bytes, and a dynamic ``-lz`` would take whatever deflate the host has
(zlib-ng, a patched or newer zlib emit different streams for the same input).  The linked
implementation's identity is ``native.deflate_id()``, pinned by ``numerics.DEFLATE_ID``.
"""
from __future__ import annotations

import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = HERE / "src" / "native.cpp"
SOURCES = [SRC, HERE / "src" / "secp256k1.cpp", HERE / "src" / "h264.cpp"]
ZLIB_STATIC = ("/usr/lib/x86_64-linux-gnu/libz.a", "/usr/lib64/libz.a", "/usr/lib/libz.a")
HEADERS = [HERE / "src" / "secp256k1.h", HERE / "src" / "h264.h"]


def target() -> Path:
    return HERE / ("_native" + sysconfig.get_config_var("EXT_SUFFIX"))


def build(force: bool = False) -> Path:
    out = target()
    if out.exists() and not force and all(out.stat().st_mtime >= f.stat().st_mtime for f in SOURCES + HEADERS):
        return out
    import pybind11
    # x86-64-v2 (SSE4.2): every x86 server CPU since 2009; lets the H.264 quantiser loops use pmulld
    libz = next((p for p in ZLIB_STATIC if Path(p).exists()), None)
    if libz is None:
        raise RuntimeError("static zlib (libz.a) not found: the PNG encoder must not depend on the host's libz")
    cmd = ["g++", "-O3", "-march=x86-64-v2", "-shared", "-fPIC", "-std=c++17", "-fvisibility=hidden", "-pthread",
           "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"], *map(str, SOURCES), libz,
           "-Wl,--exclude-libs,ALL", "-Wl,-Bsymbolic", "-o", str(out)]
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
