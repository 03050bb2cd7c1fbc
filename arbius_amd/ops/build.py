"""Build the gfx950 HIP kernel library in-tree (``arbius_amd/ops/libarbius_kernels.so``).

Plain ``hipcc --offload-arch=gfx950 -shared`` over ``csrc/*.hip`` - no torch
headers, so a rebuild takes seconds; the library is loaded with ctypes and
launched on PyTorch's current HIP stream (graph-capture safe).

    python -m arbius_amd.ops.build [--force] [--jobs N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
OBJ = HERE / "build_obj"
LIB = HERE / "libarbius_kernels.so"
ARCH = os.environ.get("ARBIUS_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build arbius_amd kernels)")


def sources():
    return sorted(CSRC.glob("*.hip"))


def _needs(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    deps = [src] + list(CSRC.glob("*.h")) + list(CSRC.glob("*.inc"))
    return any(d.stat().st_mtime > t for d in deps)


def build(force: bool = False, jobs: int = 8, verbose: bool = False) -> Path:
    hipcc = _hipcc()
    OBJ.mkdir(exist_ok=True)
    srcs = sources()
    flags = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-I", str(CSRC),
             "-Wno-unused-result", "-munsafe-fp-atomics"]

    def compile_one(src: Path):
        obj = OBJ / (src.stem + ".o")
        if force or _needs(obj, src):
            cmd = [hipcc, *flags, "-c", str(src), "-o", str(obj)]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr}")
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(compile_one, srcs))
    if force or not LIB.exists() or any(o.stat().st_mtime > LIB.stat().st_mtime for o in objs):
        cmd = [hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", *map(str, objs), "-o", str(LIB)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    # every symbol must resolve (hipcc can emit a kernel launch whose host stub it silently dropped)
    import ctypes
    try:
        ctypes.CDLL(str(LIB), mode=os.RTLD_NOW | os.RTLD_LOCAL)
    except OSError as e:
        raise RuntimeError(f"built {LIB.name} does not load: {e}") from None
    return LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    p = build(a.force, a.jobs, a.verbose)
    print(p)


if __name__ == "__main__":
    main()
