#!/usr/bin/env python3
"""Where the CPU time of one RVM task goes after the GPU matting (bench clip, 1080p x 48 frames).

Runs the bench's synthetic clip through the matting pipeline once (warm-up) and once timed, then
times the output path piece by piece: ``list(out)`` + ``np.stack`` (what ``encode_mp4`` did), the
native intra encode at 1 and 16 threads, and the CID.  Saves a few output frames (``--save``) so
the encoder can be tuned on the CPU against real matting output.

    python scripts/rvm_encode_probe.py [--save gpurun_out/rvm_frames.npz]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--save", default=None)
    a = ap.parse_args()
    import numpy as np
    import torch

    from arbius_amd import native
    from arbius_amd.models.registry import build_pipeline
    from arbius_amd.node.solver import solve_files
    from arbius_amd.utils import mp4
    pipe = build_pipeline("robust_video_matting", device=torch.device("cuda", 0))
    F, H, W = 48, 1080, 1920
    rng = np.random.default_rng(1234)
    yy, xx = np.mgrid[0:H, 0:W]
    base = ((xx[None] + 7 * np.arange(F)[:, None, None]) % 256).astype(np.uint8)
    clip = np.stack([base, (yy[None] % 256).astype(np.uint8).repeat(F, 0),
                     rng.integers(0, 256, base.shape, dtype=np.uint8)], axis=-1)
    pipe(clip, "green-screen")
    torch.cuda.synchronize()
    r = {}
    t0 = time.perf_counter()
    out = pipe(clip, "green-screen")
    r["matting_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    st = np.stack(list(out))
    r["stack_s"] = time.perf_counter() - t0
    for th in (1, 16):
        t0 = time.perf_counter()
        _, _, nals = native.h264_encode_rgb(st, mp4.INTRA_QP, th)
        r[f"encode_t{th}_s"] = time.perf_counter() - t0
    r["nal_bytes"] = sum(len(n) for n in nals)
    t0 = time.perf_counter()
    data = mp4.encode_mp4(list(out), 24)
    r["encode_mp4_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    sol = solve_files([("out-1.mp4", data)])
    r["cid_s"] = time.perf_counter() - t0
    r["mp4_bytes"] = len(data)
    r["cid"] = sol.cid
    r["cpus"] = len(os.sched_getaffinity(0))
    print(json.dumps(r))
    if a.save:
        os.makedirs(os.path.dirname(a.save) or ".", exist_ok=True)
        np.savez_compressed(a.save, frames=out[::12].copy())


if __name__ == "__main__":
    main()
