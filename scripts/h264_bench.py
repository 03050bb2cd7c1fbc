#!/usr/bin/env python3
"""GPU avc-intra encode (ops.h264_intra_encode, csrc/h264_intra.hip) vs the native host encoder on one
RVM-sized clip (48 pictures of 1920x1080, macroblock-padded 4:2:0): GPU time per clip (events, the
encoder's 5 launches), host CPU time of the native encode at 1 and N threads, host time of the GPU
path's tail (emulation prevention), output equality.  One JSON line.

    python scripts/h264_bench.py [--frames 48] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=48)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import numpy as np
    import torch

    from arbius_amd import native, ops
    from arbius_amd.utils.mp4 import INTRA_QP
    F, H16, W16 = a.frames, 1088, 1920
    rng = np.random.default_rng(0)
    yy, xx = np.mgrid[0:H16, 0:W16]
    # a matting-like picture: smooth background, textured foreground, noise
    y = np.stack([((xx // 2 + yy // 3 + 5 * t) % 200 + 20 + rng.integers(0, 12, (H16, W16))
                   + ((xx - 900 - 4 * t) ** 2 + (yy - 540) ** 2 < 300 ** 2) * ((xx * yy) % 37))
                  for t in range(F)]).clip(1, 254).astype(np.uint8)
    yc, xc = np.mgrid[0:H16 // 2, 0:W16 // 2]
    cb = np.stack([(xc // 3 + 2 * yc // 5 + t) % 150 + 50 for t in range(F)]).astype(np.uint8)
    cr = np.stack([(xc // 4 + yc // 2 + 3 * t) % 160 + 40 for t in range(F)]).astype(np.uint8)
    dev = torch.device("cuda", 0)
    tp = [torch.from_numpy(p).to(dev) for p in (y, cb, cr)]
    ops.h264_intra_encode(*tp, INTRA_QP)
    torch.cuda.synchronize()
    from arbius_amd.ops import _lib
    _lib.lib().arb_set_h264_sync(1)             # agent-scope hand-off between diagonals (A/B)
    agent = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.h264_intra_encode(*tp, INTRA_QP)
        e1.record()
        e1.synchronize()
        agent.append(e0.elapsed_time(e1))
    _lib.lib().arb_set_h264_sync(0)
    times = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out, meta = ops.h264_intra_encode(*tp, INTRA_QP)
        e1.record()
        e1.synchronize()
        times.append(e0.elapsed_time(e1))
    m = meta.cpu().numpy()
    buf = out[:int(m[F])].cpu().numpy()
    c0 = time.process_time()
    t0 = time.perf_counter()
    nals = native.h264_nals_from_rbsp(buf, m, F, 1)
    tail_s = time.perf_counter() - t0
    tail_cpu = time.process_time() - c0
    c0 = time.process_time()
    t0 = time.perf_counter()
    _, _, ref1 = native.h264_encode_yuv420_frames(y, cb, cr, W16, H16, INTRA_QP, 1)
    host1_s = time.perf_counter() - t0
    host1_cpu = time.process_time() - c0
    t0 = time.perf_counter()
    _, _, refn = native.h264_encode_yuv420_frames(y, cb, cr, W16, H16, INTRA_QP, a.threads)
    hostn_s = time.perf_counter() - t0
    print(json.dumps({"frames": F, "size": [W16, H16], "gpu_encode_ms": round(min(times), 2),
                      "gpu_encode_ms_all": [round(t, 2) for t in times],
                      "gpu_encode_ms_agent_sync": round(min(agent), 2), "host_tail_ms": round(tail_s * 1e3, 2),
                      "host_tail_cpu_ms": round(tail_cpu * 1e3, 2), "native_1thread_s": round(host1_s, 3),
                      "native_1thread_cpu_s": round(host1_cpu, 3), f"native_{a.threads}threads_s": round(hostn_s, 3),
                      "bytes": int(sum(len(n) for n in nals)), "equal": nals == ref1 == refn}), flush=True)


if __name__ == "__main__":
    main()
