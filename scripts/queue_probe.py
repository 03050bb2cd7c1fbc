#!/usr/bin/env python3
"""Do HIP streams that share a hardware queue run their kernels one after the other?

HIP maps every stream onto one of GPU_MAX_HW_QUEUES (default 4) HSA queues per process; past
that count a new stream shares the least-used queue.  A HIP dispatch packet carries the AQL
barrier bit (in-order stream semantics), so two streams on ONE queue cannot overlap their kernels
even when the CUs are idle.  This probe measures it directly with a one-workgroup spin kernel
(``torch.cuda._sleep``, occupies one CU for a fixed cycle count):

  * pool: k = 1..8 streams from PyTorch's pool (in creation order), one spin kernel each,
    all launched back to back; wall / single-kernel time = how many ran one after another.
  * forks: the same test on the streams of C pipeline forks of the real model (as the node and
    bench.py create them, after one warm-up solve per fork so every side stream exists).

    python scripts/queue_probe.py [--forks 4] [--model anythingv3]
Prints one JSON line per measurement.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def spin_wall(torch, streams, cycles, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in streams:
            with torch.cuda.stream(s):
                torch.cuda._sleep(cycles)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--forks", type=int, default=0)
    ap.add_argument("--model", default="anythingv3")
    ap.add_argument("--cycles", type=int, default=50_000_000)
    a = ap.parse_args()
    import torch
    print(json.dumps({"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}), flush=True)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    one = spin_wall(torch, [torch.cuda.current_stream()], a.cycles)
    print(json.dumps({"probe": "single", "ms": round(one * 1e3, 2)}), flush=True)
    if a.forks <= 0:
        pool = [torch.cuda.Stream() for _ in range(8)]
        for k in range(1, 9):
            w = spin_wall(torch, pool[:k], a.cycles)
            print(json.dumps({"probe": "pool", "streams": k, "ms": round(w * 1e3, 2),
                              "serial_rounds": round(w / one, 2)}), flush=True)
        return
    import bench
    from arbius_amd.models.registry import build_pipeline
    from arbius_amd.node.solver import infer_images
    args = bench.parse_args(["--model", a.model, "--concurrent", str(a.forks), "--steps", "1", "--warmup", "1"])
    pipe = build_pipeline(a.model, device=dev, init=True, use_graphs=True)
    forks = [pipe.fork() for _ in range(a.forks)]
    for j, f in enumerate(forks):      # one small solve per fork: captures, side streams, VAE
        inps = [{"prompt": f"probe {j}.{g}", "negative_prompt": "", "width": args.res, "height": args.res,
                 "num_inference_steps": 2, "guidance_scale": 7.0, "scheduler": "DPMSolverMultistep",
                 "seed": 1 + g} for g in range(4)]
        infer_images(f, inps)
    torch.cuda.synchronize()
    for k in range(1, a.forks + 1):
        w = spin_wall(torch, [f.stream for f in forks[:k]], a.cycles)
        print(json.dumps({"probe": "forks", "streams": k, "ms": round(w * 1e3, 2),
                          "serial_rounds": round(w / one, 2)}), flush=True)
    # the forks' streams beside the default stream (which the text graphs' warm-up used)
    w = spin_wall(torch, [torch.cuda.default_stream()] + [f.stream for f in forks], a.cycles)
    print(json.dumps({"probe": "forks+default", "streams": a.forks + 1, "ms": round(w * 1e3, 2),
                      "serial_rounds": round(w / one, 2)}), flush=True)


if __name__ == "__main__":
    main()
