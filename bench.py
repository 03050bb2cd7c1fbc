#!/usr/bin/env python3
"""Headline benchmark: tasks solved / hour (whole node) + p50 task latency,
anythingv3 (SD1.5 architecture) 512x512, 50 denoising steps (BASELINE.json).

One "step" = every rank solves ONE complete task end to end: CLIP text encode,
50 CFG (batch 2) UNet evaluations + sampler, VAE decode, deterministic PNG
encode, wrapped-directory CIDv0 and the solution commitment.  Synthetic
prompts, random-init weights of the real architecture (no checkpoints offline).

N GPUs = N independent task workers (task-level data parallel, weak scaling);
rank 0 initialises the weights and RCCL-broadcasts them over xGMI (outside the
timed region, reported separately).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="anythingv3",
                    choices=["anythingv3", "kandinsky2", "zeroscopev2xl", "damo", "robust_video_matting"],
                    help="anythingv3 = BASELINE headline config; kandinsky2 = config #3; zeroscopev2xl = #4; "
                         "robust_video_matting = #5 (1080p clip per task)")
    ap.add_argument("--frames", type=int, default=None,
                    help="video models: frames (config #4: 24); matting: clip length (default 48 = 2 s at 24 fps)")
    ap.add_argument("--concurrent", type=int, default=2,
                    help="tasks solved concurrently per GPU (pipeline forks on private HIP streams)")
    ap.add_argument("--group", type=int, default=4,
                    help="SD family: tasks solved lock-step per stream (one batch-2k UNet launch sequence; "
                         "batch-invariant plans keep every CID equal to its solo solve)")
    ap.add_argument("--res", type=int, default=None, help="default 512 (anythingv3) / 768 (kandinsky2)")
    ap.add_argument("--denoise-steps", type=int, default=None, help="default 50 / 100")
    ap.add_argument("--scheduler", default="DPMSolverMultistep")
    ap.add_argument("--guidance", type=float, default=12.0)
    ap.add_argument("--reference-ops", action="store_true", help="A/B: PyTorch ops instead of HIP kernels")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--tiny", action="store_true", help="tiny config (CPU plumbing check only)")
    ap.add_argument("--device", default=None)
    args = ap.parse_args()
    k2 = args.model == "kandinsky2"
    vid = args.model in ("zeroscopev2xl", "damo")
    rvm = args.model == "robust_video_matting"
    args.frames = args.frames or (48 if rvm else 24)
    args.res = args.res or (768 if k2 else 576 if args.model == "zeroscopev2xl" else 256 if vid else
                            1920 if rvm else 512)
    args.height = 320 if args.model == "zeroscopev2xl" else 1080 if rvm else args.res
    args.denoise_steps = args.denoise_steps or (100 if k2 else 50)

    from arbius_amd import ops
    from arbius_amd.models.registry import build_pipeline
    from arbius_amd.node.solver import solve_image
    from arbius_amd.parallel import dist as D
    from arbius_amd.utils.protocol import generate_commitment, taskid2seed
    from arbius_amd.utils.keccak import keccak256

    if args.reference_ops:
        ops.set_reference_ops(True)
    dev_type = "cuda" if (args.device or ("cuda" if torch.cuda.is_available() else "cpu")).startswith("cuda") else "cpu"
    rank, local, world, dev = D.init(device_type=dev_type)
    n = world

    t_init = time.perf_counter()
    pipe = build_pipeline(args.model, device=dev, tiny=args.tiny, init=(rank == 0),
                          use_graphs=(dev.type == "cuda" and not args.no_graphs))
    bstats = D.broadcast_modules(pipe.modules().values())
    t_init = time.perf_counter() - t_init

    wallet = "0x" + "11" * 20
    lat = []
    C = max(1, args.concurrent) if hasattr(pipe, "fork") else 1
    forks = [pipe.fork() for _ in range(C)] if C > 1 else [pipe]

    if rvm:   # BASELINE config #5: a synthetic 1080p clip (moving gradient + noise), green-screen output
        import numpy as np
        rng = np.random.default_rng(1234 + rank)
        yy, xx = np.mgrid[0:args.height, 0:args.res]
        base = ((xx[None] + 7 * np.arange(args.frames)[:, None, None]) % 256).astype(np.uint8)
        clip = np.stack([base, (yy[None] % 256).astype(np.uint8).repeat(args.frames, 0),
                         rng.integers(0, 256, base.shape, dtype=np.uint8)], axis=-1)

    def one_task(i, pipe=pipe):
        taskid = "0x" + keccak256(f"bench-task-{rank}-{i}".encode()).hex()
        if rvm:
            from arbius_amd.node.solver import solve_files
            from arbius_amd.utils.mp4 import encode_mp4
            t0 = time.perf_counter()
            out = pipe(clip, "green-screen")
            t1 = time.perf_counter()
            tm = dict(pipe.timings)
            tm.update({"infer_s": t1 - t0})
            sol = solve_files([("out-1.mp4", encode_mp4(list(out), 24))], tm)
            sol.timings["encode_cid_s"] = time.perf_counter() - t1
            generate_commitment(wallet, taskid, sol.cid)
            lat.append(time.perf_counter() - t0)
            return sol
        if vid:  # BASELINE config #4: 576x320x24f text-to-video
            inp = {"prompt": f"a red cat walking on a castle wall, cinematic, task {i}", "num_frames": args.frames,
                   "width": args.res, "height": args.height, "num_inference_steps": args.denoise_steps,
                   "seed": taskid2seed(taskid), "fps": 24}
            t0 = time.perf_counter()
            sol = pipe.solve(inp)
            generate_commitment(wallet, taskid, sol.cid)
            lat.append(time.perf_counter() - t0)
            return sol
        if k2 and args.group > 1:
            from arbius_amd.node.solver import solve_images
            pipe.cfg.num_steps = args.denoise_steps
            inps = []
            for j in range(args.group):
                tid = "0x" + keccak256(f"bench-task-{rank}-{i}-{j}".encode()).hex()
                inps.append({"prompt": f"a red cat sitting on a castle wall, oil painting, task {i}.{j}",
                             "width": args.res, "height": args.res, "seed": taskid2seed(tid)})
            t0 = time.perf_counter()
            sols = solve_images(pipe, inps)
            for sol in sols:
                generate_commitment(wallet, taskid, sol.cid)
            lat.extend([time.perf_counter() - t0] * len(sols))
            return sols[-1]
        if k2:   # templates/kandinsky2.json inputs; hidden defaults 100 steps, guidance 4, prior 5 steps
            pipe.cfg.num_steps = args.denoise_steps
            inp = {"prompt": f"a red cat sitting on a castle wall, oil painting, task {i}",
                   "width": args.res, "height": args.res, "seed": taskid2seed(taskid)}
            t0 = time.perf_counter()
            sol = pipe.solve(inp)
            generate_commitment(wallet, taskid, sol.cid)
            lat.append(time.perf_counter() - t0)
            return sol
        if args.group > 1:
            from arbius_amd.node.solver import solve_images
            inps = []
            for j in range(args.group):
                tid = "0x" + keccak256(f"bench-task-{rank}-{i}-{j}".encode()).hex()
                inps.append({"prompt": f"a detailed anime illustration of a castle on a hill, task {i}.{j}",
                             "negative_prompt": "lowres, bad anatomy, bad hands, text, error",
                             "width": args.res, "height": args.res, "num_inference_steps": args.denoise_steps,
                             "guidance_scale": args.guidance, "scheduler": args.scheduler,
                             "seed": taskid2seed(tid)})
            t0 = time.perf_counter()
            sols = solve_images(pipe, inps)
            for j, sol in enumerate(sols):
                generate_commitment(wallet, taskid, sol.cid)
            dt = time.perf_counter() - t0
            lat.extend([dt] * len(sols))
            return sols[-1]
        inp = {
            "prompt": f"a detailed anime illustration of a castle on a hill, task {i}",
            "negative_prompt": "lowres, bad anatomy, bad hands, text, error",
            "width": args.res, "height": args.res,
            "num_inference_steps": args.denoise_steps,
            "guidance_scale": args.guidance,
            "scheduler": args.scheduler,
            "seed": taskid2seed(taskid),
        }
        t0 = time.perf_counter()
        sol = solve_image(pipe, inp)
        generate_commitment(wallet, taskid, sol.cid)
        lat.append(time.perf_counter() - t0)
        return sol

    from concurrent.futures import ThreadPoolExecutor
    ex = ThreadPoolExecutor(C) if C > 1 else None

    def one_step(i):
        """One bench step = C tasks, concurrently on C pipeline forks (C = 1: one task)."""
        if ex is None:
            return one_task(i)
        futs = [ex.submit(one_task, i * C + j, forks[j]) for j in range(C)]
        return [f.result() for f in futs][-1]

    for i in range(args.warmup):
        if ex is None:
            one_task(-1 - i)
        else:               # capture every fork's graphs once, one after the other
            for j in range(C):
                one_task(-1 - i * C - j, forks[j])
    lat.clear()
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    D.barrier(dev)
    sync()
    t0 = time.perf_counter()
    last = None
    for i in range(args.steps):
        last = one_step(i)
    sync()
    D.barrier(dev)
    elapsed = time.perf_counter() - t0
    ms_per_step = D.max_over_ranks(elapsed * 1000.0 / args.steps, dev)
    all_lat = D.all_gather_floats(lat, dev)
    flat = sorted(x for r in all_lat for x in r)
    p50 = statistics.median(flat) * 1000.0 if flat else float("nan")

    if rank == 0:
        G = args.group if not (vid or rvm) else 1
        tasks_per_hour = n * C * G * 3600.0 * 1000.0 / ms_per_step
        out = {
            "metric": "tasks_solved_per_hour",
            "value": round(tasks_per_hour, 2),
            "unit": "tasks/hour",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("fp16" if rvm else "bf16") if dev.type == "cuda" else "fp32",
            "data": ("synthetic 1080p clip, random-init weights (RVM MobileNetV3 architecture)" if rvm else
                     "synthetic prompts, random-init weights (%s architecture)" % (
                         "Kandinsky 2.1" if k2 else "UNet3D text-to-video" if vid else "SD1.5")),
            "config": {
                "model": ("robust_video_matting (MobileNetV3 + LR-ASPP + ConvGRU decoder + DGF), "
                          f"{args.frames}-frame {args.res}x{args.height} clip" if rvm else
                          "kandinsky2 (Kandinsky 2.1: prior + GLIDE UNet + MoVQ + XLM-R/CLIP text)" if k2 else
                          f"{args.model} (UNet3D + KL-VAE + OpenCLIP ViT-H text), {args.frames} frames" if vid else
                          "anythingv3 (SD1.5 UNet + KL-VAE + CLIP ViT-L/14 text)") + (" TINY" if args.tiny else ""),
                "global_batch": n * C * G,
                "concurrent_tasks_per_gpu": C * G,
                "streams_per_gpu": C,
                "lockstep_group": G,
                "seq_len": (args.res // 8) * (args.height // 8),
                "resolution": f"{args.res}x{args.height}" if (vid or rvm) else args.res,
                "denoise_steps": None if rvm else args.denoise_steps,
                "scheduler": None if rvm else "p_sampler" if k2 else "DPMSolverMultistep" if vid else args.scheduler,
                "cfg_batch": 1 if rvm else 2,
                "parallelism": f"task-dp{n}",
            },
            "p50_task_latency_ms": round(p50, 2),
            **({"frames_per_second": round(n * C * args.frames * 1000.0 / ms_per_step, 1)} if (rvm or vid) else {}),
            "stage_s": {k: round(v, 4) for k, v in (last.timings.items() if last else [])},
            "weight_broadcast": {"bytes": bstats["bytes"], "seconds": round(bstats["seconds"], 4)},
            "init_s": round(t_init, 2),
            "native_kernels_loaded": ops.native_loaded(),
            "reference_ops": bool(args.reference_ops),
        }
        print(json.dumps(out), flush=True)
    if D.is_dist():
        import torch.distributed as tdist
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
