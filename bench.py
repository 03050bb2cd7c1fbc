#!/usr/bin/env python3
"""Headline benchmark: tasks solved / hour (whole node) + p50 task latency,
anythingv3 (SD1.5 architecture) 512x512, 50 denoising steps (BASELINE.json).

One "step" = every rank solves its task slots end to end: CLIP text encode,
50 CFG (batch 2) UNet evaluations + sampler, VAE decode, deterministic PNG
encode, wrapped-directory CIDv0 and the solution commitment.  Synthetic
prompts, random-init weights of the real architecture (no checkpoints offline;
``--weights-dir`` loads real safetensors on rank 0 instead).

N GPUs = N independent task workers, one process per GPU (task-level data
parallel, weak scaling).  Rank 0 materialises the weights (random init or
safetensors) and RCCL-broadcasts them over xGMI to every other rank (outside the
timed region, reported as ``weight_broadcast``).  There are no per-step
collectives; the timed region is bracketed by a barrier + device sync on both
sides and ms/step is the MAX over ranks.

  python bench.py [--gpus N] [--steps K] [--warmup W]      # N > 1: spawns N rank processes
  torchrun --nproc-per-node N bench.py --gpus N ...         # one rank per process (driver path)
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse_args(argv=None):
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
    ap.add_argument("--concurrent", type=int, default=None,
                    help="task streams per GPU (pipeline forks on private HIP streams); default: the node's "
                         "(mi355x.workers_per_gpu = 4, capped per model by mi355x.model_streams: anythingv3 3, "
                         "kandinsky2 2, video / matting 2)")
    ap.add_argument("--group", type=int, default=None,
                    help="image models: tasks solved lock-step per stream (one batch-2k UNet launch sequence; "
                         "batch-invariant plans keep every CID equal to its solo solve); default: the node's "
                         "(mi355x.model_lockstep: 8 for anythingv3 / kandinsky2, else mi355x.lockstep_group = 4)")
    ap.add_argument("--res", type=int, default=None, help="default 512 (anythingv3) / 768 (kandinsky2)")
    ap.add_argument("--height", type=int, default=None,
                    help="image height when it differs from --res (default: --res; zeroscope 320, matting 1080)")
    ap.add_argument("--denoise-steps", type=int, default=None, help="default 50 / 100")
    ap.add_argument("--scheduler", default="DPMSolverMultistep")
    ap.add_argument("--guidance", type=float, default=12.0)
    ap.add_argument("--weights-dir", default=None, help="safetensors dir (rank 0 loads, RCCL-broadcast)")
    ap.add_argument("--reference-ops", action="store_true", help="A/B: PyTorch ops instead of HIP kernels")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--tiny", action="store_true", help="tiny config (CPU plumbing check only)")
    ap.add_argument("--device", default=None, help="cuda (default when a GPU is visible) or cpu (gloo ranks)")
    ap.add_argument("--rccl-group", action="store_true",
                    help="form the process group at N = 1 too: the weight broadcast then runs through a one-rank "
                         "RCCL communicator (the multi-GPU code path, exercised on one GPU)")
    ap.add_argument("--node", action="store_true",
                    help="whole-node mode: tasks flow through the node's own stack (MockEngine events -> "
                         "orchestrator -> solver pool -> commit/submit); one process, N GPU worker processes")
    ap.add_argument("--dispatch-sim", action="store_true",
                    help="no GPU: the multi-GPU dispatch model (parallel/dispatch.py) under Poisson arrival at "
                         "25/50/75/100 %% of node capacity, spread vs pack policy (one JSON line per point)")
    ap.add_argument("--node-outstanding", type=int, default=0,
                    help="--node: tasks kept in flight (default 2 x pool capacity: a saturated node)")
    args = ap.parse_args(argv)
    from arbius_amd.config.mining_config import DEFAULT_MODEL_LOCKSTEP, DEFAULT_MODEL_STREAMS, MI355XConfig
    # no --concurrent / --group: the node's shipped pool config (node bench: workers_per_gpu slots, capped
    # per model by model_streams, model_lockstep groups - e.g. anythingv3 4 slots on 3 forks x groups of 8)
    args.shipped_pool = args.concurrent is None and args.group is None
    if args.concurrent is None:
        args.concurrent = DEFAULT_MODEL_STREAMS.get(args.model, MI355XConfig().workers_per_gpu)
    if args.group is None:
        args.group = DEFAULT_MODEL_LOCKSTEP.get(args.model, MI355XConfig().lockstep_group)
    k2 = args.model == "kandinsky2"
    vid = args.model in ("zeroscopev2xl", "damo")
    rvm = args.model == "robust_video_matting"
    args.frames = args.frames or (48 if rvm else 24)
    args.res = args.res or (768 if k2 else 576 if args.model == "zeroscopev2xl" else 256 if vid else
                            1920 if rvm else 512)
    args.height = args.height or (320 if args.model == "zeroscopev2xl" else 1080 if rvm else args.res)
    args.denoise_steps = args.denoise_steps or (100 if k2 else 50)
    return args


def _device_type(args) -> str:
    """cuda / cpu WITHOUT initialising HIP (device_count does not; is_available may)."""
    if args.device:
        return "cuda" if args.device.startswith("cuda") else "cpu"
    import torch
    return "cuda" if torch.cuda.device_count() > 0 else "cpu"


def run(args):
    dump = float(os.environ.get("ARBIUS_BENCH_STACKDUMP", "0") or 0)
    if dump > 0:        # diagnosis of a stalled run: every thread's Python stack to stderr periodically
        import faulthandler
        faulthandler.dump_traceback_later(dump, repeat=True, file=sys.stderr)
    import torch

    from arbius_amd import ops
    from arbius_amd.models import graphs
    from arbius_amd.models.registry import build_pipeline
    from arbius_amd.node.solver import solve_image
    from arbius_amd.parallel import dist as D
    from arbius_amd.utils.keccak import keccak256
    from arbius_amd.utils.protocol import generate_commitment, taskid2seed

    k2 = args.model == "kandinsky2"
    vid = args.model in ("zeroscopev2xl", "damo")
    rvm = args.model == "robust_video_matting"
    if args.reference_ops:
        ops.set_reference_ops(True)
    rank, local, world, dev = D.init(device_type=_device_type(args), force_group=args.rccl_group)
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the process group has {world} ranks")
    if world > 1:
        # N ranks share the host: keep each rank's CPU-side work (tokenizer, noise, PNG) off the
        # other ranks' cores
        torch.set_num_threads(max(1, min(torch.get_num_threads(), 4)))
    n = world

    t_init = time.perf_counter()
    src = rank == 0
    pipe = build_pipeline(args.model, device=dev, tiny=args.tiny, init=src and not args.weights_dir,
                          weights_dir=args.weights_dir if src else None,
                          tokenizer_dir=args.weights_dir,
                          use_graphs=(dev.type == "cuda" and not args.no_graphs))
    winfo = D.world_info(dev)
    if rank == 0:
        print(f"[bench] world: {json.dumps(winfo)}", file=sys.stderr, flush=True)
    if os.environ.get("ARBIUS_FAULT_INJECTION") == "1" and os.environ.get("ARBIUS_FAULT_BCAST_DIE_RANK") == str(rank):
        os._exit(17)        # test hook: a rank lost right before / during the weight broadcast
    bstats = D.broadcast_modules(pipe.modules().values())
    if hasattr(pipe, "_reset_graphs"):
        pipe._reset_graphs()
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

    def tid_of(i, j=None):
        return "0x" + keccak256((f"bench-task-{rank}-{i}" + ("" if j is None else f"-{j}")).encode()).hex()

    def finish_group(t0, tids, imgs, tm):
        """CPU tail of a lock-step group (PNG + CID of every image, commitments): runs on the slot's
        tail thread while the slot's stream already solves its next group, as the node's pools do."""
        from arbius_amd.node.solver import encode_images
        sols = encode_images(imgs, tm)
        for tid, sol in zip(tids, sols):
            generate_commitment(wallet, tid, sol.cid)
        lat.extend([time.perf_counter() - t0] * len(sols))
        return sols[-1]

    def finish_clip(t0, tid, raw):
        """CPU tail of an RVM task: MP4 encode + CID + commitment."""
        sol = type(pipe).finish(raw)
        generate_commitment(wallet, tid, sol.cid)
        lat.append(time.perf_counter() - t0)
        return sol

    def one_task(i, pipe=pipe, tail=None):
        """Solve this slot's task(s) of step i; every solution gets its own task id's commitment.
        ``tail``: executor for a lock-step group's CPU tail (returns its future)."""
        t0 = time.perf_counter()
        if rvm:
            # the node's two-phase solve (node/solver.py infer_task): matting on the slot's stream,
            # then the H.264 encode + CID (RVMPipeline.finish, CPU only) on the slot's tail thread
            # while the stream mattes the next clip
            out = pipe.matte_for_encode(clip, "green-screen")      # as RVMPipeline.infer
            tm = dict(pipe.timings)
            tm.update({"infer_s": time.perf_counter() - t0})
            raw = (out, 24, tm)
            if tail is not None:
                return tail.submit(finish_clip, t0, tid_of(i), raw)
            return finish_clip(t0, tid_of(i), raw)
        elif vid:  # BASELINE config #4: 576x320x24f text-to-video
            inp = {"prompt": f"a red cat walking on a castle wall, cinematic, task {i}", "num_frames": args.frames,
                   "width": args.res, "height": args.height, "num_inference_steps": args.denoise_steps,
                   "seed": taskid2seed(tid_of(i)), "fps": 24}
            done = [(tid_of(i), pipe.solve(inp))]
        elif k2:   # templates/kandinsky2.json inputs; hidden defaults 100 steps, guidance 4, prior 5 steps
            from arbius_amd.node.solver import solve_images
            pipe.cfg.num_steps = args.denoise_steps
            tids = [tid_of(i, j) for j in range(max(1, args.group))]
            inps = [{"prompt": f"a red cat sitting on a castle wall, oil painting, task {i}.{j}",
                     "width": args.res, "height": args.height, "seed": taskid2seed(t)} for j, t in enumerate(tids)]
            if tail is not None and len(inps) > 1:
                from arbius_amd.node.solver import infer_images
                return tail.submit(finish_group, t0, tids, *infer_images(pipe, inps))
            done = list(zip(tids, solve_images(pipe, inps) if len(inps) > 1 else [pipe.solve(inps[0])]))
        else:
            from arbius_amd.node.solver import solve_images
            tids = [tid_of(i, j) for j in range(max(1, args.group))]
            inps = [{"prompt": f"a detailed anime illustration of a castle on a hill, task {i}.{j}",
                     "negative_prompt": "lowres, bad anatomy, bad hands, text, error",
                     "width": args.res, "height": args.height, "num_inference_steps": args.denoise_steps,
                     "guidance_scale": args.guidance, "scheduler": args.scheduler,
                     "seed": taskid2seed(t)} for j, t in enumerate(tids)]
            if tail is not None and len(inps) > 1:
                from arbius_amd.node.solver import infer_images
                return tail.submit(finish_group, t0, tids, *infer_images(pipe, inps))
            sols = solve_images(pipe, inps) if len(inps) > 1 else [solve_image(pipe, inps[0])]
            done = list(zip(tids, sols))
        for tid, sol in done:
            generate_commitment(wallet, tid, sol.cid)
        dt = time.perf_counter() - t0
        lat.extend([dt] * len(done))
        return done[-1][1]

    from concurrent.futures import ThreadPoolExecutor
    ex = ThreadPoolExecutor(C) if C > 1 else None

    def one_step(i):
        """One bench step = C task slots, concurrently on C pipeline forks (C = 1: one slot)."""
        if ex is None:
            return one_task(i)
        futs = [ex.submit(one_task, i * C + j, forks[j]) for j in range(C)]
        return [f.result() for f in futs][-1]

    def progress(msg):      # stderr heartbeat: long steps (video models) must not look hung
        print(f"[bench rank {rank}] {msg} ({time.perf_counter() - t_start:.1f} s)", file=sys.stderr, flush=True)

    t_start = time.perf_counter()
    for i in range(args.warmup):
        if ex is None:
            one_task(-1 - i)
        else:               # capture every fork's graphs once, one after the other
            for j in range(C):
                one_task(-1 - i * C - j, forks[j])
                progress(f"warmup {i} slot {j} done")
        progress(f"warmup {i} done")
    lat.clear()
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    D.barrier(dev)
    sync()
    t0 = time.perf_counter()
    cpu0 = os.times()          # host CPU seconds of this process (every thread) over the timed region
    marks = os.environ.get("ARB_BENCH_MARKS") == "1"   # timed-region bounds on the trace clocks
    if marks:
        print(f"[bench] timed t0 monotonic_ns={time.monotonic_ns()} "
              f"boottime_ns={time.clock_gettime_ns(time.CLOCK_BOOTTIME)}", file=sys.stderr, flush=True)
    if os.environ.get("ARB_DUMP_MAPS"):     # library load addresses: symbolise a native crash stack offline
        with open("/proc/self/maps") as src, open(os.environ["ARB_DUMP_MAPS"], "w") as dst:
            dst.write(src.read())
    last = None
    if ex is None:
        for i in range(args.steps):
            last = one_step(i)
            progress(f"step {i} done")
    else:
        # C free-running task slots (as the node's scheduler runs them): each fork solves its K
        # tasks back to back, so one slot's CPU tail (PNG / MP4 encode + CID) overlaps the other
        # slots' GPU work instead of every slot idling the GPU at a per-step join.  Same K x C tasks.
        # A lock-step group's CPU tail (PNG + CID) runs on the slot's tail thread while the slot's
        # stream solves its next group; the clock stops only after every tail finished.
        from concurrent.futures import Future, ThreadPoolExecutor as _TPE
        tails = [_TPE(max_workers=1) for _ in range(C)]

        def run_slot(j):
            r = None
            for i in range(args.steps):
                r = one_task(i * C + j, forks[j], tails[j])
                progress(f"slot {j} task {i} done")
            return r.result() if isinstance(r, Future) else r
        futs = [ex.submit(run_slot, j) for j in range(C)]
        last = [f.result() for f in futs][-1]
        for tp in tails:
            tp.shutdown(wait=True)
    sync()
    D.barrier(dev)
    elapsed = time.perf_counter() - t0
    cpu1 = os.times()
    my_cpu_s = (cpu1.user - cpu0.user) + (cpu1.system - cpu0.system)
    if marks:
        print(f"[bench] timed t1 monotonic_ns={time.monotonic_ns()} "
              f"boottime_ns={time.clock_gettime_ns(time.CLOCK_BOOTTIME)}", file=sys.stderr, flush=True)
    my_ms = elapsed * 1000.0 / args.steps
    ms_per_step = D.max_over_ranks(my_ms, dev)
    all_lat = D.all_gather_floats(lat, dev)
    per_rank = D.all_gather_floats([my_ms, float(len(lat)), float(bstats["bytes"]), my_cpu_s], dev)
    flat = sorted(x for r in all_lat for x in r)
    p50 = statistics.median(flat) * 1000.0 if flat else float("nan")

    if rank == 0:
        G = max(1, args.group) if not (vid or rvm) else 1
        per_gpu_tasks = C * G
        tasks_per_hour = n * per_gpu_tasks * 3600.0 * 1000.0 / ms_per_step
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
            "data": ("synthetic 1080p clip, " if rvm else "synthetic prompts, ") + (
                f"safetensors weights ({os.path.basename(os.path.normpath(args.weights_dir))})"
                if args.weights_dir else "random-init weights") + " (%s architecture)" % (
                "RVM MobileNetV3" if rvm else "Kandinsky 2.1" if k2 else "UNet3D text-to-video" if vid else "SD1.5"),
            "config": {
                "model": ("robust_video_matting (MobileNetV3 + LR-ASPP + ConvGRU decoder + DGF), "
                          f"{args.frames}-frame {args.res}x{args.height} clip" if rvm else
                          "kandinsky2 (Kandinsky 2.1: prior + GLIDE UNet + MoVQ + XLM-R/CLIP text)" if k2 else
                          f"{args.model} (UNet3D + KL-VAE + OpenCLIP ViT-H text), {args.frames} frames" if vid else
                          "anythingv3 (SD1.5 UNet + KL-VAE + CLIP ViT-L/14 text)") + (" TINY" if args.tiny else ""),
                "global_batch": n * per_gpu_tasks,
                "concurrent_tasks_per_gpu": per_gpu_tasks,
                "streams_per_gpu": C,
                "lockstep_group": G,
                "seq_len": (args.res // 8) * (args.height // 8),
                "resolution": f"{args.res}x{args.height}" if (vid or rvm or args.height != args.res) else args.res,
                "denoise_steps": None if rvm else args.denoise_steps,
                "scheduler": None if rvm else "p_sampler" if k2 else "DPMSolverMultistep" if vid else args.scheduler,
                "cfg_batch": 1 if rvm else 2,
                "parallelism": f"dp{n}",
                "parallelism_detail": f"task-level data parallel: {n} independent worker process(es), "
                                      "one per GPU, weights broadcast from rank 0, no per-step collectives",
            },
            "p50_task_latency_ms": round(p50, 2),
            "per_rank": [{"rank": r, "ms_per_step": round(v[0], 2), "tasks": int(v[1]),
                          "tasks_per_hour": round(per_gpu_tasks * 3600.0 * 1000.0 / v[0], 2),
                          "weight_broadcast_bytes": int(v[2]),
                          "host_cpu_s_per_task": round(v[3] / max(1.0, v[1]), 3),
                          "host_cores_busy": round(v[3] * 1000.0 / (v[0] * args.steps), 2)}
                         for r, v in enumerate(per_rank)],
            **({"frames_per_second": round(n * C * args.frames * 1000.0 / ms_per_step, 1)} if (rvm or vid) else {}),
            "stage_s": {k: round(v, 4) for k, v in (last.timings.items() if last else [])},
            "weight_broadcast": {"bytes": int(max(v[2] for v in per_rank)), "seconds": round(bstats["seconds"], 4),
                                 "backend": D.backend_name()},
            "world": winfo,
            "init_s": round(t_init, 2),
            "peak_hbm_gb": round(torch.cuda.max_memory_allocated(dev) / 2**30, 2) if dev.type == "cuda" else None,
            "native_kernels_loaded": ops.native_loaded(),
            "reference_ops": bool(args.reference_ops),
            "task_stream_queue_check": dict(graphs.QUEUE_STATS),
        }
        print(json.dumps(out), flush=True)
    if ex is not None:
        ex.shutdown()
    D.shutdown()


def run_node(args):
    """``--node``: the node as shipped (arbius_amd/node/nodebench.py) instead of bare pipeline loops."""
    from arbius_amd import ops
    from arbius_amd.node.nodebench import run_node_bench
    dev = _device_type(args)
    device = "cuda:0" if dev == "cuda" else "cpu"
    if args.reference_ops:
        ops.set_reference_ops(True)
    r = run_node_bench(args, device)
    per_step_ms = r["elapsed_s"] * 1000.0 / args.steps
    k2 = args.model == "kandinsky2"
    out = {
        "metric": "tasks_solved_per_hour",
        "value": round(r["tasks"] * 3600.0 / r["elapsed_s"], 2),
        "unit": "tasks/hour",
        "n_gpus": args.gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(per_step_ms, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if dev == "cuda" else "fp32",
        "data": "synthetic prompts submitted to an in-process MockEngine, random-init weights" + (
            " (TINY)" if args.tiny else ""),
        "config": {"model": args.model + (" TINY" if args.tiny else ""), "mode": "node",
                   "global_batch": r["capacity"], "seq_len": (args.res // 8) * (args.height // 8),
                   "resolution": args.res, "denoise_steps": args.denoise_steps,
                   "scheduler": "p_sampler" if k2 else args.scheduler, "cfg_batch": 2,
                   "streams_per_gpu": args.concurrent, "lockstep_group": args.group,
                   "parallelism": f"dp{args.gpus}",
                   "parallelism_detail": "node stack: event poll -> task/solve jobs -> solver pool -> "
                                         "commit/submit; pool slots = GPUs x streams x lock-step group"},
        "p50_task_latency_ms": round(r["p50_s"] * 1000.0, 2),
        "p90_task_latency_ms": round(r["p90_s"] * 1000.0, 2),
        "tasks_timed": r["tasks"],
        "pool_capacity": r["capacity"],
        "tasks_outstanding": r["outstanding"],
        "pins_ok": r["pins_ok"],
        "jobs": r["jobs"],
        "stage_p50_s": r["stage_p50_s"],
        "init_s": round(r["init_s"], 2),
        "native_kernels_loaded": ops.native_loaded(),
    }
    print(json.dumps(out), flush=True)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank: int, world: int, port: int, argv):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    run(parse_args(argv))


def spawn(argv, world: int) -> int:
    """``python bench.py --gpus N`` without torchrun: N fresh rank processes (spawn context - the
    parent never touches the GPU).  A rank that fails takes the others down (they would wait in
    the next collective forever); the exit code is the first failure's."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, argv), daemon=False) for r in range(world)]
    for p in procs:
        p.start()
    rc = 0
    while any(p.is_alive() for p in procs):
        for p in procs:
            p.join(0.2)
            if p.exitcode not in (None, 0) and rc == 0:
                rc = p.exitcode if p.exitcode > 0 else 1
                for q in procs:
                    if q.is_alive():
                        q.terminate()
    for p in procs:
        p.join()
        if p.exitcode not in (0, None) and rc == 0:
            rc = p.exitcode if p.exitcode > 0 else 1
    return rc


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.dispatch_sim:
        from arbius_amd.parallel.dispatch import SERVICE_MODELS, node_capacity_per_s, simulate
        n = max(1, args.gpus)
        sm = SERVICE_MODELS.get(args.model)
        if sm is None:
            raise SystemExit(f"--dispatch-sim: no service model for {args.model} ({sorted(SERVICE_MODELS)})")
        cap = node_capacity_per_s(n_gpus=n, streams=args.concurrent, group=args.group, model=sm)
        for frac in (0.25, 0.5, 0.75, 1.0):
            for pol in ("spread", "pack"):
                r = simulate(pol, cap * frac, n_gpus=n, streams=args.concurrent, group=args.group, model=sm,
                             n_tasks=4000)
                print(json.dumps(dict(r, load=frac, n_gpus=n, streams=args.concurrent, group=args.group,
                                      model=f"{args.model} service model (measured r5 points)")), flush=True)
        return
    launched = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if args.node:
        if launched > 1:
            raise SystemExit("--node runs the whole node in ONE process (it spawns its GPU workers): no torchrun")
        return run_node(args)
    if launched == 0 and args.gpus > 1:
        sys.exit(spawn(argv, args.gpus))
    run(args)


if __name__ == "__main__":
    main()
