#!/usr/bin/env python3
"""Per-op / per-shape GPU time of one lock-step SD1.5 (or Kandinsky2) solve, eager (no hipGraphs):
every HIP op entry point in ``ops._lib`` is wrapped with a pair of HIP events, so the table says
which conv / GEMM / norm / attention shapes carry the time (rocprofv3's summary only names kernels).

    python scripts/layer_prof.py [--model anythingv3|kandinsky2] [--group 4] [--res 512] [--steps 2]
        [--json out.jsonl]
"""
import argparse
import json
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd.ops import _lib  # noqa: E402

REC = []
SLEEP_CYCLES = 400_000
WRAPPED = ("conv2d_nhwc", "gemm", "gemm_geglu", "group_norm_table", "norm_table_apply", "layer_norm",
           "flash_attention", "group_norm_nhwc", "group_norm_mod_nhwc", "softmax_rows", "sampler_step", "silu",
           "geglu", "temporal_attention", "gemm_ln", "row_stats")


def _key(name, a, k):
    def sh(t):
        return tuple(t.shape) if hasattr(t, "shape") else None
    if name == "conv2d_nhwc":
        x, w = a[0], a[1]
        return (sh(x), sh(w), "s%d" % k.get("stride", a[7] if len(a) > 7 else 1),
                "up" if (a[4] if len(a) > 4 else k.get("upsample")) else "", "cat" if k.get("x2") is not None else "",
                "norm" if k.get("norm") is not None else "")
    if name in ("gemm", "gemm_geglu", "gemm_ln"):
        return (sh(a[0]), sh(a[1]))
    if name == "flash_attention":
        return (sh(a[0]), sh(a[1]), "prefix" if (a[5] if len(a) > 5 else k.get("kv_prefix")) is not None else "")
    if name == "sampler_step":
        return (len(a[0]),)
    return tuple(sh(t) for t in a[:2] if hasattr(t, "shape"))


def wrap():
    for name in WRAPPED:
        f = getattr(_lib, name, None)
        if f is None:
            continue

        def g(*a, __f=f, __n=name, **k):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # keep the GPU busy while the host enqueues (start event, op, end event): the events then
            # bracket GPU execution only, not the host's launch gaps of an eager run
            torch.cuda._sleep(SLEEP_CYCLES)
            s.record()
            r = __f(*a, **k)
            e.record()
            REC.append((__n, _key(__n, a, k), s, e))
            return r
        setattr(_lib, name, g)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="anythingv3")
    ap.add_argument("--group", type=int, default=4)
    ap.add_argument("--res", type=int, default=None)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--json", default=None)
    ap.add_argument("--top", type=int, default=60)
    args = ap.parse_args()
    from arbius_amd.models.registry import build_pipeline
    from arbius_amd.node.solver import solve_images
    k2 = args.model == "kandinsky2"
    res = args.res or (768 if k2 else 512)
    pipe = build_pipeline(args.model, device="cuda:0", use_graphs=False)
    if k2:
        pipe.cfg.num_steps = args.steps
    inps = [{"prompt": f"castle {j}", "negative_prompt": "x", "width": res, "height": res,
             "num_inference_steps": args.steps, "guidance_scale": 7, "scheduler": "DPMSolverMultistep",
             "seed": 1000 + j} for j in range(args.group)]
    solve_images(pipe, inps)            # warm: plans, workspaces, caches
    torch.cuda.synchronize()
    wrap()
    solve_images(pipe, inps)
    torch.cuda.synchronize()
    agg = defaultdict(lambda: [0.0, 0])
    for n, key, s, e in REC:
        a = agg[(n, key)]
        a[0] += s.elapsed_time(e) * 1000.0
        a[1] += 1
    total = sum(v[0] for v in agg.values())
    by_op = defaultdict(float)
    for (n, _), v in agg.items():
        by_op[n] += v[0]
    print(f"total op time {total / 1000:.2f} ms over {len(REC)} calls ({args.model}, group {args.group}, "
          f"{args.steps} steps, eager)")
    for n, t in sorted(by_op.items(), key=lambda kv: -kv[1]):
        print(f"  {n:20s} {100 * t / total:5.1f} %  {t / 1000:8.2f} ms")
    print("| % | ms | calls | avg us | op | shape |")
    print("|---:|---:|---:|---:|---|---|")
    rows = sorted(agg.items(), key=lambda kv: -kv[1][0])
    for (n, key), (t, c) in rows[:args.top]:
        print(f"| {100 * t / total:.1f} | {t / 1000:.2f} | {c} | {t / c:.1f} | {n} | {key} |")
    if args.json:
        with open(args.json, "w") as f:
            for (n, key), (t, c) in rows:
                f.write(json.dumps({"op": n, "key": repr(key), "us": t, "calls": c}) + "\n")


if __name__ == "__main__":
    main()
