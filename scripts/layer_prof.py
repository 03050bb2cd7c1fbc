#!/usr/bin/env python3
"""Per-op / per-shape GPU time of one lock-step SD1.5 (or Kandinsky2) solve, eager (no hipGraphs):
every HIP op entry point in ``ops._lib`` is wrapped with a pair of HIP events, so the table says
which conv / GEMM / norm / attention shapes carry the time (rocprofv3's summary only names kernels).
Each row carries the useful FLOPs of the call, the achieved TFLOP/s and - for conv / GEMM launches -
the tile family and split-K the launch runs (``_lib.conv_choice`` / ``gemm_choice``: the canonical
plan at its split, on the family tuned for the actual shape).

    python scripts/layer_prof.py [--model anythingv3|kandinsky2] [--group 4] [--res 512] [--steps 2]
        [--streams 1] [--json out.jsonl] [--md out.md]
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
_ORIG = {}
_DEPTH = [0]


def _arg(a, k, i, name, default=None):
    if len(a) > i:
        return a[i]
    return k.get(name, default)


def _sh(t):
    return tuple(t.shape) if hasattr(t, "shape") else None


def _info(name, a, k):
    """(key, flops, family) of one call."""
    if name == "conv2d_nhwc":
        x, w = a[0], a[1]
        pad, up = _arg(a, k, 3, "padding", 1), bool(_arg(a, k, 4, "upsample", False))
        stride = _arg(a, k, 7, "stride", 1)
        x2 = k.get("x2")
        B, H, W, Cin = x.shape
        if x2 is not None:
            Cin += x2.shape[-1]
        Cout, kh, kw, _ = w.shape
        kcode = 31 if (kh, kw) == (3, 1) else kh
        Hl, Wl = (2 * H, 2 * W) if up else (H, W)
        Ho = (Hl + 2 * pad - kh) // stride + 1
        Wo = (Wl + 2 * (0 if kcode == 31 else pad) - kw) // stride + 1
        M, N, K = B * Ho * Wo, Cout, kh * kw * Cin
        plan_b = k.get("plan_b")
        cfg, split = _ORIG["conv_choice"](B, H, W, Cin, Cout, kcode, pad, up, stride, plan_b)
        temb, res = _arg(a, k, 6, "temb"), _arg(a, k, 5, "residual")
        flags = ("up" if up else "", "cat" if x2 is not None else "", "norm" if k.get("norm") is not None else "",
                 "temb" if temb is not None else "", "res" if res is not None else "")
        key = ("conv%dx%d" % (kh, kw), _sh(x), Cout, "s%d" % stride) + flags
        return key, 2.0 * M * N * K, (M, N, K, _lib.cfg_name(cfg), split)
    if name in ("gemm", "gemm_geglu", "gemm_ln"):
        x, w = a[0], a[1]
        K, N = x.shape[-1], w.shape[0]
        M = x.numel() // K
        cfg, split = _ORIG["gemm_choice"](M, N, K, k.get("plan_batch"))
        return (_sh(x), _sh(w)), 2.0 * M * N * K, (M, N, K, _lib.cfg_name(cfg), split)
    if name == "flash_attention":
        q, kk = a[0], a[1]
        B, Nq, H, D = q.shape
        kvp = _arg(a, k, 5, "kv_prefix")
        Nk = kk.shape[1] + (kvp[0].shape[1] if kvp is not None else 0)
        return (_sh(q), _sh(kk), "prefix" if kvp is not None else ""), 4.0 * B * H * Nq * Nk * D, None
    if name == "temporal_attention":
        q = a[0]
        B, F, P, H, D = q.shape
        return (_sh(q),), 4.0 * B * P * H * F * F * D, None
    if name == "sampler_step":
        return (len(a[0]),), 0.0, None
    return tuple(_sh(t) for t in a[:2] if hasattr(t, "shape")), 0.0, None


def wrap():
    _ORIG["conv_choice"] = _lib.conv_choice
    _ORIG["gemm_choice"] = _lib.gemm_choice
    for name in WRAPPED:
        f = getattr(_lib, name, None)
        if f is None:
            continue

        def g(*a, __f=f, __n=name, **k):
            if _DEPTH[0]:                   # an op inside a timed op (e.g. the d=512 attention's GEMMs)
                return __f(*a, **k)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # keep the GPU busy while the host enqueues (start event, op, end event): the events then
            # bracket GPU execution only, not the host's launch gaps of an eager run
            torch.cuda._sleep(SLEEP_CYCLES)
            s.record()
            _DEPTH[0] += 1
            try:
                r = __f(*a, **k)
            finally:
                _DEPTH[0] -= 1
            e.record()
            key, flops, fam = _info(__n, a, k)
            REC.append((__n, key, flops, fam, s, e))
            return r
        setattr(_lib, name, g)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="anythingv3")
    ap.add_argument("--group", type=int, default=4)
    ap.add_argument("--res", type=int, default=None)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--json", default=None)
    ap.add_argument("--md", default=None)
    ap.add_argument("--top", type=int, default=80)
    ap.add_argument("--frames", type=int, default=24, help="video models: frames per clip")
    args = ap.parse_args()
    from arbius_amd.models.registry import build_pipeline
    from arbius_amd.node.solver import solve_images
    k2 = args.model == "kandinsky2"
    vid = args.model in ("zeroscopev2xl", "damo")
    res = args.res or (768 if k2 else 576 if args.model == "zeroscopev2xl" else 256 if vid else 512)
    pipe = build_pipeline(args.model, device="cuda:0", use_graphs=False)
    if k2:
        pipe.cfg.num_steps = args.steps
    if k2:      # templates/kandinsky2.json inputs (hidden defaults: p_sampler, guidance 4, prior 5 steps)
        inps = [{"prompt": f"castle {j}", "width": res, "height": res, "num_inference_steps": args.steps,
                 "seed": 1000 + j} for j in range(args.group)]
    else:
        inps = [{"prompt": f"castle {j}", "negative_prompt": "x", "width": res, "height": res,
                 "num_inference_steps": args.steps, "guidance_scale": 7, "scheduler": "DPMSolverMultistep",
                 "seed": 1000 + j} for j in range(args.group)]
    if vid:     # one clip (BASELINE config #4: 576x320, 24 frames); lock-step groups do not apply
        height = 320 if args.model == "zeroscopev2xl" else 256
        vinp = {"prompt": "a red cat walking", "negative_prompt": "blurry", "num_frames": args.frames,
                "width": res, "height": height, "num_inference_steps": args.steps, "guidance_scale": 9.0,
                "fps": 8, "seed": 1337}
        args.group = 1

        def run():
            pipe.solve(vinp)
    else:
        def run():
            solve_images(pipe, inps)
    run()                               # warm: plans, workspaces, caches
    torch.cuda.synchronize()
    wrap()
    run()
    torch.cuda.synchronize()
    agg = defaultdict(lambda: [0.0, 0, 0.0, None])
    for n, key, flops, fam, s, e in REC:
        a = agg[(n, key)]
        a[0] += s.elapsed_time(e) * 1000.0
        a[1] += 1
        a[2] += flops
        a[3] = fam
    total = sum(v[0] for v in agg.values())
    tot_fl = sum(v[2] for v in agg.values())
    by_op = defaultdict(float)
    for (n, _), v in agg.items():
        by_op[n] += v[0]
    what = (f"{res}x{vinp['height']}x{args.frames}f, CFG batch 2" if vid else
            f"{res}^2, group {args.group} = batch {2 * args.group}")
    lines = [f"total op time {total / 1000:.2f} ms over {len(REC)} calls ({args.model} {what}, "
             f"{args.steps} steps, eager, each op timed in isolation); "
             f"{tot_fl / 1e12:.1f} TFLOP of matmul work -> {tot_fl / (total * 1e-6) / 1e12:.0f} TFLOP/s overall", ""]
    lines += ["| op | % | ms |", "|---|---:|---:|"]
    for n, t in sorted(by_op.items(), key=lambda kv: -kv[1]):
        lines.append(f"| {n} | {100 * t / total:.1f} | {t / 1000:.2f} |")
    lines += ["", "| % | ms | calls | avg us | TFLOP/s | op | shape | M x N x K | family | split |",
              "|---:|---:|---:|---:|---:|---|---|---|---|---:|"]
    rows = sorted(agg.items(), key=lambda kv: -kv[1][0])
    for (n, key), (t, c, fl, fam) in rows[:args.top]:
        tf = f"{fl / (t * 1e-6) / 1e12:.0f}" if fl else "-"
        mnk = f"{fam[0]}x{fam[1]}x{fam[2]}" if fam else ""
        fname, split = (fam[3], fam[4]) if fam else ("", "")
        lines.append(f"| {100 * t / total:.1f} | {t / 1000:.2f} | {c} | {t / c:.1f} | {tf} | {n} | {key} | {mnk} | "
                     f"{fname} | {split} |")
    text = "\n".join(lines)
    print(text)
    if args.md:
        with open(args.md, "w") as f:
            f.write(text + "\n")
    if args.json:
        with open(args.json, "w") as f:
            for (n, key), (t, c, fl, fam) in rows:
                f.write(json.dumps({"op": n, "key": repr(key), "us": t, "calls": c, "flops": fl,
                                    "family": fam}) + "\n")


if __name__ == "__main__":
    main()
