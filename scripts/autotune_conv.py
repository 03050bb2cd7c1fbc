#!/usr/bin/env python3
"""Offline autotuner for the implicit-GEMM conv/GEMM kernel (csrc/conv.hip).

Enumerates every conv and residual-GEMM shape of the SD1.5 UNet (batch 2, 512^2)
and VAE decoder (batch 1) by running the models on the meta device, times every
(tile cfg, split-K) candidate on the GPU with hipGraph-captured launches (so CPU
launch cost is excluded), and writes the winners as a pinned table
(``csrc/conv_plans.inc``).  The table is keyed by the GEMM dims (M, N, K): the
plan stays a pure function of the shape, identical on every GPU (determinism).

    python scripts/autotune_conv.py OUT_DIR
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd import ops  # noqa: E402
from arbius_amd.ops import _lib  # noqa: E402

NCFG = 20  # 0-9: LDS-DMA multi-stage, 10-19: register-staged, 20-23: 8-wave LDS-DMA (KBIG)
SPLITS = (1, 2, 3, 4, 6, 8)


def _run_meta(models, res, batch=2):
    """Run the selected model families on the meta device (shapes only)."""
    with torch.device("meta"):
        if "sd15" in models:
            from arbius_amd.models.unet2d import UNet2DCondition, UNetConfig
            from arbius_amd.models.vae import VAEDecoder
            UNet2DCondition(UNetConfig())(torch.zeros(batch, res // 8, res // 8, 4), torch.tensor([500.0]),
                                          torch.zeros(batch, 77, 768))
            VAEDecoder()(torch.zeros(1, res // 8, res // 8, 4))
        if "kandinsky2" in models:
            from arbius_amd.models.glide_unet import GlideUNet
            from arbius_amd.models.movq import MoVQDecoder
            GlideUNet()(torch.zeros(batch, 96, 96, 4), torch.tensor([500.0]), torch.zeros(batch, 77, 1024),
                        torch.zeros(batch, 768), torch.zeros(batch, 768))
            MoVQDecoder()(torch.zeros(1, 96, 96, 4))
        if "kandinsky2_prior" in models:   # the diffusion prior (CFG batch 2 per task): M = batch x 81 tokens
            from arbius_amd.models.clip_text import CLIPTextConfig
            from arbius_amd.models.prior import PriorConfig, PriorTransformer
            pcfg = PriorConfig.kandinsky21()
            prior = PriorTransformer(pcfg)
            lens = [5, 77] * (batch // 2)
            layout = prior.layout(lens, torch.device("meta"))
            prior(torch.zeros(batch, pcfg.clip_dim), 500, torch.zeros(batch, 77, CLIPTextConfig.vit_l14().width),
                  torch.zeros(batch, pcfg.clip_dim), lens, layout)
        if "video" in models:   # BASELINE config #4: zeroscope 576x320x24f; VAE in chunks of 8 frames
            from arbius_amd.models.unet3d import UNet3DCondition
            from arbius_amd.models.vae import VAEDecoder
            UNet3DCondition()(torch.zeros(48, 40, 72, 4), torch.tensor([500.0]), torch.zeros(2, 77, 1024), frames=24)
            VAEDecoder()(torch.zeros(8, 40, 72, 4))


def collect_shapes(models=("sd15",), res=512, batch=2):
    convs, gemms = set(), set()
    orig_conv, orig_lin = ops.conv2d, ops.linear

    def conv(x, w, b=None, stride=1, padding=1, upsample=False, residual=None, temb=None, norm=None):
        if x.shape[-1] % 64 == 0 and w.shape[0] % 8 == 0:
            B, H, W, C = x.shape
            convs.add((B, H, W, C, w.shape[0], w.shape[1], w.shape[2], padding, int(bool(upsample)), stride))
        return orig_conv(x, w, b, stride, padding, upsample, residual, temb, norm)

    def lin(x, w, b=None, residual=None, act=None):
        # every linear: under batch-invariant planning plain projections run on this kernel too
        if x.shape[-1] % 64 == 0 and w.shape[0] % 8 == 0:
            gemms.add((x.numel() // x.shape[-1], x.shape[-1], w.shape[0], residual is not None))
        return orig_lin(x, w, b, residual, act=act)

    orig_ln, orig_lng, orig_geglu = ops.ln_linear, ops.ln_linear_geglu, ops.linear_geglu

    def note(x, w, residual=None):
        if x.shape[-1] % 64 == 0 and w.shape[0] % 8 == 0:
            gemms.add((x.numel() // x.shape[-1], x.shape[-1], w.shape[0], residual is not None))

    def ln_lin(x, gamma, beta, eps, w, b=None, residual=None, act=None):
        note(x, w, residual)    # LayerNorm-folded GEMMs share the (M, N, K) plan table
        return orig_ln(x, gamma, beta, eps, w, b, residual=residual, act=act)

    def ln_lin_geglu(x, gamma, beta, eps, w, b=None):
        note(x, w)
        return orig_lng(x, gamma, beta, eps, w, b)

    def lin_geglu(x, w, b=None):
        note(x, w)
        return orig_geglu(x, w, b)

    ops.conv2d, ops.linear = conv, lin
    ops.ln_linear, ops.ln_linear_geglu, ops.linear_geglu = ln_lin, ln_lin_geglu, lin_geglu
    try:
        _run_meta(models, res, batch)
    finally:
        ops.conv2d, ops.linear = orig_conv, orig_lin
        ops.ln_linear, ops.ln_linear_geglu, ops.linear_geglu = orig_ln, orig_lng, orig_geglu
    return sorted(convs), sorted(gemms)


def read_table(path):
    """Existing conv_plans.inc -> {(M, N, K): (cfg, split)}."""
    out = {}
    if not os.path.exists(path):
        return out
    for line in open(path):
        line = line.strip()
        if line.startswith("{") and line.endswith("},"):
            M, N, K, c, sp = (int(v) for v in line[1:-2].split(","))
            out[(M, N, K)] = (c, sp)
    return out


def candidates(M, N, K, mode):
    """(cfg, split) pairs worth timing: split-K only when the grid is short of 2 waves."""
    deep = list(range(28, 28 + len(KDEEP)))
    xreg = list(range(32, 32 + len(KXREG)))
    stag = list(range(36, 36 + len(KSTAG)))
    big = list(range(20, 20 + len(KBIG))) + list(range(24, 24 + len(KPERSIST))) + deep + xreg + stag
    cfgs = {"legacy": range(10, NCFG), "big": big, "glds": list(range(10)) + big, "deep": deep}.get(
        mode, list(range(NCFG)) + big)
    for cfg in cfgs:
        bn, bm = (KSTAG[cfg - 36] if cfg >= 36 else KXREG[cfg - 32] if cfg >= 32 else KDEEP[cfg - 28]
                  if cfg >= 28 else KPERSIST[cfg - 24] if cfg >= 24 else KBIG[cfg - 20] if cfg >= 20
                  else KCFG[cfg % 10])
        if cfg >= 20 and bn > N + N // 2:
            continue
        if 24 <= cfg < 28:      # persistent short-K kernel: no split-K
            if K <= 2560:
                yield cfg, 1
            continue
        tiles = -(-N // bn) * -(-M // bm)
        for sp in SPLITS:
            if sp > 1 and (sp > (K // 64) // 2 or tiles >= (256 if cfg >= 20 else 512)):
                continue
            yield cfg, sp


KCFG = [(128, 128), (64, 128), (128, 64), (64, 64), (160, 64), (160, 128), (320, 32), (256, 64), (128, 256), (64, 256)]
KBIG = [(256, 256), (320, 128), (256, 128), (320, 192)]
KPERSIST = [(128, 128), (256, 128), (160, 128), (128, 64)]
KDEEP = [(128, 256), (256, 128), (192, 192), (320, 64)]     # 8-wave, 3-stage ring
KXREG = [(160, 256), (128, 256), (160, 128), (256, 128)]     # 8-wave, activation operand in VGPRs
# 8-wave, two groups a barrier apart, 3-stage ring
KSTAG = [(256, 128), (128, 256), (192, 192), (320, 64), (160, 256), (160, 128),
         (320, 128), (256, 256), (256, 192)]   # 42-44: K-half slot ring


def _agrees(y, ref):
    return ((y.float() - ref.float()).norm() / ref.float().norm().clamp_min(1e-6)).item() < 1e-2


CONC = 1   # concurrent copies timed together (2 = the miner's two task streams per GPU)


def graph_time(fn, reps=10, rounds=5):
    """Median us per call of fn, hipGraph-replayed.  With CONC > 1 the graph runs CONC copies on
    parallel streams and the time is per call of the aggregate (the throughput a kernel keeps
    while sharing the GPU with the other task stream - what the default deployment sees)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    side = [torch.cuda.Stream() for _ in range(CONC)] if CONC > 1 else []
    with torch.cuda.graph(g):
        if side:
            cap = torch.cuda.current_stream()
            for st in side:
                st.wait_stream(cap)
                with torch.cuda.stream(st):
                    for _ in range(reps):
                        fn()
            for st in side:
                cap.wait_stream(st)
        else:
            for _ in range(reps):
                fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1000 / (reps * max(1, CONC)))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir", nargs="?", default="gpurun_out")
    ap.add_argument("--models", default="sd15", help="comma list: sd15,kandinsky2,video")
    ap.add_argument("--legacy-only", action="store_true", help="time only the register-staged cfgs (10-19)")
    ap.add_argument("--conc", type=int, default=1, help="time CONC concurrent copies (2 = two task streams)")
    ap.add_argument("--mode", default="all", help="all | glds (LDS-DMA cfgs vs the current plan) | big | legacy")
    ap.add_argument("--big-only", action="store_true",
                    help="time only the 8-wave cfgs (20-23) against the current plan; re-pin where they win")
    ap.add_argument("--merge", default=None, help="existing conv_plans.inc to keep entries from")
    ap.add_argument("--batch", type=int, default=2, help="SD UNet batch for shape collection (8 = groups of 4)")
    ap.add_argument("--gemms-only", action="store_true", help="tune the linear (GEMM) shapes only")
    ap.add_argument("--convs-only", action="store_true", help="tune the conv shapes only")
    args = ap.parse_args()
    out_dir = args.out_dir
    os.makedirs(out_dir, exist_ok=True)
    dev = torch.device("cuda")
    convs, gemms = collect_shapes(tuple(args.models.split(",")), batch=args.batch)
    if args.gemms_only:
        convs = []
    if args.convs_only:
        gemms = []
    mode = "big" if args.big_only else "legacy" if args.legacy_only else args.mode
    global CONC
    CONC = args.conc
    results = []
    pinned = read_table(args.merge) if args.merge else {}
    print(f"{len(convs)} conv shapes, {len(gemms)} gemm shapes, {len(pinned)} pinned kept", flush=True)
    for (B, H, W, C, Co, kh, kw, pad, up, st) in convs:
        x = torch.randn(B, H, W, C, device=dev).bfloat16()
        w = (torch.randn(Co, kh, kw, C, device=dev) / math.sqrt(kh * kw * C)).bfloat16()
        b = torch.randn(Co, device=dev).bfloat16()
        Hl, Wl = (2 * H, 2 * W) if up else (H, W)
        padw = 0 if kw != kh else pad
        Ho, Wo = (Hl + 2 * pad - kh) // st + 1, (Wl + 2 * padw - kw) // st + 1
        M, K = B * Ho * Wo, kh * kw * C
        auto = _lib.conv_plan(B, H, W, C, Co, 31 if kw != kh else kh, pad, up, st)
        y_ref = _lib.conv2d_nhwc(x, w, b, pad, up, None, None, st)
        t_auto = graph_time(lambda: _lib.conv2d_nhwc(x, w, b, pad, up, None, None, st))
        best = (t_auto, auto[0], auto[1]) if mode in ("big", "glds", "deep") else None
        for cfg, sp in candidates(M, Co, K, mode):
            if True:
                try:
                    if not _agrees(_lib.conv2d_nhwc(x, w, b, pad, up, None, None, st, cfg, sp), y_ref):
                        print("MISMATCH conv", (B, H, W, C, Co, kh, pad, up, st), cfg, sp, flush=True)
                        continue
                    t = graph_time(lambda: _lib.conv2d_nhwc(x, w, b, pad, up, None, None, st, cfg, sp))
                except Exception as e:  # noqa: BLE001
                    print("skip", cfg, sp, e, flush=True)
                    continue
                if best is None or t < best[0]:
                    best = (t, cfg, sp)
        fl = 2.0 * M * Co * K
        rec = {"kind": "conv", "shape": [B, H, W, C, Co, kh, kw, pad, up, st], "MNK": [M, Co, K],
               "best_us": round(best[0], 2),
               "best_cfg": best[1], "best_split": best[2], "best_tflops": round(fl / best[0] / 1e6, 1),
               "auto_cfg": auto, "auto_us": round(t_auto, 2)}
        results.append(rec)
        if best[1] >= 0:
            pinned[(M, Co, K)] = (best[1], best[2])
        print(json.dumps(rec), flush=True)
    # a shape used both with and without residual is tuned once, with it (the slower epilogue)
    gemm_res = {}
    for (M, K, N, has_res) in gemms:
        gemm_res[(M, K, N)] = gemm_res.get((M, K, N), False) or has_res
    for (M, K, N), has_res in sorted(gemm_res.items()):
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
        b = torch.randn(N, device=dev).bfloat16()
        r = torch.randn(M, N, device=dev).bfloat16() if has_res else None
        y_ref = _lib.gemm(x, w, b, r)
        best = None
        if mode in ("big", "glds", "deep"):
            best = (graph_time(lambda: _lib.gemm(x, w, b, r)), *pinned.get((M, N, K), (-1, 1)))
        for cfg, sp in candidates(M, N, K, mode):
            if True:
                try:
                    if not _agrees(_lib.gemm(x, w, b, r, cfg, sp), y_ref):
                        print("MISMATCH gemm", (M, N, K), cfg, sp, flush=True)
                        continue
                    t = graph_time(lambda: _lib.gemm(x, w, b, r, cfg, sp))
                except Exception as e:  # noqa: BLE001
                    continue
                if best is None or t < best[0]:
                    best = (t, cfg, sp)
        t_blas = graph_time(lambda: torch.addmm(r, x, w.t()).add_(b)) if has_res else graph_time(
            lambda: torch.nn.functional.linear(x, w, b))
        fl = 2.0 * M * N * K
        rec = {"kind": "gemm_res" if has_res else "gemm", "MNK": [M, N, K], "best_us": round(best[0], 2),
               "best_cfg": best[1],
               "best_split": best[2], "best_tflops": round(fl / best[0] / 1e6, 1),
               "hipblaslt_addmm_add_us": round(t_blas, 2)}
        results.append(rec)
        if best[1] >= 0 and (M, N, K) not in {tuple(r["MNK"]) for r in results if r["kind"] == "conv"}:
            pinned[(M, N, K)] = (best[1], best[2])
        print(json.dumps(rec), flush=True)
    json.dump(results, open(os.path.join(out_dir, "autotune_conv.json"), "w"), indent=1)
    lines = ["// Generated by scripts/autotune_conv.py on MI355X: (M, N, K) -> (tile cfg, split-K).",
             "// Shapes not listed fall back to the cost model in conv.hip.",
             "static const PinnedPlan kPinnedPlans[] = {"]
    for (M, N, K), (c, sp) in sorted(pinned.items()):
        lines.append(f"    {{{M}, {N}, {K}, {c}, {sp}}},")
    lines.append("};")
    open(os.path.join(out_dir, "conv_plans.inc"), "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
