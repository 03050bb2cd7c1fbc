#!/usr/bin/env python3
"""Conv kernel lab: the hot SD1.5 batch-8 conv shapes under every tile family, against the
hipBLASLt bar (torch.matmul of the same M x K x N GEMM, i.e. a conv with its im2col for free).

    python scripts/conv_lab.py sweep        # one JSON line per shape: us per cfg, TFLOP/s, bar
    python scripts/conv_lab.py pmc SHAPE    # the planned kernel of one shape in a loop (rocprofv3 --pmc)

Random data (cdna_hip_programming.md §5.4 rule 25); hipGraph replay, median of rounds.
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd.ops import _lib  # noqa: E402
from scripts.autotune_conv import graph_time  # noqa: E402

# (B, H, W, Cin, Cout, k): the SD1.5 UNet convs at lock-step batch 8 (2 streams x group 4 x CFG 2 / 2)
SHAPES = {
    "l0_320": (8, 64, 64, 320, 320, 3), "l0_640": (8, 64, 64, 640, 320, 3), "l0_960": (8, 64, 64, 960, 320, 3),
    "l1_640": (8, 32, 32, 640, 640, 3), "l1_1280": (8, 32, 32, 1280, 640, 3), "l1_1920": (8, 32, 32, 1920, 640, 3),
    "l2_1280": (8, 16, 16, 1280, 1280, 3), "l2_2560": (8, 16, 16, 2560, 1280, 3),
    "s0_320": (2, 64, 64, 320, 320, 3),
}
CFGS = [int(c) for c in os.environ.get("LAB_CFGS", "5,15,10,0,20,21,22,23,28,29,30,31").split(",")]


def make(shape, dev):
    B, H, W, C, Co, k = shape
    x = torch.randn(B, H, W, C, device=dev).bfloat16()
    w = (torch.randn(Co, k, k, C, device=dev) / math.sqrt(k * k * C)).bfloat16()
    b = torch.randn(Co, device=dev).bfloat16()
    return x, w, b


def sweep():
    dev = torch.device("cuda")
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else list(SHAPES)
    for name in names:
        shape = SHAPES[name]
        B, H, W, C, Co, k = shape
        x, w, b = make(shape, dev)
        M, K = B * H * W, k * k * C
        fl = 2.0 * M * Co * K
        res = {"plan": round(graph_time(lambda: _lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1)), 1)}
        for cfg in CFGS:
            for sp in (1, 2) if M <= 8192 else (1,):
                try:
                    t = graph_time(lambda: _lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1, cfg, sp))
                except Exception as e:  # noqa: BLE001 - unsupported cfg for this shape
                    t = float("nan")
                    print(f"# {name} cfg {cfg}: {e}", file=sys.stderr)
                res[f"{cfg}/{sp}"] = round(t, 1)
        a = torch.randn(M, K, device=dev).bfloat16()
        wt = torch.randn(K, Co, device=dev).bfloat16()
        t_bar = graph_time(lambda: torch.matmul(a, wt))
        best = min((k_ for k_ in res if res[k_] == res[k_]), key=res.get)
        print(json.dumps({"shape": name, "MNK": [M, Co, K], "us": res, "best": best,
                          "best_tflops": round(fl / res[best] / 1e6, 1),
                          "plan_tflops": round(fl / res["plan"] / 1e6, 1),
                          "hipblaslt_us": round(t_bar, 1), "hipblaslt_tflops": round(fl / t_bar / 1e6, 1)}),
              flush=True)


def libs_ab():
    """In-process A/B of kernel-library builds (LAB_LIBS=a.so,b.so in arbius_amd/ops/): the planned
    conv of every shape through each library's arb_conv2d_nhwc, interleaved per round (same
    clock / thermal state for both arms)."""
    import ctypes
    dev = torch.device("cuda")
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "arbius_amd", "ops")
    names = os.environ.get("LAB_LIBS", "libarbius_kernels_base.so,libarbius_kernels.so").split(",")
    fns = {}
    for n in names:
        L = ctypes.CDLL(os.path.join(here, n))
        f = L.arb_conv2d_nhwc
        f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p] * 8 + [ctypes.c_int] * 12 + [ctypes.c_void_p]
        ws = L.arb_conv2d_workspace
        ws.restype, ws.argtypes = ctypes.c_size_t, [ctypes.c_int] * 11
        fns[n] = (f, ws)
    shapes = sys.argv[2].split(",") if len(sys.argv) > 2 else list(SHAPES)
    cfg = int(os.environ.get("LAB_CFG", "-1"))
    for name in shapes:
        B, H, W, C, Co, k = SHAPES[name]
        x, w, b = make(SHAPES[name], dev)
        y = torch.empty(B, H, W, Co, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * B * H * W * Co * k * k * C
        P = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731
        calls, outs = {}, {}
        for n, (f, wsf) in fns.items():
            nbytes = wsf(B, H, W, C, Co, k, 1, 0, 1, cfg, 1)
            ws = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=dev)

            def call(f=f, ws=ws):
                rc = f(P(x), P(w), P(b), P(None), P(None), P(y), P(ws), P(None), B, H, W, C, Co, k, 1, 0, 1,
                       cfg, 1, 0, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                assert rc == 0, rc
            calls[n] = call
            call()
            torch.cuda.synchronize()
            outs[n] = y.clone()
        same = all(torch.equal(outs[names[0]], o) for o in outs.values())
        res = {n: [] for n in names}
        for _ in range(int(os.environ.get("LAB_ROUNDS", "3"))):
            for n in names:
                res[n].append(graph_time(calls[n]))
        med = {n: round(sorted(v)[len(v) // 2], 1) for n, v in res.items()}
        print(json.dumps({"shape": name, "us": med, "tflops": {n: round(fl / t / 1e6, 1) for n, t in med.items()},
                          "bitwise_equal": same}), flush=True)


GN_SHAPES = [(8, 4096, 320), (8, 4096, 640), (8, 4096, 960), (8, 1024, 640), (8, 1024, 1280), (8, 1024, 1920),
             (8, 256, 1280), (8, 256, 2560), (8, 64, 1280), (2, 4096, 320)]


def gn_ab():
    """GroupNorm-table (stats + table) per library build, interleaved; GB/s of the one read of x."""
    import ctypes
    dev = torch.device("cuda")
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "arbius_amd", "ops")
    names = os.environ.get("LAB_LIBS", "libarbius_kernels_base.so,libarbius_kernels.so").split(",")
    fns = {}
    for n in names:
        L = ctypes.CDLL(os.path.join(here, n))
        f = L.arb_group_norm_table
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_float] + [ctypes.c_void_p] * 2 + [ctypes.c_int] * 4 + \
            [ctypes.c_float, ctypes.c_void_p]
        ws = L.arb_group_norm_workspace
        ws.restype, ws.argtypes = ctypes.c_size_t, [ctypes.c_int] * 4
        fns[n] = (f, ws)
    P = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731
    for (B, HW, C) in GN_SHAPES:
        x = (torch.randn(B, HW, C, device=dev) * 2 + 0.5).bfloat16()
        g = (torch.rand(C, device=dev) + 0.5).bfloat16()
        bt = torch.randn(C, device=dev).bfloat16()
        calls, tabs = {}, {}
        for n, (f, wsf) in fns.items():
            ws = torch.empty(max(16, int(wsf(B, HW, C, 32))), dtype=torch.uint8, device=dev)
            tab = torch.empty(B, C, 2, device=dev)

            def call(f=f, ws=ws, tab=tab):
                rc = f(P(x), P(g), P(bt), P(None), 0.0, P(ws), P(tab), B, HW, C, 32, 1e-5,
                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                assert rc == 0, rc
            calls[n] = call
            call()
            torch.cuda.synchronize()
            tabs[n] = tab.clone()
        ref = tabs[names[0]]
        err = max(float((t - ref).abs().max() / ref.abs().max()) for t in tabs.values())
        res = {n: [] for n in names}
        for _ in range(3):
            for n in names:
                res[n].append(graph_time(calls[n]))
        med = {n: round(sorted(v)[1], 1) for n, v in res.items()}
        gbs = {n: round(B * HW * C * 2 / t / 1e3, 0) for n, t in med.items()}
        print(json.dumps({"gn": [B, HW, C], "us": med, "GBps": gbs, "max_rel_diff": err}), flush=True)


def pmc():
    dev = torch.device("cuda")
    shape = SHAPES[sys.argv[2]]
    cfg = int(sys.argv[3]) if len(sys.argv) > 3 else -1
    x, w, b = make(shape, dev)
    for _ in range(int(os.environ.get("LAB_ITERS", "20"))):
        _lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1, cfg, 1)
    torch.cuda.synchronize()
    print("pmc done", sys.argv[2], cfg)


if __name__ == "__main__":
    {"sweep": sweep, "pmc": pmc, "ab": libs_ab, "gn": gn_ab}[sys.argv[1]]()
