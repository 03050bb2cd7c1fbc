#!/usr/bin/env python3
"""Kandinsky 2.1 text + prior stage: linears on the implicit-GEMM kernel (default) vs the library GEMM
(the pre-r2.5 routing of residual-free linears), interleaved, one MI355X."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd import ops  # noqa: E402
from arbius_amd.models.registry import build_pipeline  # noqa: E402


def main():
    dev = torch.device("cuda")
    pipe = build_pipeline("kandinsky2", device=dev)
    orig = ops.linear

    def lib_linear(x, w, b=None, residual=None):
        if residual is None:
            return torch.nn.functional.linear(x, w, b)
        return orig(x, w, b, residual)

    def stage():
        gen = torch.Generator().manual_seed(1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h, p, lens = pipe.encode_clip("a red fox in the snow, watercolor")
        t1 = time.perf_counter()
        pipe.sample_prior(h, p, lens, gen, 5, 4.0)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        pipe.encode_xlmr("a red fox in the snow, watercolor")
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        return t1 - t0, t2 - t1, t3 - t2

    res = {"hip": [], "lib": []}
    for r in range(4):
        for arm in ("hip", "lib"):
            ops.linear = orig if arm == "hip" else lib_linear
            res[arm].append(stage())
    ops.linear = orig
    for arm, v in res.items():
        v = v[1:]
        print(json.dumps({"arm": arm, "clip_s": min(x[0] for x in v), "prior_s": min(x[1] for x in v),
                          "xlmr_s": min(x[2] for x in v)}), flush=True)
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA, ProfilerActivity.CPU]) as prof:
        stage()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=15))


if __name__ == "__main__":
    main()
