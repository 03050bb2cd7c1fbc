"""Timing experiment: one SD1.5 UNet eval (hipGraph) at CFG batch 2 vs 4 vs 8 (2/4 tasks lock-step)."""
import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd.models.registry import build_pipeline

pipe = build_pipeline("anythingv3", device="cuda")
for B in (2, 4, 8):
    x = torch.randn(B, 64, 64, 4, device="cuda").bfloat16()
    ctx = torch.randn(B, 77, 768, device="cuda").bfloat16()
    for _ in range(3):
        pipe._unet_eval(x, 500, ctx)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        pipe._unet_eval(x, 500, ctx)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 20 * 1000
    print(f"batch {B}: {dt:.2f} ms/eval  {dt / (B // 2):.2f} ms per task-eval", flush=True)
