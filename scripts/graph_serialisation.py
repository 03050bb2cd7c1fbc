#!/usr/bin/env python3
"""Why a hipGraph-replayed VAE decode stalls the 2-stream SD1.5 pipeline.

Two pipeline forks (private HIP streams, as in bench.py) solve lock-step groups of 4 concurrently;
every VAE decode and every UNet evaluation is bracketed by timing events on its own stream, and
the host time spent inside each VAE call is recorded.  For each decode the report gives:

* host_ms  - wall time of the decode call on the CPU (graph replay + the copy out + D2H),
* gpu_ms   - its stream's event span (when the stream reached the decode -> decode finished),
* other_unet - how many UNet evaluations of the OTHER stream overlap that span, and their mean
  GPU time vs. the other stream's UNet evaluations that overlap no decode.

A decode whose GPU span holds many of the other stream's evaluations while its own kernels take
~40 ms means the two streams were serialised on the device; a long host_ms with a short gpu_ms
means the host blocked in the replay call.  Run it with and without ``--vae-graph`` (same process
cannot switch: the switch is read at import).

    python scripts/graph_serialisation.py [--vae-graph] [--groups 3] [--json out.json]
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vae-graph", action="store_true")
    ap.add_argument("--groups", type=int, default=3, help="lock-step groups per stream (after 1 warm-up)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    if a.vae_graph:
        os.environ["ARB_VAE_GRAPH"] = "1"
    import torch

    from arbius_amd.models import sd15
    from arbius_amd.models.registry import build_pipeline
    dev = torch.device("cuda", 0)
    base = build_pipeline("anythingv3", device=dev)
    forks = [base.fork(), base.fork()]
    rec = {0: {"unet": [], "vae": []}, 1: {"unet": [], "vae": []}}
    t_base = torch.cuda.Event(enable_timing=True)
    t_base.record()
    local = threading.local()
    orig_unet, orig_decode = sd15.SD15Pipeline._unet_eval, sd15.SD15Pipeline.decode

    def unet_eval(self, *args):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = orig_unet(self, *args)
        e1.record()
        if getattr(local, "on", False):
            rec[local.k]["unet"].append((e0, e1))
        return out

    def decode(self, latent):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        h0 = time.perf_counter()
        out = orig_decode(self, latent)
        host = (time.perf_counter() - h0) * 1e3
        e1.record()
        if getattr(local, "on", False):
            rec[local.k]["vae"].append((e0, e1, host))
        return out

    sd15.SD15Pipeline._unet_eval, sd15.SD15Pipeline.decode = unet_eval, decode
    inps = [{"prompt": f"arbius test {j}", "negative_prompt": "", "width": 512, "height": 512, "seed": 7 + j,
             "num_inference_steps": a.steps, "guidance_scale": 12.0, "scheduler": "DPMSolverMultistep"}
            for j in range(4)]

    def worker(k):
        local.k = k
        p = forks[k]
        with p._stream_ctx():
            local.on = False
            p.run_group(inps)                       # warm-up: graphs captured, caches filled
            torch.cuda.current_stream().synchronize()
            barrier.wait()
            local.on = True
            for _ in range(a.groups):
                p.run_group(inps)
            torch.cuda.current_stream().synchronize()

    barrier = threading.Barrier(2)
    th = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    w0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - w0
    torch.cuda.synchronize()

    def ts(e):
        return t_base.elapsed_time(e)

    rows = []
    for k in (0, 1):
        other = [(ts(e0), ts(e1)) for e0, e1 in rec[1 - k]["unet"]]
        spans = []
        for e0, e1, host in rec[k]["vae"]:
            s, e = ts(e0), ts(e1)
            inside = [b - a_ for a_, b in other if a_ < e and b > s]      # overlapping the decode span
            spans.append((s, e))
            rows.append({"stream": k, "host_ms": round(host, 2), "gpu_ms": round(e - s, 2),
                         "other_unet_inside": len(inside),
                         "other_unet_inside_mean_ms": round(statistics.mean(inside), 2) if inside else None})
    outside = []
    for k in (0, 1):
        spans = [(ts(e0), ts(e1)) for e0, e1, _ in rec[1 - k]["vae"]]
        for e0, e1 in rec[k]["unet"]:
            s, e = ts(e0), ts(e1)
            if not any(s < b and e > a_ for a_, b in spans):
                outside.append(e - s)
    summ = {"vae_graph": a.vae_graph, "wall_s": round(wall, 2), "groups_per_stream": a.groups,
            "decodes": len(rows), "decode_host_ms_median": statistics.median(r["host_ms"] for r in rows),
            "decode_gpu_ms_median": statistics.median(r["gpu_ms"] for r in rows),
            "other_unet_inside_per_decode": statistics.mean(r["other_unet_inside"] for r in rows),
            "other_unet_ms_overlapping_decodes": round(statistics.mean(
                [r["other_unet_inside_mean_ms"] for r in rows if r["other_unet_inside_mean_ms"]] or [0]), 2),
            "unet_eval_ms_outside_decodes_median": round(statistics.median(outside), 2) if outside else None,
            "tasks_per_hour": round(2 * 4 * a.groups * 3600 / wall, 1)}
    print(json.dumps(summ))
    for r in rows[:8]:
        print(json.dumps(r))
    if a.json:
        json.dump({"summary": summ, "decodes": rows}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
