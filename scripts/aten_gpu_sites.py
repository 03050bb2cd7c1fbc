#!/usr/bin/env python3
"""GPU time of the ATen kernels left on a model's path, by the model source line that launched them.

Runs one solve of the model (after a warm-up solve) under torch.profiler with Python stacks.
Each ATen CPU op's device kernels are attributed to the innermost ``arbius_amd/models`` frame
(outside ``ops/``).  Prints one JSON line per call site, ordered by GPU time.  The static twin is
``scripts/aten_audit.py``, which counts launches on the meta device without a GPU.

    python scripts/aten_gpu_sites.py kandinsky2 [--steps 20] [--res 768]
"""
import argparse
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model", nargs="?", default="kandinsky2")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--res", type=int, default=None)
    a = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile

    from arbius_amd.models.registry import build_pipeline
    dev = torch.device("cuda", 0)
    # eager: kernels inside a replayed hipGraph carry no ATen op / Python stack to attribute them to
    pipe = build_pipeline(a.model, device=dev, init=True, use_graphs=False)
    res = a.res or (768 if a.model == "kandinsky2" else 512)
    inp = {"prompt": "a lighthouse on a cliff at dusk", "negative_prompt": "", "width": res, "height": res,
           "num_inference_steps": a.steps, "seed": 7}
    if a.model == "kandinsky2":
        pipe.cfg.num_steps = a.steps
    if a.model in ("zeroscopev2xl", "damo"):   # BASELINE config #4: 576 x 320 x 24 frames
        inp.update(width=a.res or 576, height=320 if a.model == "zeroscopev2xl" else inp["height"], num_frames=24)
    if hasattr(pipe, "solve"):
        run = lambda: pipe.solve(inp)  # noqa: E731
    else:                              # image pipelines: the node's solve path
        from arbius_amd.node.solver import solve_image
        inp.update(guidance_scale=7, scheduler="DPMSolverMultistep")
        run = lambda: solve_image(pipe, inp)  # noqa: E731
    run()
    torch.cuda.synchronize()
    # every tensor copy that touches the GPU (device <-> host, device <-> device), by the model source line:
    # hipMemcpy* calls have no Python stack in the profiler, the dispatch mode sees the ATen op and the stack
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    copies = collections.Counter()

    class CopySites(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = str(func)
            if name.startswith(("aten.copy_", "aten._to_copy", "aten.clone", "aten._copy_from")):
                devs = {str(t.device) for t in list(args) + list((kwargs or {}).values()) if torch.is_tensor(t)}
                dst = (kwargs or {}).get("device")
                if dst is not None:
                    devs.add(str(dst))
                if any(d.startswith("cuda") for d in devs):
                    site = "?"
                    for fr in reversed(traceback.extract_stack()[:-1]):
                        if "/arbius_amd/" in fr.filename:
                            site = f"{fr.filename.split('/arbius_amd/')[1]}:{fr.lineno}"
                            break
                    copies[(name.split(".")[1] if "." in name else name, "->".join(sorted(devs)), site)] += 1
            return func(*args, **(kwargs or {}))

    with CopySites():
        run()
        torch.cuda.synchronize()
    for (op, devs, site), n in copies.most_common(25):
        print(json.dumps({"copy_op": op, "devices": devs, "site": site, "calls": n}), flush=True)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        run()
        torch.cuda.synchronize()
    sites = collections.defaultdict(lambda: [0.0, 0, set()])
    for ev in prof.events():
        if ev.device_type.name != "CPU" or not ev.name.startswith("aten::"):
            continue
        dev_us = sum(k.duration for k in ev.kernels) if ev.kernels else 0.0
        if dev_us <= 0:
            continue
        where = "?"
        for fr in ev.stack or []:
            if "/arbius_amd/" in fr and "/ops/" not in fr:
                where = fr.split("/arbius_amd/")[1]
                break
        s = sites[(ev.name, where)]
        s[0] += dev_us
        s[1] += 1
        s[2].update(k.name[:60] for k in ev.kernels)
    total = sum(v[0] for v in sites.values())
    print(json.dumps({"model": a.model, "steps": a.steps, "aten_gpu_ms": round(total / 1e3, 3)}), flush=True)
    for (name, where), (us, n, ks) in sorted(sites.items(), key=lambda kv: -kv[1][0])[:40]:
        print(json.dumps({"op": name, "site": where, "gpu_ms": round(us / 1e3, 3), "calls": n,
                          "kernels": sorted(ks)[:3]}), flush=True)


if __name__ == "__main__":
    main()
