"""Task solver: hydrated template input -> output files -> solution CID.

This is the in-process replacement of ``EnabledModels[..].getfiles`` + ``default__getcid``
(``miner/src/index.ts:781-877``, ``miner/src/models.ts:34-54``): instead of an HTTP
POST to a Cog container and a kubo ``addAll``, the GPU worker runs the pipeline,
encodes a deterministic PNG and computes the wrapped-directory CIDv0 locally.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

from ..ipfs.unixfs import DagResult, wrap_directory
from ..utils.png import encode_png

EVIL_CID = "0x1220" + "66" * 32  # miner/src/models.ts:40-42 (evilmode fault injection)


@dataclass
class Solution:
    files: List[Tuple[str, bytes]]
    cid: str                       # 0x1220... (34 bytes hex)
    dag: DagResult = None
    timings: Dict[str, float] = field(default_factory=dict)


def solve_image(pipe, inp: dict, png_level: int = 6) -> Solution:
    """SD-family text-to-image task (anythingv3 template semantics)."""
    t0 = time.perf_counter()
    img = pipe(
        prompt=inp["prompt"],
        negative_prompt=inp.get("negative_prompt", ""),
        width=int(inp.get("width", 768)),
        height=int(inp.get("height", 768)),
        num_inference_steps=int(inp.get("num_inference_steps", 20)),
        guidance_scale=float(inp.get("guidance_scale", 12)),
        scheduler=inp.get("scheduler", "DPMSolverMultistep"),
        seed=int(inp["seed"]),
    )
    t1 = time.perf_counter()
    png = encode_png(img, png_level)
    dag = wrap_directory([("out-1.png", png)])
    t2 = time.perf_counter()
    tm = dict(getattr(pipe, "timings", {}))
    tm.update({"infer_s": t1 - t0, "encode_cid_s": t2 - t1})
    return Solution([("out-1.png", png)], dag.cid_hex, dag, tm)


_ENCODE_POOL = None


def _encode_pool():
    """Threads for the per-image PNG + CID work of a group (the native PNG encoder and hashlib
    release the GIL, so a group's images encode in parallel)."""
    global _ENCODE_POOL
    if _ENCODE_POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _ENCODE_POOL = ThreadPoolExecutor(max_workers=8, thread_name_prefix="png")
    return _ENCODE_POOL


def infer_images(pipe, inps: List[dict]):
    """The GPU part of ``solve_images``: k compatible SD-family tasks lock-step (``run_group``) ->
    (uint8 images, timings).  Returning here lets a task slot hand its pipeline to the next group
    while ``encode_images`` runs on the CPU."""
    t0 = time.perf_counter()
    imgs = pipe.run_group(list(inps))
    tm = dict(getattr(pipe, "timings", {}))
    tm.update({"infer_s": time.perf_counter() - t0, "group": len(inps)})
    return imgs, tm


def _one_png(img, png_level):
    png = encode_png(img, png_level)
    dag = wrap_directory([("out-1.png", png)])
    return Solution([("out-1.png", png)], dag.cid_hex, dag, {})


def encode_images(imgs, tm: dict, png_level: int = 6) -> List[Solution]:
    """PNG + wrapped-directory CID of every image of a group, the images in parallel (bytes are
    independent of the thread that encodes them)."""
    t1 = time.perf_counter()
    if len(imgs) > 1:
        out = list(_encode_pool().map(lambda im: _one_png(im, png_level), imgs))
    else:
        out = [_one_png(im, png_level) for im in imgs]
    tm = dict(tm)
    tm["encode_cid_s"] = time.perf_counter() - t1
    for s in out:
        s.timings = dict(tm)
    return out


def solve_images(pipe, inps: List[dict], png_level: int = 6) -> List[Solution]:
    """k compatible SD-family tasks solved lock-step (``run_group``): same bytes as k solo solves."""
    if len(inps) == 1 or not hasattr(pipe, "run_group"):     # e.g. Kandinsky 2: one at a time
        return [pipe.solve(i) if hasattr(pipe, "solve") else solve_image(pipe, i, png_level) for i in inps]
    imgs, tm = infer_images(pipe, inps)
    return encode_images(imgs, tm, png_level)


# Per-family defaults of the lock-step key fields (what each pipeline's ``run_group`` fills in for a
# missing input): SD-family templates (anythingv3) vs the Kandinsky 2 container's hidden defaults.
_GROUP_DEFAULTS = {"kandinsky2": (768, 768, 100, "p_sampler")}
_SD_DEFAULTS = (768, 768, 20, "DPMSolverMultistep")


def group_key(inp: dict, model: str = None):
    """Tasks with equal keys can share lock-step launches (image templates): resolution, step count
    and scheduler, missing fields filled with the MODEL FAMILY's defaults - a Kandinsky2 task without
    ``num_inference_steps`` runs 100 steps, not the SD default 20, so it must not join a group of
    explicit 20-step tasks."""
    w, h, n, sch = _GROUP_DEFAULTS.get(model, _SD_DEFAULTS)
    return (int(inp.get("width", w)), int(inp.get("height", h)), int(inp.get("num_inference_steps", n)),
            str(inp.get("scheduler", sch)))


def take_group(jobs, first, lockstep: int, kind_of, inp_of, model_of):
    """Lock-step batching for a task-slot loop: after ``first`` came off the ``jobs`` queue, take
    up to ``lockstep - 1`` more queued jobs that can share its launches (image tasks of the same
    model with equal ``group_key``) without waiting; anything else goes back on the queue."""
    batch = [first]
    if lockstep <= 1 or kind_of(first) != "image":
        return batch
    import queue as _q
    key = (model_of(first), group_key(inp_of(first), model_of(first)))
    back = []
    while len(batch) < lockstep:
        try:
            m = jobs.get_nowait()
        except _q.Empty:
            break
        if m is not None and kind_of(m) == "image" and (model_of(m), group_key(inp_of(m), model_of(m))) == key:
            batch.append(m)
        else:
            back.append(m)
            if m is None:
                break
    for m in back:
        jobs.put(m)
    return batch


def solve_files(files, timings=None) -> Solution:
    dag = wrap_directory(list(files))
    return Solution(list(files), dag.cid_hex, dag, dict(timings or {}))


def solve_task(model, pipe, inp: dict) -> Solution:
    """Dispatch by template output kind: image -> out-1.png, video/matting -> out-1.mp4."""
    if hasattr(pipe, "solve"):
        return pipe.solve(inp)
    if model.kind == "image":
        return solve_image(pipe, inp)
    raise ValueError(f"no solver for model kind {model.kind}")


def infer_task(model, pipe, inp: dict):
    """Two-phase solve for task slots: the GPU part runs now, while the caller holds the pipeline;
    the returned callable is the CPU tail (encode + CID) and touches no pipeline state, so the slot
    can hand its pipeline / stream to the next task first.  Pipelines with a separable tail expose
    ``infer(inp) -> raw`` and a static ``finish(raw) -> Solution`` (RVM: the 1080p H.264 encode is
    longer than the matting); for the rest the tail is the finished solution.  Same bytes as
    ``solve_task``."""
    if hasattr(pipe, "infer") and hasattr(type(pipe), "finish"):
        raw = pipe.infer(inp)
        fin = type(pipe).finish
        return lambda: fin(raw)
    sol = solve_task(model, pipe, inp)
    return lambda: sol
