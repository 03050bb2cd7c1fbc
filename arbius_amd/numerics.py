"""Consensus numerics: the version of this node's output bytes, the golden CIDs that pin it on
gfx950, and the env knobs that would change it.

A solution is valid only if every honest miner produces the same bytes, and
CIDs are hardware-specific (``docs/src/pages/register-model.mdx:78-80``): the reference pins one
A100 CID in its boot self-test (``miner/src/index.ts:981-1001``).  This node pins a set of
golden tasks per (hardware, weights) in ``tests/golden_cids.json``; every kernel, plan, sampler
or encoder change that flips one output bit fails ``tests/test_golden_gpu.py`` until
``NUMERICS_VERSION`` is bumped and the goldens are re-pinned (``scripts/pin_goldens.py``).  Two
nodes on the same NUMERICS_VERSION produce the same CIDs; nodes on different versions would
contest each other and must not mine the same model registration.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Tuple

# bump on ANY change of output bytes (kernels, conv plans, sampler arithmetic, PNG/MP4 encoders)
NUMERICS_VERSION = "r5.2-gn-slice-one-launch"
# The deflate implementation behind every PNG's IDAT stream (consensus bytes: zlib-ng or another zlib
# version emits different streams for the same pixels).  The native runtime links this one statically
# (native/build.py); ``check_mining_env`` refuses any other, and tests/test_encoder_golden.py pins the
# exact PNG / MP4 bytes of fixed inputs on the CPU.
DEFLATE_ID = "zlib-1.2.11"

# Environment knobs that select a different kernel library, plan table, tiling or reference ops.
# They exist for A/B measurement only; ``start`` refuses to mine with any of them set.
NUMERICS_ENV_KNOBS = (
    "ARBIUS_PLAN_CANON", "ARB_CONV_PLANS", "ARB_GN_GROUP", "ARBIUS_NORM_PROLOGUE", "ARBIUS_KERNEL_LIB",
    "ARBIUS_EXPERIMENT_SKIP", "ARBIUS_REFERENCE_OPS", "ARB_ATTN_GLDS", "ARB_ATTN_QT", "ARB_LN_ROWS",
    "ARB_SPLITK_INLAUNCH", "ARBIUS_GEGLU_FUSED", "ARBIUS_CROSS_KV_HOIST", "ARBIUS_FAULT_INJECTION",
    "ARBIUS_SAMPLER_REF", "ARB_GN_TABLE_LDS", "ARB_VAE_GRAPH", "ARB_PINNED_D2H", "ARB_PRIOR_GRAPH",
    "ARB_ATTN_PP", "ARB_LN_FOLD_NARROW", "ARB_LN_FOLD_NARROW_N", "ARBIUS_LIBRARY_FALLBACK", "ARB_ATTN_PRESCALE",
    # tile-family / layout switches read by the kernel library (bitwise-neutral by test, but their
    # neutrality then rests on a run-time file or an untested combination: refused all the same)
    "ARB_CONV_FAMILY", "ARB_NO_FAMILY", "ARB_DMA_BUF", "ARB_STAG2_PD", "ARB_GN_APPLY2", "ARB_GN_FUSED",
    "ARB_LN_PACKED", "ARB_ATTN512", "ARB_CAPTURE_SIDE", "ARB_QUEUE_CHECK", "ARB_RVM_GPU_YUV",
    "ARB_RVM_BLOCKING_SYNC", "ARB_K2_SPLIT_CFG", "ARB_GN_TAIL", "ARB_GN_SLICE", "ARB_ATTN_ILP",
)


def numerics_env_overrides(env=None) -> Dict[str, str]:
    env = os.environ if env is None else env
    return {k: env[k] for k in NUMERICS_ENV_KNOBS if env.get(k, "") != ""}


def deflate_identity() -> str:
    """The deflate that would encode this node's PNGs: the native module's static zlib, else the
    Python ``zlib`` module's runtime library (the pure-Python encoder path)."""
    from . import native
    if native.loaded:
        return native.deflate_id()
    import zlib
    return f"zlib-{zlib.ZLIB_RUNTIME_VERSION}"


def check_mining_env(env=None, deflate_id=None) -> None:
    """Refuse to mine with a numerics-changing knob set, or with a PNG deflate other than the pinned
    one: either would produce non-consensus CIDs."""
    bad = numerics_env_overrides(env)
    if bad:
        raise SystemExit("refusing to mine: numerics-changing environment knobs are set "
                         f"({', '.join(f'{k}={v}' for k, v in sorted(bad.items()))}); their outputs differ from "
                         f"every other node on NUMERICS_VERSION {NUMERICS_VERSION}. Unset them.")
    got = deflate_identity() if deflate_id is None else deflate_id
    if got != DEFLATE_ID:
        raise SystemExit(f"refusing to mine: the PNG encoder's deflate is {got}, consensus pins {DEFLATE_ID} "
                         "(NUMERICS_VERSION " + NUMERICS_VERSION + "): its IDAT bytes - and every image CID - would "
                         "differ. Rebuild the native runtime (python -m arbius_amd.native.build) against the "
                         "pinned static zlib.")


# ---------------------------------------------------------------------------------------------
# golden tasks (run on one GPU by tests/test_golden_gpu.py and scripts/pin_goldens.py)
def _sd_inp(prompt, seed, res, steps, sched, g, neg="blurry, lowres"):
    return {"prompt": prompt, "negative_prompt": neg, "width": res, "height": res, "num_inference_steps": steps,
            "guidance_scale": g, "scheduler": sched, "seed": seed}


SD_SOLO = _sd_inp("arbius test cat", 1337, 512, 4, "DPMSolverMultistep", 12.0)
SD_GROUP = [_sd_inp(f"a detailed anime illustration of a castle, golden {i}", 2000 + i, 512, 4,
                    "DPMSolverMultistep", 7.0 + i) for i in range(8)]
SD_SCHEDULERS = ("DDIM", "K_EULER", "K_EULER_ANCESTRAL", "DPMSolverMultistep", "PNDM", "KLMS")


def golden_cases(device) -> List[Tuple[str, Callable[[], object]]]:
    """(name, fn) pairs; fn() -> a CID hex string or a list of them.  Pipelines are built lazily
    and shared between cases of one family."""
    from .models.registry import build_pipeline
    from .node.solver import solve_image, solve_images

    cache: Dict[str, object] = {}

    def pipe(name):
        if name not in cache:
            cache[name] = build_pipeline(name, device=device)
        return cache[name]

    def sd_solo():
        return solve_image(pipe("anythingv3"), SD_SOLO).cid

    def sd_group_streams():
        """8 tasks as 2 concurrent streams x lock-step groups of 4 (the bench configuration):
        every CID must equal its solo CID."""
        from concurrent.futures import ThreadPoolExecutor
        base = pipe("anythingv3")
        forks = [base.fork(), base.fork()]
        with ThreadPoolExecutor(2) as ex:
            futs = [ex.submit(solve_images, forks[j], SD_GROUP[4 * j:4 * j + 4]) for j in range(2)]
            grouped = [s.cid for f in futs for s in f.result()]
        solo = [solve_image(base, i).cid for i in SD_GROUP]
        if grouped != solo:
            raise AssertionError(f"lock-step/stream CIDs differ from solo: {grouped} vs {solo}")
        return grouped

    def sd_group(k):
        """one stream, a lock-step group of k (k = 2, 3: the batch-4 / batch-6 tile-family entries of
        csrc/conv_family.inc) - every CID must equal its solo CID (also pinned by name)."""
        def f():
            base = pipe("anythingv3")
            grouped = [s.cid for s in solve_images(base, SD_GROUP[:k])]
            solo = [solve_image(base, i).cid for i in SD_GROUP[:k]]
            if grouped != solo:
                raise AssertionError(f"lock-step group of {k} differs from solo: {grouped} vs {solo}")
            return grouped
        return f

    def sd_template_default():
        """anythingv3's template defaults (templates/anythingv3.json: 768^2, 20 steps, guidance 12,
        DPMSolverMultistep) with the template's default negative prompt."""
        from .node.models import hydrate_input, load_template
        tpl = load_template("anythingv3")
        neg = next(f["default"] for f in tpl["input"] if f["variable"] == "negative_prompt")   # required field
        inp, err, msg = hydrate_input({"prompt": "arbius test cat", "negative_prompt": neg}, tpl)
        if err:
            raise AssertionError(msg)
        inp["seed"] = 1337
        return solve_image(pipe("anythingv3"), inp).cid

    def k2_group2():
        """Kandinsky2 768^2, a lock-step group of 2 with different guidance / prior settings: batched
        text towers + prior + batch-4 GLIDE UNet launches; CIDs equal the solo solves."""
        from .node.solver import solve_images as group_solve
        p = pipe("kandinsky2")
        inps = [{"prompt": f"arbius test cat {j}", "width": 768, "height": 768, "seed": 4000 + j,
                 "num_inference_steps": 2, "prior_steps": "2", "guidance_scale": 4.0 + j, "prior_cf_scale": 4 - j}
                for j in range(2)]
        grouped = [s.cid for s in group_solve(p, inps)]
        solo = [p.solve(i).cid for i in inps]
        if grouped != solo:
            raise AssertionError(f"K2 lock-step group differs from solo: {grouped} vs {solo}")
        return grouped

    def k2_sampler(name):
        def f():
            return pipe("kandinsky2").solve({"prompt": "arbius test cat", "width": 768, "height": 768, "seed": 1337,
                                             "num_inference_steps": 4, "prior_steps": "2",
                                             "scheduler": name}).cid
        return f

    def sd_sched(s):
        return lambda: solve_image(pipe("anythingv3"), _sd_inp("arbius test cat", 42, 256, 3, s, 7.0)).cid

    def k2():
        p = pipe("kandinsky2")
        old = (p.cfg.num_steps, p.cfg.prior_steps)
        p.cfg.num_steps, p.cfg.prior_steps = 2, 2
        try:
            return p.solve({"prompt": "arbius test cat", "width": 768, "height": 768, "seed": 1337}).cid
        finally:
            p.cfg.num_steps, p.cfg.prior_steps = old

    def video(name):
        def f():
            if name == "damo":      # templates/damo.json inputs only (no negative prompt / size / guidance)
                inp = {"prompt": "a red cat walking on a castle wall", "num_frames": 8, "num_inference_steps": 2,
                       "fps": 8, "seed": 1337}
            else:
                inp = {"prompt": "a red cat walking on a castle wall", "negative_prompt": "blurry", "num_frames": 8,
                       "width": 256, "height": 256, "num_inference_steps": 2, "guidance_scale": 9.0, "fps": 8,
                       "seed": 1337}
            return pipe(name).solve(inp).cid
        return f

    def rvm():
        import numpy as np

        from .node.solver import solve_files
        from .utils.mp4 import encode_mp4
        rng = np.random.default_rng(1337)
        clip = rng.integers(0, 256, (8, 180, 320, 3), dtype=np.uint8)
        out = pipe("robust_video_matting")(clip, "green-screen")
        return solve_files([("out-1.mp4", encode_mp4(list(out), 24))]).cid

    def sd_1024():
        """the largest anythingv3 size (1024^2: 16,384-token spatial attention), 2 steps"""
        inp = _sd_inp("arbius test cat", 1337, 1024, 2, "DPMSolverMultistep", 12.0)
        return solve_image(pipe("anythingv3"), inp).cid

    def k2_1024():
        """kandinsky2 at its largest template size (1024^2), 2 decoder + 2 prior steps"""
        return pipe("kandinsky2").solve({"prompt": "arbius test cat", "width": 1024, "height": 1024, "seed": 1337,
                                         "num_inference_steps": 2, "prior_steps": "2"}).cid

    def zeroscope_template_default():
        """zeroscopev2xl at its template defaults (templates/zeroscopev2xl.json: 1024x576, 24 frames,
        guidance 17.5, fps 24; spatial attention over 9,216 tokens) with 2 denoising steps"""
        from .node.models import hydrate_input, load_template
        tpl = load_template("zeroscopev2xl")
        inp, err, msg = hydrate_input({"prompt": "a red cat walking on a castle wall",
                                       "negative_prompt": "noisy, washed out, ugly, distorted, broken",
                                       "num_inference_steps": 2}, tpl)
        if err:
            raise AssertionError(msg)
        inp["seed"] = 1337
        return pipe("zeroscopev2xl").solve(inp).cid

    cases = [("sd15_512_dpm4_solo", sd_solo), ("sd15_512_dpm4_2streams_group4", sd_group_streams)]
    cases += [(f"sd15_256_{s}_3", sd_sched(s)) for s in SD_SCHEDULERS]
    cases += [("sd15_512_dpm4_group2", sd_group(2)), ("sd15_512_dpm4_group3", sd_group(3)),
              ("sd15_768_dpm20_template_default", sd_template_default)]
    cases += [("kandinsky2_768_group2", k2_group2)]
    cases += [(f"kandinsky2_768_{n}_4", k2_sampler(n)) for n in ("ddim_sampler", "pims_sampler")]
    cases += [("kandinsky2_768_2+2", k2), ("zeroscopev2xl_256x256x8_2", video("zeroscopev2xl")),
              ("damo_256x256x8_2", video("damo")), ("rvm_320x180x8", rvm)]
    cases += [("sd15_1024_dpm2", sd_1024), ("kandinsky2_1024_2+2", k2_1024),
              ("zeroscopev2xl_1024x576x24_2_template_default", zeroscope_template_default)]
    return cases


def selftest_cids(device, names=("kandinsky2", "anythingv3")) -> Dict[str, str]:
    """The boot self-test tasks of ``config/selftest.json`` solved exactly as ``Miner.self_test``
    does (template hydration + the task's seed + ``solve_task``) -> {model: CID}."""
    import json
    from pathlib import Path

    from .models.registry import build_pipeline
    from .node.models import Model, hydrate_input, load_template
    from .node.solver import solve_task
    table = json.loads((Path(__file__).resolve().parent / "config" / "selftest.json").read_text())
    out = {}
    for name in names:
        tpl = load_template(name)
        inp, err, msg = hydrate_input(dict(table[name]["input"]), tpl)
        if err:
            raise ValueError(f"self test input of {name}: {msg}")
        inp["seed"] = table[name]["input"]["seed"]
        pipe = build_pipeline(name, device=device)
        out[name] = solve_task(Model("0x0", name, tpl), pipe, inp).cid
        del pipe
    return out
