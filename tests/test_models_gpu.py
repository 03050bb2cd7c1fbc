"""Model-level GPU checks: every family runs on the HIP kernels (native library
loaded, no eager fallback), is bitwise deterministic run-to-run, and tracks the
fp32 PyTorch reference ops within bf16 tolerance."""
import numpy as np
import pytest
import torch

from arbius_amd import ops
from arbius_amd.models.registry import build_pipeline

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_glide_unet_hip_vs_reference(cuda):
    from arbius_amd.models.glide_unet import GlideUNet, GlideUNetConfig
    from arbius_amd.models.layers import init_weights
    cfg = GlideUNetConfig(model_channels=128, channel_mult=(1, 2), num_res_blocks=1, attention_ds=(2,),
                          head_channels=64, text_dim=128, pooled_dim=128, encoder_channels=128,
                          image_embed_dim=128, image_tokens=2, groups=32)
    m = init_weights(torch.nn.ModuleDict({"u": GlideUNet(cfg)}), 3)["u"].to(cuda, torch.bfloat16).eval()
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 32, 32, 4, generator=g).to(cuda, torch.bfloat16)
    t = torch.tensor([500.0], device=cuda)
    tt = torch.randn(2, 77, 128, generator=g).to(cuda, torch.bfloat16)
    tp = torch.randn(2, 128, generator=g).to(cuda, torch.bfloat16)
    ie = torch.randn(2, 128, generator=g).to(cuda, torch.bfloat16)
    with torch.no_grad():
        y = m(x, t, tt, tp, ie)
        assert ops.native_loaded()
        ops.set_reference_ops(True)
        try:
            r = m(x, t, tt, tp, ie)
        finally:
            ops.set_reference_ops(False)
    assert _rel(y, r) < 5e-2


def test_kandinsky_full_arch_768_two_steps(cuda):
    pipe = build_pipeline("kandinsky2", device=cuda)
    kw = dict(width=768, height=768, seed=1337, num_inference_steps=2, prior_steps=2)
    a = pipe("arbius test cat", **kw)
    b = pipe("arbius test cat", **kw)
    assert ops.native_loaded()
    assert a.shape == (768, 768, 3) and a.dtype == np.uint8
    assert (a == b).all(), "kandinsky2 must be bitwise deterministic"


def test_sd15_full_arch_128_deterministic(cuda):
    pipe = build_pipeline("anythingv3", device=cuda)
    kw = dict(width=128, height=128, num_inference_steps=3, scheduler="DPMSolverMultistep", seed=7)
    a = pipe("arbius test cat", **kw)
    b = pipe("arbius test cat", **kw)
    assert ops.native_loaded() and (a == b).all()


def test_sd15_unet_hip_vs_reference(cuda):
    pipe = build_pipeline("anythingv3", device=cuda, use_graphs=False)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 32, 32, 4, generator=g).to(cuda, torch.bfloat16)
    ctx = torch.randn(2, 77, 768, generator=g).to(cuda, torch.bfloat16)
    t = torch.tensor([400.0], device=cuda)
    with torch.no_grad():
        y = pipe.unet(x, t, ctx)
        ops.set_reference_ops(True)
        try:
            r = pipe.unet(x, t, ctx)
        finally:
            ops.set_reference_ops(False)
    assert _rel(y, r) < 5e-2


def test_unet3d_hip_vs_reference(cuda):
    from arbius_amd.models.layers import init_weights
    from arbius_amd.models.unet3d import UNet3DCondition, UNet3DConfig
    cfg = UNet3DConfig(block_channels=(64, 128, 128, 128), layers_per_block=1, head_dim=64, in_heads=2,
                       cross_dim=64, groups=32, time_dim=64)
    m = init_weights(torch.nn.ModuleDict({"u": UNet3DCondition(cfg)}), 5)["u"].to(cuda, torch.bfloat16).eval()
    g = torch.Generator().manual_seed(0)
    F = 6
    x = torch.randn(2 * F, 16, 16, 4, generator=g).to(cuda, torch.bfloat16)
    ctx = torch.randn(2, 77, 64, generator=g).to(cuda, torch.bfloat16)
    t = torch.tensor([300.0], device=cuda)
    with torch.no_grad():
        y = m(x, t, ctx, frames=F)
        ops.set_reference_ops(True)
        try:
            r = m(x, t, ctx, frames=F)
        finally:
            ops.set_reference_ops(False)
    assert _rel(y, r) < 5e-2


def test_zeroscope_full_arch_small_mp4(cuda):
    pipe = build_pipeline("zeroscopev2xl", device=cuda)
    inp = {"prompt": "arbius test cat", "num_frames": 8, "width": 256, "height": 256, "num_inference_steps": 2,
           "seed": 11, "fps": 8}
    a, b = pipe.solve(inp), pipe.solve(inp)
    assert ops.native_loaded()
    assert a.files[0][0] == "out-1.mp4" and a.cid == b.cid, "video solutions must be deterministic"


def test_rvm_1080p_fp16_deterministic(cuda):
    import numpy as np
    pipe = build_pipeline("robust_video_matting", device=cuda)
    frames = np.random.default_rng(0).integers(0, 256, (6, 1080, 1920, 3), dtype=np.uint8)
    a = pipe(frames, "green-screen")
    b = pipe(frames, "green-screen")
    assert a.shape == frames.shape and (a == b).all()
    assert ops.native_loaded()


def test_concurrent_streams_bitwise_equal_solo(cuda):
    """Two pipeline forks on private HIP streams, solving concurrently from two threads,
    produce exactly the solo CIDs (hipGraph capture is thread-local and serialised)."""
    from concurrent.futures import ThreadPoolExecutor
    from arbius_amd.node.solver import solve_image
    pipe = build_pipeline("anythingv3", device=cuda)
    inps = [{"prompt": f"cat {i}", "negative_prompt": "", "width": 256, "height": 256, "num_inference_steps": 4,
             "guidance_scale": 7.5, "scheduler": "DPMSolverMultistep", "seed": 100 + i} for i in range(2)]
    solo = [solve_image(pipe, inp).cid for inp in inps]
    forks = [pipe.fork() for _ in range(2)]
    for f, inp in zip(forks, inps):          # capture each fork's graph first
        solve_image(f, inp)
    with ThreadPoolExecutor(2) as ex:
        for _ in range(3):
            conc = list(ex.map(lambda a: solve_image(a[0], a[1]).cid, zip(forks, inps)))
            assert conc == solo


def test_rvm_hip_convs_match_library_path(cuda):
    """The MFMA fp16 conv route of the matting network == the library (MIOpen) convs within
    fp16 rounding: output frames differ by at most a couple of 8-bit levels on average."""
    import numpy as np
    pipe = build_pipeline("robust_video_matting", device=cuda)
    frames = np.random.default_rng(1).integers(0, 256, (4, 360, 640, 3), dtype=np.uint8)
    a = pipe(frames, "alpha-mask").astype(np.float32)
    ops.set_reference_ops(True)
    try:
        b = pipe(frames, "alpha-mask").astype(np.float32)
    finally:
        ops.set_reference_ops(False)
    assert np.abs(a - b).mean() < 2.0, np.abs(a - b).mean()


def test_lockstep_group_bitwise_equals_solo(cuda):
    """Batch-invariant plans: k tasks solved lock-step in ONE batch-2k UNet launch sequence give
    exactly the solo CIDs (consensus must not depend on which tasks shared a launch)."""
    from arbius_amd.node.solver import solve_image, solve_images
    pipe = build_pipeline("anythingv3", device=cuda)
    inps = [{"prompt": f"castle {i}", "negative_prompt": "blurry", "width": 256, "height": 256,
             "num_inference_steps": 4, "guidance_scale": 7.0 + i, "scheduler": "DPMSolverMultistep",
             "seed": 40 + i} for i in range(3)]
    solo = [solve_image(pipe, i).cid for i in inps]
    assert [s.cid for s in solve_images(pipe, inps)] == solo
    assert [s.cid for s in solve_images(pipe, inps[:2])] == solo[:2]


def test_lockstep_group_of_8_at_512_bitwise_equals_solo(cuda):
    """The deployed SD1.5 groups of 8 (batch 16, mi355x.model_lockstep) run the batch-8 canonical plans'
    splits on tile families tuned for the batch-16 shapes (ratio-0 entries of conv_family.inc): every
    task's CID is its solo CID at the benchmark resolution, where those families apply."""
    from arbius_amd.node.solver import solve_image, solve_images
    pipe = build_pipeline("anythingv3", device=cuda)
    inps = [{"prompt": f"harbour at dawn {i}", "negative_prompt": "", "width": 512, "height": 512,
             "num_inference_steps": 3, "guidance_scale": 7.5, "scheduler": "DPMSolverMultistep",
             "seed": 70 + i} for i in range(8)]
    solo = [solve_image(pipe, i).cid for i in inps]
    assert [s.cid for s in solve_images(pipe, inps)] == solo


def test_local_pool_lockstep_groups_match_solo(cuda):
    """The node's single-GPU pool batches queued compatible tasks into lock-step groups; the
    solutions are the solo ones."""
    import asyncio
    from arbius_amd.node.models import default_models
    from arbius_amd.node.pool import LocalSolverPool
    from arbius_amd.node.solver import solve_image
    model = next(m for m in default_models({"anythingv3": "0x" + "ab" * 32}).values() if m.name == "anythingv3")
    pool = LocalSolverPool(cuda, capacity=1, lockstep=3)
    inps = [{"prompt": f"tower {i}", "negative_prompt": "", "width": 256, "height": 256,
             "num_inference_steps": 3, "guidance_scale": 7.5, "scheduler": "DDIM", "seed": 70 + i} for i in range(3)]

    async def go():
        return await asyncio.gather(*[pool.solve(model, f"t{i}", inp) for i, inp in enumerate(inps)])

    sols = asyncio.run(go())
    pipe = pool.pipes["anythingv3"]
    assert [s.cid for s in sols] == [solve_image(pipe, inp).cid for inp in inps]
    assert pool.capacity == 6       # 1 stream x group of 3 running + one group queued (pool depth 2)


def test_kandinsky2_lockstep_group_bitwise_equals_solo(cuda):
    from arbius_amd.node.solver import solve_images
    pipe = build_pipeline("kandinsky2", device=cuda)
    pipe.cfg.num_steps = 3
    inps = [{"prompt": f"arbius test cat {i}", "width": 256, "height": 256, "seed": 1337 + i} for i in range(2)]
    solo = [pipe.solve(i).cid for i in inps]
    assert [s.cid for s in solve_images(pipe, inps)] == solo


def test_kandinsky2_group_of_8_at_768_bitwise_equals_solo(cuda):
    """The shipped Kandinsky2 lock-step group (8 tasks = UNet batch 16 on the batch-16 tile families at
    the pinned splits, config/mining_config.py DEFAULT_MODEL_LOCKSTEP) at the template's 768^2: every
    CID equals its solo solve."""
    from arbius_amd.node.solver import solve_images
    pipe = build_pipeline("kandinsky2", device=cuda)
    pipe.cfg.num_steps = 3
    inps = [{"prompt": f"arbius group {i}" + " long" * (3 * i), "width": 768, "height": 768, "seed": 4242 + i}
            for i in range(8)]
    solo = [pipe.solve(i).cid for i in inps]
    assert [s.cid for s in solve_images(pipe, inps)] == solo


def _clear_derived_caches(pipe):
    ops._LN_FOLD.clear()
    ops._GEGLU_W.clear()
    ops._PAD_W.clear()
    unet = getattr(pipe, "unet", None)
    if unet is not None and hasattr(unet, "_temb_cache"):
        unet._temb_cache = None


@pytest.mark.parametrize("graphs", [False, True])
def test_cold_cache_concurrent_first_use_matches_solo(cuda, graphs):
    """Derived-weight caches (LayerNorm fold, GEGLU interleave, padded conv weights, batched time
    projection) are shared by pipeline forks on other threads and HIP streams: two forks whose FIRST
    solve races on an empty cache still give the solo CIDs (an entry is published only after the
    kernels that computed it finished - ``ops.derived_ready``)."""
    from concurrent.futures import ThreadPoolExecutor
    from arbius_amd.node.solver import solve_image
    pipe = build_pipeline("anythingv3", device=cuda, use_graphs=graphs)
    inps = [{"prompt": f"lake {i}", "negative_prompt": "", "width": 128, "height": 128, "num_inference_steps": 3,
             "guidance_scale": 7.5, "scheduler": "DPMSolverMultistep", "seed": 300 + i} for i in range(2)]
    solo = [solve_image(pipe, inp).cid for inp in inps]
    for _ in range(2):
        _clear_derived_caches(pipe)
        forks = [pipe.fork() for _ in range(2)]
        with ThreadPoolExecutor(2) as ex:
            conc = list(ex.map(lambda a: solve_image(a[0], a[1]).cid, zip(forks, inps)))
        assert conc == solo


def test_kandinsky2_prior_graph_bitwise_equals_eager(cuda):
    """The hipGraph replay of the diffusion-prior step (``prior_graph``, default on) gives the eager CIDs:
    a lock-step group of 2 with different prompt lengths and a mixed prior_steps group."""
    from arbius_amd.node.solver import solve_images
    pipe = build_pipeline("kandinsky2", device=cuda)
    pipe.cfg.num_steps = 2
    inps = [{"prompt": "cat", "width": 256, "height": 256, "seed": 5},
            {"prompt": "a very long prompt about a castle on a hill at dawn", "width": 256, "height": 256,
             "seed": 6, "prior_steps": "3"},
            {"prompt": "dog on a boat", "width": 256, "height": 256, "seed": 7}]
    pipe.prior_graph = False
    eager = [s.cid for s in solve_images(pipe, inps)]
    pipe.prior_graph = True
    graph = [s.cid for s in solve_images(pipe, inps)]
    assert graph == eager
    assert [pipe.solve(i).cid for i in inps] == eager


def test_kandinsky2_group_with_mixed_steps_splits(cuda):
    """A K2 group whose tasks differ in step count runs as separate lock-step groups (no failure)."""
    from arbius_amd.node.solver import solve_images
    pipe = build_pipeline("kandinsky2", device=cuda)
    inps = [{"prompt": "cat", "width": 256, "height": 256, "seed": 5, "num_inference_steps": 2},
            {"prompt": "cat", "width": 256, "height": 256, "seed": 6, "num_inference_steps": 3}]
    assert [s.cid for s in solve_images(pipe, inps)] == [pipe.solve(i).cid for i in inps]


def test_vae_graph_two_concurrent_forks_bitwise_equal_eager(cuda, monkeypatch):
    """the VAE decode replayed as a hipGraph on 2 forks solving concurrently from two
    threads gives the eager CIDs.  Every replay first checks that each captured input and output buffer
    is still the tensor the graph was captured on (GraphedCall.check_live)."""
    from concurrent.futures import ThreadPoolExecutor
    from arbius_amd.models import sd15
    from arbius_amd.node.solver import solve_image
    pipe = build_pipeline("anythingv3", device=cuda)
    inps = [{"prompt": f"harbour {i}", "negative_prompt": "", "width": 256, "height": 256,
             "num_inference_steps": 3, "guidance_scale": 7.5, "scheduler": "DPMSolverMultistep",
             "seed": 500 + i} for i in range(2)]
    eager = [solve_image(pipe, inp).cid for inp in inps]
    monkeypatch.setattr(sd15, "_VAE_GRAPH", True)
    forks = [pipe.fork() for _ in range(2)]
    with ThreadPoolExecutor(2) as ex:
        for _ in range(3):
            conc = list(ex.map(lambda a: solve_image(a[0], a[1]).cid, zip(forks, inps)))
            assert conc == eager
    assert all(len(f._vae_graph.graphs) == 1 for f in forks)


def test_kandinsky2_split_cfg_latency_mode_bitwise_equals_batch2(cuda):
    """Latency mode: a solo task's cond / uncond UNet rows as two batch-1 graph replays on two hardware
    queues give exactly the batch-2 solo bytes (and so the lock-step group's)."""
    pipe = build_pipeline("kandinsky2", device=cuda)
    pipe.cfg.num_steps = 4
    inps = [{"prompt": "a red fox in snow", "width": 768, "height": 768, "seed": 21},
            {"prompt": "harbour at night", "width": 512, "height": 512, "seed": 22}]
    pipe.split_cfg = False
    ref = [pipe.solve(i).cid for i in inps]
    pipe.split_cfg = True
    assert [pipe.solve(i).cid for i in inps] == ref
    assert pipe._split is not None
