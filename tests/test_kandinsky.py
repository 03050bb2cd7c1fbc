"""Kandinsky 2.1 family (BASELINE config #3, the model enabled on mainnet):
sampler, padding-free encoders, fused modulated GroupNorm reference, and the
tiny-width pipeline through the whole node on CPU."""
import asyncio
import json
import math

import numpy as np
import pytest
import torch

from arbius_amd import ops
from arbius_amd.models.kandinsky2 import Kandinsky2Config, Kandinsky2Pipeline
from arbius_amd.models.layers import init_weights
from arbius_amd.models.prior import PriorConfig, PriorTransformer
from arbius_amd.models.schedulers import GaussianDiffusion, TaskSampler, space_timesteps
from arbius_amd.models.xlmr import MCLIPText, XLMRConfig
from arbius_amd.node.pool import LocalSolverPool

from test_node_e2e import _full_cycle, make_miner, make_world


def test_space_timesteps_matches_guided_diffusion():
    assert space_timesteps(1000, 5) == [0, 250, 500, 749, 999]
    s = space_timesteps(1000, 100)
    assert len(s) == 100 and s[0] == 0 and s[-1] == 999 and s[1] == 10


def test_gaussian_diffusion_last_step_is_mean_and_var_range():
    sched = GaussianDiffusion(10, predict="eps", learned_var=True)
    x = torch.randn(1, 4, 4, 4)
    eps = torch.randn_like(x)
    g = torch.Generator().manual_seed(0)
    ts = TaskSampler(sched, x, g, "cpu")
    assert ts.noise.shape[0] == 9                         # no draw at the final (j == 0) step
    out = torch.cat([eps, torch.zeros_like(eps)], -1)      # eps + learned-variance channels
    from arbius_amd import ops
    ops.ref.sampler_step([ts.task_args(9, out, out, 1.0)])
    a = float(sched.ac[0])
    x0 = (x - math.sqrt(1 - a) * eps) / math.sqrt(a)
    # j == 0: ac_prev = 1 -> posterior mean is exactly x0, no noise
    assert torch.allclose(ts.x, x0, atol=1e-5)
    # var = +1 -> log beta ; var = -1 -> clipped posterior log variance
    j = 5
    b = float(sched.betas[j])
    assert b > math.exp(float(sched.post_logvar[j]))


def test_group_norm_mod_reference_matches_composite():
    torch.manual_seed(0)
    x = torch.randn(2, 8, 12, 64)
    mod = torch.randn(2, 2, 3, 128)
    gm, bt = torch.rand(64) + 0.5, torch.randn(64)
    y = ops.spatial_norm(x, mod, gm, bt, 8, 1e-6, silu=True)
    gn = torch.nn.functional.group_norm(x.permute(0, 3, 1, 2), 8, gm, bt, 1e-6).permute(0, 2, 3, 1)
    up = mod.repeat_interleave(4, 1).repeat_interleave(4, 2)
    ref = torch.nn.functional.silu(gn * up[..., :64] + up[..., 64:])
    assert torch.allclose(y, ref, atol=1e-4)
    ss = torch.randn(2, 128)
    y2 = ops.scale_shift_norm(x, ss, gm, bt, 8, 1e-5, silu=False)
    gn = torch.nn.functional.group_norm(x.permute(0, 3, 1, 2), 8, gm, bt, 1e-5).permute(0, 2, 3, 1)
    assert torch.allclose(y2, gn * (1 + ss[:, None, None, :64]) + ss[:, None, None, 64:], atol=1e-4)


def _masked_attn(q, k, v, mask):
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) / math.sqrt(q.shape[-1])
    s = s.masked_fill(~mask[:, None], float("-inf"))
    return torch.einsum("bhqk,bkhd->bqhd", s.softmax(-1), v)


def test_xlmr_kv_slicing_equals_key_padding_mask():
    """Slicing K/V to the real length == the reference's key-padding mask (all 77 outputs)."""
    cfg = XLMRConfig.tiny()
    m = init_weights(torch.nn.ModuleDict({"x": MCLIPText(cfg)}), 1)["x"].eval()
    n = 9
    ids = torch.tensor([[0] + list(range(5, 5 + n - 2)) + [2] + [1] * (77 - n)])
    full, pooled = m(ids, n)
    # reference: masked attention over all 77 keys
    pos = torch.arange(77)
    pos = torch.where(pos < n, pos + 2, torch.full_like(pos, 1))
    x = m.ln(m.tok(ids) + m.pos(pos)[None] + m.tok_type.weight[0])
    mask = (torch.arange(77) < n)[None, None, :].expand(1, 77, 77)
    for layer in m.layers:
        B, N, C = x.shape
        qkv = layer.qkv(x).view(B, N, 3, layer.heads, C // layer.heads)
        o = _masked_attn(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], mask)
        x = layer.ln1(layer.out(o.reshape(B, N, C), residual=x))
        x = layer.ln2(layer.fc2(torch.nn.functional.gelu(layer.fc1(x)), residual=x))
    assert torch.allclose(full, x, atol=1e-5)
    assert torch.allclose(pooled, m.proj(x[:, :n].mean(1)), atol=1e-5)


def test_prior_pad_removal_equals_causal_plus_padding_mask():
    cfg = PriorConfig.tiny()
    p = init_weights(torch.nn.ModuleDict({"p": PriorTransformer(cfg)}), 2)["p"].eval()
    d, n = cfg.clip_dim, 6
    torch.manual_seed(0)
    xt, states, pooled = torch.randn(1, d), torch.randn(1, 77, d), torch.randn(1, d)
    got = p(xt, 500, states, pooled, [n])
    # reference: full 81-token sequence, causal mask AND text-padding mask
    from arbius_amd.models.layers import timestep_embedding
    w = cfg.width
    temb = p.time2(torch.nn.functional.silu(p.time1(timestep_embedding(torch.tensor([500.0]), w))))
    seq = torch.cat([p.text_enc_proj(states), p.text_emb_proj(pooled)[:, None], temb[:, None],
                     p.img_proj(xt)[:, None], p.query[None, None]], dim=1) + p.pos[None]
    L = seq.shape[1]
    keep = torch.cat([torch.arange(77) < n, torch.ones(4, dtype=torch.bool)])
    mask = torch.tril(torch.ones(L, L, dtype=torch.bool)) & keep[None, :]
    h = seq
    for blk in p.blocks:
        B, N, C = h.shape
        qkv = blk.qkv(blk.ln1(h)).view(B, N, 3, blk.heads, C // blk.heads)
        o = _masked_attn(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], mask[None])
        h = blk.out(o.reshape(B, N, C), residual=h)
        h = blk.fc2(torch.nn.functional.gelu(blk.fc1(blk.ln2(h))), residual=h)
    ref = p.out_proj(p.final_ln(h[:, -1]))
    assert torch.allclose(got, ref, atol=1e-5)


def test_prior_batched_rows_with_different_lengths_equal_solo():
    """Rows padded to 81 tokens with trailing pads: a batch of sequences of different prompt lengths
    gives each row its solo result (causal attention never reaches a trailing pad)."""
    cfg = PriorConfig.tiny()
    p = init_weights(torch.nn.ModuleDict({"p": PriorTransformer(cfg)}), 3)["p"].eval()
    d = cfg.clip_dim
    torch.manual_seed(1)
    xt, states, pooled = torch.randn(3, d), torch.randn(3, 77, d), torch.randn(3, d)
    ns = [4, 11, 77]
    got = p(xt, 250, states, pooled, ns)
    for b, n in enumerate(ns):
        solo = p(xt[b:b + 1], 250, states[b:b + 1], pooled[b:b + 1], [n])
        assert torch.allclose(got[b:b + 1], solo, atol=1e-5)


def test_k2_template_surface_and_group_on_cpu():
    """The documented Kandinsky 2 inputs (num_inference_steps, guidance_scale, scheduler in
    {p_sampler, ddim_sampler, pims_sampler}, prior_cf_scale, prior_steps) change the output; a
    lock-step group with mixed guidance / prior settings matches the solo solves."""
    pipe = Kandinsky2Pipeline(Kandinsky2Config.tiny(), device="cpu")
    base = {"prompt": "arbius test cat", "width": 64, "height": 64, "seed": 7, "num_inference_steps": 4}
    outs = {}
    for key, val in (("scheduler", "p_sampler"), ("scheduler", "ddim_sampler"), ("scheduler", "pims_sampler"),
                     ("guidance_scale", 9.0), ("prior_cf_scale", 1), ("prior_steps", "3")):
        outs[(key, val)] = pipe.run_group([dict(base, **{key: val})])[0]
    ref = outs[("scheduler", "p_sampler")]
    for k, v in outs.items():
        if k != ("scheduler", "p_sampler"):
            assert not (v == ref).all(), k
    with pytest.raises(ValueError):
        pipe.run_group([dict(base, scheduler="euler")])
    inps = [dict(base, prompt=f"cat {i}", seed=20 + i, guidance_scale=4.0 + i, prior_cf_scale=1 + i,
                 prior_steps="3" if i == 1 else "5", scheduler="ddim_sampler") for i in range(3)]
    grp = pipe.run_group(inps)
    for inp, g in zip(inps, grp):
        solo = pipe.run_group([inp])[0]
        assert np.abs(solo.astype(int) - g.astype(int)).max() <= 1


def test_kandinsky_tiny_deterministic():
    pipe = Kandinsky2Pipeline(Kandinsky2Config.tiny(), device="cpu")
    a = pipe("arbius test cat", width=64, height=64, seed=1337)
    b = pipe("arbius test cat", width=64, height=64, seed=1337)
    c = pipe("arbius test cat", width=64, height=64, seed=1338)
    assert a.shape == (64, 64, 3) and a.dtype == np.uint8
    assert (a == b).all() and not (a == c).all()


def test_kandinsky_tiny_through_node():
    """Template kandinsky2 (768^2 default input) through boot/poll/solve/claim on CPU."""
    e, tok, mid = make_world("kandinsky2")
    pool = LocalSolverPool("cpu", tiny=True)
    m = make_miner(e, mid, pool, model="kandinsky2")
    tid = asyncio.run(_full_cycle(e, mid, m, {"prompt": "arbius test cat"}))
    model = m.models[mid.lower()]
    row = json.loads(m.db.get_task_input(tid, e.tasks[tid].cid)["data"])
    assert row == {"prompt": "arbius test cat", "width": 768, "height": 768, "seed": row["seed"]}
    assert pool.solve_sync(model, tid, row).cid == e.solutions[tid].cid
