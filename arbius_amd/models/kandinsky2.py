"""Kandinsky 2.1 text-to-image pipeline - the only model enabled on mainnet
(``miner/src/index.ts:844-876``, template ``templates/kandinsky2.json``; hidden
Cog defaults per ``docs/src/pages/register-model.mdx:140-185``: 100 steps,
guidance 4, ``p_sampler``, prior_cf_scale 4, prior_steps 5; 768^2 default).

    prompt ---> CLIP ViT-L/14 text ---> diffusion prior (5 steps, CFG 4, x0-pred,
            |                           causal transformer) --> CLIP image embedding
            '-> XLM-R (M-CLIP) -----> text states + pooled
    seed -> CPU generator -> prior noise, latent noise, per-step noise
    100 x { CFG batch-2 GLIDE UNet (hipGraph replay) -> guided eps + learned var
            -> ancestral p_sample }   (latent 4 x H/8 x W/8)
    MoVQ decode (SpatialNorm conditioned on the latent) -> uint8 RGB -> PNG

Unconditional branches: the empty prompt for both text towers and, for the
decoder, the CLIP image embedding of a blank image (``zero_img_emb``, a
checkpoint buffer; the reference computes it with the CLIP vision tower).
Random-init weights are deterministic per seed (BASELINE.json: synthetic
weights); byte-parity with the kasumi-1 container is "parity unpinned".
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn

from .. import ops
from ..utils.png import encode_png
from ..utils.progress import beat
from .clip_text import CLIPTextConfig, CLIPTextEncoder
from .glide_unet import GlideUNet, GlideUNetConfig
from .graphs import GraphCache, PipelineBase
from .layers import Linear, init_weights
from .movq import MoVQConfig, MoVQDecoder
from .prior import PriorConfig, PriorTransformer
from .schedulers import GaussianDiffusion, GroupSampler, TaskSampler
from .tokenizer import CLIPTokenizer
from .xlmr import MCLIPText, XLMRConfig, XLMRTokenizer


@dataclass
class Kandinsky2Config:
    unet: GlideUNetConfig = field(default_factory=GlideUNetConfig.kandinsky21)
    movq: MoVQConfig = field(default_factory=MoVQConfig.kandinsky21)
    prior: PriorConfig = field(default_factory=PriorConfig.kandinsky21)
    clip_text: CLIPTextConfig = field(default_factory=CLIPTextConfig.vit_l14)
    xlmr: XLMRConfig = field(default_factory=XLMRConfig.large)
    num_steps: int = 100
    guidance_scale: float = 4.0
    prior_cf_scale: float = 4.0
    prior_steps: int = 5
    latent_clamp: float = 2.0      # denoised_fn clamp(-2, 2)

    @staticmethod
    def tiny():
        return Kandinsky2Config(unet=GlideUNetConfig.tiny(), movq=MoVQConfig.tiny(), prior=PriorConfig.tiny(),
                                clip_text=CLIPTextConfig.tiny(32), xlmr=XLMRConfig.tiny(), num_steps=4)


class _Buffers(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.zero_img_emb = nn.Parameter(torch.zeros(d), requires_grad=False)

    def reset(self, gen):
        self.zero_img_emb.data.normal_(0.0, 0.5, generator=gen)


class Kandinsky2Pipeline(PipelineBase):
    def __init__(self, cfg: Kandinsky2Config = None, device="cpu", dtype=None, weight_seed: int = 0,
                 use_graphs: Optional[bool] = None, tokenizer_dir: Optional[str] = None, init=True):
        self.cfg = cfg = cfg or Kandinsky2Config()
        self.device = torch.device(device)
        if dtype is None:
            dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.dtype = dtype
        d = cfg.prior.clip_dim
        self.unet = GlideUNet(cfg.unet)
        self.movq = MoVQDecoder(cfg.movq)
        self.prior = PriorTransformer(cfg.prior)
        self.clip = CLIPTextEncoder(cfg.clip_text)
        self.clip_proj = Linear(cfg.clip_text.width, d, bias=False)
        self.xlmr = MCLIPText(cfg.xlmr)
        self.buffers = _Buffers(d)
        mods = self.modules()
        if init:
            for i, (name, m) in enumerate(mods.items()):
                init_weights(nn.ModuleDict({"m_" + name: m}), weight_seed + i)
        for m in mods.values():
            m.to(device=self.device, dtype=dtype).eval()
        self.clip_tok = CLIPTokenizer(tokenizer_dir, cfg.clip_text.max_len, cfg.clip_text.vocab)
        self.xlmr_tok = XLMRTokenizer(cfg.xlmr.vocab, cfg.xlmr.max_len, tokenizer_dir)
        self.use_graphs = (self.device.type == "cuda") if use_graphs is None else use_graphs
        self._unet = GraphCache(self.unet, self.use_graphs)
        self.timings: Dict[str, float] = {}

    def _reset_graphs(self):
        self._unet = GraphCache(self.unet, self.use_graphs)

    def modules(self) -> Dict[str, nn.Module]:
        return {"unet": self.unet, "movq": self.movq, "prior": self.prior, "clip": self.clip,
                "clip_proj": self.clip_proj, "xlmr": self.xlmr, "buffers": self.buffers}

    # ------------------------------------------------------------------------------------------
    def _clip_len(self, ids):
        eos = ids[-1]
        return ids.index(eos) + 1

    @torch.no_grad()
    def encode_clip(self, prompt: str):
        ids = [self.clip_tok(prompt), self.clip_tok("")]
        lens = [self._clip_len(i) for i in ids]
        hidden, pooled = self.clip(torch.tensor(ids, dtype=torch.long, device=self.device))
        return hidden, self.clip_proj(pooled), lens

    @torch.no_grad()
    def encode_xlmr(self, prompt: str):
        full, pooled = [], []
        for text in (prompt, ""):
            ids, n = self.xlmr_tok(text)
            f, p = self.xlmr(torch.tensor([ids], dtype=torch.long, device=self.device), n)
            full.append(f)
            pooled.append(p)
        return torch.cat(full), torch.cat(pooled)

    @torch.no_grad()
    def sample_prior(self, hidden, pooled, lens, gen, steps: int, cf_scale: float):
        d = self.cfg.prior.clip_dim
        sched = GaussianDiffusion(steps, schedule="cosine", predict="x0", learned_var=False)
        x = torch.randn((1, d), generator=gen, dtype=torch.float32)
        ts = TaskSampler(sched, x.view(d // 4, 4), gen, self.device)
        xin = torch.empty((d // 4, 4), dtype=self.dtype, device=self.device)

        def rows(k, out):     # out = (cond, uncond) prior outputs [1, d]
            return (None if out is None else out[1].reshape(-1, 4), None if out is None else out[0].reshape(-1, 4),
                    xin, None)

        samp = GroupSampler([ts], [float(cf_scale)], xin, rows)
        samp.write_input(0)
        for i, t in enumerate(sched.timesteps):
            beat()
            xv = xin.view(1, d)
            c = self.prior(xv, t, hidden[0:1], pooled[0:1], lens[0]).contiguous()
            u = self.prior(xv, t, hidden[1:2], pooled[1:2], lens[1]).contiguous()
            samp.step(i, (c, u))
        x = ts.x.view(1, d)
        return (x * self.prior.clip_std.float() + self.prior.clip_mean.float()).to(self.dtype)

    def _group_sampler(self, tasks, h, w):
        """k decoder tasks on one batch-2k GLIDE UNet input: rows 2k / 2k+1 = (cond, uncond); the
        cond row's channels 4..7 are the learned variance of p_sample."""
        zc = self.cfg.unet.in_channels
        xin = torch.empty((2 * len(tasks), h, w, zc), dtype=self.dtype, device=self.device)

        def rows(k, out):
            return (None if out is None else out[2 * k + 1], None if out is None else out[2 * k],
                    xin[2 * k], xin[2 * k + 1])

        samp = GroupSampler(tasks, [float(self.cfg.guidance_scale)] * len(tasks), xin, rows)
        samp.write_input(0)
        return samp

    @torch.no_grad()
    def __call__(self, prompt: str, width: int = 768, height: int = 768, seed: int = 0,
                 num_inference_steps: Optional[int] = None, guidance_scale: Optional[float] = None,
                 prior_cf_scale: Optional[float] = None, prior_steps: Optional[int] = None):
        with self._stream_ctx():
            return self._run(prompt, width, height, seed, num_inference_steps, guidance_scale, prior_cf_scale,
                             prior_steps)

    def _run(self, prompt, width, height, seed, num_inference_steps, guidance_scale, prior_cf_scale, prior_steps):
        cfg = self.cfg
        steps = num_inference_steps or cfg.num_steps
        g = cfg.guidance_scale if guidance_scale is None else guidance_scale
        sync = self._sync
        t0 = time.perf_counter()
        gen = torch.Generator(device="cpu").manual_seed(int(seed))
        hidden, pooled, lens = self.encode_clip(prompt)
        img_emb = self.sample_prior(hidden, pooled, lens, gen, prior_steps or cfg.prior_steps,
                                    cfg.prior_cf_scale if prior_cf_scale is None else prior_cf_scale)
        text_full, text_pooled = self.encode_xlmr(prompt)
        img_embs = torch.cat([img_emb, self.buffers.zero_img_emb[None].to(self.dtype)])
        sync()
        t1 = time.perf_counter()
        h, w = height // 8, width // 8
        zc = cfg.unet.in_channels
        x = torch.randn((1, zc, h, w), generator=gen, dtype=torch.float32).permute(0, 2, 3, 1).contiguous()
        sched = GaussianDiffusion(steps, schedule="linear", predict="eps", learned_var=True, clamp=cfg.latent_clamp)
        ts = TaskSampler(sched, x, gen, self.device)
        samp = self._group_sampler([ts], h, w)
        samp.g = [float(g)]
        tbuf = torch.zeros(1, dtype=torch.float32, device=self.device)
        for i, t in enumerate(sched.timesteps):
            beat()
            tbuf.fill_(float(t))
            with ops.plan_batch(2):      # batch-invariant plans: solo == lock-step group bytes
                out = self._unet(samp.xin, tbuf, text_full, text_pooled, img_embs)
            samp.step(i, out)            # ONE fused CFG + p_sample launch (learned variance, clamp)
        sync()
        t2 = time.perf_counter()
        img = self.decode(ts.x)
        sync()
        t3 = time.perf_counter()
        self.timings = {"text_prior_s": t1 - t0, "denoise_s": t2 - t1, "movq_s": t3 - t2}
        return img

    @torch.no_grad()
    def run_group(self, inps: List[dict]) -> List[np.ndarray]:
        """Lock-step solve of k tasks of one resolution: text encoders, prior, noise, sampler and
        MoVQ per task; every GLIDE UNet step runs the k (cond, uncond) pairs as one batch-2k
        launch sequence under batch-invariant plans (bitwise the solo outputs)."""
        sizes = {(int(i.get("width", 768)), int(i.get("height", 768))) for i in inps}
        if len(sizes) != 1:
            raise ValueError(f"run_group needs one resolution, got {sorted(sizes)}")
        width, height = sizes.pop()
        cfg = self.cfg
        with self._stream_ctx():
            sync = self._sync
            t0 = time.perf_counter()
            gens, xs, tf, tp, ie = [], [], [], [], []
            h, w = height // 8, width // 8
            zc = cfg.unet.in_channels
            for inp in inps:
                gen = torch.Generator(device="cpu").manual_seed(int(inp["seed"]))
                hidden, pooled, lens = self.encode_clip(inp["prompt"])
                img_emb = self.sample_prior(hidden, pooled, lens, gen, cfg.prior_steps, cfg.prior_cf_scale)
                text_full, text_pooled = self.encode_xlmr(inp["prompt"])
                tf.append(text_full)
                tp.append(text_pooled)
                ie.append(torch.cat([img_emb, self.buffers.zero_img_emb[None].to(self.dtype)]))
                x = torch.randn((1, zc, h, w), generator=gen, dtype=torch.float32).permute(0, 2, 3, 1).contiguous()
                sched = GaussianDiffusion(cfg.num_steps, schedule="linear", predict="eps", learned_var=True,
                                          clamp=cfg.latent_clamp)
                xs.append(TaskSampler(sched, x, gen, self.device))    # draws this task's noise now
                gens.append(gen)
            text_full, text_pooled, img_embs = torch.cat(tf), torch.cat(tp), torch.cat(ie)
            sync()
            t1 = time.perf_counter()
            samp = self._group_sampler(xs, h, w)
            tbuf = torch.zeros(1, dtype=torch.float32, device=self.device)
            for i, t in enumerate(xs[0].sched.timesteps):
                beat()
                tbuf.fill_(float(t))
                with ops.plan_batch(2):
                    out = self._unet(samp.xin, tbuf, text_full, text_pooled, img_embs)
                samp.step(i, out)
            sync()
            t2 = time.perf_counter()
            imgs = [self.decode(ts.x) for ts in xs]
            sync()
            self.timings = {"text_prior_s": t1 - t0, "denoise_s": t2 - t1, "movq_s": time.perf_counter() - t2}
            return imgs

    @torch.no_grad()
    def decode(self, latent):
        img = self.movq(latent.to(self.dtype))[0].float()
        img = ((img + 1.0) * 127.5).clamp(0, 255).round().to(torch.uint8)
        return img.cpu().numpy()

    def solve(self, inp: dict):
        """Template inputs (prompt, width, height, seed) -> ``out-1.png`` solution."""
        from ..node.solver import solve_files
        t0 = time.perf_counter()
        img = self(prompt=inp["prompt"], width=int(inp.get("width", 768)), height=int(inp.get("height", 768)),
                   seed=int(inp["seed"]))
        t1 = time.perf_counter()
        png = encode_png(img, 6)
        tm = dict(self.timings)
        tm.update({"infer_s": t1 - t0, "encode_cid_s": time.perf_counter() - t1})
        return solve_files([("out-1.png", png)], tm)
