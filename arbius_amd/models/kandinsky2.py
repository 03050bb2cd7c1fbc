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

import os
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
from .graphs import GraphCache, PipelineBase, task_stream
from .layers import Linear, init_weights
from .movq import MoVQConfig, MoVQDecoder
from .prior import PriorConfig, PriorTransformer
from .schedulers import K2_SCHEDULERS, GaussianDiffusion, GroupSampler, TaskSampler, k2_decoder_scheduler
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
    prior_steps: str = "5"          # template type "string" (guided-diffusion respacing spec)
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


# Each diffusion-prior step replays as a hipGraph (bitwise equal to eager; +1.3 % on the 2-stream
# bench, no stream serialisation: profiles/ab_r4_k2.md).  ARB_PRIOR_GRAPH=0 = eager (A/B only).
_PRIOR_GRAPH = os.environ.get("ARB_PRIOR_GRAPH", "1") == "1"
# ARB_K2_SPLIT_CFG=1: a solo task's cond / uncond UNet rows run as two overlapping batch-1 graph replays
# on two hardware queues (latency mode; bitwise the batch-2 bytes by test)
_SPLIT_CFG = os.environ.get("ARB_K2_SPLIT_CFG", "0") == "1"


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
        self._prior_graph = GraphCache(self._prior_step, self.use_graphs)
        # A/B switch (bitwise-equal paths, tests/test_models_gpu.py): replay each prior step as a hipGraph
        self.prior_graph = _PRIOR_GRAPH
        # latency mode: a solo task's cond / uncond UNet rows on two hardware queues (_unet_split)
        self.split_cfg = _SPLIT_CFG
        self._split = None
        self.timings: Dict[str, float] = {}

    def _prior_step(self, xin, tt, hidden, pooled, idx, q):
        return self.prior(xin, None, hidden, pooled, None, (idx, q), tt=tt)

    def _reset_graphs(self):
        self._unet = GraphCache(self.unet, self.use_graphs)
        self._prior_graph = GraphCache(self._prior_step, self.use_graphs)
        self._split = None

    def modules(self) -> Dict[str, nn.Module]:
        return {"unet": self.unet, "movq": self.movq, "prior": self.prior, "clip": self.clip,
                "clip_proj": self.clip_proj, "xlmr": self.xlmr, "buffers": self.buffers}

    # ------------------------------------------------------------------------------------------
    def settings(self, inp: dict) -> dict:
        """A task's sampling settings: the template inputs (docs/src/pages/register-model.mdx:141-185:
        num_inference_steps, guidance_scale, scheduler, prior_cf_scale, prior_steps) over the hidden
        defaults of the mainnet template (templates/kandinsky2.json exposes only prompt / size)."""
        cfg = self.cfg
        sched = str(inp.get("scheduler", "p_sampler"))
        if sched not in K2_SCHEDULERS:
            raise ValueError(f"kandinsky2: unknown scheduler {sched!r}")
        prior_steps = inp.get("prior_steps", cfg.prior_steps)
        return {"steps": int(inp.get("num_inference_steps", cfg.num_steps)),
                "guidance": float(inp.get("guidance_scale", cfg.guidance_scale)),
                "scheduler": sched,
                "prior_cf_scale": float(inp.get("prior_cf_scale", cfg.prior_cf_scale)),
                "prior_steps": str(prior_steps).strip()}

    def _clip_len(self, ids):
        eos = ids[-1]
        return ids.index(eos) + 1

    @torch.no_grad()
    def encode_text(self, prompts: List[str]):
        """Both text towers for k prompts in ONE batch of 2k sequences (rows 2i / 2i+1 = prompt i /
        the empty prompt), under batch-invariant plans: each row's bytes are its solo bytes.
        -> CLIP hidden [2k,77,w], CLIP pooled (projected) [2k,d], CLIP lengths, XLM-R full [2k,77,W],
        XLM-R pooled [2k,proj]."""
        texts = [t for p in prompts for t in (p, "")]
        cids = [self.clip_tok(t) for t in texts]
        lens = [self._clip_len(i) for i in cids]
        xt = [self.xlmr_tok(t) for t in texts]
        with ops.plan_batch(1):
            hidden, pooled = self.clip(torch.tensor(cids, dtype=torch.long, device=self.device))
            pooled = self.clip_proj(pooled)
            full, xpooled = self.xlmr(torch.tensor([i for i, _ in xt], dtype=torch.long, device=self.device),
                                      [n for _, n in xt])
        return hidden, pooled, lens, full, xpooled

    def _prior_stats(self):
        return self.prior.clip_std.float(), self.prior.clip_mean.float()

    @torch.no_grad()
    def sample_prior(self, hidden, pooled, lens, gens, steps, cf_scales: List[float]):
        """The diffusion prior of k tasks as ONE batch of 2k padded sequences per step (fused CFG +
        x0-pred p_sample per task, each with its own generator) -> image embeddings [k, d]."""
        k = len(gens)
        d = self.cfg.prior.clip_dim
        sched = GaussianDiffusion(steps, schedule="cosine", predict="x0", learned_var=False)
        tasks = [TaskSampler(sched, torch.randn((1, d), generator=g, dtype=torch.float32).view(d // 4, 4), g,
                             self.device) for g in gens]
        xin = torch.empty((2 * k, d), dtype=self.dtype, device=self.device)

        def rows(i, out):     # out = prior outputs [2k, d]: rows 2i / 2i+1 = (cond, uncond)
            return (None if out is None else out[2 * i + 1].reshape(-1, 4),
                    None if out is None else out[2 * i].reshape(-1, 4),
                    xin[2 * i].view(-1, 4), xin[2 * i + 1].view(-1, 4))

        samp = GroupSampler(tasks, [float(c) for c in cf_scales], xin, rows)
        samp.write_input(0)
        layout = self.prior.layout(lens, self.device)
        for i, t in enumerate(sched.timesteps):
            beat()
            with ops.plan_batch(2):
                if self.use_graphs and self.prior_graph:
                    tbuf = torch.full((1,), float(t), dtype=torch.float32, device=self.device)
                    out = self._prior_graph(xin, tbuf, hidden, pooled, layout[0], layout[1]).contiguous()
                else:
                    out = self.prior(xin, t, hidden, pooled, lens, layout).contiguous()
            samp.step(i, out)
        std, mean = self._prior_stats()
        return torch.stack([(ts.x.view(d) * std + mean) for ts in tasks]).to(self.dtype)

    def _split_ok(self) -> bool:
        return self.split_cfg and self.use_graphs and self.device.type == "cuda"

    def _unet_split(self, xin, tbuf, text_full, text_pooled, img_embs):
        """Latency mode of a solo task: the cond row's UNet on the calling stream and the uncond row's on
        a second task stream (its own hardware queue, ``graphs.task_stream``), as two batch-1 graph
        replays that overlap, joined before the sampler step.  Batch-1 launches under plan_batch(1)
        plan at the same canonical batch as the batch-2 solo launch and every UNet op is row-local, so
        each row's bytes are the batch-2 row's (tests/test_models_gpu.py)."""
        dev = self.device
        cur = torch.cuda.current_stream(dev)
        if self._split is None:
            peers = [cur] if cur != torch.cuda.default_stream(dev) else []
            self._split = (task_stream(dev, peers), GraphCache(self.unet, True), GraphCache(self.unet, True),
                           torch.cuda.Event(), torch.cuda.Event())
        s2, una, unb, ev_in, ev_b = self._split
        ev_in.record(cur)
        with torch.cuda.stream(s2):
            s2.wait_event(ev_in)
            with ops.plan_batch(1):
                ob = unb(xin[1:2], tbuf, text_full[1:2], text_pooled[1:2], img_embs[1:2])
            ev_b.record(s2)
        with ops.plan_batch(1):
            oa = una(xin[0:1], tbuf, text_full[0:1], text_pooled[0:1], img_embs[0:1])
        cur.wait_event(ev_b)
        return torch.cat([oa, ob])

    def _group_sampler(self, tasks, h, w, guidance: List[float]):
        """k decoder tasks on one batch-2k GLIDE UNet input: rows 2k / 2k+1 = (cond, uncond); the
        cond row's channels 4..7 are the learned variance of p_sample."""
        zc = self.cfg.unet.in_channels
        xin = torch.empty((2 * len(tasks), h, w, zc), dtype=self.dtype, device=self.device)

        def rows(k, out):
            return (None if out is None else out[2 * k + 1], None if out is None else out[2 * k],
                    xin[2 * k], xin[2 * k + 1])

        samp = GroupSampler(tasks, [float(g) for g in guidance], xin, rows)
        samp.write_input(0)
        return samp

    @torch.no_grad()
    def __call__(self, prompt: str, width: int = 768, height: int = 768, seed: int = 0,
                 num_inference_steps: Optional[int] = None, guidance_scale: Optional[float] = None,
                 prior_cf_scale: Optional[float] = None, prior_steps=None, scheduler: str = "p_sampler"):
        inp = {"prompt": prompt, "width": width, "height": height, "seed": seed, "scheduler": scheduler}
        for k, v in (("num_inference_steps", num_inference_steps), ("guidance_scale", guidance_scale),
                     ("prior_cf_scale", prior_cf_scale), ("prior_steps", prior_steps)):
            if v is not None:
                inp[k] = v
        return self.run_group([inp])[0]

    @torch.no_grad()
    def run_group(self, inps: List[dict]) -> List[np.ndarray]:
        """Lock-step solve of k tasks of one resolution / step count / scheduler (a solo task is
        k = 1, the same code): both text towers and the prior run as one batch per step, every
        GLIDE UNet step runs the k (cond, uncond) pairs as one batch-2k launch sequence, all under
        batch-invariant plans (bitwise the solo outputs); guidance, prior_cf_scale, noise and MoVQ
        are per task.  Tasks whose prior_steps differ run their priors as separate batches."""
        sizes = {(int(i.get("width", 768)), int(i.get("height", 768))) for i in inps}
        if len(sizes) != 1:
            raise ValueError(f"run_group needs one resolution, got {sorted(sizes)}")
        width, height = sizes.pop()
        st = [self.settings(i) for i in inps]
        kinds = sorted({(s["steps"], s["scheduler"]) for s in st})
        if len(kinds) != 1:
            # tasks that cannot share decoder launches run as separate lock-step groups (same bytes)
            out = [None] * len(inps)
            for kd in kinds:
                sel = [j for j, s in enumerate(st) if (s["steps"], s["scheduler"]) == kd]
                for j, im in zip(sel, self.run_group([inps[j] for j in sel])):
                    out[j] = im
            return out
        cfg = self.cfg
        with self._stream_ctx():
            sync = self._sync
            t0 = time.perf_counter()
            k = len(inps)
            gens = [torch.Generator(device="cpu").manual_seed(int(i["seed"])) for i in inps]
            hidden, pooled, lens, text_full, text_pooled = self.encode_text([i["prompt"] for i in inps])
            img = [None] * k
            for ps in sorted({s["prior_steps"] for s in st}):
                sel = [j for j in range(k) if st[j]["prior_steps"] == ps]
                r = [r for j in sel for r in (2 * j, 2 * j + 1)]
                steps = int(ps) if ps.isdigit() else ps
                emb = self.sample_prior(hidden[r], pooled[r], [lens[x] for x in r], [gens[j] for j in sel], steps,
                                        [st[j]["prior_cf_scale"] for j in sel])
                for q, j in enumerate(sel):
                    img[j] = emb[q]
            zero = self.buffers.zero_img_emb.to(self.dtype)
            img_embs = torch.stack([e for j in range(k) for e in (img[j], zero)])
            h, w = height // 8, width // 8
            zc = cfg.unet.in_channels
            tasks = []
            for j in range(k):
                x = torch.randn((1, zc, h, w), generator=gens[j], dtype=torch.float32).permute(0, 2, 3, 1).contiguous()
                sched = k2_decoder_scheduler(st[j]["scheduler"], st[j]["steps"], cfg.latent_clamp)
                tasks.append(TaskSampler(sched, x, gens[j], self.device))    # draws this task's noise now
            sync()
            t1 = time.perf_counter()
            samp = self._group_sampler(tasks, h, w, [s["guidance"] for s in st])
            tbuf = torch.zeros(1, dtype=torch.float32, device=self.device)
            split = k == 1 and self._split_ok()
            for i, t in enumerate(tasks[0].sched.timesteps):
                beat()
                tbuf.fill_(float(t))
                if split:
                    out = self._unet_split(samp.xin, tbuf, text_full, text_pooled, img_embs)
                else:
                    with ops.plan_batch(2):      # batch-invariant plans: solo == lock-step group bytes
                        out = self._unet(samp.xin, tbuf, text_full, text_pooled, img_embs)
                samp.step(i, out)            # ONE fused CFG + sampler launch for the group
            sync()
            t2 = time.perf_counter()
            imgs = [self.decode(ts.x) for ts in tasks]
            sync()
            self.timings = {"text_prior_s": t1 - t0, "denoise_s": t2 - t1, "movq_s": time.perf_counter() - t2}
            return imgs

    @torch.no_grad()
    def decode(self, latent):
        img = self.movq(latent.to(self.dtype))[0]
        if img.is_cuda and img.dtype == torch.bfloat16 and not ops.reference_ops():
            img = ops.image_u8(img, 1)            # one HIP pass, the ATen chain's bytes
        else:
            img = ((img.float() + 1.0) * 127.5).clamp(0, 255).round().to(torch.uint8)
        return img.cpu().numpy()

    def solve(self, inp: dict):
        """Template inputs (prompt, width, height, seed + the documented sampling inputs) ->
        ``out-1.png`` solution."""
        from ..node.solver import solve_files
        t0 = time.perf_counter()
        img = self.run_group([inp])[0]
        t1 = time.perf_counter()
        png = encode_png(img, 6)
        tm = dict(self.timings)
        tm.update({"infer_s": t1 - t0, "encode_cid_s": time.perf_counter() - t1})
        return solve_files([("out-1.png", png)], tm)
