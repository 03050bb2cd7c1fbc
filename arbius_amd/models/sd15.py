"""anythingv3 / SD1.5 text-to-image pipeline (the in-process replacement of the
Cog container's ``POST /predictions``, ``miner/src/index.ts:852-875``).

  prompt, negative_prompt -> CLIP text encoder (once)
  seed -> deterministic Gaussian latent (CPU generator -> identical on every GPU)
  N x { CFG batch-2 UNet (replayed hipGraph) -> guidance combine -> sampler step }
  VAE decode -> uint8 RGB -> deterministic PNG bytes

On a GPU the UNet forward for a fixed (batch, latent shape) is captured once
into a hipGraph (torch.cuda.CUDAGraph on ROCm) and replayed for every
denoising step: the ~600 kernel launches of one UNet evaluation cost one
graph launch, so the step is bound by the kernels, not by Python.
"""
from __future__ import annotations

import os

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import ops
from ..utils.trace import span
from ..utils.progress import beat
from .clip_text import CLIPTextConfig, CLIPTextEncoder
from .graphs import CAPTURE_LOCK, GraphCache, PipelineBase, capture_stream, check_live, live_table
from .layers import init_weights
from .schedulers import GroupSampler, TaskSampler, make_scheduler
from .tokenizer import CLIPTokenizer
from .unet2d import CrossAttention, UNet2DCondition, UNetConfig, cross_kv_mode
from .vae import VAEConfig, VAEDecoder


@dataclass
class SD15Config:
    unet: UNetConfig = field(default_factory=UNetConfig.sd15)
    vae: VAEConfig = field(default_factory=VAEConfig)
    text: CLIPTextConfig = field(default_factory=CLIPTextConfig.vit_l14)

    @staticmethod
    def tiny():
        return SD15Config(unet=UNetConfig.tiny(), vae=VAEConfig.tiny(), text=CLIPTextConfig.tiny(32))


class _GraphedUNet:
    """Static-shape hipGraph wrapper around one UNet forward.

    Two graphs: ``kv_graph`` projects the text context through every cross-attention to_kv
    (replayed once per new context, i.e. once per task / lock-step group), ``graph`` is the
    per-step UNet that reads those K/V buffers instead of re-projecting the constant context
    at every denoising step (unet2d.cross_kv_mode)."""

    def __init__(self, unet, x_shape, ctx, dtype):
        dev = ctx.device
        self.unet = unet
        self.x = torch.zeros(x_shape, dtype=dtype, device=dev)
        self.t = torch.zeros(1, dtype=torch.float32, device=dev)
        self.ctx = ctx.clone()
        self.kv = {}
        self._ctx_obj = None
        CAPTURE_LOCK.acquire()
        try:
            self._capture(unet, dev)
        finally:
            CAPTURE_LOCK.release()

    HOIST = os.environ.get("ARBIUS_CROSS_KV_HOIST", "1") != "0"   # A/B switch (same numerics)

    def _project_kv(self, unet):
        if not self.HOIST:
            return
        for m in unet.modules():
            if isinstance(m, CrossAttention):
                self.kv[id(m)] = m.context_kv(self.ctx)

    def _capture(self, unet, dev):
        s = capture_stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(2):  # warm-up: allocator + kernel-library load outside capture
                self._project_kv(unet)
                with cross_kv_mode("consume" if self.HOIST else None, self.kv):
                    self.out = unet(self.x, self.t, self.ctx)
        torch.cuda.current_stream(dev).wait_stream(s)
        self.kv_graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.kv_graph, stream=s, capture_error_mode="thread_local"):
            self._project_kv(unet)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=s, capture_error_mode="thread_local"):
            with cross_kv_mode("consume" if self.HOIST else None, self.kv):
                self.out = unet(self.x, self.t, self.ctx)
        self._live = live_table([self.x, self.t, self.ctx, self.out] + list(self.kv.values()))

    def __call__(self, x, t, ctx):
        check_live(self._live)
        if x.data_ptr() != self.x.data_ptr():       # the sampler writes the static buffer itself
            self.x.copy_(x)
        self.t.fill_(float(t))
        if ctx is not self._ctx_obj:
            # a new context object = a new task / group (the reference is held, so identity
            # cannot be recycled by the allocator while it is cached)
            self.ctx.copy_(ctx)
            self.kv_graph.replay()
            self._ctx_obj = ctx
        self.graph.replay()
        return self.out


# A/B switches (bitwise-equal paths): ARB_VAE_GRAPH=0 runs the VAE decode eagerly instead of as one
# hipGraph replay per image (r5, 4 x 4 bench on one box: 30,960 graph vs 30,308-30,572 eager; the r4
# "VAE-graph stall" was two task streams bound to one hardware queue - profiles/graph_serialisation_r5.md);
# ARB_PINNED_D2H=1 copies the image to the host through a pinned buffer instead of a pageable ``.cpu()``
_VAE_GRAPH = os.environ.get("ARB_VAE_GRAPH", "1") == "1"
_PINNED_D2H = os.environ.get("ARB_PINNED_D2H", "0") == "1"


def _to_host(img):
    """Device uint8 image -> numpy (pinned staging buffer, async copy and a wait on the current
    stream only, with ARB_PINNED_D2H=1)."""
    if not img.is_cuda or not _PINNED_D2H:
        return img.cpu().numpy()
    host = torch.empty(img.shape, dtype=img.dtype, pin_memory=True)
    host.copy_(img, non_blocking=True)
    torch.cuda.current_stream(img.device).synchronize()
    return host.numpy()


class SD15Pipeline(PipelineBase):
    def __init__(self, cfg: SD15Config = None, device="cpu", dtype=None, weight_seed: int = 0,
                 use_graphs: Optional[bool] = None, tokenizer_dir: Optional[str] = None, init=True):
        self.cfg = cfg or SD15Config()
        self.device = torch.device(device)
        if dtype is None:
            dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.dtype = dtype
        self.unet = UNet2DCondition(self.cfg.unet)
        self.vae = VAEDecoder(self.cfg.vae)
        self.text = CLIPTextEncoder(self.cfg.text)
        if init:
            init_weights(self.unet, weight_seed)
            init_weights(self.vae, weight_seed + 1)
            init_weights(self.text, weight_seed + 2)
        for m in (self.unet, self.vae, self.text):
            m.to(device=self.device, dtype=dtype).eval()
        self.tokenizer = CLIPTokenizer(tokenizer_dir, self.cfg.text.max_len, self.cfg.text.vocab)
        self.use_graphs = (self.device.type == "cuda") if use_graphs is None else use_graphs
        self._graphs: Dict[tuple, _GraphedUNet] = {}
        # the CLIP text tower as one graph replay per task (~150 small launches eager; same kernels,
        # same bytes); the graph's output buffer is static, so encode_prompt copies it out
        self._text_graph = GraphCache(self._text_hidden, self.use_graphs)
        self._vae_graph = GraphCache(self._vae_image, self.use_graphs)
        self.timings: Dict[str, float] = {}

    def modules(self):
        return {"unet": self.unet, "vae": self.vae, "text": self.text}

    def _reset_graphs(self):
        self._graphs = {}
        self._text_graph = GraphCache(self._text_hidden, self.use_graphs)
        self._vae_graph = GraphCache(self._vae_image, self.use_graphs)

    def _text_hidden(self, ids):
        return self.text(ids)[0]

    def _vae_image(self, z):
        return self.vae(z)[0]

    # ------------------------------------------------------------------------------------------
    @torch.no_grad()
    def encode_prompt(self, prompt: str, negative_prompt: str = ""):
        ids = torch.tensor([self.tokenizer(negative_prompt), self.tokenizer(prompt)], dtype=torch.long,
                           device=self.device)
        if self.use_graphs:
            return self._text_graph(ids).clone()   # [2, 77, C]: (uncond, cond)
        hidden, _ = self.text(ids)
        return hidden  # [2, 77, C]: (uncond, cond)

    @staticmethod
    def initial_noise(seed: int, h: int, w: int, channels: int = 4):
        g = torch.Generator(device="cpu").manual_seed(int(seed))
        n = torch.randn((1, channels, h, w), generator=g, dtype=torch.float32)
        return n.permute(0, 2, 3, 1).contiguous(), g  # NHWC

    def _unet_eval(self, x2, t, ctx):
        # batch-invariant plans (ops.plan_batch): one CFG pair is the planning unit, so a
        # lock-step group of k tasks (batch 2k) computes each task's bytes exactly as solo
        with ops.plan_batch(2):
            if not self.use_graphs:
                return self.unet(x2, torch.tensor([float(t)], device=self.device), ctx)
            return self._graph(tuple(x2.shape), ctx)(x2, t, ctx)

    def _graph(self, shape, ctx):
        with ops.plan_batch(2):
            if shape not in self._graphs:
                self._graphs[shape] = _GraphedUNet(self.unet, shape, ctx, self.dtype)
            return self._graphs[shape]

    @torch.no_grad()
    def __call__(self, prompt: str, negative_prompt: str = "", width: int = 512, height: int = 512,
                 num_inference_steps: int = 50, guidance_scale: float = 7.5, scheduler: str = "DDIM",
                 seed: int = 0, output: str = "uint8"):
        with self._stream_ctx():
            return self._run(prompt, negative_prompt, width, height, num_inference_steps, guidance_scale,
                             scheduler, seed)

    def _run(self, prompt, negative_prompt, width, height, num_inference_steps, guidance_scale, scheduler, seed):
        sync = self._sync
        tm: Dict[str, float] = {}
        with span("text_s", tm, sync):
            ctx = self.encode_prompt(prompt, negative_prompt)
            h, w = height // 8, width // 8
            x, gen = self.initial_noise(seed, h, w, self.cfg.unet.in_channels)
            sched = make_scheduler(scheduler, num_inference_steps)
            samp = self._group_sampler([TaskSampler(sched, x * sched.init_noise_sigma, gen, self.device)],
                                       [guidance_scale], h, w, ctx)
        with span("denoise_s", tm, sync):
            for i, t in enumerate(sched.timesteps):
                beat()
                samp.step(i, self._unet_eval(samp.xin, t, ctx))   # UNet, then ONE fused CFG+sampler launch
        with span("vae_s", tm, sync):
            img = self.decode(samp.latent(0))
        self.timings = tm
        return img

    def _group_sampler(self, tasks, guidance, h, w, ctx):
        """Sampler for k tasks sharing one batch-2k UNet input: rows 2k / 2k+1 = (uncond, cond).
        With hipGraphs the sampler writes the next input straight into the graph's static buffer."""
        shape = (2 * len(tasks), h, w, self.cfg.unet.in_channels)
        xin = self._graph(shape, ctx).x if self.use_graphs else torch.empty(shape, dtype=self.dtype,
                                                                              device=self.device)

        def rows(k, out):
            return (None if out is None else out[2 * k], None if out is None else out[2 * k + 1],
                    xin[2 * k], xin[2 * k + 1])

        samp = GroupSampler(tasks, [float(g) for g in guidance], xin, rows)
        samp.write_input(0)
        return samp

    @torch.no_grad()
    def run_group(self, inps: List[dict]) -> List[np.ndarray]:
        """Lock-step solve of k compatible tasks (same width / height / steps / scheduler): every
        UNet evaluation runs the k CFG pairs as ONE batch-2k launch sequence (k x the rows per
        GEMM / conv -> fuller tiles, 1/k of the launches per task), while text encoding, noise,
        the sampler state and the VAE stay per task.  With batch-invariant plans each output
        is bitwise the solo output (tests/test_models_gpu.py)."""
        keys = {(int(i.get("width", 768)), int(i.get("height", 768)), int(i.get("num_inference_steps", 20)),
                 i.get("scheduler", "DPMSolverMultistep")) for i in inps}
        if len(keys) != 1:
            raise ValueError(f"run_group needs identical width/height/steps/scheduler, got {sorted(keys)}")
        width, height, steps, scheduler = keys.pop()
        with self._stream_ctx():
            sync = self._sync
            tm: Dict[str, float] = {}
            with span("text_s", tm, sync):
                ctxs, tasks = [], []
                for inp in inps:
                    ctxs.append(self.encode_prompt(inp["prompt"], inp.get("negative_prompt", "")))
                    x, gen = self.initial_noise(int(inp["seed"]), height // 8, width // 8,
                                                self.cfg.unet.in_channels)
                    sched = make_scheduler(scheduler, steps)
                    tasks.append(TaskSampler(sched, x * sched.init_noise_sigma, gen, self.device))
                ctx = torch.cat(ctxs)
                samp = self._group_sampler(tasks, [float(inp.get("guidance_scale", 12)) for inp in inps],
                                           height // 8, width // 8, ctx)
            with span("denoise_s", tm, sync):
                for i, t in enumerate(tasks[0].sched.timesteps):
                    beat()
                    samp.step(i, self._unet_eval(samp.xin, t, ctx))
            with span("vae_s", tm, sync):
                imgs = [self.decode(samp.latent(k)) for k in range(len(tasks))]
            self.timings = tm
            return imgs

    @torch.no_grad()
    def decode(self, latent):
        z = (latent / self.cfg.vae.scaling_factor).to(self.dtype)
        if "vae" in ops._EXP_SKIP:      # ablation runs only (numerics knob): no VAE decode
            return np.zeros((z.shape[1] * 8, z.shape[2] * 8, 3), np.uint8)
        if self.use_graphs and _VAE_GRAPH:
            img = self._vae_graph(z).clone()      # a copy out of the graph's static output
        else:
            img = self.vae(z)[0]
        if img.is_cuda and img.dtype == torch.bfloat16 and not ops.reference_ops():
            img = ops.image_u8(img, 0)            # one HIP pass, the ATen chain's bytes
        else:
            img = ((img.float() / 2 + 0.5).clamp(0, 1) * 255).round().to(torch.uint8)
        return _to_host(img)  # [H, W, 3]
