"""Text-to-video pipelines: zeroscopev2xl and damo (``templates/zeroscopev2xl.json``,
``templates/damo.json``; SURVEY.md §2.6(c), BASELINE config #4).

    prompt, negative -> OpenCLIP ViT-H/14 text (penultimate layer) [2, 77, 1024]
    seed -> CPU generator -> latent noise [1, 4, F, h, w] -> frame-major NHWC
    N x { CFG batch-2 UNet3D over [2F, h, w, 4] (hipGraph replay) -> guidance
          -> sampler step }
    KL-VAE decode per frame (chunks) -> uint8 RGB frames -> deterministic MP4
    (H.264 avc-intra, utils/mp4.py; the solve path encodes on the GPU, ops.h264_intra_encode,
    same bytes) -> out-1.mp4

damo has no negative prompt input (empty uncond).  Random-init weights
(BASELINE.json); byte-parity with the Replicate containers is "parity unpinned".
"""
from __future__ import annotations

import functools
import os
import time
from dataclasses import dataclass, field
from typing import Dict, Optional

import torch

from ..utils.mp4 import encode_mp4
from ..utils.progress import beat

from .clip_text import CLIPTextConfig, CLIPTextEncoder
from .. import ops
from .graphs import GraphCache, PipelineBase
from .layers import init_weights
from .schedulers import GroupSampler, TaskSampler, make_scheduler
from .tokenizer import CLIPTokenizer
from .unet3d import UNet3DCondition, UNet3DConfig
from .vae import VAEConfig, VAEDecoder

# the solve path encodes the decoded frames on the GPU (ARB_VIDEO_GPU_H264=0: host encode, A/B; same bytes)
_GPU_H264 = os.environ.get("ARB_VIDEO_GPU_H264", "1") != "0"


@dataclass
class VideoConfig:
    name: str = "zeroscopev2xl"
    unet: UNet3DConfig = field(default_factory=UNet3DConfig.zeroscope)
    vae: VAEConfig = field(default_factory=VAEConfig)
    text: CLIPTextConfig = field(default_factory=CLIPTextConfig.vit_h14)
    width: int = 1024
    height: int = 576
    num_frames: int = 24
    num_inference_steps: int = 50
    guidance_scale: float = 17.5
    fps: int = 24
    negative_prompt: str = "noisy, washed out, ugly, distorted, broken"
    scheduler: str = "DPMSolverMultistep"
    vae_chunk: int = 8

    @staticmethod
    def for_model(name: str):
        if name == "zeroscopev2xl":
            return VideoConfig()
        if name == "damo":
            return VideoConfig(name="damo", width=256, height=256, num_frames=16, guidance_scale=9.0, fps=8,
                               negative_prompt="")
        raise ValueError(name)

    @staticmethod
    def tiny(name: str = "zeroscopev2xl"):
        c = VideoConfig.for_model(name)
        c.unet, c.vae, c.text = UNet3DConfig.tiny(), VAEConfig.tiny(), CLIPTextConfig.tiny(32)
        c.unet.cross_dim = 32
        return c


class VideoPipeline(PipelineBase):
    def __init__(self, cfg: VideoConfig = None, device="cpu", dtype=None, weight_seed: int = 0,
                 use_graphs: Optional[bool] = None, tokenizer_dir: Optional[str] = None, init=True):
        self.cfg = cfg = cfg or VideoConfig()
        self.device = torch.device(device)
        if dtype is None:
            dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.dtype = dtype
        self.unet = UNet3DCondition(cfg.unet)
        self.vae = VAEDecoder(cfg.vae)
        self.text = CLIPTextEncoder(cfg.text)
        if init:
            init_weights(self.unet, weight_seed)
            init_weights(self.vae, weight_seed + 1)
            init_weights(self.text, weight_seed + 2)
        for m in (self.unet, self.vae, self.text):
            m.to(device=self.device, dtype=dtype).eval()
        self.tokenizer = CLIPTokenizer(tokenizer_dir, cfg.text.max_len, cfg.text.vocab)
        self.use_graphs = (self.device.type == "cuda") if use_graphs is None else use_graphs
        self._graphs: Dict[int, GraphCache] = {}
        self.timings: Dict[str, float] = {}

    def modules(self):
        return {"unet": self.unet, "vae": self.vae, "text": self.text}

    def _reset_graphs(self):
        self._graphs = {}

    def _unet(self, frames):
        if frames not in self._graphs:
            self._graphs[frames] = GraphCache(functools.partial(self.unet, frames=frames), self.use_graphs)
        return self._graphs[frames]

    @torch.no_grad()
    def __call__(self, prompt: str, negative_prompt: Optional[str] = None, num_frames: Optional[int] = None,
                 width: Optional[int] = None, height: Optional[int] = None,
                 num_inference_steps: Optional[int] = None, guidance_scale: Optional[float] = None,
                 seed: int = 0, for_encode: bool = False):
        """uint8 RGB frames [F, H, W, 3]; ``for_encode`` on a GPU: the clip already encoded there
        (``utils.mp4.H264IntraClip``, the avc-intra bytes of those frames)."""
        with self._stream_ctx():
            return self._run(prompt, negative_prompt, num_frames, width, height, num_inference_steps,
                             guidance_scale, seed, for_encode)

    def _run(self, prompt, negative_prompt, num_frames, width, height, num_inference_steps, guidance_scale, seed,
             for_encode=False):
        cfg = self.cfg
        F = int(num_frames or cfg.num_frames)
        W, H = int(width or cfg.width), int(height or cfg.height)
        steps = int(num_inference_steps or cfg.num_inference_steps)
        g = cfg.guidance_scale if guidance_scale is None else float(guidance_scale)
        neg = cfg.negative_prompt if negative_prompt is None else negative_prompt
        sync = self._sync
        t0 = time.perf_counter()
        ids = torch.tensor([self.tokenizer(neg), self.tokenizer(prompt)], dtype=torch.long, device=self.device)
        ctx, _ = self.text(ids)                                   # [2, 77, 1024]: (uncond, cond)
        gen = torch.Generator(device="cpu").manual_seed(int(seed))
        zc = cfg.unet.in_channels
        x = torch.randn((1, zc, F, H // 8, W // 8), generator=gen, dtype=torch.float32)
        x = x[0].permute(1, 2, 3, 0).contiguous()                 # [F, h, w, 4] frame-major NHWC
        sched = make_scheduler(cfg.scheduler, steps)
        ts = TaskSampler(sched, x * sched.init_noise_sigma, gen, self.device)
        xin = torch.empty((2 * F,) + tuple(x.shape[1:]), dtype=self.dtype, device=self.device)

        def rows(k, out):       # frames of the uncond pass, then the cond pass
            return (None if out is None else out[:F], None if out is None else out[F:], xin[:F], xin[F:])

        samp = GroupSampler([ts], [g], xin, rows)
        samp.write_input(0)
        tbuf = torch.zeros(1, dtype=torch.float32, device=self.device)
        unet = self._unet(F)
        sync()
        t1 = time.perf_counter()
        for i, t in enumerate(sched.timesteps):
            beat()
            tbuf.fill_(float(t))
            # UNet3D, then ONE fused CFG + sampler launch.  No plan_batch scope here: the video
            # linears (M = 2F x HW rows) stay on hipBLASLt, measured faster than the implicit-GEMM
            # kernel's cost-model plans at these shapes (zeroscope 928 vs 693 tasks/h).
            samp.step(i, unet(xin, tbuf, ctx))
        sync()
        t2 = time.perf_counter()
        frames = self.decode(ts.x, for_encode)
        sync()
        t3 = time.perf_counter()
        self.timings = {"text_s": t1 - t0, "denoise_s": t2 - t1, "vae_s": t3 - t2}
        return frames

    @torch.no_grad()
    def decode(self, latent, for_encode: bool = False):
        z = (latent / self.cfg.vae.scaling_factor).to(self.dtype)
        if for_encode and _GPU_H264 and z.is_cuda:
            return self._decode_encoded(z)
        out = []
        for i in range(0, z.shape[0], self.cfg.vae_chunk):
            beat()
            out.append(ops.image_u8(self.vae(z[i:i + self.cfg.vae_chunk]), 0).cpu())
        return torch.cat(out).numpy()                             # [F, H, W, 3]

    def _decode_encoded(self, z):
        """Decoded frames -> 4:2:0 planes -> avc-intra slices, all on the GPU; only the compressed
        slices come back (``utils.mp4.H264IntraClip``).  A clip the encoder flags (output capacity)
        returns the RGB frames for the host encoder (same bytes)."""
        from ..utils.mp4 import INTRA_QP, H264IntraClip
        u8 = torch.cat([ops.image_u8(self.vae(z[i:i + self.cfg.vae_chunk]), 0)
                        for i in range(0, z.shape[0], self.cfg.vae_chunk)])
        F, H, W, _ = u8.shape
        enc, meta = ops.h264_intra_encode(*ops.rgb_to_yuv420(u8), INTRA_QP)
        m = meta.cpu().numpy()
        if m[F + 1] != 0:
            return u8.cpu().numpy()
        return H264IntraClip(enc[:int(m[F])].cpu().numpy(), m, W, H, INTRA_QP)

    def solve(self, inp: dict):
        from ..node.solver import solve_files
        t0 = time.perf_counter()
        frames = self(prompt=inp["prompt"], negative_prompt=inp.get("negative_prompt"),
                      num_frames=inp.get("num_frames"), width=inp.get("width"), height=inp.get("height"),
                      num_inference_steps=inp.get("num_inference_steps"), guidance_scale=inp.get("guidance_scale"),
                      seed=int(inp["seed"]), for_encode=True)
        t1 = time.perf_counter()
        mp4 = encode_mp4(frames if not hasattr(frames, "ndim") else list(frames), int(inp.get("fps", self.cfg.fps)))
        tm = dict(self.timings)
        tm.update({"infer_s": t1 - t0, "encode_cid_s": time.perf_counter() - t1})
        return solve_files([("out-1.mp4", mp4)], tm)
