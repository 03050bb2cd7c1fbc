"""Shape audit of the template operating range (no GPU needed).

Every model of every template runs its forward passes on the META device with ``ops._lib`` in audit
mode: the real host-side code of every op runs - eligibility tests, the zero-padding onto the
kernels, shape / stride validation, the batch-invariant plan selection (canonical-batch plan at its
split-K, tile family for the actual shape, both looked up in the built library's pinned tables) -
and only the launch itself is replaced by a recording stub.  A shape that no HIP kernel serves
raises ``ops.LibraryFallback`` (GPU tensors never take a library path), so a clean audit proves
that every conv / GEMM / attention / norm of the audited inputs lands on a HIP kernel with a plan
that is a pure function of the shape.

The template ranges (``config/templates/*.json``):

* anythingv3: width, height in {128, 256, 512, 640, 768, 896, 1024} - solo (CFG batch 2) and a
  lock-step group of 4 (batch 8);
* kandinsky2: width, height in {768, 1024} (solo and group of 4);
* zeroscopev2xl: width in {256 .. 1920} (14), height in {256 .. 896} (11), num_frames 1 .. 96;
* damo: 256 x 256, num_frames >= 1 (the template's max 500 is not enforced under the reference's
  hydration quirks).

Frame counts only scale the row count M of the video UNet's launches (no kernel's eligibility or
tile choice depends on M), so the video audit takes a few frame counts per resolution.
"""
from __future__ import annotations

import contextlib
from typing import Dict, Iterable, List

import torch

from . import _lib, plan_batch

SD_SIZES = (128, 256, 512, 640, 768, 896, 1024)
K2_SIZES = (768, 1024)
ZS_WIDTHS = (1920, 1792, 1664, 1536, 1408, 1280, 1152, 1024, 896, 768, 640, 512, 384, 256)
ZS_HEIGHTS = (896, 832, 768, 704, 640, 576, 512, 448, 384, 320, 256)


@contextlib.contextmanager
def audit():
    """Run the body with every HIP launch recorded (not executed); yields the record list."""
    if _lib.auditing():
        raise RuntimeError("audit() does not nest")
    _lib.lib()                         # host-side plan tables come from the built library
    rec: List[Dict] = []
    _lib._AUDIT = rec
    try:
        with torch.no_grad():
            yield rec
    finally:
        _lib._AUDIT = None


def _meta(shape, dtype=torch.bfloat16):
    return torch.empty(shape, dtype=dtype, device="meta")


def _build(cls, cfg):
    with torch.device("meta"):
        m = cls(cfg)
    return m.to(torch.bfloat16).eval()


def launches(rec: Iterable[Dict]) -> List[Dict]:
    return [r for r in rec if r["kind"] in ("conv", "gemm")]


def check_invariance(solo: Iterable[Dict], group: Iterable[Dict]) -> List[str]:
    """Batch invariance of a lock-step group against its solo tasks, launch by launch (same op
    sequence): every conv / GEMM whose row count grows with the group must be planned under
    ``ops.plan_batch`` and run the solo launch's split-K (the reduction order of each output); its
    tile family may differ (families are bitwise interchangeable at a fixed split).  Launches whose
    shape does not depend on the group (e.g. the timestep embedding, M = 1) are equal anyway."""
    a, b = launches(solo), launches(group)
    if len(a) != len(b):
        return [f"solo and group runs launch {len(a)} vs {len(b)} convs / GEMMs"]
    bad = []
    for x, y in zip(a, b):
        tag = f"{y['kind']} {y['M']}x{y['N']}x{y['K']}"
        if (x["kind"], x["N"], x["K"]) != (y["kind"], y["N"], y["K"]):
            bad.append(f"{tag}: launch sequence differs from the solo run ({x['kind']} {x['N']}x{x['K']})")
        elif x["M"] != y["M"] and not (x.get("plan_b") and y.get("plan_b")):
            bad.append(f"{tag}: row count depends on the group but planned outside ops.plan_batch")
        elif x["split"] != y["split"]:
            bad.append(f"{tag}: split-K {y['split']} in the group vs {x['split']} solo")
    return bad


def sd15(width: int, height: int, group: int = 1):
    """One SD1.5 UNet evaluation (CFG batch 2 per task), the VAE decode and the CLIP text tower."""
    from ..models.clip_text import CLIPTextConfig, CLIPTextEncoder
    from ..models.unet2d import UNet2DCondition, UNetConfig
    from ..models.vae import VAEConfig, VAEDecoder
    unet = _build(UNet2DCondition, UNetConfig.sd15())
    with audit() as rec:
        with plan_batch(2):
            unet(_meta((2 * group, height // 8, width // 8, 4)), torch.tensor([500.0], device="meta"),
                 _meta((2 * group, 77, 768)))
        del unet
        vae = _build(VAEDecoder, VAEConfig())
        vae(_meta((1, height // 8, width // 8, 4)))
        del vae
        text = _build(CLIPTextEncoder, CLIPTextConfig())
        with plan_batch(1):
            text(torch.zeros(2, 77, dtype=torch.long, device="meta"))
    return rec


def kandinsky2(width: int, height: int, group: int = 1):
    """Kandinsky 2.1: GLIDE UNet step (batch 2 per task), MoVQ decode, prior step, both text towers."""
    from ..models.clip_text import CLIPTextConfig, CLIPTextEncoder
    from ..models.glide_unet import GlideUNet, GlideUNetConfig
    from ..models.movq import MoVQConfig, MoVQDecoder
    from ..models.prior import PriorConfig, PriorTransformer
    from ..models.xlmr import MCLIPText, XLMRConfig
    ucfg = GlideUNetConfig.kandinsky21()
    unet = _build(GlideUNet, ucfg)
    b = 2 * group
    with audit() as rec:
        with plan_batch(2):
            unet(_meta((b, height // 8, width // 8, ucfg.in_channels)), torch.tensor([500.0], device="meta"),
                 _meta((b, 77, ucfg.text_dim)), _meta((b, ucfg.pooled_dim)), _meta((b, ucfg.image_embed_dim)))
        del unet
        movq = _build(MoVQDecoder, MoVQConfig.kandinsky21())
        movq(_meta((1, height // 8, width // 8, 4)))
        del movq
        pcfg = PriorConfig.kandinsky21()
        prior = _build(PriorTransformer, pcfg)
        lens = [5, 77] * group
        with plan_batch(2):
            layout = prior.layout(lens, torch.device("meta"))
            prior(_meta((b, pcfg.clip_dim)), 500, _meta((b, 77, CLIPTextConfig.vit_l14().width)),
                  _meta((b, pcfg.clip_dim)), lens, layout)   # CLIP-L hidden states [2k, 77, 768]
        del prior
        clip = _build(CLIPTextEncoder, CLIPTextConfig.vit_l14())
        xlmr = _build(MCLIPText, XLMRConfig.large())
        with plan_batch(1):
            clip(torch.zeros(b, 77, dtype=torch.long, device="meta"))
            xlmr(torch.zeros(b, 77, dtype=torch.long, device="meta"), [5, 77] * group)
    return rec


def video(name: str, width: int, height: int, frames: int):
    """One UNet3D evaluation (CFG batch 2) at ``frames`` frames and one VAE decode chunk."""
    from ..models.unet3d import UNet3DCondition, UNet3DConfig
    from ..models.vae import VAEConfig, VAEDecoder
    from ..models.video import VideoConfig
    vc = VideoConfig.for_model(name)
    ucfg = UNet3DConfig.zeroscope() if name == "zeroscopev2xl" else vc.unet
    unet = _build(UNet3DCondition, ucfg)
    with audit() as rec:     # as VideoPipeline: no lock-step groups, plans for the actual shapes
        unet(_meta((2 * frames, height // 8, width // 8, 4)), torch.tensor([500.0], device="meta"),
             _meta((2, 77, ucfg.cross_dim)), frames=frames)
        del unet
        vae = _build(VAEDecoder, VAEConfig())
        vae(_meta((min(frames, vc.vae_chunk), height // 8, width // 8, 4)))
    return rec
