"""Real-checkpoint loading - nothing in a weights file is ever executed (safetensors, or a plain
tensor state dict through ``torch.load(weights_only=True)``).

The reference miner never touches weights: its Cog containers bake them in
(``templates/*.json`` ``meta.docker``; SURVEY.md §5.4 "model weights from safetensors, loaded
by one rank and RCCL-broadcast").  This module maps the PUBLIC checkpoint layouts of every
template's model family onto this engine's module tree:

* ``anythingv3`` (SD1.5, diffusers): ``unet/``, ``vae/``, ``text_encoder/``.
* ``kandinsky2`` (Kandinsky 2.1), either layout:
  - the ORIGINAL release the mainnet container ships (``decoder_fp16.ckpt``, ``prior_fp16.ckpt``,
    ``movq_final.ckpt``, ``ViT-L-14_stats.th``, ``text_encoder/``, OpenAI CLIP ViT-L/14 state dict;
    optionally under ``2_1/``) - used whenever ``decoder_fp16.ckpt`` is present;
  - diffusers ``kandinsky-community/kandinsky-2-1`` at the root and ``kandinsky-2-1-prior`` under
    ``prior/``: ``unet/``, ``movq/``, ``text_encoder/`` (M-CLIP XLM-R), ``prior/prior/``,
    ``prior/text_encoder/`` (CLIP ViT-L/14 + projection), ``prior/image_encoder/`` (only to
    compute the decoder's zero-image embedding once).
* ``zeroscopev2xl`` / ``damo`` (diffusers ``UNet3DConditionModel`` text-to-video): ``unet/``,
  ``vae/``, ``text_encoder/`` (OpenCLIP ViT-H as ``CLIPTextModel``; its 23-layer export drops the
  unused last layer, which stays optional here).
* ``robust_video_matting``: the upstream ``rvm_mobilenetv3`` state dict (``.safetensors`` or the
  released ``.pth`` tensor dict); BatchNorms are folded into the conv weights at load.
* **native layout** for any family, per module: ``<module>.safetensors`` with this engine's own
  parameter names (``save_native``; ``python -m arbius_amd.models.weights convert``).  A native
  file present for a module takes precedence over the public mapping of that module.

Layout differences handled here, MI355X-first design choices of the engine's modules:
conv weights are stored OHWI (channels-last implicit GEMM), 1x1 ``proj_in``/``proj_out`` convs
are plain linears, Q/K/V (and K/V) projections are ONE fused GEMM, the MoVQ SpatialNorm
``conv_y``/``conv_b`` pair is one 1x1 conv, temporal Conv3d (3,1,1) weights are [Cout, 3, 1, Cin]
taps.  Every target parameter must be filled exactly once, with the right shape, or loading
fails loudly (no silent partial random init).  Byte parity of outputs with the reference's
containers is "parity unpinned" (no public vector exists); the mappings are pinned by
export -> load round trips and, for the text towers, by numerical parity with transformers.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass
from typing import Callable, Dict, Iterable, List, Optional, Tuple

import torch

Tensor = torch.Tensor


# --------------------------------------------------------------------------- checkpoint IO
def read_safetensors(path: str) -> Dict[str, Tensor]:
    from safetensors.torch import load_file
    return load_file(path, device="cpu")


def read_checkpoint(path: str) -> Dict[str, Tensor]:
    """safetensors, or a ``.pth``/``.pt``/``.bin`` tensor state dict loaded with the weights-only
    unpickler (which refuses anything but tensors and plain containers)."""
    if path.endswith(".safetensors"):
        return read_safetensors(path)
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(obj, dict) and "state_dict" in obj and isinstance(obj["state_dict"], dict):
        obj = obj["state_dict"]
    if not isinstance(obj, dict) or not all(torch.is_tensor(v) for v in obj.values()):
        raise ValueError(f"{path}: not a tensor state dict")
    return dict(obj)


def write_safetensors(state: Dict[str, Tensor], path: str):
    from safetensors.torch import save_file
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    save_file({k: v.detach().contiguous().cpu() for k, v in state.items()}, path)


# --------------------------------------------------------------------------- name rules
# A rule maps a TARGET (engine) name pattern to one or more SOURCE names; ``#`` captures an index.
# kind: "copy" | "conv" (OIHW -> OHWI) | "lin1x1" (1x1 conv OI11 -> linear OI) | "cat" (concat dim 0)
#       | "convcat" (OIHW convs concatenated on O, -> OHWI) | "conv3d" ([O, I, 3, 1, 1] -> [O, 3, 1, I])
#       | "unsq1" / "unsq2" (leading singleton dims dropped) | "bnw@eps" / "bnb@eps" (BatchNorm fold:
#       srcs (conv.w, bn.w, bn.var) / (bn.w, bn.b, bn.mean, bn.var))
Rule = Tuple[str, str, Tuple[str, ...]]


def _wb(R: List[Rule], dst: str, src: str, kind: str = "copy", bias: bool = True):
    R.append((f"{dst}.weight", kind, (f"{src}.weight",)))
    if bias:
        R.append((f"{dst}.bias", "copy", (f"{src}.bias",)))


def _sd15_unet_rules() -> List[Rule]:
    R: List[Rule] = []

    def res(dst, src):
        for a, b in (("norm1", "norm1"), ("norm2", "norm2")):
            R.extend([(f"{dst}.{a}.weight", "copy", (f"{src}.{b}.weight",)),
                      (f"{dst}.{a}.bias", "copy", (f"{src}.{b}.bias",))])
        for a, b in (("conv1", "conv1"), ("conv2", "conv2"), ("shortcut", "conv_shortcut")):
            R.extend([(f"{dst}.{a}.weight", "conv", (f"{src}.{b}.weight",)),
                      (f"{dst}.{a}.bias", "copy", (f"{src}.{b}.bias",))])
        R.extend([(f"{dst}.temb_proj.weight", "copy", (f"{src}.time_emb_proj.weight",)),
                  (f"{dst}.temb_proj.bias", "copy", (f"{src}.time_emb_proj.bias",))])

    def attn(dst, src):
        R.extend(_transformer2d_rules(dst, src))

    R.extend([("conv_in.weight", "conv", ("conv_in.weight",)), ("conv_in.bias", "copy", ("conv_in.bias",)),
              ("time_lin1.weight", "copy", ("time_embedding.linear_1.weight",)),
              ("time_lin1.bias", "copy", ("time_embedding.linear_1.bias",)),
              ("time_lin2.weight", "copy", ("time_embedding.linear_2.weight",)),
              ("time_lin2.bias", "copy", ("time_embedding.linear_2.bias",)),
              ("norm_out.weight", "copy", ("conv_norm_out.weight",)),
              ("norm_out.bias", "copy", ("conv_norm_out.bias",)),
              ("conv_out.weight", "conv", ("conv_out.weight",)), ("conv_out.bias", "copy", ("conv_out.bias",))])
    res("down.#.resnets.#", "down_blocks.#.resnets.#")
    attn("down.#.attns.#", "down_blocks.#.attentions.#")
    R.extend([("down.#.downsample.conv.weight", "conv", ("down_blocks.#.downsamplers.0.conv.weight",)),
              ("down.#.downsample.conv.bias", "copy", ("down_blocks.#.downsamplers.0.conv.bias",))])
    res("mid_res1", "mid_block.resnets.0")
    res("mid_res2", "mid_block.resnets.1")
    attn("mid_attn", "mid_block.attentions.0")
    res("up.#.resnets.#", "up_blocks.#.resnets.#")
    attn("up.#.attns.#", "up_blocks.#.attentions.#")
    R.extend([("up.#.upsample.conv.weight", "conv", ("up_blocks.#.upsamplers.0.conv.weight",)),
              ("up.#.upsample.conv.bias", "copy", ("up_blocks.#.upsamplers.0.conv.bias",))])
    return R


def _transformer2d_rules(dst: str, src: str) -> List[Rule]:
    """diffusers ``Transformer2DModel`` (one BasicTransformerBlock, self + cross attention, GEGLU)."""
    t = f"{src}.transformer_blocks.0"
    R: List[Rule] = [
        (f"{dst}.norm.weight", "copy", (f"{src}.norm.weight",)),
        (f"{dst}.norm.bias", "copy", (f"{src}.norm.bias",)),
        (f"{dst}.proj_in.weight", "lin1x1", (f"{src}.proj_in.weight",)),
        (f"{dst}.proj_in.bias", "copy", (f"{src}.proj_in.bias",)),
        (f"{dst}.proj_out.weight", "lin1x1", (f"{src}.proj_out.weight",)),
        (f"{dst}.proj_out.bias", "copy", (f"{src}.proj_out.bias",)),
        (f"{dst}.block.attn1.to_qkv.weight", "cat",
         (f"{t}.attn1.to_q.weight", f"{t}.attn1.to_k.weight", f"{t}.attn1.to_v.weight")),
        (f"{dst}.block.attn1.to_out.weight", "copy", (f"{t}.attn1.to_out.0.weight",)),
        (f"{dst}.block.attn1.to_out.bias", "copy", (f"{t}.attn1.to_out.0.bias",)),
        (f"{dst}.block.attn2.to_q.weight", "copy", (f"{t}.attn2.to_q.weight",)),
        (f"{dst}.block.attn2.to_kv.weight", "cat", (f"{t}.attn2.to_k.weight", f"{t}.attn2.to_v.weight")),
        (f"{dst}.block.attn2.to_out.weight", "copy", (f"{t}.attn2.to_out.0.weight",)),
        (f"{dst}.block.attn2.to_out.bias", "copy", (f"{t}.attn2.to_out.0.bias",)),
        (f"{dst}.block.ff.proj.weight", "copy", (f"{t}.ff.net.0.proj.weight",)),
        (f"{dst}.block.ff.proj.bias", "copy", (f"{t}.ff.net.0.proj.bias",)),
        (f"{dst}.block.ff.out.weight", "copy", (f"{t}.ff.net.2.weight",)),
        (f"{dst}.block.ff.out.bias", "copy", (f"{t}.ff.net.2.bias",)),
    ]
    for n in ("norm1", "norm2", "norm3"):
        R.extend([(f"{dst}.block.{n}.weight", "copy", (f"{t}.{n}.weight",)),
                  (f"{dst}.block.{n}.bias", "copy", (f"{t}.{n}.bias",))])
    return R


def _vae_decoder_rules() -> List[Rule]:
    R: List[Rule] = []

    def res(dst, src):
        for n in ("norm1", "norm2"):
            R.extend([(f"{dst}.{n}.weight", "copy", (f"{src}.{n}.weight",)),
                      (f"{dst}.{n}.bias", "copy", (f"{src}.{n}.bias",))])
        for a, b in (("conv1", "conv1"), ("conv2", "conv2"), ("shortcut", "conv_shortcut")):
            R.extend([(f"{dst}.{a}.weight", "conv", (f"{src}.{b}.weight",)),
                      (f"{dst}.{a}.bias", "copy", (f"{src}.{b}.bias",))])

    d = "decoder"
    R.extend([("post_quant.weight", "conv", ("post_quant_conv.weight",)),
              ("post_quant.bias", "copy", ("post_quant_conv.bias",)),
              ("conv_in.weight", "conv", (f"{d}.conv_in.weight",)), ("conv_in.bias", "copy", (f"{d}.conv_in.bias",)),
              ("norm_out.weight", "copy", (f"{d}.conv_norm_out.weight",)),
              ("norm_out.bias", "copy", (f"{d}.conv_norm_out.bias",)),
              ("conv_out.weight", "conv", (f"{d}.conv_out.weight",)),
              ("conv_out.bias", "copy", (f"{d}.conv_out.bias",))])
    res("mid_res1", f"{d}.mid_block.resnets.0")
    res("mid_res2", f"{d}.mid_block.resnets.1")
    a = f"{d}.mid_block.attentions.0"
    R.extend([("mid_attn.norm.weight", "copy", (f"{a}.group_norm.weight",)),
              ("mid_attn.norm.bias", "copy", (f"{a}.group_norm.bias",)),
              ("mid_attn.to_qkv.weight", "cat", (f"{a}.to_q.weight", f"{a}.to_k.weight", f"{a}.to_v.weight")),
              ("mid_attn.to_qkv.bias", "cat", (f"{a}.to_q.bias", f"{a}.to_k.bias", f"{a}.to_v.bias")),
              ("mid_attn.to_out.weight", "copy", (f"{a}.to_out.0.weight",)),
              ("mid_attn.to_out.bias", "copy", (f"{a}.to_out.0.bias",))])
    res("up.#.resnets.#", f"{d}.up_blocks.#.resnets.#")
    R.extend([("up.#.upsample.weight", "conv", (f"{d}.up_blocks.#.upsamplers.0.conv.weight",)),
              ("up.#.upsample.bias", "copy", (f"{d}.up_blocks.#.upsamplers.0.conv.bias",))])
    return R


# diffusers < 0.15 VAE attention names -> current ones
_VAE_LEGACY = {".query.": ".to_q.", ".key.": ".to_k.", ".value.": ".to_v.", ".proj_attn.": ".to_out.0."}


def normalize_vae_names(src: Dict[str, Tensor]) -> Dict[str, Tensor]:
    for old, new in _VAE_LEGACY.items():
        src = {k.replace(old, new): v for k, v in src.items()}
    return src


def _clip_text_rules() -> List[Rule]:
    L = "text_model.encoder.layers.#"
    R: List[Rule] = [("tok.weight", "copy", ("text_model.embeddings.token_embedding.weight",)),
                     ("pos.weight", "copy", ("text_model.embeddings.position_embedding.weight",)),
                     ("final_ln.weight", "copy", ("text_model.final_layer_norm.weight",)),
                     ("final_ln.bias", "copy", ("text_model.final_layer_norm.bias",))]
    for p in ("weight", "bias"):
        R.extend([(f"layers.#.qkv.{p}", "cat", (f"{L}.self_attn.q_proj.{p}", f"{L}.self_attn.k_proj.{p}",
                                                 f"{L}.self_attn.v_proj.{p}")),
                  (f"layers.#.out.{p}", "copy", (f"{L}.self_attn.out_proj.{p}",)),
                  (f"layers.#.ln1.{p}", "copy", (f"{L}.layer_norm1.{p}",)),
                  (f"layers.#.ln2.{p}", "copy", (f"{L}.layer_norm2.{p}",)),
                  (f"layers.#.fc1.{p}", "copy", (f"{L}.mlp.fc1.{p}",)),
                  (f"layers.#.fc2.{p}", "copy", (f"{L}.mlp.fc2.{p}",))])
    return R


def _xlmr_rules() -> List[Rule]:
    """M-CLIP XLM-Roberta-Large text tower (Kandinsky 2.1): HF ``XLMRobertaModel`` names under the
    M-CLIP ``transformer.`` prefix, + ``LinearTransformation`` (1024 -> 768)."""
    E, L = "transformer.embeddings", "transformer.encoder.layer.#"
    R: List[Rule] = [("tok.weight", "copy", (f"{E}.word_embeddings.weight",)),
                     ("pos.weight", "copy", (f"{E}.position_embeddings.weight",)),
                     ("tok_type.weight", "copy", (f"{E}.token_type_embeddings.weight",)),
                     ("ln.weight", "copy", (f"{E}.LayerNorm.weight",)), ("ln.bias", "copy", (f"{E}.LayerNorm.bias",)),
                     ("proj.weight", "copy", ("LinearTransformation.weight",)),
                     ("proj.bias", "copy", ("LinearTransformation.bias",))]
    for p in ("weight", "bias"):
        R.extend([(f"layers.#.qkv.{p}", "cat", (f"{L}.attention.self.query.{p}", f"{L}.attention.self.key.{p}",
                                                 f"{L}.attention.self.value.{p}")),
                  (f"layers.#.out.{p}", "copy", (f"{L}.attention.output.dense.{p}",)),
                  (f"layers.#.ln1.{p}", "copy", (f"{L}.attention.output.LayerNorm.{p}",)),
                  (f"layers.#.fc1.{p}", "copy", (f"{L}.intermediate.dense.{p}",)),
                  (f"layers.#.fc2.{p}", "copy", (f"{L}.output.dense.{p}",)),
                  (f"layers.#.ln2.{p}", "copy", (f"{L}.output.LayerNorm.{p}",))])
    return R


def normalize_clip_names(src: Dict[str, Tensor]) -> Dict[str, Tensor]:
    """transformers >= 5 drops the ``text_model.`` prefix of CLIPTextModel state dicts; the files of
    public SD checkpoints keep it.  Accept both."""
    if any(k.startswith("text_model.") for k in src):
        return src
    return {("text_model." + k if k.startswith(("embeddings.", "encoder.", "final_layer_norm.")) else k): v
            for k, v in src.items()}


# ---- Kandinsky 2.1 (diffusers kandinsky-community layout)
def _glide_unet_rules(m) -> List[Rule]:
    """diffusers ``UNet2DConditionModel`` of Kandinsky 2.1 (scale-shift ResBlocks with resnet
    up/down-sampling, ``SimpleCrossAttn`` blocks with added K/V, ``text_image`` embeddings) ->
    ``GlideUNet`` (models/glide_unet.py)."""
    R: List[Rule] = []
    cfg = m.cfg

    def res(dst, src, blk):
        _wb(R, f"{dst}.norm1", f"{src}.norm1")
        _wb(R, f"{dst}.conv1", f"{src}.conv1", "conv")
        _wb(R, f"{dst}.emb", f"{src}.time_emb_proj")
        _wb(R, f"{dst}.norm2", f"{src}.norm2")
        _wb(R, f"{dst}.conv2", f"{src}.conv2", "conv")
        if blk.skip is not None:
            _wb(R, f"{dst}.skip", f"{src}.conv_shortcut", "conv")

    def attn(dst, src):
        _wb(R, f"{dst}.norm", f"{src}.group_norm")
        for p in ("weight", "bias"):
            R.append((f"{dst}.qkv.{p}", "cat", (f"{src}.to_q.{p}", f"{src}.to_k.{p}", f"{src}.to_v.{p}")))
            R.append((f"{dst}.ctx_kv.{p}", "cat", (f"{src}.add_k_proj.{p}", f"{src}.add_v_proj.{p}")))
        _wb(R, f"{dst}.out", f"{src}.to_out.0")

    _wb(R, "time1", "time_embedding.linear_1")
    _wb(R, "time2", "time_embedding.linear_2")
    _wb(R, "img_emb", "add_embedding.image_proj")
    _wb(R, "text_pool", "add_embedding.text_proj")
    _wb(R, "text_norm", "add_embedding.text_norm")
    _wb(R, "img_tokens", "encoder_hid_proj.image_embeds")
    _wb(R, "text_proj", "encoder_hid_proj.text_proj")
    _wb(R, "conv_in", "conv_in", "conv")
    _wb(R, "norm_out", "conv_norm_out")
    _wb(R, "conv_out", "conv_out", "conv")
    i, nlev = 0, len(cfg.channel_mult)
    for lvl in range(nlev):
        for j in range(cfg.num_res_blocks):
            blk = m.down[i]
            res(f"down.{i}.res", f"down_blocks.{lvl}.resnets.{j}", blk.res)
            if blk.attn is not None:
                attn(f"down.{i}.attn", f"down_blocks.{lvl}.attentions.{j}")
            i += 1
        if lvl != nlev - 1:
            res(f"down.{i}.res", f"down_blocks.{lvl}.downsamplers.0", m.down[i].res)
            i += 1
    res("mid1", "mid_block.resnets.0", m.mid1)
    attn("mid_attn", "mid_block.attentions.0")
    res("mid2", "mid_block.resnets.1", m.mid2)
    i = 0
    for b in range(nlev):
        for j in range(cfg.num_res_blocks + 1):
            blk = m.up[i]
            res(f"up.{i}.res", f"up_blocks.{b}.resnets.{j}", blk.res)
            if blk.attn is not None:
                attn(f"up.{i}.attn", f"up_blocks.{b}.attentions.{j}")
            if blk.upsample is not None:
                res(f"up.{i}.upsample", f"up_blocks.{b}.upsamplers.0", blk.upsample)
            i += 1
    return R


def _movq_rules(m) -> List[Rule]:
    """diffusers ``VQModel`` (norm_type "spatial", the Kandinsky MoVQ) decoder -> ``MoVQDecoder``."""
    R: List[Rule] = []
    d = "decoder"

    def sn(dst, src):
        R.append((f"{dst}.weight", "copy", (f"{src}.norm_layer.weight",)))
        R.append((f"{dst}.bias", "copy", (f"{src}.norm_layer.bias",)))
        R.append((f"{dst}.yb.weight", "convcat", (f"{src}.conv_y.weight", f"{src}.conv_b.weight")))
        R.append((f"{dst}.yb.bias", "cat", (f"{src}.conv_y.bias", f"{src}.conv_b.bias")))

    def res(dst, src, blk):
        sn(f"{dst}.norm1", f"{src}.norm1")
        _wb(R, f"{dst}.conv1", f"{src}.conv1", "conv")
        sn(f"{dst}.norm2", f"{src}.norm2")
        _wb(R, f"{dst}.conv2", f"{src}.conv2", "conv")
        if blk.skip is not None:
            _wb(R, f"{dst}.skip", f"{src}.conv_shortcut", "conv")

    def attn(dst, src):
        sn(f"{dst}.norm", f"{src}.spatial_norm")
        for p in ("weight", "bias"):
            R.append((f"{dst}.qkv.{p}", "cat", (f"{src}.to_q.{p}", f"{src}.to_k.{p}", f"{src}.to_v.{p}")))
        _wb(R, f"{dst}.out", f"{src}.to_out.0")

    _wb(R, "post_quant", "post_quant_conv", "conv")
    _wb(R, "conv_in", f"{d}.conv_in", "conv")
    res("mid1", f"{d}.mid_block.resnets.0", m.mid1)
    attn("mid_attn", f"{d}.mid_block.attentions.0")
    res("mid2", f"{d}.mid_block.resnets.1", m.mid2)
    for i, blk in enumerate(m.up):
        for j, rb in enumerate(blk.res):
            res(f"up.{i}.res.{j}", f"{d}.up_blocks.{i}.resnets.{j}", rb)
        for j in range(len(blk.attn)):
            attn(f"up.{i}.attn.{j}", f"{d}.up_blocks.{i}.attentions.{j}")
        if blk.upsample is not None:
            _wb(R, f"up.{i}.upsample", f"{d}.up_blocks.{i}.upsamplers.0.conv", "conv")
    sn("norm_out", f"{d}.conv_norm_out")
    _wb(R, "conv_out", f"{d}.conv_out", "conv")
    return R


def _prior_rules(m) -> List[Rule]:
    """diffusers ``PriorTransformer`` (kandinsky-2-1-prior) -> ``PriorTransformer`` (models/prior.py)."""
    R: List[Rule] = [("pos", "unsq1", ("positional_embedding",)), ("query", "unsq2", ("prd_embedding",)),
                     ("clip_mean", "unsq1", ("clip_mean",)), ("clip_std", "unsq1", ("clip_std",))]
    _wb(R, "text_enc_proj", "encoder_hidden_states_proj")
    _wb(R, "text_emb_proj", "embedding_proj")
    _wb(R, "img_proj", "proj_in")
    _wb(R, "time1", "time_embedding.linear_1")
    _wb(R, "time2", "time_embedding.linear_2")
    _wb(R, "final_ln", "norm_out")
    _wb(R, "out_proj", "proj_to_clip_embeddings")
    t = "transformer_blocks.#"
    _wb(R, "blocks.#.ln1", f"{t}.norm1")
    for p in ("weight", "bias"):
        R.append((f"blocks.#.qkv.{p}", "cat", (f"{t}.attn1.to_q.{p}", f"{t}.attn1.to_k.{p}", f"{t}.attn1.to_v.{p}")))
    _wb(R, "blocks.#.out", f"{t}.attn1.to_out.0")
    _wb(R, "blocks.#.ln2", f"{t}.norm3")
    _wb(R, "blocks.#.fc1", f"{t}.ff.net.0.proj")
    _wb(R, "blocks.#.fc2", f"{t}.ff.net.2")
    return R


# ---- Kandinsky 2.1 ORIGINAL layout: the ai-forever ``Kandinsky_2.1`` release the kasumi-1 container
# bakes in (templates/kandinsky2.json:1): ``decoder_fp16.ckpt`` (guided-diffusion ``Text2ImUNet``),
# ``prior_fp16.ckpt`` (DALL-E 2 style prior under ``model.``), ``movq_final.ckpt`` (taming-style MoVQ),
# ``ViT-L-14_stats.th`` (CLIP image-embedding mean / std), ``text_encoder/`` (M-CLIP, HF names) and
# the OpenAI CLIP ViT-L/14 state dict (``ViT-L-14.pt`` / ``.safetensors``; a TorchScript archive is
# refused by the weights-only loader - save its ``state_dict()`` once).  The names follow the
# original module trees; the head interleaving of the fused QKV projections is undone at load.
def _k2_orig_unet_rules(m) -> List[Rule]:
    """guided-diffusion ``Text2ImUNet`` (input_blocks / middle_block / output_blocks; ResBlock
    in_layers / emb_layers / out_layers / skip_connection; AttentionBlock norm / qkv / encoder_kv /
    proj_out as conv1d with per-head [q|k|v] rows) -> ``GlideUNet``."""
    R: List[Rule] = []
    hd = m.cfg.head_channels

    def res(dst, src, blk):
        _wb(R, f"{dst}.norm1", f"{src}.in_layers.0")
        _wb(R, f"{dst}.conv1", f"{src}.in_layers.2", "conv")
        _wb(R, f"{dst}.emb", f"{src}.emb_layers.1")
        _wb(R, f"{dst}.norm2", f"{src}.out_layers.0")
        _wb(R, f"{dst}.conv2", f"{src}.out_layers.3", "conv")
        if blk.skip is not None:
            _wb(R, f"{dst}.skip", f"{src}.skip_connection", "conv")

    def attn(dst, src):
        _wb(R, f"{dst}.norm", f"{src}.norm")
        R.append((f"{dst}.qkv.weight", f"heads1d@3@{hd}", (f"{src}.qkv.weight",)))
        R.append((f"{dst}.qkv.bias", f"headsb@3@{hd}", (f"{src}.qkv.bias",)))
        R.append((f"{dst}.ctx_kv.weight", f"heads1d@2@{hd}", (f"{src}.encoder_kv.weight",)))
        R.append((f"{dst}.ctx_kv.bias", f"headsb@2@{hd}", (f"{src}.encoder_kv.bias",)))
        R.append((f"{dst}.out.weight", "lin1d", (f"{src}.proj_out.weight",)))
        R.append((f"{dst}.out.bias", "copy", (f"{src}.proj_out.bias",)))

    _wb(R, "time1", "time_embed.0")
    _wb(R, "time2", "time_embed.2")
    _wb(R, "img_emb", "img_layer")
    _wb(R, "text_pool", "proj_n")
    _wb(R, "text_norm", "ln_model_n")
    _wb(R, "img_tokens", "clip_to_seq")
    _wb(R, "text_proj", "to_model_dim_n")
    _wb(R, "conv_in", "input_blocks.0.0", "conv")
    _wb(R, "norm_out", "out.0")
    _wb(R, "conv_out", "out.2", "conv")
    for i, blk in enumerate(m.down):                     # input_blocks[i + 1] = [ResBlock, (Attention)]
        res(f"down.{i}.res", f"input_blocks.{i + 1}.0", blk.res)
        if getattr(blk, "attn", None) is not None:
            attn(f"down.{i}.attn", f"input_blocks.{i + 1}.1")
    res("mid1", "middle_block.0", m.mid1)
    attn("mid_attn", "middle_block.1")
    res("mid2", "middle_block.2", m.mid2)
    for i, blk in enumerate(m.up):                       # output_blocks[i] = [ResBlock, (Attention), (up ResBlock)]
        res(f"up.{i}.res", f"output_blocks.{i}.0", blk.res)
        k = 1
        if blk.attn is not None:
            attn(f"up.{i}.attn", f"output_blocks.{i}.1")
            k = 2
        if blk.upsample is not None:
            res(f"up.{i}.upsample", f"output_blocks.{i}.{k}", blk.upsample)
    return R


def _k2_orig_movq_rules(m) -> List[Rule]:
    """taming / MoVQ ``decoder`` (up.{level} in resolution order, highest first; mid.block_1 /
    attn_1 / block_2; 1x1-conv q / k / v / proj_out; SpatialNorm norm_layer / conv_y / conv_b;
    nin_shortcut) -> ``MoVQDecoder`` (whose up[0] is the first, lowest-resolution stage)."""
    R: List[Rule] = []
    d = "decoder"

    def sn(dst, src):
        R.append((f"{dst}.weight", "copy", (f"{src}.norm_layer.weight",)))
        R.append((f"{dst}.bias", "copy", (f"{src}.norm_layer.bias",)))
        R.append((f"{dst}.yb.weight", "convcat", (f"{src}.conv_y.weight", f"{src}.conv_b.weight")))
        R.append((f"{dst}.yb.bias", "cat", (f"{src}.conv_y.bias", f"{src}.conv_b.bias")))

    def res(dst, src, blk):
        sn(f"{dst}.norm1", f"{src}.norm1")
        _wb(R, f"{dst}.conv1", f"{src}.conv1", "conv")
        sn(f"{dst}.norm2", f"{src}.norm2")
        _wb(R, f"{dst}.conv2", f"{src}.conv2", "conv")
        if blk.skip is not None:
            _wb(R, f"{dst}.skip", f"{src}.nin_shortcut", "conv")

    def attn(dst, src):
        sn(f"{dst}.norm", f"{src}.norm")
        R.append((f"{dst}.qkv.weight", "catlin1x1", (f"{src}.q.weight", f"{src}.k.weight", f"{src}.v.weight")))
        R.append((f"{dst}.qkv.bias", "cat", (f"{src}.q.bias", f"{src}.k.bias", f"{src}.v.bias")))
        R.append((f"{dst}.out.weight", "lin1x1", (f"{src}.proj_out.weight",)))
        R.append((f"{dst}.out.bias", "copy", (f"{src}.proj_out.bias",)))

    _wb(R, "post_quant", "post_quant_conv", "conv")
    _wb(R, "conv_in", f"{d}.conv_in", "conv")
    res("mid1", f"{d}.mid.block_1", m.mid1)
    attn("mid_attn", f"{d}.mid.attn_1")
    res("mid2", f"{d}.mid.block_2", m.mid2)
    n = len(m.up)
    for i, blk in enumerate(m.up):
        lvl = n - 1 - i
        for j, rb in enumerate(blk.res):
            res(f"up.{i}.res.{j}", f"{d}.up.{lvl}.block.{j}", rb)
        for j in range(len(blk.attn)):
            attn(f"up.{i}.attn.{j}", f"{d}.up.{lvl}.attn.{j}")
        if blk.upsample is not None:
            _wb(R, f"up.{i}.upsample", f"{d}.up.{lvl}.upsample.conv", "conv")
    sn("norm_out", f"{d}.norm_out")
    _wb(R, "conv_out", f"{d}.conv_out", "conv")
    return R


def _k2_orig_prior_rules(m) -> List[Rule]:
    """DALL-E 2 style ``PriorTransformer`` under ``model.`` (glide-text2im ``Transformer``:
    resblocks.N.attn.c_qkv with per-head [q|k|v] rows, c_proj, ln_1, mlp.c_fc / c_proj, ln_2) +
    the CLIP image-embedding statistics -> ``PriorTransformer``."""
    hd = m.cfg.width // m.cfg.heads
    p = "model"
    R: List[Rule] = [("pos", "unsq1", (f"{p}.positional_embedding",)), ("query", "unsq2", (f"{p}.prd_emb",)),
                     ("clip_mean", "unsq1", ("clip_mean",)), ("clip_std", "unsq1", ("clip_std",))]
    _wb(R, "text_enc_proj", f"{p}.text_enc_proj")
    _wb(R, "text_emb_proj", f"{p}.text_emb_proj")
    _wb(R, "img_proj", f"{p}.clip_img_proj")
    _wb(R, "time1", f"{p}.time_embed.0")
    _wb(R, "time2", f"{p}.time_embed.2")
    _wb(R, "final_ln", f"{p}.final_ln")
    _wb(R, "out_proj", f"{p}.out_proj")
    t = f"{p}.transformer.resblocks.#"
    _wb(R, "blocks.#.ln1", f"{t}.ln_1")
    R.append(("blocks.#.qkv.weight", f"heads@3@{hd}", (f"{t}.attn.c_qkv.weight",)))
    R.append(("blocks.#.qkv.bias", f"headsb@3@{hd}", (f"{t}.attn.c_qkv.bias",)))
    _wb(R, "blocks.#.out", f"{t}.attn.c_proj")
    _wb(R, "blocks.#.ln2", f"{t}.ln_2")
    _wb(R, "blocks.#.fc1", f"{t}.mlp.c_fc")
    _wb(R, "blocks.#.fc2", f"{t}.mlp.c_proj")
    return R


def _openai_clip_text_rules() -> List[Rule]:
    """OpenAI CLIP (``clip`` package) text tower names -> ``CLIPTextEncoder``."""
    L = "transformer.resblocks.#"
    R: List[Rule] = [("tok.weight", "copy", ("token_embedding.weight",)),
                     ("pos.weight", "copy", ("positional_embedding",)),
                     ("final_ln.weight", "copy", ("ln_final.weight",)), ("final_ln.bias", "copy", ("ln_final.bias",)),
                     ("layers.#.qkv.weight", "copy", (f"{L}.attn.in_proj_weight",)),
                     ("layers.#.qkv.bias", "copy", (f"{L}.attn.in_proj_bias",))]
    for p in ("weight", "bias"):
        R.extend([(f"layers.#.out.{p}", "copy", (f"{L}.attn.out_proj.{p}",)),
                  (f"layers.#.ln1.{p}", "copy", (f"{L}.ln_1.{p}",)),
                  (f"layers.#.ln2.{p}", "copy", (f"{L}.ln_2.{p}",)),
                  (f"layers.#.fc1.{p}", "copy", (f"{L}.mlp.c_fc.{p}",)),
                  (f"layers.#.fc2.{p}", "copy", (f"{L}.mlp.c_proj.{p}",))])
    return R


def openai_visual_to_hf(src: Dict[str, Tensor]) -> Dict[str, Tensor]:
    """OpenAI CLIP ``visual.*`` names -> transformers ``CLIPVisionModelWithProjection`` names (the
    decoder's zero-image embedding is computed through transformers)."""
    out: Dict[str, Tensor] = {}
    V, H = "visual.", "vision_model."
    direct = {"class_embedding": "embeddings.class_embedding", "conv1.weight": "embeddings.patch_embedding.weight",
              "positional_embedding": "embeddings.position_embedding.weight", "ln_pre.weight": "pre_layrnorm.weight",
              "ln_pre.bias": "pre_layrnorm.bias", "ln_post.weight": "post_layernorm.weight",
              "ln_post.bias": "post_layernorm.bias"}
    for k, v in src.items():
        if not k.startswith(V):
            continue
        r = k[len(V):]
        if r in direct:
            out[H + direct[r]] = v
        elif r == "proj":
            out["visual_projection.weight"] = v.t().contiguous()
        elif r.startswith("transformer.resblocks."):
            i, rest = r[len("transformer.resblocks."):].split(".", 1)
            L = f"{H}encoder.layers.{i}."
            if rest in ("attn.in_proj_weight", "attn.in_proj_bias"):
                kind = "weight" if rest.endswith("weight") else "bias"
                for name, part in zip(("q_proj", "k_proj", "v_proj"), v.chunk(3, 0)):
                    out[f"{L}self_attn.{name}.{kind}"] = part.contiguous()
            else:
                ren = {"attn.out_proj.": "self_attn.out_proj.", "ln_1.": "layer_norm1.", "ln_2.": "layer_norm2.",
                       "mlp.c_fc.": "mlp.fc1.", "mlp.c_proj.": "mlp.fc2."}
                for a, b in ren.items():
                    if rest.startswith(a):
                        out[L + b + rest[len(a):]] = v
    return out


def _k2_stats(weights_dir: str) -> Dict[str, Tensor]:
    """``ViT-L-14_stats.th``: (mean, std) of the CLIP image embeddings (tuple, list or dict)."""
    for rel in ("ViT-L-14_stats.th", "2_1/ViT-L-14_stats.th"):
        path = os.path.join(weights_dir, rel)
        if os.path.isfile(path):
            obj = torch.load(path, map_location="cpu", weights_only=True)
            if isinstance(obj, dict):
                return {"clip_mean": obj["clip_mean"] if "clip_mean" in obj else obj["mean"],
                        "clip_std": obj["clip_std"] if "clip_std" in obj else obj["std"]}
            mean, std = obj
            return {"clip_mean": mean, "clip_std": std}
    return {}


# ---- text-to-video UNet3D (diffusers UNet3DConditionModel: zeroscope_v2_XL, text-to-video-ms-1.7b)
def _temporal_transformer_rules(dst: str, src: str) -> List[Rule]:
    """diffusers ``TransformerTemporalModel`` (double self-attention over frames, GEGLU FF)."""
    t = f"{src}.transformer_blocks.0"
    R: List[Rule] = []
    _wb(R, f"{dst}.norm", f"{src}.norm")
    _wb(R, f"{dst}.proj_in", f"{src}.proj_in", "lin1x1")
    _wb(R, f"{dst}.proj_out", f"{src}.proj_out", "lin1x1")
    for i in (1, 2):
        R.append((f"{dst}.qkv{i}.weight", "cat",
                  (f"{t}.attn{i}.to_q.weight", f"{t}.attn{i}.to_k.weight", f"{t}.attn{i}.to_v.weight")))
        _wb(R, f"{dst}.out{i}", f"{t}.attn{i}.to_out.0")
    for n in ("norm1", "norm2", "norm3"):
        _wb(R, f"{dst}.{n}", f"{t}.{n}")
    _wb(R, f"{dst}.ff.proj", f"{t}.ff.net.0.proj")
    _wb(R, f"{dst}.ff.out", f"{t}.ff.net.2")
    return R


def _unet3d_rules(m) -> List[Rule]:
    R: List[Rule] = []

    def res(dst, src, rb):
        _wb(R, f"{dst}.norm1", f"{src}.norm1")
        _wb(R, f"{dst}.conv1", f"{src}.conv1", "conv")
        _wb(R, f"{dst}.temb_proj", f"{src}.time_emb_proj")
        _wb(R, f"{dst}.norm2", f"{src}.norm2")
        _wb(R, f"{dst}.conv2", f"{src}.conv2", "conv")
        if rb.shortcut is not None:
            _wb(R, f"{dst}.shortcut", f"{src}.conv_shortcut", "conv")

    def tconv(dst, src):
        for i in range(4):
            _wb(R, f"{dst}.norms.{i}", f"{src}.conv{i + 1}.0")
            _wb(R, f"{dst}.convs.{i}", f"{src}.conv{i + 1}.{2 if i == 0 else 3}", "conv3d")

    def layer(dst, blk, j, lyr):
        res(f"{dst}.res", f"{blk}.resnets.{j}", lyr.res)
        tconv(f"{dst}.tconv", f"{blk}.temp_convs.{j}")
        if lyr.attn is not None:
            R.extend(_transformer2d_rules(f"{dst}.attn", f"{blk}.attentions.{j}"))
            R.extend(_temporal_transformer_rules(f"{dst}.tattn", f"{blk}.temp_attentions.{j}"))

    _wb(R, "conv_in", "conv_in", "conv")
    _wb(R, "time_lin1", "time_embedding.linear_1")
    _wb(R, "time_lin2", "time_embedding.linear_2")
    R.extend(_temporal_transformer_rules("transformer_in", "transformer_in"))
    for i, blk in enumerate(m.down):
        for j, lyr in enumerate(blk.layers):
            layer(f"down.{i}.layers.{j}", f"down_blocks.{i}", j, lyr)
        if blk.downsample is not None:
            _wb(R, f"down.{i}.downsample.conv", f"down_blocks.{i}.downsamplers.0.conv", "conv")
    res("mid_in.res", "mid_block.resnets.0", m.mid_in.res)
    tconv("mid_in.tconv", "mid_block.temp_convs.0")
    R.extend(_transformer2d_rules("mid_attn", "mid_block.attentions.0"))
    R.extend(_temporal_transformer_rules("mid_tattn", "mid_block.temp_attentions.0"))
    res("mid_out.res", "mid_block.resnets.1", m.mid_out.res)
    tconv("mid_out.tconv", "mid_block.temp_convs.1")
    for i, blk in enumerate(m.up):
        for j, lyr in enumerate(blk.layers):
            layer(f"up.{i}.layers.{j}", f"up_blocks.{i}", j, lyr)
        if blk.upsample is not None:
            _wb(R, f"up.{i}.upsample.conv", f"up_blocks.{i}.upsamplers.0.conv", "conv")
    _wb(R, "norm_out", "conv_norm_out")
    _wb(R, "conv_out", "conv_out", "conv")
    return R


# ---- Robust Video Matting (upstream rvm_mobilenetv3 state dict; BatchNorm folded at load)
_MBV3_BN_EPS = 1e-3       # torchvision MobileNetV3 norm_layer = BatchNorm2d(eps=0.001)
_BN_EPS = 1e-5            # nn.BatchNorm2d default (LR-ASPP, decoder, refiner)


def _rvm_rules(m) -> List[Rule]:
    R: List[Rule] = []

    def bn(dst, conv, norm, eps):
        R.append((f"{dst}.weight", f"bnw@{eps}", (f"{conv}.weight", f"{norm}.weight", f"{norm}.running_var")))
        R.append((f"{dst}.bias", f"bnb@{eps}",
                  (f"{norm}.weight", f"{norm}.bias", f"{norm}.running_mean", f"{norm}.running_var")))

    feats = m.backbone.features
    bn("backbone.features.0.conv", "backbone.features.0.0", "backbone.features.0.1", _MBV3_BN_EPS)
    for i in range(1, len(feats) - 1):
        ir, j, src = feats[i], 0, f"backbone.features.{i}.block"
        if ir.expand is not None:
            bn(f"backbone.features.{i}.expand.conv", f"{src}.0.0", f"{src}.0.1", _MBV3_BN_EPS)
            j += 1
        bn(f"backbone.features.{i}.dw.conv", f"{src}.{j}.0", f"{src}.{j}.1", _MBV3_BN_EPS)
        j += 1
        if ir.se is not None:
            _wb(R, f"backbone.features.{i}.se.fc1", f"{src}.{j}.fc1")
            _wb(R, f"backbone.features.{i}.se.fc2", f"{src}.{j}.fc2")
            j += 1
        bn(f"backbone.features.{i}.project.conv", f"{src}.{j}.0", f"{src}.{j}.1", _MBV3_BN_EPS)
    last = len(feats) - 1
    bn(f"backbone.features.{last}.conv", f"backbone.features.{last}.0", f"backbone.features.{last}.1",
       _MBV3_BN_EPS)
    bn("aspp.aspp1.conv", "aspp.aspp1.0", "aspp.aspp1.1", _BN_EPS)
    R.append(("aspp.aspp2.weight", "copy", ("aspp.aspp2.1.weight",)))
    _wb(R, "decoder.decode4.gru.ih", "decoder.decode4.gru.ih.0")
    _wb(R, "decoder.decode4.gru.hh", "decoder.decode4.gru.hh.0")
    for n in (3, 2, 1):
        bn(f"decoder.decode{n}.conv.conv", f"decoder.decode{n}.conv.0", f"decoder.decode{n}.conv.1", _BN_EPS)
        _wb(R, f"decoder.decode{n}.gru.gru.ih", f"decoder.decode{n}.gru.ih.0")
        _wb(R, f"decoder.decode{n}.gru.gru.hh", f"decoder.decode{n}.gru.hh.0")
    bn("decoder.out0.conv", "decoder.decode0.conv.0", "decoder.decode0.conv.1", _BN_EPS)
    bn("decoder.out1.conv", "decoder.decode0.conv.3", "decoder.decode0.conv.4", _BN_EPS)
    _wb(R, "project", "project_mat.conv")
    bn("refiner.c1.conv", "refiner.conv.0", "refiner.conv.1", _BN_EPS)
    bn("refiner.c2.conv", "refiner.conv.3", "refiner.conv.4", _BN_EPS)
    _wb(R, "refiner.c3", "refiner.conv.6")
    return R


# legacy name table kept for callers / tests that address the SD1.5 + text-tower rules directly
RULES: Dict[str, Callable[[], List[Rule]]] = {
    "unet": _sd15_unet_rules, "vae": _vae_decoder_rules, "text": _clip_text_rules, "mclip": _xlmr_rules}


def _pattern(p: str) -> re.Pattern:
    return re.compile("^" + re.escape(p).replace("\\#", r"(\d+)") + "$")


def _fill(p: str, idx: Iterable[str]) -> str:
    it = iter(idx)
    return re.sub("#", lambda _: next(it), p)


def _bn_scale(gamma: Tensor, var: Tensor, eps: float) -> Tensor:
    return gamma.double() / torch.sqrt(var.double() + eps)


def _heads_split(kind: str):
    """"heads@N@HD" / "heads1d@N@HD" / "headsb@N@HD" -> (N, HD): a fused projection whose output rows
    are interleaved PER HEAD ([head][q|k|v][HD], guided-diffusion / GLIDE / DALL-E 2 QKV attention),
    against the engine's [q | k | v] concatenation of whole projections."""
    _, n, hd = kind.split("@")
    return int(n), int(hd)


def _to_target(kind: str, srcs: List[Tensor], like: Tensor) -> Tensor:
    if kind.startswith(("heads@", "heads1d@", "headsb@")):
        n, hd = _heads_split(kind)
        t = srcs[0]
        t = t.reshape(t.shape[0], -1) if t.dim() > 1 else t           # conv1d [O, I, 1] -> [O, I]
        rest = tuple(t.shape[1:])
        return t.reshape(-1, n, hd, *rest).transpose(0, 1).reshape(t.shape)
    if kind == "T":
        return srcs[0].t()
    if kind == "catlin1x1":
        return torch.cat([s.reshape(s.shape[0], s.shape[1]) for s in srcs], 0)
    if kind == "conv":
        t = srcs[0]
        t = t.permute(0, 2, 3, 1) if t.dim() == 4 else t      # OIHW -> OHWI
        if t.dim() == 2 and like.dim() == 4:                     # linear stored for a 1x1 conv
            t = t[:, None, None, :]
    elif kind == "lin1x1":
        t = srcs[0]
        t = t.reshape(t.shape[0], t.shape[1]) if t.dim() > 2 else t    # 1x1 conv2d / conv1d -> linear
    elif kind == "cat":
        t = torch.cat(srcs, 0)
    elif kind == "convcat":
        t = torch.cat(srcs, 0).permute(0, 2, 3, 1)
    elif kind == "conv3d":                                      # [O, I, kt, 1, 1] -> [O, kt, 1, I]
        t = srcs[0]
        t = t.reshape(t.shape[0], t.shape[1], t.shape[2]).permute(0, 2, 1)[:, :, None, :]
    elif kind in ("unsq1", "unsq2"):
        t = srcs[0].reshape(like.shape)
    elif kind == "lin1d":                                       # conv1d [O, I, 1] -> linear
        t = srcs[0].reshape(srcs[0].shape[0], -1)
    elif kind.startswith("bnw@"):
        w, g, var = srcs
        s = _bn_scale(g, var, float(kind[4:]))
        t = (w.double() * s.view(-1, *([1] * (w.dim() - 1)))).to(w.dtype)
    elif kind.startswith("bnb@"):
        g, b, mean, var = srcs
        t = (b.double() - mean.double() * _bn_scale(g, var, float(kind[4:]))).to(b.dtype)
    else:
        t = srcs[0]
    return t


def convert(rules: List[Rule], target: Dict[str, Tensor], source: Dict[str, Tensor],
            optional: Tuple[str, ...] = ()) -> Dict[str, Tensor]:
    """source (checkpoint names) -> target (engine names), checked: every target key filled once,
    exact shapes.  ``optional`` target-name regexes may stay unfilled (kept as-is)."""
    out: Dict[str, Tensor] = {}
    pats = [(_pattern(dst), kind, srcs) for dst, kind, srcs in rules]
    for name, like in target.items():
        for pat, kind, srcs in pats:
            m = pat.match(name)
            if m is None:
                continue
            keys = [_fill(s, m.groups()) for s in srcs]
            missing = [k for k in keys if k not in source]
            if missing:
                if kind == "conv" and name.endswith(("shortcut.weight", "shortcut.bias")):
                    break     # the block has no shortcut in this checkpoint either -> reported below
                if any(re.search(o, name) for o in optional):
                    break
                raise KeyError(f"checkpoint lacks {missing} for {name}")
            t = _to_target(kind, [source[k] for k in keys], like)
            if tuple(t.shape) != tuple(like.shape):
                raise ValueError(f"{name}: checkpoint shape {tuple(t.shape)} != engine {tuple(like.shape)}")
            out[name] = t
            break
    unfilled = [n for n in target if n not in out and not any(re.search(o, n) for o in optional)]
    if unfilled:
        raise KeyError(f"{len(unfilled)} engine parameters have no checkpoint tensor, e.g. {unfilled[:5]}")
    return out


def load_state(module: torch.nn.Module, state: Dict[str, Tensor]):
    """Copy converted tensors into the module in place (dtype/device of the module)."""
    params = dict(module.named_parameters())
    with torch.no_grad():
        for k, v in state.items():
            params[k].copy_(v.to(dtype=params[k].dtype))


# --------------------------------------------------------------------------- layouts
def _ident(src):
    return src


def _no_optional(m):
    return ()


def _clip_optional(m):
    """A penultimate-layer text tower (skip_last) never runs its last layer(s); public exports of
    such towers (SD2 / zeroscope text_encoder, 23 of 24 OpenCLIP layers) omit them."""
    n = getattr(m.cfg, "skip_last", 0)
    return tuple(rf"^layers\.{len(m.layers) - 1 - i}\." for i in range(n))


def _no_extra(weights_dir):
    return {}


@dataclass
class Source:
    """Where one engine module's tensors live in a public checkpoint directory."""
    files: Tuple[str, ...]                         # candidate relative paths; the first existing wins
    rules: Callable[[torch.nn.Module], List[Rule]]
    rename: Callable[[Dict[str, Tensor]], Dict[str, Tensor]] = _ident
    optional: Callable[[torch.nn.Module], Tuple[str, ...]] = _no_optional
    extra: Callable[[str], Dict[str, Tensor]] = _no_extra     # side files merged into the source tensors


_DIFF = "diffusion_pytorch_model.safetensors"
_SD_VAE = Source((f"vae/{_DIFF}",), lambda m: _vae_decoder_rules(), normalize_vae_names)
_CLIP = Source(("text_encoder/model.safetensors",), lambda m: _clip_text_rules(), normalize_clip_names,
               _clip_optional)
_VIDEO = {"unet": Source((f"unet/{_DIFF}",), _unet3d_rules), "vae": _SD_VAE, "text": _CLIP}
LAYOUTS: Dict[str, Dict[str, Source]] = {
    "anythingv3": {"unet": Source((f"unet/{_DIFF}",), lambda m: _sd15_unet_rules()), "vae": _SD_VAE,
                   "text": _CLIP},
    "kandinsky2": {
        "unet": Source((f"unet/{_DIFF}",), _glide_unet_rules),
        "movq": Source((f"movq/{_DIFF}",), _movq_rules, normalize_vae_names),
        "prior": Source((f"prior/prior/{_DIFF}",), _prior_rules),
        "clip": Source(("prior/text_encoder/model.safetensors",), lambda m: _clip_text_rules(),
                       normalize_clip_names),
        "clip_proj": Source(("prior/text_encoder/model.safetensors",),
                            lambda m: [("weight", "copy", ("text_projection.weight",))]),
        "xlmr": Source(("text_encoder/model.safetensors",), lambda m: _xlmr_rules()),
    },
    # the original release (see _k2_orig_unet_rules); used when its decoder checkpoint is present
    "kandinsky2_original": {
        "unet": Source(("decoder_fp16.ckpt", "2_1/decoder_fp16.ckpt"), _k2_orig_unet_rules),
        "movq": Source(("movq_final.ckpt", "2_1/movq_final.ckpt"), _k2_orig_movq_rules),
        "prior": Source(("prior_fp16.ckpt", "2_1/prior_fp16.ckpt"), _k2_orig_prior_rules, extra=_k2_stats),
        "clip": Source(("ViT-L-14.safetensors", "ViT-L-14.pt", "2_1/ViT-L-14.safetensors", "2_1/ViT-L-14.pt"),
                       lambda m: _openai_clip_text_rules()),
        "clip_proj": Source(("ViT-L-14.safetensors", "ViT-L-14.pt", "2_1/ViT-L-14.safetensors", "2_1/ViT-L-14.pt"),
                            lambda m: [("weight", "T", ("text_projection",))]),
        "xlmr": Source(("text_encoder/model.safetensors", "text_encoder/pytorch_model.bin",
                        "2_1/text_encoder/model.safetensors", "2_1/text_encoder/pytorch_model.bin"),
                       lambda m: _xlmr_rules()),
    },
    "zeroscopev2xl": _VIDEO,
    "damo": _VIDEO,
    "robust_video_matting": {"net": Source(("rvm_mobilenetv3.safetensors", "rvm_mobilenetv3.pth"), _rvm_rules)},
}
# kept for callers that address the SD1.5 diffusers files by module name
_DIFFUSERS = {name: src.files[0] for name, src in LAYOUTS["anythingv3"].items()}


def _k2_zero_image_embed(weights_dir: str, like: Tensor) -> Tensor:
    """Kandinsky 2.1's unconditional decoder image embedding: the CLIP ViT-L/14 image embedding of
    an all-zero image (diffusers ``KandinskyPriorPipeline.get_zero_embed``), computed once at load
    from ``prior/image_encoder`` (safetensors only) on the CPU in fp32."""
    d = os.path.join(weights_dir, "prior", "image_encoder")
    if not os.path.isfile(os.path.join(d, "model.safetensors")):
        raise FileNotFoundError(f"{d}/model.safetensors (CLIP vision tower for the zero-image embedding) or a "
                                f"native buffers.safetensors is required")
    from transformers import CLIPVisionConfig, CLIPVisionModelWithProjection
    cfg = CLIPVisionConfig.from_pretrained(d, local_files_only=True)
    model = CLIPVisionModelWithProjection(cfg).eval()
    state = read_safetensors(os.path.join(d, "model.safetensors"))
    missing, unexpected = model.load_state_dict(state, strict=False)
    missing = [k for k in missing if not k.endswith("position_ids")]
    if missing:
        raise KeyError(f"{d}: CLIP vision tower lacks {missing[:5]}")
    with torch.no_grad():
        emb = model(pixel_values=torch.zeros(1, 3, cfg.image_size, cfg.image_size)).image_embeds[0]
    if tuple(emb.shape) != tuple(like.shape):
        raise ValueError(f"zero-image embedding {tuple(emb.shape)} != engine {tuple(like.shape)}")
    return emb


def _k2_zero_image_embed_openai(path: str, like: Tensor) -> Tensor:
    """The zero-image embedding from an OpenAI-layout CLIP state dict (original Kandinsky 2.1
    release): ``visual.*`` mapped onto transformers' CLIP vision tower, config read off the shapes."""
    from transformers import CLIPVisionConfig, CLIPVisionModelWithProjection
    src = read_checkpoint(path)
    if "visual.conv1.weight" not in src:
        raise KeyError(f"{path}: no visual.* tensors (CLIP vision tower for the zero-image embedding)")
    width, patch = src["visual.conv1.weight"].shape[0], src["visual.conv1.weight"].shape[-1]
    grid = int(round((src["visual.positional_embedding"].shape[0] - 1) ** 0.5))
    layers = len({k.split(".")[3] for k in src if k.startswith("visual.transformer.resblocks.")})
    inter = src["visual.transformer.resblocks.0.mlp.c_fc.weight"].shape[0]
    cfg = CLIPVisionConfig(hidden_size=width, intermediate_size=inter, num_hidden_layers=layers,
                           num_attention_heads=max(1, width // 64), image_size=grid * patch, patch_size=patch,
                           projection_dim=src["visual.proj"].shape[1], hidden_act="quick_gelu", layer_norm_eps=1e-5)
    model = CLIPVisionModelWithProjection(cfg).eval()
    missing, _ = model.load_state_dict(openai_visual_to_hf(src), strict=False)
    missing = [k for k in missing if not k.endswith("position_ids")]
    if missing:
        raise KeyError(f"{path}: CLIP vision tower lacks {missing[:5]}")
    with torch.no_grad():
        emb = model(pixel_values=torch.zeros(1, 3, cfg.image_size, cfg.image_size)).image_embeds[0]
    if tuple(emb.shape) != tuple(like.shape):
        raise ValueError(f"zero-image embedding {tuple(emb.shape)} != engine {tuple(like.shape)}")
    return emb


def _layout(weights_dir: str, model: str) -> Tuple[Dict[str, Source], str]:
    """The public layout present in ``weights_dir`` (Kandinsky: the original release when its
    decoder checkpoint is there, else the diffusers conversion)."""
    if model == "kandinsky2":
        orig = LAYOUTS["kandinsky2_original"]
        if _first_file(weights_dir, orig["unet"].files) is not None:
            return orig, "kandinsky2_original"
    return LAYOUTS.get(model, {}), model


def _native_path(weights_dir: str, name: str) -> str:
    return os.path.join(weights_dir, f"{name}.safetensors")


def load_native_module(name: str, mod: torch.nn.Module, weights_dir: str):
    state = read_safetensors(_native_path(weights_dir, name))
    target = dict(mod.named_parameters())
    if set(state) != set(target):
        raise KeyError(f"{name}.safetensors: names differ from the engine module "
                       f"(missing {sorted(set(target) - set(state))[:3]}, "
                       f"extra {sorted(set(state) - set(target))[:3]})")
    for k, v in state.items():
        if tuple(v.shape) != tuple(target[k].shape):
            raise ValueError(f"{name}.{k}: shape {tuple(v.shape)} != {tuple(target[k].shape)}")
    load_state(mod, state)


def load_native(pipe, weights_dir: str):
    for name, mod in pipe.modules().items():
        load_native_module(name, mod, weights_dir)


def save_native(pipe, weights_dir: str):
    for name, mod in pipe.modules().items():
        write_safetensors(dict(mod.named_parameters()), _native_path(weights_dir, name))


def _first_file(weights_dir: str, files: Tuple[str, ...]) -> Optional[str]:
    for f in files:
        p = os.path.join(weights_dir, f)
        if os.path.isfile(p):
            return p
    return None


def load_pipeline(pipe, weights_dir: str, model: str):
    """Fill every module of ``pipe`` from ``weights_dir``: per module the native file if present,
    else the family's public layout (``LAYOUTS``).  Missing files / tensors are errors."""
    layout, variant = _layout(weights_dir, model)
    cache: Dict[str, Dict[str, Tensor]] = {}
    problems = []
    for name, mod in pipe.modules().items():
        if os.path.isfile(_native_path(weights_dir, name)):
            load_native_module(name, mod, weights_dir)
            continue
        if model == "kandinsky2" and name == "buffers":
            clip_file = _first_file(weights_dir, LAYOUTS["kandinsky2_original"]["clip"].files)
            if variant == "kandinsky2" and os.path.isdir(os.path.join(weights_dir, "prior")):
                with torch.no_grad():
                    mod.zero_img_emb.copy_(_k2_zero_image_embed(weights_dir, mod.zero_img_emb))
                continue
            if variant == "kandinsky2_original" and clip_file is not None:
                with torch.no_grad():
                    mod.zero_img_emb.copy_(_k2_zero_image_embed_openai(clip_file, mod.zero_img_emb))
                continue
            problems.append(f"{name}.safetensors, prior/image_encoder/ or an OpenAI CLIP ViT-L/14 state dict")
            continue
        src = layout.get(name)
        path = _first_file(weights_dir, src.files) if src is not None else None
        if path is None:
            problems.append(f"{name}.safetensors" + (f" or {' / '.join(src.files)}" if src is not None else ""))
            continue
        if path not in cache:
            cache[path] = read_checkpoint(path)
        state = src.rename(cache[path])
        extra = src.extra(weights_dir)
        if extra:
            state = {**state, **extra}
        target = dict(mod.named_parameters())
        load_state(mod, convert(src.rules(mod), target, state, src.optional(mod)))
    if problems:
        raise FileNotFoundError(f"{weights_dir}: no weights for {model} module(s): " + "; ".join(problems))
    if hasattr(pipe, "_reset_graphs"):
        pipe._reset_graphs()


def load_sd15(pipe, weights_dir: str):
    """anythingv3 / SD1.5 weights (diffusers or native layout) into an ``SD15Pipeline``."""
    return load_pipeline(pipe, weights_dir, "anythingv3")


# --------------------------------------------------------------------------- export (tests, tools)
def _from_target(kind: str, t: Tensor, keys: List[str], out: Dict[str, Tensor]):
    """Inverse of ``_to_target``: engine tensor -> the public tensors it was built from."""
    if kind.startswith(("heads@", "heads1d@", "headsb@")):
        n, hd = _heads_split(kind)
        rest = tuple(t.shape[1:])
        r = t.reshape(n, -1, hd, *rest).transpose(0, 1).reshape(t.shape)
        out[keys[0]] = (r[..., None] if kind.startswith("heads1d@") else r).contiguous()
        return
    if kind == "T":
        out[keys[0]] = t.t().contiguous()
        return
    if kind == "catlin1x1":
        for k, part in zip(keys, t.chunk(len(keys), 0)):
            out[k] = part[:, :, None, None].contiguous()
        return
    if kind == "lin1d":
        out[keys[0]] = t[:, :, None].contiguous()
        return
    if kind == "conv":
        out[keys[0]] = t.permute(0, 3, 1, 2).contiguous()
    elif kind == "lin1x1":
        out[keys[0]] = t[:, :, None, None].contiguous()
    elif kind == "cat":
        for k, part in zip(keys, t.chunk(len(keys), 0)):
            out[k] = part.contiguous()
    elif kind == "convcat":
        for k, part in zip(keys, t.permute(0, 3, 1, 2).chunk(len(keys), 0)):
            out[k] = part.contiguous()
    elif kind == "conv3d":
        out[keys[0]] = t[:, :, 0, :].permute(0, 2, 1)[:, :, :, None, None].contiguous()
    elif kind == "unsq1":
        out[keys[0]] = t[None].contiguous()
    elif kind == "unsq2":
        out[keys[0]] = t[None, None].contiguous()
    elif kind.startswith("bnw@"):      # identity BatchNorm: gamma 1, var 1 - eps (beta / mean set by bnb)
        eps = float(kind[4:])
        out[keys[0]] = t.contiguous()
        out[keys[1]] = torch.ones(t.shape[0], dtype=t.dtype)
        out[keys[2]] = torch.full((t.shape[0],), 1.0 - eps, dtype=torch.float64).to(t.dtype)
    elif kind.startswith("bnb@"):
        out[keys[1]] = t.contiguous()
        out[keys[2]] = torch.zeros_like(t)
    else:
        out[keys[0]] = t.contiguous()


def export_public(pipe, model: str) -> Dict[str, Dict[str, Tensor]]:
    """The engine's weights under the public layout of ``model``: {relative file: state dict}
    (used by the round-trip tests and to hand weights to other tools).  Kandinsky's zero-image
    embedding has no public tensor; it is exported as a native ``buffers.safetensors``."""
    files: Dict[str, Dict[str, Tensor]] = {}
    for name, mod in pipe.modules().items():
        src = LAYOUTS[model].get(name)
        if src is None:
            files[f"{name}.safetensors"] = {k: v.detach().float().cpu().contiguous()
                                            for k, v in mod.named_parameters()}
            continue
        pats = [(_pattern(dst), kind, srcs) for dst, kind, srcs in src.rules(mod)]
        out = files.setdefault(src.files[0], {})
        for tname, t in mod.named_parameters():
            for pat, kind, srcs in pats:
                m = pat.match(tname)
                if m is None:
                    continue
                _from_target(kind, t.detach().float().cpu(), [_fill(s, m.groups()) for s in srcs], out)
                break
    return files


def export_diffusers(pipe) -> Dict[str, Dict[str, Tensor]]:
    """SD1.5 weights under diffusers / transformers names, keyed by module name."""
    by_file = export_public(pipe, "anythingv3")
    return {name: by_file[path] for name, path in _DIFFUSERS.items()}


def write_public(pipe, model: str, weights_dir: str):
    """Write ``export_public`` files: safetensors, or a plain tensor dict (``torch.save``) for the
    ``.ckpt`` / ``.pt`` / ``.bin`` names of layouts that use them."""
    for rel, state in export_public(pipe, model).items():
        path = os.path.join(weights_dir, rel)
        if path.endswith(".safetensors"):
            write_safetensors(state, path)
        else:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            torch.save({k: v.detach().contiguous().cpu() for k, v in state.items()}, path)


def main(argv: Optional[List[str]] = None):
    """python -m arbius_amd.models.weights convert MODEL SRC_DIR DST_DIR: public layout -> native."""
    import argparse
    ap = argparse.ArgumentParser(prog="arbius_amd.models.weights")
    ap.add_argument("action", choices=["convert"])
    ap.add_argument("model")
    ap.add_argument("src")
    ap.add_argument("dst")
    a = ap.parse_args(argv)
    from .registry import build_pipeline
    pipe = build_pipeline(a.model, device="cpu", init=False, weights_dir=a.src)
    save_native(pipe, a.dst)
    print(f"wrote {sorted(pipe.modules())} to {a.dst}")  # noqa: T201 (CLI output)


if __name__ == "__main__":
    main()
