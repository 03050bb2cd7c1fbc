"""Real-checkpoint loading (safetensors only - nothing in a weights file is ever executed).

The reference miner never touches weights: its Cog containers bake them in
(``templates/*.json`` ``meta.docker``; SURVEY.md §5.4 "model weights from safetensors, loaded
by one rank and RCCL-broadcast").  This module maps the public checkpoint layouts onto this
engine's module tree:

* **diffusers layout** (what anythingv3 / SD1.5 checkpoints ship as):
  ``unet/diffusion_pytorch_model.safetensors``, ``vae/diffusion_pytorch_model.safetensors``,
  ``text_encoder/model.safetensors`` (transformers ``CLIPTextModel`` names).
* **native layout**: ``<module>.safetensors`` per ``pipe.modules()`` entry with this engine's own
  parameter names (``save_native``) - what ``python -m arbius_amd.models.weights convert`` writes once,
  so later boots skip the renaming.

Layout differences handled here, MI355X-first design choices of the engine's modules:
conv weights are stored OHWI (channels-last implicit GEMM), 1x1 ``proj_in``/``proj_out`` convs
are plain linears, self-attention Q/K/V (and cross-attention K/V, and CLIP's q/k/v) are ONE
fused projection.  Every target parameter must be filled exactly once, with the right shape,
or loading fails loudly (no silent partial random init).
"""
from __future__ import annotations

import os
import re
from typing import Callable, Dict, Iterable, List, Optional, Tuple

import torch

Tensor = torch.Tensor


# --------------------------------------------------------------------------- safetensors IO
def read_safetensors(path: str) -> Dict[str, Tensor]:
    from safetensors.torch import load_file
    return load_file(path, device="cpu")


def write_safetensors(state: Dict[str, Tensor], path: str):
    from safetensors.torch import save_file
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    save_file({k: v.detach().contiguous().cpu() for k, v in state.items()}, path)


# --------------------------------------------------------------------------- name rules
# A rule maps a TARGET (engine) name pattern to one or more SOURCE names; ``#`` captures an index.
# kind: "copy" | "conv" (OIHW -> OHWI) | "lin1x1" (1x1 conv OI11 -> linear OI) | "cat" (concat dim 0)
Rule = Tuple[str, str, Tuple[str, ...]]


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
        t = f"{src}.transformer_blocks.0"
        R.extend([
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
        ])
        for n in ("norm1", "norm2", "norm3"):
            R.extend([(f"{dst}.block.{n}.weight", "copy", (f"{t}.{n}.weight",)),
                      (f"{dst}.block.{n}.bias", "copy", (f"{t}.{n}.bias",))])

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


RULES: Dict[str, Callable[[], List[Rule]]] = {
    "unet": _sd15_unet_rules, "vae": _vae_decoder_rules, "text": _clip_text_rules, "mclip": _xlmr_rules}


def _pattern(p: str) -> re.Pattern:
    return re.compile("^" + re.escape(p).replace("\\#", r"(\d+)") + "$")


def _fill(p: str, idx: Iterable[str]) -> str:
    it = iter(idx)
    return re.sub("#", lambda _: next(it), p)


def _to_target(kind: str, srcs: List[Tensor], like: Tensor) -> Tensor:
    if kind == "conv":
        t = srcs[0]
        t = t.permute(0, 2, 3, 1) if t.dim() == 4 else t      # OIHW -> OHWI
        if t.dim() == 2 and like.dim() == 4:                     # linear stored for a 1x1 conv
            t = t[:, None, None, :]
    elif kind == "lin1x1":
        t = srcs[0]
        t = t.reshape(t.shape[0], t.shape[1]) if t.dim() == 4 else t
    elif kind == "cat":
        t = torch.cat(srcs, 0)
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


# --------------------------------------------------------------------------- pipelines
_DIFFUSERS = {"unet": "unet/diffusion_pytorch_model.safetensors",
              "vae": "vae/diffusion_pytorch_model.safetensors",
              "text": "text_encoder/model.safetensors"}


def _layout(weights_dir: str, modules: Dict[str, torch.nn.Module]) -> str:
    if all(os.path.exists(os.path.join(weights_dir, f"{n}.safetensors")) for n in modules):
        return "native"
    if all(os.path.exists(os.path.join(weights_dir, _DIFFUSERS[n])) for n in modules if n in _DIFFUSERS):
        return "diffusers"
    raise FileNotFoundError(f"{weights_dir}: neither <module>.safetensors ({sorted(modules)}) nor the diffusers "
                            f"layout ({sorted(_DIFFUSERS.values())}) found")


def load_native(pipe, weights_dir: str):
    for name, mod in pipe.modules().items():
        state = read_safetensors(os.path.join(weights_dir, f"{name}.safetensors"))
        target = dict(mod.named_parameters())
        if set(state) != set(target):
            raise KeyError(f"{name}.safetensors: names differ from the engine module "
                           f"(missing {sorted(set(target) - set(state))[:3]}, "
                           f"extra {sorted(set(state) - set(target))[:3]})")
        for k, v in state.items():
            if tuple(v.shape) != tuple(target[k].shape):
                raise ValueError(f"{name}.{k}: shape {tuple(v.shape)} != {tuple(target[k].shape)}")
        load_state(mod, state)


def save_native(pipe, weights_dir: str):
    for name, mod in pipe.modules().items():
        write_safetensors(dict(mod.named_parameters()), os.path.join(weights_dir, f"{name}.safetensors"))


def load_sd15(pipe, weights_dir: str):
    """anythingv3 / SD1.5 weights (diffusers or native layout) into an ``SD15Pipeline``."""
    mods = pipe.modules()
    if _layout(weights_dir, mods) == "native":
        return load_native(pipe, weights_dir)
    for name, mod in mods.items():
        src = read_safetensors(os.path.join(weights_dir, _DIFFUSERS[name]))
        if name == "vae":
            for old, new in _VAE_LEGACY.items():
                src = {k.replace(old, new): v for k, v in src.items()}
        if name == "text":
            src = normalize_clip_names(src)
        target = {k: v for k, v in mod.named_parameters()}
        load_state(mod, convert(RULES[name](), target, src))
    if hasattr(pipe, "_reset_graphs"):
        pipe._reset_graphs()


def load_pipeline(pipe, weights_dir: str, model: str):
    """Dispatch by template name; families without a public-layout mapping load native files."""
    if model == "anythingv3":
        return load_sd15(pipe, weights_dir)
    return load_native(pipe, weights_dir)


# --------------------------------------------------------------------------- export (tests, tools)
def export_diffusers(pipe) -> Dict[str, Dict[str, Tensor]]:
    """Inverse of ``load_sd15``: the engine's SD1.5 weights under diffusers / transformers names
    (used by the round-trip test and to hand weights to other tools)."""
    out: Dict[str, Dict[str, Tensor]] = {}
    for name, mod in pipe.modules().items():
        target = dict(mod.named_parameters())
        pats = [(_pattern(dst), kind, srcs) for dst, kind, srcs in RULES[name]()]
        src: Dict[str, Tensor] = {}
        for tname, t in target.items():
            for pat, kind, srcs in pats:
                m = pat.match(tname)
                if m is None:
                    continue
                keys = [_fill(s, m.groups()) for s in srcs]
                t = t.detach().float().cpu()
                if kind == "conv":
                    src[keys[0]] = t.permute(0, 3, 1, 2).contiguous()
                elif kind == "lin1x1":
                    src[keys[0]] = t[:, :, None, None].contiguous()
                elif kind == "cat":
                    for k, part in zip(keys, t.chunk(len(keys), 0)):
                        src[k] = part.contiguous()
                else:
                    src[keys[0]] = t.contiguous()
                break
        out[name] = src
    return out


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
