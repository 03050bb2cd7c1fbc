"""Template name -> in-process pipeline factory (replaces the per-model Cog
containers referenced by ``templates/*.json`` ``meta.docker``)."""
from __future__ import annotations

from typing import Optional


def _load(pipe, name: str, weights_dir: Optional[str]):
    """Real weights (safetensors; models/weights.py) when a weights dir is configured, else the
    deterministic random init (benchmarks; BASELINE.json 'random-init weights')."""
    if weights_dir:
        from .weights import load_pipeline
        load_pipeline(pipe, weights_dir, name)
    return pipe


def build_pipeline(name: str, device="cpu", tiny: bool = False, weights_dir: Optional[str] = None,
                   weight_seed: int = 0, **kw):
    """``tokenizer_dir`` defaults to ``weights_dir``: tokenizer files are auto-discovered there
    (models/tokenizer.py ``TOKENIZER_SUBDIRS``), so real weights always run with their real
    tokenizers."""
    if kw.get("tokenizer_dir") is None and weights_dir:
        kw["tokenizer_dir"] = weights_dir
    if name == "anythingv3":
        from .sd15 import SD15Config, SD15Pipeline
        cfg = SD15Config.tiny() if tiny else SD15Config()
        pipe = SD15Pipeline(cfg, device=device, weight_seed=weight_seed, **kw)
        return _load(pipe, name, weights_dir)
    if name == "kandinsky2":
        from .kandinsky2 import Kandinsky2Config, Kandinsky2Pipeline
        cfg = Kandinsky2Config.tiny() if tiny else Kandinsky2Config()
        return _load(Kandinsky2Pipeline(cfg, device=device, weight_seed=weight_seed, **kw), name, weights_dir)
    if name in ("zeroscopev2xl", "damo"):
        from .video import VideoConfig, VideoPipeline
        cfg = VideoConfig.tiny(name) if tiny else VideoConfig.for_model(name)
        return _load(VideoPipeline(cfg, device=device, weight_seed=weight_seed, **kw), name, weights_dir)
    if name == "robust_video_matting":
        from .rvm import RVMConfig, RVMPipeline
        cfg = RVMConfig.tiny() if tiny else RVMConfig()
        return _load(RVMPipeline(cfg, device=device, weight_seed=weight_seed, **kw), name, weights_dir)
    raise ValueError(f"unknown model template {name!r}")
