"""Per-task spans: host timing + roctx ranges.

``span(name, sink)`` times a stage on the host and, when a GPU is present, brackets
it with a roctx range (``torch.cuda.nvtx`` is backed by roctx on ROCm), so a
``rocprofv3 --marker-trace`` run shows text-encode / denoise / decode / encode
ranges over the kernel timeline.  ``sink`` is a dict that receives
``{name: seconds}`` (pipelines put it into ``Solution.timings``, the miner
exports it as ``arbius_stage_<name>`` on /metrics).
"""
from __future__ import annotations

import time
from contextlib import contextmanager
from typing import Dict, Optional

_ROCTX = None


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        try:
            import torch
            _ROCTX = torch.cuda.nvtx if torch.cuda.is_available() else False
        except Exception:  # noqa: BLE001
            _ROCTX = False
    return _ROCTX


@contextmanager
def span(name: str, sink: Optional[Dict[str, float]] = None, sync=None):
    """Time ``name``; ``sync`` (e.g. torch.cuda.synchronize) makes the host time cover GPU work."""
    rt = _roctx()
    if rt:
        rt.range_push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if sync is not None:
            sync()
        if rt:
            rt.range_pop()
        if sink is not None:
            sink[name] = sink.get(name, 0.0) + time.perf_counter() - t0
