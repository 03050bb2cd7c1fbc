"""Per-model host-CPU admission for the multi-GPU pool.

Every GPU worker also needs host cores: a task stream's driver thread and the CPU tail of each solve
(PNG / MP4 encode, CID).  Measured per GPU at each model's shipped configuration
(``profiles/cpu_budget_r5.md``, ``bench.py`` ``host_cores_busy``): the diffusion models need 3-5
cores; robust video matting needs ~2 with the GPU H.264 encoder (``profiles/r6/rvm_streams.jsonl``)
and 13.4 when its 48-frame 1080p clips are encoded on the host (``ARB_RVM_GPU_H264=0``) - an 8-GPU
node on a 64-core host that runs host-encoded RVM on every GPU gets ~60 % of the GPU rate and
starves its own control plane.  So at boot the pool compares the cores this process may use
(``os.sched_getaffinity``) with each model's budget and lets a model's tasks onto at most
``floor((cores - reserve) / budget)`` workers (the lowest ranks; the others keep every other model).
The cap is logged; ``mi355x.host_cores`` overrides the core count, ``mi355x.cpu_admission = false``
turns the cap off.
"""
from __future__ import annotations

import logging
import math
import os
from typing import Dict, Iterable, Optional

log = logging.getLogger("arbius.cpu_budget")

# host cores busy per GPU at full rate (profiles/cpu_budget_r5.md; kandinsky2 at its 4 x 4 default:
# profiles/sweep_r5.md "host cores"; RVM with the GPU encoder: profiles/r6/rvm_streams.jsonl, 1.7-2.2)
CORES_PER_GPU = {"anythingv3": 5.1, "kandinsky2": 5.2, "zeroscopev2xl": 3.0, "damo": 3.0,
                 "robust_video_matting": 2.2}
RVM_HOST_ENCODE_CORES = 13.4


def cores_per_gpu(model: str) -> Optional[float]:
    if model == "robust_video_matting" and os.environ.get("ARB_RVM_GPU_H264", "1") == "0":
        return RVM_HOST_ENCODE_CORES
    return CORES_PER_GPU.get(model)
RESERVE_CORES = 2.0          # event loop, RPC server, IPFS pins, SQLite


def host_cores() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:                # non-Linux
        return os.cpu_count() or 1


def model_gpu_caps(models: Iterable[str], n_gpus: int, cores: Optional[int] = None) -> Dict[str, int]:
    """Workers (GPUs) that may take each model's tasks, by the host-core budget; only models whose
    budget does not fit every GPU appear."""
    cores = host_cores() if cores is None else int(cores)
    caps = {}
    for m in models:
        need = cores_per_gpu(m)
        if not need:
            continue
        fit = max(1, int(math.floor(max(0.0, cores - RESERVE_CORES) / need)))
        if fit < n_gpus:
            caps[m] = fit
            log.warning("host-CPU admission: %s needs ~%.1f cores per GPU, this process has %d cores: its tasks "
                        "go to %d of %d GPUs (mi355x.host_cores / cpu_admission to change)", m, need, cores, fit,
                        n_gpus)
    return caps
