"""One-process-per-GPU runtime helpers: rendezvous, RCCL weight broadcast,
health barriers.

The node is task-parallel: every GPU runs an independent worker holding ALL
model weights resident in its 288 GB of HBM; there are no per-step
collectives.  RCCL (torch.distributed backend "nccl" on ROCm) is used for
the boot-time weight broadcast from rank 0 over xGMI and for barriers.

Broadcast design: parameters are packed into a few large flat buckets
(default 1 GiB) so each broadcast is one big ring collective - per-link
bandwidth bound on point-to-point xGMI, not latency bound - and the packing
is a device-local copy.  On CPU/gloo the same code runs for tests.
"""
from __future__ import annotations

import os
import time
from typing import Dict, Iterable, List

import torch
import torch.distributed as dist


def env_rank():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def init(backend: str = None, device_type: str = "cuda"):
    """Initialise torch.distributed from torchrun env vars (no-op at world size 1)."""
    rank, local, world = env_rank()
    if device_type == "cuda" and torch.cuda.is_available():
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if dev.type == "cuda" else "gloo"
        kw = {"device_id": dev} if dev.type == "cuda" else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, local, world, dev


def is_dist():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def backend_name() -> str:
    """'nccl' (= RCCL on ROCm), 'gloo', or 'none' at world size 1."""
    return str(dist.get_backend()) if is_dist() else "none"


def shutdown():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def barrier(dev=None):
    if is_dist():
        if dev is not None and dev.type == "cuda":
            dist.barrier(device_ids=[dev.index])
        else:
            dist.barrier()


def broadcast_tensors(tensors: List[torch.Tensor], src: int = 0, bucket_bytes: int = 1 << 30) -> Dict[str, float]:
    """Broadcast a list of same-device tensors from ``src`` in packed buckets."""
    stats = {"bytes": 0, "buckets": 0, "seconds": 0.0}
    if not is_dist() or not tensors:
        return stats
    t0 = time.perf_counter()
    by_dtype: Dict[torch.dtype, List[torch.Tensor]] = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    for dtype, ts in by_dtype.items():
        i = 0
        while i < len(ts):
            group, nbytes = [], 0
            while i < len(ts) and (not group or nbytes + ts[i].numel() * ts[i].element_size() <= bucket_bytes):
                group.append(ts[i])
                nbytes += ts[i].numel() * ts[i].element_size()
                i += 1
            flat = torch.cat([g.reshape(-1) for g in group]) if dist.get_rank() == src else \
                torch.empty(sum(g.numel() for g in group), dtype=dtype, device=group[0].device)
            dist.broadcast(flat, src=src)
            if dist.get_rank() != src:
                off = 0
                for g in group:
                    g.copy_(flat[off:off + g.numel()].view_as(g))
                    off += g.numel()
            stats["bytes"] += nbytes
            stats["buckets"] += 1
    if tensors[0].is_cuda:
        torch.cuda.synchronize(tensors[0].device)
    stats["seconds"] = time.perf_counter() - t0
    return stats


def broadcast_modules(modules: Iterable[torch.nn.Module], src: int = 0, bucket_bytes: int = 1 << 30):
    ts = []
    for m in modules:
        ts.extend(p.data for p in m.parameters())
        ts.extend(b for b in m.buffers())
    return broadcast_tensors(ts, src, bucket_bytes)


def all_gather_floats(values: List[float], dev) -> List[List[float]]:
    """Gather a small float vector from every rank (bench metrics)."""
    if not is_dist():
        return [list(values)]
    t = torch.tensor(values, dtype=torch.float64, device=dev)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def max_over_ranks(v: float, dev) -> float:
    if not is_dist():
        return v
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
