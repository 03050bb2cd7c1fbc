"""One-process-per-GPU runtime helpers: rendezvous, RCCL weight broadcast,
health barriers.

The node is task-parallel: every GPU runs an independent worker holding ALL
model weights resident in its 288 GB of HBM; there are no per-step
collectives.  RCCL (torch.distributed backend "nccl" on ROCm) is used for
the boot-time weight broadcast from rank 0 over xGMI and for barriers.

Broadcast design: parameters are re-homed into a few large flat buckets (default
1 GiB) that the modules then VIEW (every tensor at a 256-byte aligned offset, so the
HIP kernels' 16-byte operand loads stay aligned), and each bucket is broadcast in
place: one big ring collective per bucket - per-link bandwidth bound on
point-to-point xGMI, not latency bound - with no concatenated copy on the source
and no copy-back on the receivers.  On CPU/gloo the same code runs for tests.

Failure handling: the process group has a finite timeout (``ARBIUS_DIST_TIMEOUT_S``,
default 600 s), so a collective with a dead peer raises instead of waiting forever,
and ``shutdown`` is bounded (``destroy_process_group`` runs in a helper thread and
is abandoned after ``timeout`` seconds).
"""
from __future__ import annotations

import datetime
import logging
import os
import threading
import time
from typing import Dict, Iterable, List

import torch
import torch.distributed as dist

log = logging.getLogger("arbius.dist")
ALIGN_BYTES = 256


def pg_timeout() -> datetime.timedelta:
    return datetime.timedelta(seconds=float(os.environ.get("ARBIUS_DIST_TIMEOUT_S", "600")))


def env_rank():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def init(backend: str = None, device_type: str = "cuda", force_group: bool = False):
    """Initialise torch.distributed from torchrun env vars (no-op at world size 1 unless
    ``force_group``: then a one-rank group is formed too - on a GPU a one-rank RCCL communicator, so
    the weight broadcast runs the same RCCL code path as on an 8-GPU node)."""
    rank, local, world = env_rank()
    if device_type == "cuda" and torch.cuda.is_available():
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if (world > 1 or force_group) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        if backend is None:
            backend = "nccl" if dev.type == "cuda" else "gloo"
        kw = {"device_id": dev} if dev.type == "cuda" else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, timeout=pg_timeout(), **kw)
    return rank, local, world, dev


def world_info(dev) -> Dict[str, object]:
    """The world this rank actually joined (logged, and reported in the bench JSON): backend, size,
    every rank's device and host, the RCCL version, the HIP / RCCL environment that shapes it."""
    info: Dict[str, object] = {"backend": backend_name(), "world_size": dist.get_world_size() if in_group() else 1,
                               "torch": torch.__version__, "hip": getattr(torch.version, "hip", None)}
    try:
        v = torch.cuda.nccl.version() if torch.cuda.is_available() else None
        info["rccl"] = ".".join(str(x) for x in v) if isinstance(v, tuple) else v
    except Exception:  # noqa: BLE001
        info["rccl"] = None
    import socket
    me = f"{socket.gethostname()}:{dev}"
    if is_dist():
        everyone = [None] * dist.get_world_size()
        dist.all_gather_object(everyone, me)
        info["ranks"] = everyone
    else:
        info["ranks"] = [me]
    info["env"] = {k: os.environ[k] for k in sorted(os.environ)
                   if k.startswith(("NCCL_", "RCCL_", "HSA_", "HIP_VISIBLE", "ROCR_VISIBLE", "TORCH_NCCL"))}
    return info


def is_dist():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def in_group() -> bool:
    """A process group exists (possibly of one rank: ``init(force_group=True)``)."""
    return dist.is_available() and dist.is_initialized()


def backend_name() -> str:
    """'nccl' (= RCCL on ROCm) or 'gloo' when a process group exists (any size), else 'none'."""
    return str(dist.get_backend()) if in_group() else "none"


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def shutdown(timeout: float = 30.0) -> bool:
    """Bounded teardown: ``destroy_process_group`` can block on a dead or wedged peer, so it runs in a
    daemon thread that is abandoned after ``timeout`` seconds.  Returns True when it completed."""
    if not (dist.is_available() and dist.is_initialized()):
        return True
    err: List[BaseException] = []

    def _destroy():
        try:
            dist.destroy_process_group()
        except BaseException as e:  # noqa: BLE001
            err.append(e)

    th = threading.Thread(target=_destroy, name="arbius-pg-destroy", daemon=True)
    th.start()
    th.join(timeout)
    if th.is_alive():
        log.error("destroy_process_group did not return within %.0f s (dead peer?): abandoned", timeout)
        return False
    if err:
        log.warning("destroy_process_group raised %r", err[0])
    return not err


def barrier(dev=None):
    if is_dist():
        if dev is not None and dev.type == "cuda":
            dist.barrier(device_ids=[dev.index])
        else:
            dist.barrier()


def _aligned(numel: int, elem: int) -> int:
    step = max(1, ALIGN_BYTES // elem)
    return -(-numel // step) * step


def rehome_flat(group: List[torch.Tensor], copy: bool) -> torch.Tensor:
    """Allocate one flat buffer for ``group`` (same dtype / device) and make every tensor a view of it
    at an aligned offset (``t.data = view``: every holder of the tensor object sees the new storage).
    ``copy``: carry the current values over (the broadcast source); receivers skip the copy - the
    broadcast fills the buffer in place."""
    with torch.no_grad():
        return _rehome(group, copy)


def _rehome(group: List[torch.Tensor], copy: bool) -> torch.Tensor:
    elem = group[0].element_size()
    sizes = [_aligned(t.numel(), elem) for t in group]
    flat = torch.empty(sum(sizes), dtype=group[0].dtype, device=group[0].device)
    off = 0
    for t, n in zip(group, sizes):
        view = flat[off:off + t.numel()].view(t.shape)
        if copy:
            view.copy_(t)
        t.data = view
        off += n
    return flat


def broadcast_tensors(tensors: List[torch.Tensor], src: int = 0, bucket_bytes: int = 1 << 30) -> Dict[str, float]:
    """Broadcast a list of same-device tensors from ``src`` in flat buckets the tensors are re-homed
    into (views): the collective runs straight on the buckets on every rank.  Runs whenever a
    process group exists - also a one-rank group (``init(force_group=True)``), where the RCCL
    collective is trivial but the whole path (re-homing, buckets, communicator) executes."""
    stats = {"bytes": 0, "buckets": 0, "seconds": 0.0}
    if not in_group() or not tensors:
        return stats
    t0 = time.perf_counter()
    by_dtype: Dict[torch.dtype, List[torch.Tensor]] = {}
    seen = set()
    for t in tensors:
        if id(t) in seen:               # a tied weight listed twice
            continue
        seen.add(id(t))
        by_dtype.setdefault(t.dtype, []).append(t)
    me = dist.get_rank()
    for dtype, ts in by_dtype.items():
        i = 0
        while i < len(ts):
            group, nbytes = [], 0
            while i < len(ts) and (not group or nbytes + ts[i].numel() * ts[i].element_size() <= bucket_bytes):
                group.append(ts[i])
                nbytes += ts[i].numel() * ts[i].element_size()
                i += 1
            flat = rehome_flat(group, copy=(me == src))
            dist.broadcast(flat, src=src)
            stats["bytes"] += nbytes
            stats["buckets"] += 1
    if tensors[0].is_cuda:
        torch.cuda.synchronize(tensors[0].device)
    stats["seconds"] = time.perf_counter() - t0
    return stats


def broadcast_modules(modules: Iterable[torch.nn.Module], src: int = 0, bucket_bytes: int = 1 << 30):
    ts = []
    for m in modules:
        ts.extend(m.parameters())       # the Parameter objects themselves: re-homing sets their .data
        ts.extend(m.buffers())
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
