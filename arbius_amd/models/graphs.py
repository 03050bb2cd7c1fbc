"""Static-shape hipGraph capture of a module forward (torch.cuda.CUDAGraph on ROCm).

The ~500-900 kernels of one denoiser evaluation are replayed as one graph
launch per sampler step, so the step is bound by the kernels, not by Python or
launch latency.  Inputs are copied into the graph's static buffers (a no-op
when the caller passes the static buffer itself).
"""
from __future__ import annotations

import contextlib
import copy
import os
import threading
import time
from typing import Callable, Sequence

import torch

# Captures are serialised process-wide; "thread_local" capture mode lets other threads keep
# launching work on their own streams while one thread captures (concurrent task streams).
CAPTURE_LOCK = threading.Lock()
# ARB_GRAPH_DEBUG=1: log every capture and every replay whose host call takes > 20 ms (stderr)
_DEBUG = os.environ.get("ARB_GRAPH_DEBUG", "0") == "1"


def _dbg(msg):
    import logging
    logging.getLogger("arbius_amd.graphs").warning("[graph %.3f %s] %s", time.perf_counter(),
                                                   threading.current_thread().name, msg)


_SIDE = {}
# ARB_CAPTURE_SIDE=1: warm up and capture on one process-wide side stream instead (A/B; same graphs)
_CAPTURE_SIDE = os.environ.get("ARB_CAPTURE_SIDE", "0") == "1"


def capture_stream(dev) -> "torch.cuda.Stream":
    """The stream a graph is warmed up and captured on: the calling pipeline fork's own stream (the
    stream its replays run on), never a new one.  HIP maps streams onto GPU_MAX_HW_QUEUES (4) hardware
    queues and two streams on one queue run their kernels one after the other
    (profiles/queues_r5_sd15.md), so every extra stream is a chance to land on a task stream's queue.
    Only an unforked pipeline (current stream = the default stream, which cannot capture) uses one
    process-wide side stream."""
    cur = torch.cuda.current_stream(dev)
    if cur != torch.cuda.default_stream(dev) and not _CAPTURE_SIDE:
        return cur
    key = torch.device(dev).index
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=dev)
    return _SIDE[key]


_HELD = []              # rejected candidates, kept alive so their queue stays counted
QUEUE_STATS = {"checked": 0, "rejected": 0, "shared": 0}
_SPIN = 4_000_000       # torch.cuda._sleep cycles: ~1.7 ms on MI355X (50M cycles = 20.9 ms, queue_probe_r5)


def _spin_wall(dev, streams) -> float:
    best = float("inf")
    for _ in range(2):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for s in streams:
            with torch.cuda.stream(s):
                torch.cuda._sleep(_SPIN)
        torch.cuda.synchronize(dev)
        best = min(best, time.perf_counter() - t0)
    return best


def task_stream(dev, peers=()) -> "torch.cuda.Stream":
    """A stream for one concurrent task (a pipeline fork) on a hardware queue that none of ``peers``
    (the other task streams of the same pipeline) uses.  HIP binds a stream to one of
    GPU_MAX_HW_QUEUES (4) HSA queues at its first use, and two streams on one queue run their kernels
    strictly one after the other.  Which queue a stream gets depends on which streams were used before
    it, so changing an unrelated side stream can put two task streams on one queue.  Round 5 measured
    exactly that: slots 2 and 3 of the 4-stream SD bench ran at half the rate of slots 0 and 1
    (profiles/queues_r5_sd15.md).  This function does not assume any mapping; it measures it.  It runs
    a one-workgroup spin kernel on the candidate together with every peer.  If the run takes more than
    1.5 spin lengths, the candidate shares a queue.  The candidate is then held (so its queue stays
    counted) and the next one is tried.  Past GPU_MAX_HW_QUEUES task streams, sharing cannot be avoided
    and the stream is taken as is.  ARB_QUEUE_CHECK=0 turns the check off (A/B)."""
    dev = torch.device(dev)
    if dev.type != "cuda":
        return None
    live = list(peers)
    nq = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    cand = torch.cuda.Stream(device=dev)
    if live and len(live) < nq and os.environ.get("ARB_QUEUE_CHECK", "1") != "0":
        QUEUE_STATS["checked"] += 1
        one = _spin_wall(dev, [cand])
        for _ in range(4 * nq):
            if _spin_wall(dev, live + [cand]) < 1.5 * one:
                break
            QUEUE_STATS["rejected"] += 1
            _HELD.append(cand)
            cand = torch.cuda.Stream(device=dev)
        else:
            QUEUE_STATS["shared"] += 1
            import logging
            logging.getLogger("arbius_amd.graphs").warning(
                "task stream %d shares a hardware queue with another task stream", len(live))
    return cand


def live_table(tensors) -> list:
    """(tensor, address, storage bytes) of every buffer a captured graph reads or writes; the tensors
    are held by the table, so the caching allocator cannot hand their blocks to anyone else."""
    return [(t, t.data_ptr(), t.untyped_storage().nbytes()) for t in tensors]


def check_live(table) -> None:
    """Before a replay: every captured buffer is still the tensor it was captured on (same address, same
    storage size).  A replay into a moved or re-sized block would write another tensor's memory."""
    for t, ptr, nbytes in table:
        if t.data_ptr() != ptr or t.untyped_storage().nbytes() != nbytes:
            raise RuntimeError(f"graph buffer moved: {ptr:#x} -> {t.data_ptr():#x} "
                               f"({nbytes} -> {t.untyped_storage().nbytes()} bytes)")


class GraphedCall:
    def __init__(self, fn: Callable, example_args: Sequence[torch.Tensor], warmup: int = 2):
        dev = example_args[0].device
        self.fn = fn
        self.inputs = [a.detach().clone() for a in example_args]
        if _DEBUG:
            _dbg(f"capture {getattr(fn, '__qualname__', fn)} {[tuple(a.shape) for a in example_args]}")
        with CAPTURE_LOCK:
            s = capture_stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                for _ in range(warmup):   # allocator + kernel-library load outside capture
                    self.out = fn(*self.inputs)
            torch.cuda.current_stream(dev).wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=s, capture_error_mode="thread_local"):
                self.out = fn(*self.inputs)
        outs = self.out if isinstance(self.out, (tuple, list)) else [self.out]
        self._live = live_table(list(self.inputs) + [o for o in outs if isinstance(o, torch.Tensor)])

    def check_live(self):
        check_live(self._live)

    def __call__(self, *args):
        check_live(self._live)
        for dst, src in zip(self.inputs, args):
            if src.data_ptr() != dst.data_ptr():
                dst.copy_(src)
        if _DEBUG:
            t0 = time.perf_counter()
            self.graph.replay()
            dt = time.perf_counter() - t0
            if dt > 0.02:
                _dbg(f"replay {getattr(self.fn, '__qualname__', self.fn)} took {dt * 1e3:.1f} ms on the host")
            return self.out
        self.graph.replay()
        return self.out


class GraphCache:
    """Graphs keyed by input shapes (one per resolution / batch)."""

    def __init__(self, fn: Callable, enabled: bool):
        self.fn, self.enabled = fn, enabled
        self.graphs = {}

    def __call__(self, *args):
        if not self.enabled:
            return self.fn(*args)
        key = tuple(tuple(a.shape) for a in args)
        g = self.graphs.get(key)
        if g is None:
            g = self.graphs[key] = GraphedCall(self.fn, args)
        return g(*args)


class PipelineBase:
    """Stream-aware pipeline plumbing shared by every model family.

    ``fork()`` returns a clone that SHARES the weights but owns its hipGraphs and a
    private HIP stream: N forks solve N tasks concurrently on one GPU (their kernels
    overlap and fill CUs a single small-latent task leaves idle).  Outputs are bitwise
    identical to a solo run - the same kernels and plans run, only interleaved."""

    stream = None

    def _reset_graphs(self):
        raise NotImplementedError

    def fork(self):
        peers = self.__dict__.setdefault("_fork_streams", [])   # shared by every fork of this pipeline
        c = copy.copy(self)
        c._reset_graphs()
        c.stream = task_stream(self.device, peers) if self.device.type == "cuda" else None
        if c.stream is not None:
            peers.append(c.stream)
        c.timings = {}
        return c

    def _stream_ctx(self):
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
