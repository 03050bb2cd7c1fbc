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

    def __call__(self, *args):
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
        c = copy.copy(self)
        c._reset_graphs()
        c.stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None
        c.timings = {}
        return c

    def _stream_ctx(self):
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
