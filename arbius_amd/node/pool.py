"""GPU task-worker pools behind the orchestrator's ``solve`` jobs.

* ``LocalSolverPool``  - pipelines in this process on one device (CPU plumbing
  config, single-GPU node); inference runs in a worker thread so the asyncio
  control plane keeps polling events / serving RPC.
* ``parallel.workers.MultiGPUSolverPool`` - one process per GPU (8 on a node).
* ``FakeSolverPool``   - deterministic synthetic outputs (control-plane tests,
  fault injection).
"""
from __future__ import annotations

import asyncio
import hashlib
import queue
import threading
from typing import Callable, Dict, Optional

import numpy as np

from ..ipfs.unixfs import wrap_directory
from ..utils.png import encode_png
from .solver import Solution, solve_task


class FakeSolverPool:
    """Synthetic solver: a PNG derived from (model, input) only - deterministic like a real miner."""

    hardware = "fake"
    weights_id = "synthetic"

    def __init__(self, capacity: int = 1, delay: float = 0.0):
        self.capacity = capacity
        self.delay = delay
        self.calls = []
        self.fail_next = 0

    async def solve(self, model, taskid, inp) -> Solution:
        self.calls.append((model.id, taskid, dict(inp)))
        if self.fail_next:
            self.fail_next -= 1
            raise RuntimeError("injected GPU worker failure")
        if self.delay:
            await asyncio.sleep(self.delay)
        h = hashlib.sha256((model.id + repr(sorted(inp.items()))).encode()).digest()
        img = np.frombuffer(h * 48, dtype=np.uint8)[: 16 * 16 * 3].reshape(16, 16, 3)
        png = encode_png(img)
        dag = wrap_directory([("out-1.png", png)])
        return Solution([("out-1.png", png)], dag.cid_hex, dag, {})

    async def close(self):
        pass


def hardware_id(device) -> str:
    """'gfx950' for an MI355X, 'cpu' for the plumbing config (self-test table key)."""
    import torch
    dev = torch.device(device)
    if dev.type == "cuda":
        name = getattr(torch.cuda.get_device_properties(dev), "gcnArchName", "") or "cuda"
        return name.split(":")[0]
    return "cpu"


class LocalSolverPool:
    """In-process pipelines (lazily built per model) on ``device``.  ``capacity`` > 1 runs
    that many solves concurrently on pipeline forks (shared weights, private HIP stream
    and hipGraphs each) - concurrency never changes a solution's bytes."""

    def __init__(self, device="cpu", pipeline_factory: Callable = None, capacity: int = 1, **factory_kw):
        from ..models.registry import build_pipeline
        self.device = device
        self.capacity = max(1, int(capacity))
        self.factory = pipeline_factory or build_pipeline
        self.factory_kw = factory_kw
        self.pipes: Dict[str, object] = {}
        self._free: Dict[str, "queue.Queue"] = {}
        self._lock = threading.Lock()

    def _pipe(self, model):
        with self._lock:
            if model.name not in self.pipes:
                base = self.factory(model.name, device=self.device, **self.factory_kw)
                self.pipes[model.name] = base
                q = queue.Queue()
                for _ in range(self.capacity):
                    q.put(base if self.capacity == 1 or not hasattr(base, "fork") else base.fork())
                self._free[model.name] = q
            return self._free[model.name]

    def hardware(self) -> str:
        return hardware_id(self.device)

    def weights_id(self) -> str:
        wd = self.factory_kw.get("weights_dir")
        base = f"safetensors:{wd.rstrip('/').split('/')[-1]}" if wd else \
            f"random-init-seed{self.factory_kw.get('weight_seed', 0)}"
        return base + ("-tiny" if self.factory_kw.get("tiny") else "")

    def solve_sync(self, model, taskid, inp) -> Solution:
        free = self._pipe(model)
        pipe = free.get()
        try:
            return solve_task(model, pipe, inp)
        finally:
            free.put(pipe)

    async def solve(self, model, taskid, inp) -> Solution:
        loop = asyncio.get_running_loop()
        return await loop.run_in_executor(None, self.solve_sync, model, taskid, inp)

    async def close(self):
        self.pipes.clear()
