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
from .solver import Solution, infer_task


class FakeSolverPool:
    """Synthetic solver: a PNG derived from (model, input) only - deterministic like a real miner."""

    hardware = "fake"
    weights_id = "synthetic"

    def __init__(self, capacity: int = 1, delay: float = 0.0, servers: int = 0):
        """``servers`` > 0 models a GPU node: at most that many solves run at once (each ``delay``
        seconds, so the node's rate is servers / delay), the rest queue - as the real pools queue one
        more lock-step group per stream behind the running one (``capacity`` = what the orchestrator
        may hand over)."""
        self.capacity = capacity
        self.delay = delay
        self.calls = []
        self.fail_next = 0
        self.servers = servers
        self._sem = None
        self.busy_s = 0.0

    async def solve(self, model, taskid, inp) -> Solution:
        self.calls.append((model.id, taskid, dict(inp)))
        if self.fail_next:
            self.fail_next -= 1
            raise RuntimeError("injected GPU worker failure")
        if self.servers:
            if self._sem is None:
                self._sem = asyncio.Semaphore(self.servers)
            async with self._sem:
                await asyncio.sleep(self.delay)
                self.busy_s += self.delay
        elif self.delay:
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

    def __init__(self, device="cpu", pipeline_factory: Callable = None, capacity: int = 1, lockstep: int = 1,
                 model_streams: Optional[Dict[str, int]] = None, model_lockstep: Optional[Dict[str, int]] = None,
                 **factory_kw):
        from ..models.registry import build_pipeline
        self.device = device
        self.streams = max(1, int(capacity))
        # per-model cap on the streams (forks) a model gets: its solves beyond that wait for a fork
        self.model_streams = dict(model_streams or {})
        # lock-step groups only where launches are batch-invariant (the HIP kernels); the CPU
        # reference path's library GEMMs are not, so grouping there would change CIDs
        self.lockstep = max(1, int(lockstep)) if str(device).startswith("cuda") else 1
        # per-model group size (mi355x.model_lockstep), same GPU-only rule
        self.model_lockstep = ({k: max(1, int(v)) for k, v in (model_lockstep or {}).items()}
                               if str(device).startswith("cuda") else {})
        group_max = max([self.lockstep] + list(self.model_lockstep.values()))
        # concurrent solves the orchestrator may hand us: every stream takes lock-step groups, and
        # with lock-step grouping one more group per stream waits in the pool - a stream that frees
        # up must find its next FULL group already pending (a group forms from whatever is queued at
        # that instant; at depth 1 the replacements were still being leased: 3.0 tasks per group of 4)
        self.depth = 2 if group_max > 1 else 1
        self.capacity = self.streams * group_max * self.depth
        self._exec = None
        self.factory = pipeline_factory or build_pipeline
        self.factory_kw = factory_kw
        self.pipes: Dict[str, object] = {}
        self._free: Dict[str, "queue.Queue"] = {}
        self._pending: Dict[str, "queue.Queue"] = {}
        self._lock = threading.Lock()

    def _pipe(self, model):
        with self._lock:
            if model.name not in self.pipes:
                base = self.factory(model.name, device=self.device, **self.factory_kw)
                self.pipes[model.name] = base
                q = queue.Queue()
                n = max(1, min(self.streams, int(self.model_streams.get(model.name, self.streams))))
                for _ in range(n):
                    q.put(base if n == 1 or not hasattr(base, "fork") else base.fork())
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
            tail = infer_task(model, pipe, inp)
        finally:
            free.put(pipe)          # the CPU tail (encode + CID) runs after the fork is back
        return tail()

    def _solve_waiting(self, model, pending: "queue.Queue"):
        """A stream's turn: this request plus any queued compatible ones, solved lock-step.  A group's
        pipeline goes back to the pool as soon as its GPU work is done; the PNG + CID tail runs on
        this thread while the next group already uses the stream."""
        from .solver import encode_images, infer_images, take_group
        free = self._pipe(model)
        pipe = free.get()
        batch, imgs, tm, tails = [], None, None, None
        try:
            try:
                first = pending.get_nowait()
            except queue.Empty:
                return                      # an earlier turn already took this request in its group
            batch = take_group(pending, first, self.model_lockstep.get(first[0].name, self.lockstep),
                               lambda r: r[0].kind, lambda r: r[1], lambda r: r[0].name)
            if len(batch) > 1 and hasattr(pipe, "run_group"):
                imgs, tm = infer_images(pipe, [r[1] for r in batch])
            else:
                tails = [infer_task(r[0], pipe, r[1]) for r in batch]
        except BaseException as e:  # noqa: BLE001
            for r in batch:
                if not r[2].done():
                    r[2].set_exception(e)
            return
        finally:
            free.put(pipe)
        if tails is not None:           # CPU tails after the fork went back (RVM: H.264 encode)
            for r, tail in zip(batch, tails):
                try:
                    r[2].set_result(tail())
                except BaseException as e:  # noqa: BLE001
                    r[2].set_exception(e)
            return
        if imgs is None:
            return
        try:
            for r, sol in zip(batch, encode_images(imgs, tm)):
                r[2].set_result(sol)
        except BaseException as e:  # noqa: BLE001
            for r in batch:
                if not r[2].done():
                    r[2].set_exception(e)

    async def solve(self, model, taskid, inp) -> Solution:
        import time
        t0 = time.time()
        sol = await self._solve(model, taskid, inp)
        st = self.__dict__.setdefault("_gpu", {"task_s": 0.0, "tasks": 0})
        st["task_s"] += time.time() - t0
        st["tasks"] += 1
        return sol

    def gpu_stats(self):
        """Solved-task count and summed solve seconds of this process's one device (``/metrics``)."""
        return {0: dict(self.__dict__.get("_gpu", {"task_s": 0.0, "tasks": 0}))}

    async def _solve(self, model, taskid, inp) -> Solution:
        loop = asyncio.get_running_loop()
        if self.model_lockstep.get(model.name, self.lockstep) <= 1:
            return await loop.run_in_executor(None, self.solve_sync, model, taskid, inp)
        import concurrent.futures as cf
        with self._lock:
            pending = self._pending.setdefault(model.name, queue.Queue())
        fut: cf.Future = cf.Future()
        pending.put((model, inp, fut))
        with self._lock:
            if self._exec is None:   # own threads: waiting turns must not exhaust the loop's default pool
                self._exec = cf.ThreadPoolExecutor(max_workers=self.capacity, thread_name_prefix="solve")
        loop.run_in_executor(self._exec, self._solve_waiting, model, pending)
        return await asyncio.wrap_future(fut)

    async def close(self):
        if self._exec is not None:
            self._exec.shutdown(wait=False)
        self.pipes.clear()
