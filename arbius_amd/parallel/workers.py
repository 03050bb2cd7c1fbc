"""One process per GPU: the node-level task-parallel pool.

    dispatcher (asyncio control plane, no GPU)
        |-- mp.Queue --> worker 0 (cuda:0)  \
        |-- mp.Queue --> worker 1 (cuda:1)   >  torch.distributed group over RCCL/xGMI:
        ...                                  |  rank 0 materialises the weights, one
        |-- mp.Queue --> worker N-1          /  bucketed broadcast fills every HBM
        <-- result queue --------------------

* every worker keeps ALL enabled models resident (288 GB HBM per GPU);
* a solve goes to an idle worker; N solves run concurrently, no per-step collectives;
* a worker that dies (HIP fault, OOM, kill) is detected by the watchdog, its in-flight
  task fails over to the caller's retry (another worker), and the worker is respawned
  standalone (deterministic init / safetensors load instead of the broken group) -
  elastic N -> N-1 -> N;
* a worker that HANGS (a HIP kernel that never finishes blocks its host thread) is found by
  heartbeats: every busy task slot stamps a shared-memory clock at each denoising step
  (``utils.progress.beat``); a slot silent for ``hang_timeout`` seconds gets its process killed,
  and the death path above takes over;
* with ``weights_dir`` rank 0 reads the safetensors and broadcasts them; a respawned worker
  reads the same files (byte-identical weights, so the same CIDs as its peers).
* every worker has its OWN request and result queue: a process killed in the middle of
  a queue operation can leave that queue's lock held or a truncated message in its
  pipe, so both queues are replaced on respawn and no other worker's traffic shares them.
On CPU the same code runs with the gloo backend (tests, world size 2).
"""
from __future__ import annotations

import asyncio
import itertools
import logging
import multiprocessing as mp
import os
import queue as pyqueue
import socket
import time
import traceback
from typing import Dict, List, Optional

from .dispatch import POLICIES, pick_rank

log = logging.getLogger("arbius.workers")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker_main(rank: int, world: int, port: int, device_type: str, models: List[str], tiny: bool,
                 in_q, out_q, group: bool, weight_seed: int, streams: int = 1, lockstep: int = 1,
                 weights_dir: Optional[str] = None, beats=None, force_group: bool = False,
                 model_streams: Optional[Dict[str, int]] = None, model_lockstep: Optional[Dict[str, int]] = None):
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import queue as _queue
    import threading

    import torch
    import torch.distributed as dist

    from ..models.registry import build_pipeline
    from ..node.models import Model
    from ..node.solver import encode_images, infer_images, infer_task, take_group
    from . import dist as D

    try:
        if device_type == "cuda":
            torch.cuda.set_device(rank)
            dev = torch.device("cuda", rank)
        else:
            dev = torch.device("cpu")
        # the weight-broadcast group: every rank of a multi-GPU start; ``force_group`` forms it at
        # world size 1 too (a one-rank RCCL communicator: the broadcast path runs exactly as on a node)
        grouped = group and (world > 1 or force_group)
        if grouped:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            backend = "nccl" if device_type == "cuda" else "gloo"
            kw = {"device_id": dev} if device_type == "cuda" else {}
            dist.init_process_group(backend, rank=rank, world_size=world, timeout=D.pg_timeout(), **kw)
        pipes = {}
        bstats = {"bytes": 0, "seconds": 0.0}
        from ..utils import progress
        if beats is not None:
            progress.set_hook(progress.shared_stamp_hook(beats, rank * streams))
        src = (not group) or world == 1 or rank == 0     # this process materialises the weights
        for name in models:
            pipe = build_pipeline(name, device=dev, tiny=tiny, weight_seed=weight_seed,
                                  init=src and not weights_dir, weights_dir=weights_dir if src else None,
                                  tokenizer_dir=weights_dir)
            if grouped:
                if (os.environ.get("ARBIUS_FAULT_INJECTION") == "1"
                        and os.environ.get("ARBIUS_FAULT_BCAST_DIE_RANK") == str(rank)):
                    os._exit(17)                    # test hook: a rank lost in the middle of the broadcast
                st = D.broadcast_modules(pipe.modules().values())
                bstats["bytes"] += st["bytes"]
                bstats["seconds"] += st["seconds"]
                if hasattr(pipe, "_reset_graphs"):
                    pipe._reset_graphs()
            pipes[name] = pipe
        # `streams` task slots share, per model, a pool of min(streams, model cap) pipeline forks (private
        # HIP stream + hipGraphs each; ADVICE r4: one fork per slot gave a capped model - Kandinsky2,
        # video, matting - 4 graph memory pools per GPU for the 2 solves its cap allows).  A slot takes
        # a fork of its job's model for the GPU part and returns it before the CPU tail.
        caps_n = {n: max(1, min(streams, int((model_streams or {}).get(n, streams)))) for n in pipes}
        forks = {}
        for n, p in pipes.items():
            q = _queue.Queue()
            for _ in range(caps_n[n]):
                q.put(p if streams == 1 or not hasattr(p, "fork") else p.fork())
            forks[n] = q
        fork_stats = {n: {"forks": caps_n[n], "in_use": 0, "peak": 0} for n in pipes}
        fork_mu = threading.Lock()
        jobs: "_queue.Queue" = _queue.Queue()
        from concurrent.futures import ThreadPoolExecutor
        # per slot: one thread for a lock-step group's PNG + CID tail, so the slot's stream starts
        # its next group while the previous one encodes
        tails = [ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"tail{k}") for k in range(streams)]
        last_tail = [None] * streams        # a slot's solo-task tail in flight (at most one: RVM clips are 300 MB)

        def finish(batch, imgs, tm, t0, k=None):
            if k is not None:
                tail_clock(k, True)
            try:
                for m, sol in zip(batch, encode_images(imgs, tm)):
                    sol.dag = None
                    sol.timings["worker_s"] = time.perf_counter() - t0
                    sol.timings["fork_peak"] = fork_stats[m[1]]["peak"]
                    out_q.put(("ok", m[0], rank, sol))
            except Exception:  # noqa: BLE001
                for m in batch:
                    out_q.put(("err", m[0], rank, traceback.format_exc()))
            finally:
                if k is not None:
                    tail_clock(k, False)

        def tail_clock(k, on):
            if beats is not None:
                beats[(world + rank) * streams + k] = time.time() if on else 0.0

        def finish_solo(batch, tail_fns, t0, k):
            tail_clock(k, True)
            try:
                _finish_solo(batch, tail_fns, t0)
            finally:
                tail_clock(k, False)

        def _finish_solo(batch, tail_fns, t0):
            for m, fn in zip(batch, tail_fns):
                try:
                    sol = fn()
                    sol.dag = None  # blocks are recomputed by the pinner; keep the message small
                    sol.timings["worker_s"] = time.perf_counter() - t0
                    sol.timings["fork_peak"] = fork_stats[m[1]]["peak"]
                    out_q.put(("ok", m[0], rank, sol))
                except Exception:  # noqa: BLE001
                    out_q.put(("err", m[0], rank, traceback.format_exc()))

        def slot_loop(k):
            progress.set_slot(k)
            while True:
                msg = jobs.get()
                if msg is None:
                    return
                jid, mname, kind, mid, taskid, inp = msg
                # the fork FIRST, then the group: with more slots than forks of a model (4
                # slots, 3 anythingv3 forks) a slot that formed its group before waiting for a fork held
                # a partial group; now the group forms from whatever queued while it waited
                pipe = forks[mname].get()           # idle (beat 0) while every fork of the model solves
                # lock-step group: queued compatible image tasks share one batch (same bytes as solo)
                batch = take_group(jobs, msg, (model_lockstep or {}).get(msg[1], lockstep), lambda m: m[2],
                                   lambda m: m[5], lambda m: m[1])
                with fork_mu:
                    st = fork_stats[mname]
                    st["in_use"] += 1
                    st["peak"] = max(st["peak"], st["in_use"])
                progress.beat()                     # busy from now on (0 = idle)
                released = False

                def release():
                    nonlocal released
                    if not released:
                        released = True
                        with fork_mu:
                            fork_stats[mname]["in_use"] -= 1
                        forks[mname].put(pipe)
                try:
                    if inp.get("__fault__") == "hang" and os.environ.get("ARBIUS_FAULT_INJECTION") == "1":
                        while True:                 # test hook: a hung kernel - no beats, no result
                            time.sleep(1.0)
                    t0 = time.perf_counter()
                    if len(batch) > 1 and hasattr(pipe, "run_group"):
                        imgs, tm = infer_images(pipe, [m[5] for m in batch])
                        release()
                        tails[k].submit(finish, batch, imgs, tm, t0, k)
                        continue
                    # GPU part now; the CPU tail (e.g. RVM's H.264 encode) on the slot's tail thread
                    # while the slot takes its next task
                    fns = [infer_task(Model(m[3], m[1], {}, True, [], m[2]), pipe, m[5]) for m in batch]
                    release()
                    if last_tail[k] is not None:
                        last_tail[k].result()
                    last_tail[k] = tails[k].submit(finish_solo, batch, fns, t0, k)
                except Exception:  # noqa: BLE001
                    for m in batch:
                        out_q.put(("err", m[0], rank, traceback.format_exc()))
                finally:
                    release()
                    if beats is not None:
                        beats[rank * streams + k] = 0.0

        threads = [threading.Thread(target=slot_loop, args=(k,), daemon=True) for k in range(streams)]
        for t in threads:
            t.start()
        world_info = D.world_info(dev) if grouped else {"backend": "none", "world_size": 1}
        log.info("worker %d ready: %s", rank, world_info)
        from ..node.pool import hardware_id
        # the dispatcher never touches the GPU: the worker reports its device's arch (self-test key)
        out_q.put(("ready", rank, dict(bstats, world=world_info, arch=hardware_id(dev),
                                       forks={n: st["forks"] for n, st in fork_stats.items()})))
        while True:
            msg = in_q.get()
            if msg is None:
                break
            jobs.put(msg)
        for _ in threads:
            jobs.put(None)
        for t in threads:
            t.join()
        for tp in tails:
            tp.shutdown(wait=True)
    finally:
        # bounded: with a dead peer destroy_process_group can block forever, and a worker that never
        # exits would stall the pool's shutdown (close() joins it)
        if dist.is_initialized() and not D.shutdown(timeout=15.0):
            os._exit(0)


class MultiGPUSolverPool:
    def __init__(self, n: int, models: List[str], device_type: str = "cuda", tiny: bool = False,
                 weight_seed: int = 0, start_timeout: float = 1800.0, streams_per_gpu: int = 1,
                 lockstep: int = 1, weights_dir: Optional[str] = None, hang_timeout: float = 300.0,
                 force_group: bool = False, model_streams: Optional[Dict[str, int]] = None,
                 dispatch: str = "spread", model_lockstep: Optional[Dict[str, int]] = None,
                 model_gpu_cap: Optional[Dict[str, int]] = None):
        if dispatch not in POLICIES:
            raise ValueError(f"dispatch policy {dispatch!r} not in {POLICIES}")
        self.dispatch = dispatch
        self.n = n
        # host-CPU admission (parallel/cpu_budget.py): model -> how many workers (ranks 0..cap-1) take it
        self.model_gpu_cap = {k: max(1, int(v)) for k, v in (model_gpu_cap or {}).items()}
        self.model_streams = dict(model_streams or {})
        self.force_group = bool(force_group)
        self.arch = None                         # gcnArchName reported by the workers (no GPU call here)
        self.models = models
        self.device_type = device_type
        self.tiny = tiny
        self.weight_seed = weight_seed
        self.weights_dir = weights_dir
        self.hang_timeout = float(hang_timeout)
        self.ctx = mp.get_context("spawn")
        self.hangs = 0
        self.in_qs = [self.ctx.Queue() for _ in range(n)]
        self.out_qs = [self.ctx.Queue() for _ in range(n)]
        self.procs: List[Optional[mp.Process]] = [None] * n
        self.streams = max(1, int(streams_per_gpu))
        # per task slot: time of its last progress beat, 0.0 while idle (shared memory, no lock:
        # one writer per slot, the watchdog only reads)
        # second half: per task slot, the start time of its CPU tail in flight (0.0 when none; ADVICE r4:
        # a tail - RVM's H.264 encode + CID - runs after the slot's beat went idle, so the watchdog
        # times it separately)
        self.beats = self.ctx.Array("d", 2 * n * self.streams, lock=False)
        # tasks per lock-step group on one stream (HIP kernels only: batch-invariant launches)
        self.lockstep = max(1, int(lockstep)) if device_type == "cuda" else 1
        # per-model group size (mi355x.model_lockstep), same GPU-only rule
        self.model_lockstep = ({k: max(1, int(v)) for k, v in (model_lockstep or {}).items()}
                               if device_type == "cuda" else {})
        group_max = max([self.lockstep] + list(self.model_lockstep.values()))
        # one more lock-step group per stream queued in the worker (node/pool.py LocalSolverPool.depth)
        self.depth = 2 if group_max > 1 else 1
        self.slots_per_rank = max(self.model_slots(m) for m in models) if models else self.streams
        self.busy: Dict[int, int] = {}           # job id -> rank
        self._job_model: Dict[int, str] = {}     # job id -> model name (per-model admission)
        self._started: Dict[int, float] = {}     # job id -> dispatch time
        self._gpu: Dict[int, dict] = {}          # rank -> {"task_s", "tasks"} (/metrics)
        self.idle: List[int] = []                # one entry per free task slot (rank repeated)
        self.futures: Dict[int, asyncio.Future] = {}
        self._ids = itertools.count(1)
        self.broadcast_stats = {}
        self.world = None                        # the process group the workers formed (rank 0's view)
        self.restarts = 0
        port = _free_port()
        for r in range(n):
            self._spawn(r, port, group=True)
        try:
            self._await_ready(start_timeout)
        except BaseException:
            # one rank lost during start (e.g. mid-broadcast) leaves its peers blocked in a collective
            # until the process-group timeout: take every worker down now, then fail loudly
            self._kill_all()
            raise
        self.idle.sort()
        self._pump_task = None

    def _kill_all(self):
        for p in self.procs:
            if p is not None and p.is_alive():
                p.kill()
        for p in self.procs:
            if p is not None:
                p.join(10)

    def _await_ready(self, start_timeout: float):
        t0 = time.time()
        pending = set(range(self.n))
        while pending:
            if time.time() - t0 > start_timeout:
                raise TimeoutError("GPU workers did not start")
            for r in sorted(pending):
                try:
                    kind, rank, payload = self.out_qs[r].get(timeout=0.2)
                except pyqueue.Empty:
                    p = self.procs[r]
                    if p is not None and not p.is_alive():
                        raise RuntimeError(f"GPU worker {r} died during start (exit {p.exitcode})")
                    continue
                if kind == "ready":
                    pending.discard(rank)
                    self.idle.extend([rank] * self.slots_per_rank)
                    self.broadcast_stats[rank] = payload
                    self.world = payload.get("world")
                    self.arch = self.arch or payload.get("arch")

    def hardware(self) -> str:
        """The workers' device arch ('gfx950'), from their ``ready`` messages: the dispatcher process
        never initialises HIP, so every respawn is a spawned child of a GPU-free parent."""
        return self.arch or ("cpu" if self.device_type != "cuda" else "unknown")

    def weights_id(self) -> str:
        base = (f"safetensors:{os.path.basename(os.path.normpath(self.weights_dir))}" if self.weights_dir
                else f"random-init-seed{self.weight_seed}")
        return base + ("-tiny" if self.tiny else "")

    def model_slots(self, name: str) -> int:
        """Tasks of model ``name`` one worker admits: its forks (streams capped by ``model_streams``) x
        its lock-step group x queue depth (one more group per fork) - a capped model (Kandinsky2,
        video) no longer queues at the largest model's group size."""
        forks = max(1, min(self.streams, int(self.model_streams.get(name, self.streams))))
        g = self.model_lockstep.get(name, self.lockstep)
        return forks * g * (2 if g > 1 else 1)

    @property
    def capacity(self) -> int:
        return self.slots_per_rank * sum(1 for p in self.procs if p is not None and p.is_alive())

    def _spawn(self, rank, port, group):
        for k in range(self.streams):
            self.beats[rank * self.streams + k] = 0.0
            self.beats[(self.n + rank) * self.streams + k] = 0.0
        p = self.ctx.Process(target=_worker_main, daemon=True,
                             args=(rank, self.n, port, self.device_type, self.models, self.tiny,
                                   self.in_qs[rank], self.out_qs[rank], group, self.weight_seed, self.streams,
                                   self.lockstep, self.weights_dir, self.beats, group and self.force_group,
                                   self.model_streams, self.model_lockstep))
        p.start()
        self.procs[rank] = p

    def _ensure_pump(self):
        if self._pump_task is None or self._pump_task.done():
            self._pump_task = asyncio.ensure_future(self._pump())

    def _handle(self, msg):
        kind = msg[0]
        if kind == "ready":
            rank = msg[1]
            self.idle = [r for r in self.idle if r != rank] + [rank] * self.slots_per_rank
            self.arch = self.arch or msg[2].get("arch")
            return
        _, jid, rank, payload = msg
        self._job_model.pop(jid, None)
        if self.busy.pop(jid, None) is not None:
            self.idle.append(rank)
        t0 = self._started.pop(jid, None)
        if t0 is not None and kind == "ok":
            st = self._gpu.setdefault(rank, {"task_s": 0.0, "tasks": 0})
            st["task_s"] += time.time() - t0
            st["tasks"] += 1
        fut = self.futures.pop(jid, None)
        if fut is None or fut.done():
            return
        if kind == "ok":
            fut.set_result(payload)
        else:
            fut.set_exception(RuntimeError(f"worker {rank} failed:\n{payload}"))

    def _drain_nowait(self) -> int:
        n = 0
        for q in list(self.out_qs):
            while True:
                try:
                    msg = q.get_nowait()
                except pyqueue.Empty:
                    break
                self._handle(msg)
                n += 1
        return n

    async def _pump(self):
        while self.futures:
            if not self._drain_nowait():
                self._watchdog()
                await asyncio.sleep(0.005)

    def hung_ranks(self, now: Optional[float] = None) -> List[int]:
        """Workers with a busy task slot that has not beaten for ``hang_timeout`` seconds."""
        now = time.time() if now is None else now
        out = []
        for r in range(self.n):
            stamps = [self.beats[r * self.streams + k] for k in range(self.streams)]
            tails = [self.beats[(self.n + r) * self.streams + k] for k in range(self.streams)]
            if any(t > 0.0 and now - t > self.hang_timeout for t in stamps + tails):
                out.append(r)
        return out

    def _watchdog(self):
        for r in self.hung_ranks():
            p = self.procs[r]
            if p is not None and p.is_alive():
                log.error("GPU worker %d hung (no progress beat for %.0f s): killing it", r, self.hang_timeout)
                self.hangs += 1
                p.kill()
                p.join(30)
        for r, p in enumerate(self.procs):
            if p is not None and not p.is_alive():
                log.error("GPU worker %d died (exit %s): failing its tasks over, respawning", r, p.exitcode)
                for jid in [j for j, rr in self.busy.items() if rr == r]:
                    del self.busy[jid]
                    self._job_model.pop(jid, None)
                    if jid in self.futures:
                        self.futures.pop(jid).set_exception(RuntimeError(f"worker {r} died"))
                self.idle = [x for x in self.idle if x != r]
                self.restarts += 1
                # a SIGKILLed process can die holding a queue lock or mid-message: fresh queues
                self.in_qs[r] = self.ctx.Queue()
                self.out_qs[r] = self.ctx.Queue()
                self._spawn(r, _free_port(), group=False)   # standalone: deterministic init / load

    def _eligible(self, name: str) -> List[int]:
        """Ranks with a free slot that still admit a task of model ``name``."""
        cap = self.model_slots(name)
        ranks = self.model_gpu_cap.get(name, self.n)
        held: Dict[int, int] = {}
        for jid, r in self.busy.items():
            if self._job_model.get(jid) == name:
                held[r] = held.get(r, 0) + 1
        return [r for r in set(self.idle) if r < ranks and held.get(r, 0) < cap]

    async def solve(self, model, taskid, inp):
        self._watchdog()
        self._drain_nowait()
        while not self._eligible(model.name):
            await asyncio.sleep(0.01)
            self._watchdog()
            self._drain_nowait()
        # dispatch policy (parallel/dispatch.py): "spread" (default) = least-loaded GPU first - below
        # saturation a task starts at once on an idle GPU (p50 at the solo latency vs ~3.7 s when GPUs
        # are packed, profiles/dispatch_r5.md); groups still form where a GPU's own queue builds up
        cand = self._eligible(model.name)
        load = {r: sum(1 for rr in self.busy.values() if rr == r) for r in cand}
        rank = pick_rank(self.dispatch, cand, load)
        self.idle.remove(rank)
        jid = next(self._ids)
        fut = asyncio.get_running_loop().create_future()
        self.futures[jid] = fut
        self.busy[jid] = rank
        self._job_model[jid] = model.name
        self._started[jid] = time.time()
        self.in_qs[rank].put((jid, model.name, model.kind, model.id, taskid, dict(inp)))
        self._ensure_pump()
        return await fut

    def gpu_stats(self):
        """Per-GPU solved-task count and summed solve seconds (``/metrics``)."""
        return {r: dict(self._gpu.get(r, {"task_s": 0.0, "tasks": 0})) for r in range(self.n)}

    def kill_worker(self, rank: int):
        """Fault injection (tests): hard-kill one worker process."""
        p = self.procs[rank]
        if p is not None and p.is_alive():
            p.kill()
            p.join(30)   # deterministic injection: the worker is gone when this returns

    async def close(self):
        for q in self.in_qs:
            try:
                q.put(None)
            except Exception:  # noqa: BLE001
                pass
        for p in self.procs:
            if p is not None:
                p.join(timeout=10)
                if p.is_alive():
                    p.kill()
