"""Task -> GPU dispatch policy of the multi-GPU pool, and a discrete-event model of the node under
Poisson task arrival (what "least-loaded first" costs against "fill one GPU's
lock-step group first" below saturation).

Policies (``MultiGPUSolverPool(dispatch=...)``, ``mi355x.dispatch_policy``):

* ``spread`` - the GPU with the fewest tasks in flight (ties: lowest rank).  Concurrent tasks go to
  different GPUs first; a GPU only forms lock-step groups once its own queue builds up.
* ``pack``   - the GPU with the MOST tasks in flight that still has a free slot: one GPU's lock-step
  groups fill before the next GPU gets work.

The model (``simulate``) runs the pool's admission rule (slots per GPU = streams x group x depth) and
the worker's slot loop (a free stream takes up to ``group`` queued tasks as one lock-step batch) with
GPU service times fitted to measured single-GPU points (``SD15_MODEL``: profiles/bench_r4_stream_group_sweep.md
and the latency-mode line): a group of k tasks is W(k) = w0 + w1 k ms of whole-GPU work, and n
concurrent streams share the GPU at total rate eff[n] (n streams fill the chip better than one).  The
dispatch decision itself is ``pick_rank`` - the same function the pool calls.
"""
from __future__ import annotations

import random
import statistics
from dataclasses import dataclass, field
from typing import Dict, Iterable, List

POLICIES = ("spread", "pack")


def pick_rank(policy: str, idle: Iterable[int], load: Dict[int, int]) -> int:
    """The GPU a new task goes to, among ranks with a free slot (``idle``, may repeat a rank once per
    free slot); ``load``: tasks in flight per rank."""
    cand = set(idle)
    if policy == "pack":
        return max(cand, key=lambda r: (load.get(r, 0), -r))
    if policy != "spread":
        raise ValueError(f"unknown dispatch policy {policy!r}")
    return min(cand, key=lambda r: (load.get(r, 0), r))


@dataclass
class ServiceModel:
    """GPU time of a lock-step group: W(k) = w0 + w1 k (ms of the whole GPU); n concurrent streams
    progress at total rate eff[n - 1]."""
    w0: float
    w1: float
    eff: List[float]

    def work(self, k: int) -> float:
        return self.w0 + self.w1 * k


# anythingv3 512^2, 50 steps (4 streams x groups of 4: 1995 ms per round of 16 tasks; 4 x 2 / 4 x 3: 1254 /
# 1646 ms; 3 x 4 / 3 x 3: 1541 / 1281 ms; 2 x 6 / 2 x 8: 1692 / 2188 ms; 1 stream solo: 354 ms)
SD15_MODEL = ServiceModel(w0=204.5, w1=149.7, eff=[1.0, 1.30, 1.56, 1.61])


@dataclass
class _GPU:
    queue: List[tuple] = field(default_factory=list)          # (task id, arrival time)
    active: Dict[int, list] = field(default_factory=dict)     # stream -> [remaining work, tasks]
    in_flight: int = 0
    tasks: int = 0
    groups: int = 0


def simulate(policy: str, rate_per_s: float, n_gpus: int = 8, streams: int = 4, group: int = 4, depth: int = 2,
             model: ServiceModel = SD15_MODEL, n_tasks: int = 4000, seed: int = 1) -> dict:
    """Poisson arrivals at ``rate_per_s``; returns throughput, latency percentiles, mean lock-step group
    size and per-GPU task counts over the tasks after a warm-up tenth."""
    rng = random.Random(seed)
    gpus = [_GPU() for _ in range(n_gpus)]
    cap = streams * group * depth
    t = 0.0
    arrivals = []
    for i in range(n_tasks):
        t += rng.expovariate(rate_per_s) * 1000.0
        arrivals.append(t)
    pending: List[tuple] = []                     # node-level FIFO (every GPU full)
    done: Dict[int, float] = {}
    group_sizes: List[int] = []
    now = 0.0
    ai = 0

    def admit():
        while pending:
            idle = [r for r, gp in enumerate(gpus) if gp.in_flight < cap]
            if not idle:
                return
            load = {r: gpus[r].in_flight for r in idle}
            r = pick_rank(policy, idle, load)
            tid, ta = pending.pop(0)
            gp = gpus[r]
            gp.in_flight += 1
            gp.queue.append((tid, ta))

    def start_groups(gp):
        for s in range(streams):
            if s in gp.active or not gp.queue:
                continue
            batch, gp.queue = gp.queue[:group], gp.queue[group:]
            gp.active[s] = [model.work(len(batch)), batch]
            gp.groups += 1
            group_sizes.append(len(batch))

    def next_completion():
        best = None
        for r, gp in enumerate(gpus):
            n = len(gp.active)
            if not n:
                continue
            rate = model.eff[min(n, len(model.eff)) - 1] / n
            for s, (rem, _) in gp.active.items():
                dt = rem / rate
                if best is None or dt < best[0]:
                    best = (dt, r, s)
        return best

    def advance(dt):
        for gp in gpus:
            n = len(gp.active)
            if not n:
                continue
            rate = model.eff[min(n, len(model.eff)) - 1] / n
            for s in gp.active:
                gp.active[s][0] -= rate * dt

    while len(done) < n_tasks:
        nc = next_completion()
        ta = arrivals[ai] if ai < n_tasks else None
        if ta is not None and (nc is None or ta - now <= nc[0]):
            advance(ta - now)
            now = ta
            pending.append((ai, ta))
            ai += 1
        else:
            dt, r, s = nc
            advance(dt)
            now += dt
            gp = gpus[r]
            _, batch = gp.active.pop(s)
            for tid, t_arr in batch:
                done[tid] = now - t_arr
            gp.in_flight -= len(batch)
            gp.tasks += len(batch)
        admit()
        for gp in gpus:
            start_groups(gp)
    warm = n_tasks // 10
    lat = sorted(done[i] for i in range(warm, n_tasks))
    span = (arrivals[-1] - arrivals[warm]) / 1000.0
    return {"policy": policy, "rate_per_s": rate_per_s, "offered_tasks_per_h": round(rate_per_s * 3600),
            "completed_per_h": round((n_tasks - warm) / max(1e-9, (max(arrivals[-1], now) - arrivals[warm]) / 1000.0)
                                     * 3600),
            "p50_ms": round(statistics.median(lat), 1), "p90_ms": round(lat[int(0.9 * len(lat))], 1),
            "mean_group": round(sum(group_sizes) / max(1, len(group_sizes)), 2),
            "gpu_tasks": [gp.tasks for gp in gpus], "span_s": round(span, 1)}


def node_capacity_per_s(n_gpus: int = 8, streams: int = 4, group: int = 4, model: ServiceModel = SD15_MODEL) -> float:
    """Saturated node throughput of the model (every stream running full groups)."""
    per_round_ms = model.work(group) * streams / model.eff[min(streams, len(model.eff)) - 1]
    return n_gpus * streams * group / per_round_ms * 1000.0
