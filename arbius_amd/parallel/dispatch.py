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
GPU service times fitted to measured single-GPU points of the SHIPPED configurations: a group of k tasks
is W(k) = w0 + w1 k ms of whole-GPU work, and n concurrent streams share the GPU at total rate eff[n]
(n streams fill the chip better than one).  ``SERVICE_MODELS`` holds one fit per model family
(``SD15_MODEL``: anythingv3 at its 3 x 8 default, round-5 kernels; ``K2_MODEL``: Kandinsky2 at its
2 x 8 default, round-6 kernels);
``fit_points`` lists the measured (streams, group, ms per round) points each reproduces.  The
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


# anythingv3 512^2, 50 steps, round-5 kernels with the batch-16 families (profiles/sd_groups_r5.md, one box):
# 4 x 4 30,560 tasks/h = 1,885 ms per round of 16; 4 x 8 31,102 = 3,704 ms per 32; 3 x 8 (shipped) 31,245 =
# 2,765 ms per 24; 2 x 8 (batch-8 families) 30,215 = 1,906 ms per 16; solo 324 ms (profiles/bench_r5_last).
# The 4 x 4 / 4 x 8 pair pins w0 / w1 (a group of 8 costs 1.97x a group of 4 at 4 streams: batching
# saves little beyond batch 8 rows), the rest the stream efficiencies.  (The round-4 fit on 4 x 4
# groups - w0 204.5, w1 149.7 - described the batch-8 families of that round.)
SD15_MODEL = ServiceModel(w0=41.1, w1=282.9, eff=[1.0, 2.418, 2.500, 2.488])
# kandinsky2 768^2, 100 steps + prior, round-6 kernels with the batch-16 families (profiles/r6/k2/, one box
# per line): 2 x 8 (shipped) 7,300 ms per round of 16, 4 x 4 7,420, 3 x 8 11,000, 4 x 8 14,780, 5 x 4 9,733;
# solo 924 ms.  The 4 x 4 / 4 x 8 pair pins w0 / w1 (a group of 8 costs 1.99x a group of 4: the batch-16
# families make batching nearly free of fixed cost), the rest the stream efficiencies.  (Round 5 fitted
# 4 x 4 with the batch-8 families only: w0 480, w1 446.)
K2_MODEL = ServiceModel(w0=28.9, w1=895.1, eff=[1.0, 1.970, 1.961, 1.946, 1.854])
SERVICE_MODELS = {"anythingv3": SD15_MODEL, "kandinsky2": K2_MODEL}
FIT_POINTS = {"anythingv3": [(4, 4, 1885), (4, 8, 3704), (3, 8, 2765), (2, 8, 1906), (1, 1, 324)],
              "kandinsky2": [(2, 8, 7300), (4, 4, 7420), (3, 8, 11000), (4, 8, 14780), (5, 4, 9733), (1, 1, 924)]}
SHIPPED = {"anythingv3": (3, 8), "kandinsky2": (2, 8)}   # streams x lock-step group (config/mining_config.py)


def fit_points(model: str):
    """(streams, group, measured ms per round, modelled ms per round) of ``model``'s fit."""
    m = SERVICE_MODELS[model]
    return [(n, k, ms, m.work(k) * n / m.eff[n - 1]) for n, k, ms in FIT_POINTS[model]]


@dataclass
class _GPU:
    queue: List[tuple] = field(default_factory=list)          # (task id, arrival time)
    active: Dict[int, list] = field(default_factory=dict)     # stream -> [remaining work, tasks]
    in_flight: int = 0
    tasks: int = 0
    groups: int = 0


def simulate(policy: str, rate_per_s: float, n_gpus: int = 8, streams: int = 3, group: int = 8, depth: int = 2,
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

    def stream_rate(n, k):
        # n streams share the GPU at total rate eff[n]; a lone task (group of 1) never runs faster than
        # the measured solo latency (the linear fit's eff > n would otherwise let concurrent solo tasks
        # beat it - the batching gain of larger groups is folded into eff by the fit)
        r = model.eff[min(n, len(model.eff)) - 1] / n
        return min(r, 1.0) if k == 1 else r

    def next_completion():
        best = None
        for r, gp in enumerate(gpus):
            n = len(gp.active)
            if not n:
                continue
            for s, (rem, batch) in gp.active.items():
                dt = rem / stream_rate(n, len(batch))
                if best is None or dt < best[0]:
                    best = (dt, r, s)
        return best

    def advance(dt):
        for gp in gpus:
            n = len(gp.active)
            if not n:
                continue
            for s in gp.active:
                gp.active[s][0] -= stream_rate(n, len(gp.active[s][1])) * dt

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


def node_capacity_per_s(n_gpus: int = 8, streams: int = 3, group: int = 8, model: ServiceModel = SD15_MODEL) -> float:
    """Saturated node throughput of the model (every stream running full groups)."""
    per_round_ms = model.work(group) * streams / model.eff[min(streams, len(model.eff)) - 1]
    return n_gpus * streams * group / per_round_ms * 1000.0
