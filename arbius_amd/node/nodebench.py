"""Whole-node benchmark (``bench.py --node``): tasks solved / hour measured THROUGH the node's own stack.

The pipeline bench (``bench.py``) drives pipelines directly.  This mode instead submits tasks to an
in-process MockEngine (EngineV1 semantics) and lets the real orchestrator do everything the
reference miner does per task (``/root/reference/miner/src/index.ts:191-211`` event ->
``:506-564`` processTask -> ``:566-672`` processSolve):

  TaskSubmitted event poll -> ``task`` job -> tx-input recovery + template hydration + seed ->
  ``solve`` job -> solver pool (``LocalSolverPool`` on 1 GPU, ``MultiGPUSolverPool`` = one worker
  process per GPU with the RCCL weight broadcast otherwise) -> PNG / MP4 + directory CID ->
  signalCommitment -> submitSolution (checked by the MockEngine) -> claim job scheduled,
  plus the background IPFS pin of every solution (MockIPFS: blocks in memory).

The reference serialises solves (``index.ts:555-563``, ``concurrent: false``); here the pool's
capacity (GPUs x task streams x lock-step group) bounds the solves in flight.  The load is a
closed loop that keeps ``capacity`` tasks outstanding: whenever a solution lands on chain a new
task is submitted, so the scheduler, the lock-step grouping and every per-task CPU stage are in
the timed region exactly as in production.  The loop keeps ``2 x capacity`` tasks outstanding by
default (``--node-outstanding``): a node measured for throughput is a SATURATED node, whose queue
holds the next lock-step group while the current one runs; with exactly ``capacity`` outstanding
every solution's replacement is still in hydration when a slot frees up and the slots run partial
groups (measured: 3.0 tasks per group of 4, 20.2k vs 25.0k tasks/h on SD1.5).  Latency is per
task, from ``submitTask`` (the event's block) to the accepted ``submitSolution``.
"""
from __future__ import annotations

import asyncio
import json
import math
import statistics
import time
from typing import Dict, List

E18 = 10 ** 18
POLL_S = 0.05          # event poll / top-up period of the bench loop
DEPLOYER, USER, MINER = ("0x" + f"{i:040x}" for i in (1, 2, 3))


def task_input(model: str, i: int, args) -> dict:
    """The raw JSON a user would submit for the benched template (``templates/<model>.json``)."""
    if model == "kandinsky2":
        return {"prompt": f"a red cat sitting on a castle wall, oil painting, task {i}", "width": args.res,
                "height": args.res}
    if model in ("zeroscopev2xl", "damo"):
        inp = {"prompt": f"a red cat walking on a castle wall, cinematic, task {i}",
               "num_frames": args.frames, "num_inference_steps": args.denoise_steps, "fps": 24}
        if model == "zeroscopev2xl":
            inp.update(negative_prompt="blurry", width=args.res, height=args.height, guidance_scale=17)
        return inp
    return {"prompt": f"a detailed anime illustration of a castle on a hill, task {i}",
            "negative_prompt": "lowres, bad anatomy, bad hands, text, error", "width": args.res, "height": args.res,
            "num_inference_steps": args.denoise_steps, "guidance_scale": int(args.guidance),
            "scheduler": args.scheduler}


class _Timed:
    """MockChainClient wrapper stamping when each task's solution is accepted on chain."""

    def __init__(self, inner, done: Dict[str, float]):
        self._inner, self._done = inner, done

    def __getattr__(self, k):
        return getattr(self._inner, k)

    async def submit_solution(self, taskid, cid):
        r = await self._inner.submit_solution(taskid, cid)
        self._done[taskid.lower()] = time.perf_counter()
        return r


async def _run(args, device: str) -> dict:
    from ..chain.client import MockChainClient
    from ..chain.mock_engine import MockEngine, MockToken
    from ..config.mining_config import MiningConfig
    from ..ipfs.pin import LocalPinner
    from ..store.db import DB
    from .miner import Miner
    from .models import default_models, template_bytes

    model = args.model
    tok = MockToken()
    e = MockEngine(tok, owner=DEPLOYER)
    tok.mint(DEPLOYER, 2000 * E18)
    tok.mint(e.address, 597000 * E18)
    tok.transfer(DEPLOYER, MINER, 10 * E18)
    tok.approve(USER, e.address, 2 ** 256 - 1)
    mid = e.register_model(USER, USER, 0, template_bytes(model))
    C, G = max(1, args.concurrent), max(1, args.group)
    ms, ml = None, None
    if getattr(args, "shipped_pool", False):
        # the pool exactly as `start` builds it from MiningConfig defaults (cli.py): workers_per_gpu slots,
        # each model capped by model_streams forks and grouped by model_lockstep
        x = MiningConfig.from_dict({}).mi355x
        C, G, ms, ml = x.workers_per_gpu, x.lockstep_group, dict(x.model_streams), dict(x.model_lockstep)
    cfg = MiningConfig.from_dict({"db_path": ":memory:", "mi355x": {
        "selftest": False, "workers_per_gpu": C, "lockstep_group": G, "poll_interval_ms": 2}})
    t_init = time.perf_counter()
    if args.gpus > 1 or getattr(args, "rccl_group", False):
        from ..parallel.workers import MultiGPUSolverPool
        pool = MultiGPUSolverPool(args.gpus, [model], "cuda" if device.startswith("cuda") else "cpu",
                                  tiny=args.tiny, streams_per_gpu=C, lockstep=G, weights_dir=args.weights_dir,
                                  force_group=getattr(args, "rccl_group", False), model_streams=ms,
                                  model_lockstep=ml)
    else:
        from .pool import LocalSolverPool
        pool = LocalSolverPool(device, capacity=C, lockstep=G, tiny=args.tiny, weights_dir=args.weights_dir,
                               model_streams=ms, model_lockstep=ml)
    done: Dict[str, float] = {}
    chain = _Timed(MockChainClient(e, MINER), done)
    miner = Miner(cfg, DB(":memory:"), chain, LocalPinner(), pool, default_models({model: mid}),
                  clock=lambda: e.timestamp)
    await miner.boot()
    await miner.poll_events()
    await miner.drain()                              # validatorStake -> deposit
    capacity = max(1, int(getattr(pool, "capacity", 1)))
    outstanding = max(capacity, int(getattr(args, "node_outstanding", 0) or 0) or 2 * capacity)
    submitted: Dict[str, float] = {}
    counter = [0]

    def submit_one():
        i = counter[0]
        counter[0] += 1
        tid = e.submit_task(USER, 0, USER, mid, 0, json.dumps(task_input(model, i, args)).encode())
        submitted[tid.lower()] = time.perf_counter()
        return tid.lower()

    async def run_tasks(n: int) -> List[str]:
        """Closed loop: ``outstanding`` tasks in flight until ``n`` solutions are accepted."""
        mine: List[str] = []
        while len(mine) < min(n, outstanding):
            mine.append(submit_one())
        # The node's own loop polls chain events on a timer (Miner.run); here every POLL_S.  The
        # bookkeeping (top-up, invalid-task check) runs at that rate too: the event loop shares the
        # GIL with the task streams' launch threads, and a 2 ms poll + a DB query per task per pass
        # starved them (the two streams ran mostly one after the other).
        last = -1.0
        while True:
            now = time.perf_counter()
            if now - last >= POLL_S:
                last = now
                finished = sum(1 for t in mine if t in done)
                if finished >= n:
                    return mine
                while len(mine) - finished < outstanding and len(mine) < n:
                    mine.append(submit_one())
                await miner.poll_events()
                if miner.metrics.counters.get("jobs_failed_solve"):
                    raise RuntimeError("a solve job failed during the node bench")
                bad = [t for t in mine if t not in done and miner.db.get_invalid_task(t)]
                if bad:
                    raise RuntimeError(f"the node judged bench task {bad[0]} invalid (input outside the template?)")
            if await miner.process_jobs() == 0:
                await asyncio.sleep(0.005)

    per_step = capacity                              # one bench step = one task per pool slot
    if args.warmup:
        await run_tasks(args.warmup * per_step)
    t_init = time.perf_counter() - t_init
    n_timed = args.steps * per_step
    t0 = time.perf_counter()
    timed = await run_tasks(n_timed)
    elapsed = time.perf_counter() - t0
    lat = sorted(done[t] - submitted[t] for t in timed)
    for t in timed:                                  # every accepted solution is this miner's
        assert e.solutions[t].validator == MINER.lower()
    await asyncio.gather(*list(miner._bg), return_exceptions=True)   # background pins
    pins_ok = miner.metrics.counters.get("pin_cid_mismatch", 0) == 0 and not miner.metrics.counters.get("pin_failures")
    await pool.close()
    return {"tasks": len(timed), "elapsed_s": elapsed, "capacity": capacity, "outstanding": outstanding,
            "p50_s": statistics.median(lat),
            "p90_s": lat[max(0, math.ceil(0.9 * len(lat)) - 1)], "init_s": t_init, "pins_ok": pins_ok,
            "jobs": {k: v for k, v in miner.metrics.counters.items() if k.startswith("jobs_")},
            "stage_p50_s": {k[len("stage_"):]: round(miner.metrics.p50(k), 4) for k in miner.metrics.latencies
                            if k.startswith("stage_")}}


def run_node_bench(args, device: str) -> dict:
    return asyncio.run(_run(args, device))
