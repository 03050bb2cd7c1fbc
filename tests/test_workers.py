"""One-process-per-device worker pool on CPU (gloo, world size 2): weight
broadcast from rank 0, concurrent solves, cross-worker determinism, and
elastic recovery after a worker is killed."""
import asyncio

import pytest

from arbius_amd.node.models import Model, load_template
from arbius_amd.node.pool import LocalSolverPool
from arbius_amd.parallel.workers import MultiGPUSolverPool

MODEL = Model("0x" + "ab" * 32, "anythingv3", load_template("anythingv3"), True, [], "image")
INP = {"prompt": "a cat", "negative_prompt": "n", "width": 128, "height": 128, "num_inference_steps": 2,
       "guidance_scale": 7.5, "scheduler": "DDIM", "seed": 1234}


@pytest.mark.timeout(600)
def test_two_workers_broadcast_determinism_and_failover():
    ref = LocalSolverPool("cpu", tiny=True).solve_sync(MODEL, "t", INP)

    async def go():
        pool = MultiGPUSolverPool(2, ["anythingv3"], device_type="cpu", tiny=True)
        try:
            assert pool.capacity == 2
            # rank 1 received its weights by broadcast (not initialised itself)
            assert pool.broadcast_stats[1]["bytes"] > 0
            a, b = await asyncio.gather(pool.solve(MODEL, "t1", INP), pool.solve(MODEL, "t2", INP))
            assert a.cid == b.cid == ref.cid  # same bytes on every worker
            pool.kill_worker(0)
            pool.kill_worker(1)
            # both respawn standalone (deterministic init) and produce the same CID
            c = await asyncio.wait_for(pool.solve(MODEL, "t3", INP), 300)
            assert c.cid == ref.cid
            assert pool.restarts >= 2
            # a worker killed while it holds a task: that task fails (caller retries elsewhere)
            slow = dict(INP, num_inference_steps=200)
            task = asyncio.ensure_future(pool.solve(MODEL, "t4", slow))
            while not pool.busy:
                await asyncio.sleep(0.005)
            pool.kill_worker(next(iter(pool.busy.values())))
            with pytest.raises(RuntimeError):
                await asyncio.wait_for(task, 300)
            d = await asyncio.wait_for(pool.solve(MODEL, "t5", INP), 300)
            assert d.cid == ref.cid
        finally:
            await pool.close()

    asyncio.run(go())


@pytest.mark.timeout(600)
def test_two_task_streams_per_worker():
    """streams_per_gpu=2: one worker process serves two tasks at once on pipeline forks,
    with the same CIDs as a solo solve."""
    ref = [LocalSolverPool("cpu", tiny=True).solve_sync(MODEL, "t", dict(INP, seed=s)).cid for s in (1, 2)]

    async def go():
        pool = MultiGPUSolverPool(1, ["anythingv3"], device_type="cpu", tiny=True, streams_per_gpu=2)
        try:
            assert pool.capacity == 2
            a, b = await asyncio.gather(pool.solve(MODEL, "a", dict(INP, seed=1)),
                                        pool.solve(MODEL, "b", dict(INP, seed=2)))
            assert [a.cid, b.cid] == ref
        finally:
            await pool.close()

    asyncio.run(go())


@pytest.mark.timeout(300)
def test_pool_start_fails_fast_when_a_rank_dies_in_the_broadcast(monkeypatch):
    """A worker lost in the middle of the weight broadcast: the pool kills its peers (blocked in the
    collective) and raises within seconds, instead of hanging until the process-group timeout."""
    import time
    monkeypatch.setenv("ARBIUS_FAULT_INJECTION", "1")
    monkeypatch.setenv("ARBIUS_FAULT_BCAST_DIE_RANK", "1")
    monkeypatch.setenv("ARBIUS_DIST_TIMEOUT_S", "600")
    t0 = time.time()
    with pytest.raises(RuntimeError, match="died during start"):
        MultiGPUSolverPool(2, ["anythingv3"], device_type="cpu", tiny=True)
    assert time.time() - t0 < 120


@pytest.mark.timeout(300)
def test_pool_reports_the_formed_world_and_closes():
    async def go():
        pool = MultiGPUSolverPool(2, ["anythingv3"], device_type="cpu", tiny=True)
        try:
            assert pool.world["backend"] == "gloo" and pool.world["world_size"] == 2
            assert len(pool.world["ranks"]) == 2
        finally:
            await pool.close()
        assert not any(p.is_alive() for p in pool.procs)

    asyncio.run(go())


@pytest.mark.timeout(600)
def test_worker_two_phase_solve_matches_solo():
    """RVM's two-phase solve in a worker slot (matting on the slot, MP4 encode + CID on the slot's
    tail thread while the slot takes the next clip): the CIDs of solo pipeline solves."""
    import base64

    import numpy as np

    from arbius_amd.utils.mp4 import encode_mp4
    rvm = Model("0x" + "cd" * 32, "robust_video_matting", load_template("robust_video_matting"), True, [], "video")
    inps = []
    for s in (4, 5, 6):
        frames = np.random.default_rng(s).integers(0, 256, (2, 48, 64, 3), dtype=np.uint8)
        src = "data:video/mp4;base64," + base64.b64encode(encode_mp4(list(frames), 5)).decode()
        inps.append({"input_video": src, "output_type": "green-screen"})
    local = LocalSolverPool("cpu", tiny=True)
    ref = [local.solve_sync(rvm, f"r{i}", inp).cid for i, inp in enumerate(inps)]

    async def go():
        pool = MultiGPUSolverPool(1, ["robust_video_matting"], device_type="cpu", tiny=True, streams_per_gpu=2)
        try:
            sols = await asyncio.gather(*[pool.solve(rvm, f"t{i}", inp) for i, inp in enumerate(inps)])
            assert [s.cid for s in sols] == ref
            assert all("encode_cid_s" in s.timings for s in sols)
        finally:
            await pool.close()

    asyncio.run(go())


def test_capped_model_gets_cap_forks_and_never_exceeds_its_cap():
    """with 4 slots and a model capped at 2 streams the worker builds 2 forks of that model
    (not 4: each fork owns hipGraphs and their memory pools) and never solves more than 2 at once."""
    ref = [LocalSolverPool("cpu", tiny=True).solve_sync(MODEL, "t", dict(INP, seed=s)).cid for s in range(1, 7)]

    async def go():
        pool = MultiGPUSolverPool(1, ["anythingv3"], device_type="cpu", tiny=True, streams_per_gpu=4,
                                  model_streams={"anythingv3": 2})
        try:
            assert pool.broadcast_stats[0]["forks"] == {"anythingv3": 2}
            sols = await asyncio.gather(*[pool.solve(MODEL, f"t{s}", dict(INP, seed=s)) for s in range(1, 7)])
            assert [x.cid for x in sols] == ref
            assert max(x.timings["fork_peak"] for x in sols) <= 2
        finally:
            await pool.close()

    asyncio.run(go())


def test_watchdog_times_cpu_tails_too():
    """a slot's CPU tail (RVM encode + CID, a group's PNGs) runs after the slot's progress
    beat went idle; the tail's own clock (second half of the beats array) is watched as well."""
    pool = MultiGPUSolverPool.__new__(MultiGPUSolverPool)
    pool.n, pool.streams, pool.hang_timeout = 2, 2, 10.0
    pool.beats = [0.0] * (2 * pool.n * pool.streams)
    assert pool.hung_ranks(now=1000.0) == []
    pool.beats[(pool.n + 1) * pool.streams + 1] = 985.0      # rank 1, slot 1: tail started 15 s ago
    assert pool.hung_ranks(now=1000.0) == [1]
    pool.beats[(pool.n + 1) * pool.streams + 1] = 995.0
    assert pool.hung_ranks(now=1000.0) == []
    pool.beats[0 * pool.streams + 0] = 980.0                 # rank 0, slot 0: solve silent for 20 s
    assert pool.hung_ranks(now=1000.0) == [0]


def test_dispatch_policies_and_model():
    """pick_rank: spread = least-loaded GPU, pack = most-loaded GPU with a free slot; the dispatch model
    (parallel/dispatch.py) reproduces the measured single-GPU points it was fitted to, and below
    saturation spread answers faster than pack at the same completed throughput."""
    from arbius_amd.parallel.dispatch import (SERVICE_MODELS, SHIPPED, fit_points, node_capacity_per_s, pick_rank,
                                              simulate)
    load = {0: 3, 1: 0, 2: 5, 3: 1}
    assert pick_rank("spread", [0, 1, 2, 3], load) == 1
    assert pick_rank("pack", [0, 1, 2, 3], load) == 2
    with pytest.raises(ValueError):
        pick_rank("random", [0], load)
    from arbius_amd.config.mining_config import DEFAULT_MODEL_LOCKSTEP, DEFAULT_MODEL_STREAMS, MI355XConfig
    for model, (st, grp) in SHIPPED.items():      # the fits describe the configurations that ship
        assert st == DEFAULT_MODEL_STREAMS[model]
        assert grp == DEFAULT_MODEL_LOCKSTEP.get(model, MI355XConfig().lockstep_group)
        for n, k, ms, mod in fit_points(model):
            assert abs(mod - ms) / ms < 0.03, (model, n, k, ms, mod)
    for model, (st, grp) in SHIPPED.items():
        sm = SERVICE_MODELS[model]
        cap = node_capacity_per_s(streams=st, group=grp, model=sm)
        sp = simulate("spread", 0.5 * cap, streams=st, group=grp, model=sm, n_tasks=1500)
        pk = simulate("pack", 0.5 * cap, streams=st, group=grp, model=sm, n_tasks=1500)
        assert sp["p50_ms"] * 2 < pk["p50_ms"], (model, sp, pk)
        assert sp["completed_per_h"] >= 0.97 * pk["completed_per_h"]
    with pytest.raises(ValueError):
        MultiGPUSolverPool(1, ["anythingv3"], device_type="cpu", tiny=True, dispatch="random")


def test_cpu_budget_caps(monkeypatch):
    """Host-CPU admission (parallel/cpu_budget.py): with the GPU H.264 encoder RVM needs ~2.2 cores per
    GPU and fits every GPU of a 64-core host; host-encoded (ARB_RVM_GPU_H264=0) its 13.4 cores fit 4;
    the diffusion models fit all 8; no cap when everything fits."""
    from arbius_amd.parallel.cpu_budget import model_gpu_caps
    assert model_gpu_caps(["anythingv3", "kandinsky2", "robust_video_matting"], 8, cores=64) == {}
    assert model_gpu_caps(["robust_video_matting", "anythingv3"], 8, cores=16) == {"robust_video_matting": 6,
                                                                                  "anythingv3": 2}
    monkeypatch.setenv("ARB_RVM_GPU_H264", "0")
    caps = model_gpu_caps(["anythingv3", "kandinsky2", "robust_video_matting"], 8, cores=64)
    assert caps == {"robust_video_matting": 4}
    assert model_gpu_caps(["robust_video_matting"], 8, cores=128) == {}
    assert model_gpu_caps(["robust_video_matting", "anythingv3"], 8, cores=16) == {"robust_video_matting": 1,
                                                                                  "anythingv3": 2}


@pytest.mark.timeout(900)
def test_eight_workers_two_killed_under_load_keep_cids():
    """8 gloo ranks (weights broadcast from rank 0), solves in flight on 6, two workers
    hard-killed at once mid-load; their tasks fail over (the miner's retry re-dispatches them), both
    respawn, and every CID - before, during and after - equals the solo CID (16 solves in flight).  A
    host-CPU cap keeps the model's tasks on ranks 0..5."""
    seeds = list(range(16))
    ref = {s: LocalSolverPool("cpu", tiny=True).solve_sync(MODEL, "t", dict(INP, seed=s)).cid for s in seeds[:6]}

    async def solve_retry(pool, s):
        for _ in range(5):
            try:
                return s, await pool.solve(MODEL, f"t{s}", dict(INP, seed=s % 6))
            except RuntimeError:
                await asyncio.sleep(0.1)
        raise AssertionError("task never completed")

    async def go():
        pool = MultiGPUSolverPool(8, ["anythingv3"], device_type="cpu", tiny=True,
                                  model_gpu_cap={"anythingv3": 6})
        try:
            assert pool.world["world_size"] == 8 and all(pool.broadcast_stats[r]["bytes"] > 0 for r in range(8))
            ranks_seen = set()
            orig = pool.in_qs

            tasks = [asyncio.ensure_future(solve_retry(pool, s)) for s in seeds]
            while len(pool.busy) < 6:
                await asyncio.sleep(0.01)
            ranks_seen |= set(pool.busy.values())
            victims = sorted(ranks_seen)[:2]
            for r in victims:                        # two at once, both holding tasks
                p = pool.procs[r]
                p.kill()
            for r in victims:
                pool.procs[r].join(30)
            done = await asyncio.wait_for(asyncio.gather(*tasks), 600)
            for s, sol in done:
                assert sol.cid == ref[s % 6], s
            assert pool.restarts >= 2
            assert orig is pool.in_qs
            assert max(ranks_seen) < 6
            again = await asyncio.wait_for(asyncio.gather(*[solve_retry(pool, s) for s in seeds[:6]]), 300)
            assert all(sol.cid == ref[s % 6] for s, sol in again)
        finally:
            await pool.close()

    asyncio.run(go())
