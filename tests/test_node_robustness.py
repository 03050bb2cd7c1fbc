"""Failure detection / control-plane robustness on CPU:
windowed event back-fill, ambiguous-input handling, lease heartbeats, GPU-worker hang
detection, and weights_dir plumbing through the one-process-per-device pool."""
import asyncio

import pytest

from arbius_amd.node.models import Model, hydration_modes_agree, load_template
from arbius_amd.node.pool import FakeSolverPool, LocalSolverPool
from arbius_amd.parallel.workers import MultiGPUSolverPool

from test_node_e2e import MINER, make_miner, make_world, submit

SD = Model("0x" + "ab" * 32, "anythingv3", load_template("anythingv3"), True, [], "image")
INP = {"prompt": "a cat", "negative_prompt": "n", "width": 128, "height": 128, "num_inference_steps": 2,
       "guidance_scale": 7, "scheduler": "DDIM", "seed": 1234}


class _WindowLimitedChain:
    """Wraps a MockChainClient; eth_getLogs over more than ``limit`` blocks fails like a provider."""

    def __init__(self, inner, limit):
        self._inner, self.limit, self.calls = inner, limit, []

    def __getattr__(self, k):
        return getattr(self._inner, k)

    async def get_events(self, a, b):
        self.calls.append((a, b))
        if b - a + 1 > self.limit:
            raise RuntimeError("query returned more than 10000 results / block range too large")
        return await self._inner.get_events(a, b)


def test_event_backfill_in_bounded_windows():
    e, tok, mid = make_world()
    m = make_miner(e, mid, FakeSolverPool(), mi355x={"selftest": False, "log_window_blocks": 64})
    m.chain = _WindowLimitedChain(m.chain, limit=20)

    async def go():
        await m.boot()
        await m.poll_events()                  # pins the cursor
        await m.drain()
        e.mine(150)                            # a long outage: many blocks, one task in the middle
        tid = submit(e, mid, {"prompt": "late cat", "negative_prompt": "x"})
        e.mine(150)
        await m.poll_events()
        head = e.block_number
        assert m.db.get_cursor() == head        # every window persisted, up to the head
        await m.drain()
        return tid

    tid = asyncio.run(go())
    assert m.log_window <= 20                  # halved until the provider accepted it
    assert all(b - a + 1 <= 64 for a, b in m.chain.calls)
    assert tid in e.solutions and e.solutions[tid].validator == MINER.lower()


def test_ambiguous_hydration_is_neither_solved_nor_invalid():
    tpl = load_template("anythingv3")
    assert not hydration_modes_agree({"prompt": "p", "negative_prompt": "n", "guidance_scale": 7.5}, tpl)
    assert not hydration_modes_agree({"prompt": "p", "negative_prompt": "n", "num_inference_steps": 501}, tpl)
    assert hydration_modes_agree({"prompt": "p", "negative_prompt": "n", "guidance_scale": 7}, tpl)
    e, tok, mid = make_world()
    pool = FakeSolverPool()
    m = make_miner(e, mid, pool)

    async def go():
        await m.boot()
        await m.poll_events()
        await m.drain()
        tid = submit(e, mid, {"prompt": "p", "negative_prompt": "n", "guidance_scale": 7.5})
        await m.poll_events()
        await m.drain()
        return tid

    tid = asyncio.run(go())
    assert pool.calls == [] and m.db.get_invalid_task(tid) is None
    assert m.metrics.counters.get("tasks_ambiguous_input") == 1


def test_long_solve_renews_its_lease_and_runs_once():
    e, tok, mid = make_world()
    pool = FakeSolverPool(delay=1.0)            # solve outlives the 0.3 s lease 3x over
    m = make_miner(e, mid, pool, mi355x={"selftest": False, "job_lease_seconds": 0.3})

    async def go():
        await m.boot()
        await m.poll_events()
        await m.drain()
        submit(e, mid, {"prompt": "slow cat", "negative_prompt": "x"})
        await m.poll_events()
        for _ in range(60):                     # scheduler passes while the solve is in flight
            await m.process_jobs()
            await asyncio.sleep(0.05)
        await m.drain()

    asyncio.run(go())
    assert len(pool.calls) == 1


@pytest.mark.timeout(600)
def test_hung_worker_is_killed_and_failed_over(monkeypatch):
    monkeypatch.setenv("ARBIUS_FAULT_INJECTION", "1")       # inherited by the spawned workers

    async def go():
        # 45 s: a CPU-contended tiny solve (pytest -n) must not look like a hang
        pool = MultiGPUSolverPool(1, ["anythingv3"], device_type="cpu", tiny=True, hang_timeout=45.0)
        try:
            ok = await asyncio.wait_for(pool.solve(SD, "t0", INP), 300)
            with pytest.raises(RuntimeError):
                await asyncio.wait_for(pool.solve(SD, "t1", dict(INP, __fault__="hang")), 120)
            assert pool.hangs == 1 and pool.restarts == 1
            again = await asyncio.wait_for(pool.solve(SD, "t2", INP), 300)   # respawned worker
            assert again.cid == ok.cid
        finally:
            await pool.close()

    asyncio.run(go())


@pytest.mark.timeout(900)
def test_pool_loads_weights_dir_on_every_worker(tmp_path):
    """weights_dir reaches every worker: rank 0 reads the safetensors and broadcasts them, a
    respawned worker reads the same files; CIDs equal the single-process pool's and differ from
    the random-init ones."""
    from arbius_amd.models.registry import build_pipeline
    from arbius_amd.models.weights import save_native
    wd = str(tmp_path / "sd-tiny-weights")
    save_native(build_pipeline("anythingv3", tiny=True, weight_seed=77), wd)
    want = LocalSolverPool("cpu", tiny=True, weights_dir=wd).solve_sync(SD, "t", INP).cid
    rand = LocalSolverPool("cpu", tiny=True).solve_sync(SD, "t", INP).cid
    assert want != rand

    async def go():
        pool = MultiGPUSolverPool(2, ["anythingv3"], device_type="cpu", tiny=True, weights_dir=wd)
        try:
            assert pool.weights_id() == "safetensors:sd-tiny-weights-tiny"
            assert pool.broadcast_stats[1]["bytes"] > 0
            a, b = await asyncio.gather(pool.solve(SD, "a", INP), pool.solve(SD, "b", INP))
            assert a.cid == b.cid == want
            pool.kill_worker(1)
            pool.kill_worker(0)
            c = await asyncio.wait_for(pool.solve(SD, "c", INP), 300)
            assert c.cid == want                     # respawn re-read the same safetensors
        finally:
            await pool.close()

    asyncio.run(go())
