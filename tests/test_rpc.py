"""Control RPC routes and JSON shapes (miner/src/rpc.ts:11-95)."""
import asyncio

from aiohttp.test_utils import TestClient, TestServer

from arbius_amd.node.rpc import make_app
from arbius_amd.store.db import DB


def _run(coro):
    return asyncio.run(coro)


def test_rpc_routes():
    async def go():
        db = DB(":memory:")
        client = TestClient(TestServer(make_app(db)))
        await client.start_server()
        try:
            r = await client.get("/")
            assert await r.text() == "Arbius Miner RPC"
            ok = {"method": "claim", "priority": 50, "waituntil": 0, "concurrent": False, "data": {"taskid": "0x1"}}
            r = await client.post("/api/jobs/queue", json=ok)
            assert (await r.json()) == {"status": "ok"}
            r = await client.post("/api/jobs/queue", json={**ok, "priority": "50"})
            j = await r.json()
            assert j["status"] == "fail" and "expected (priority) to be type (number), got (string)" in j["e"]
            r = await client.post("/api/jobs/queue", json={"method": "x"})
            assert "missing required field (priority)" in (await r.json())["e"]
            r = await client.post("/api/jobs/get", json={})
            jobs = (await r.json())["jobs"]
            assert len(jobs) == 1 and jobs[0]["method"] == "claim" and jobs[0]["concurrent"] is False
            r = await client.post("/api/jobs/list", json={"limit": 0})
            assert (await r.json())["jobs"] == []
            r = await client.post("/api/jobs/get", json={"limit": "abc"})
            assert (await r.json())["status"] == "fail"
            r = await client.post("/api/jobs/delete", json={"id": jobs[0]["id"]})
            assert (await r.json()) == {"status": "ok"}
            assert db.get_jobs() == []
            r = await client.post("/api/db/run", json=ok)
            assert (await r.json())["status"] == "ok"
            r = await client.get("/metrics")
            assert "arbius_jobs_queued 1" in await r.text()
        finally:
            await client.close()

    _run(go())


def test_metrics_histograms_and_per_gpu_counters():
    """/metrics: cumulative Prometheus latency histograms and per-GPU solved-task counters."""
    from arbius_amd.node.miner import Metrics

    class _Pool:
        capacity, busy, restarts = 2, {}, 0

        def gpu_stats(self):
            return {0: {"task_s": 3.5, "tasks": 2}, 1: {"task_s": 1.25, "tasks": 1}}

    class _Miner:
        metrics = Metrics()
        pool = _Pool()

    for s in (0.3, 0.7, 12.0):
        _Miner.metrics.observe("solve", s)

    async def go():
        client = TestClient(TestServer(make_app(DB(":memory:"), _Miner())))
        await client.start_server()
        try:
            text = await (await client.get("/metrics")).text()
        finally:
            await client.close()
        return text

    text = _run(go())
    assert "# TYPE arbius_solve_seconds histogram" in text
    assert 'arbius_solve_seconds_bucket{le="0.5"} 1' in text
    assert 'arbius_solve_seconds_bucket{le="1"} 2' in text
    assert 'arbius_solve_seconds_bucket{le="+Inf"} 3' in text
    assert "arbius_solve_seconds_count 3" in text and "arbius_solve_seconds_sum 13.000000" in text
    assert 'arbius_gpu_tasks_total{gpu="1"} 1' in text and 'arbius_gpu_task_seconds_total{gpu="0"} 3.500' in text
