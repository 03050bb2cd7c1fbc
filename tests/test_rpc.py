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
