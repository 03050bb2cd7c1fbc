"""Control RPC server (``miner/src/rpc.ts:11-95``), same routes and JSON shapes:

  GET  /                  -> "Arbius Miner RPC"
  POST /api/jobs/queue    {method, priority, waituntil, concurrent, data} (type-checked)
  POST /api/jobs/get      {limit?} -> {status, jobs}
  POST /api/jobs/list     alias of /get (the docs' name, docs/src/pages/mining.mdx:238)
  POST /api/jobs/delete   {id}
  POST /api/db/run        unvalidated alias of queue (rpc.ts:81-95)

plus ``GET /metrics`` (Prometheus text) and ``GET /health``.
"""
from __future__ import annotations

import json
import logging

from aiohttp import web

log = logging.getLogger("arbius.rpc")

_FIELDS = [("method", str), ("priority", (int, float)), ("waituntil", (int, float)), ("concurrent", bool),
           ("data", dict)]
_JS_TYPES = {str: "string", bool: "boolean", dict: "object"}


def _js_type(v) -> str:
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, (int, float)):
        return "number"
    if isinstance(v, str):
        return "string"
    if v is None:
        return "object"
    if isinstance(v, (dict, list)):
        return "object"
    return "undefined"


def make_app(db, miner=None) -> web.Application:
    app = web.Application()

    async def root(_req):
        return web.Response(text="Arbius Miner RPC")

    async def _body(req):
        try:
            return await req.json()
        except Exception:  # noqa: BLE001
            return {}

    async def queue(req):
        body = await _body(req)
        try:
            for field, typ in _FIELDS:
                if field not in body:
                    raise ValueError(f"missing required field ({field})")
                v = body[field]
                expected = "number" if typ == (int, float) else _JS_TYPES[typ]
                if _js_type(v) != expected or (typ is dict and not isinstance(v, dict)):
                    raise ValueError(f"expected ({field}) to be type ({expected}), got ({_js_type(v)})")
            db.queue_job(body["method"], body["priority"], body["waituntil"], body["concurrent"], body["data"])
            return web.json_response({"status": "ok"})
        except Exception as e:  # noqa: BLE001
            return web.json_response({"status": "fail", "e": f"Error: {e}"})

    async def get_jobs(req):
        body = await _body(req)
        try:
            limit = 100_000
            if "limit" in body:
                try:
                    limit = int(body["limit"])
                except (TypeError, ValueError):
                    raise ValueError("limit NaN")
            jobs = db.get_jobs(limit)
            for j in jobs:
                j["concurrent"] = bool(j["concurrent"])
            return web.json_response({"status": "ok", "jobs": jobs})
        except Exception as e:  # noqa: BLE001
            return web.json_response({"status": "fail", "e": f"Error: {e}"})

    async def delete_job(req):
        body = await _body(req)
        try:
            try:
                jid = int(body.get("id"))
            except (TypeError, ValueError):
                raise ValueError("id NaN")
            db.delete_job(jid)
            return web.json_response({"status": "ok"})
        except Exception as e:  # noqa: BLE001
            return web.json_response({"status": "fail", "e": f"Error: {e}"})

    async def db_run(req):
        body = await _body(req)
        try:
            db.queue_job(body.get("method"), body.get("priority"), body.get("waituntil"), body.get("concurrent"),
                         body.get("data"))
            return web.json_response({"status": "ok"})
        except Exception as e:  # noqa: BLE001
            return web.json_response({"status": "fail", "e": json.dumps(str(e))})

    async def metrics(_req):
        lines = []
        if miner is not None:
            for k, v in sorted(miner.metrics.counters.items()):
                lines.append(f"# TYPE arbius_{k} counter")
                lines.append(f"arbius_{k} {v}")
            for k in sorted(miner.metrics.latencies):
                vals = sorted(miner.metrics.latencies[k])
                if vals:
                    lines.append(f"arbius_{k}_p50 {vals[len(vals) // 2]:.6f}")
                    lines.append(f"arbius_{k}_p99 {vals[min(len(vals) - 1, int(len(vals) * 0.99))]:.6f}")
                    lines.append(f"arbius_{k}_count {len(vals)}")
            lines.extend(miner.metrics.prometheus_histograms())
        lines.append(f"arbius_jobs_queued {len(db.get_jobs())}")
        if miner is not None:
            pool = getattr(miner, "pool", None)
            lines.append(f"arbius_gpu_workers {int(getattr(pool, 'capacity', 0) or 0)}")
            lines.append(f"arbius_gpu_workers_busy {len(getattr(pool, 'busy', {}) or {})}")
            lines.append(f"arbius_gpu_worker_restarts {int(getattr(pool, 'restarts', 0) or 0)}")
            per_gpu = getattr(pool, "gpu_stats", None)
            if callable(per_gpu):
                stats = per_gpu()
                lines.append("# TYPE arbius_gpu_task_seconds_total counter")     # summed solve durations
                lines += [f'arbius_gpu_task_seconds_total{{gpu="{g}"}} {v["task_s"]:.3f}' for g, v in stats.items()]
                lines.append("# TYPE arbius_gpu_tasks_total counter")
                lines += [f'arbius_gpu_tasks_total{{gpu="{g}"}} {v["tasks"]}' for g, v in stats.items()]
        from ..utils.gpu_metrics import gpu_gauges
        lines.extend(gpu_gauges())
        return web.Response(text="\n".join(lines) + "\n", content_type="text/plain")

    async def health(_req):
        return web.json_response({"status": "ok", "jobs": len(db.get_jobs())})

    app.router.add_get("/", root)
    app.router.add_post("/api/jobs/queue", queue)
    app.router.add_post("/api/jobs/get", get_jobs)
    app.router.add_post("/api/jobs/list", get_jobs)
    app.router.add_post("/api/jobs/delete", delete_job)
    app.router.add_post("/api/db/run", db_run)
    app.router.add_get("/metrics", metrics)
    app.router.add_get("/health", health)
    return app


async def start_rpc(db, host: str, port: int, miner=None) -> web.AppRunner:
    runner = web.AppRunner(make_app(db, miner))
    await runner.setup()
    site = web.TCPSite(runner, host, port)
    await site.start()
    log.debug("RPC server listening on %s:%s", host, port)
    return runner
