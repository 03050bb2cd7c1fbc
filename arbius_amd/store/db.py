"""SQLite persistence with the reference miner's exact schema (``miner/src/sql/*.sql``,
``miner/src/db.ts``) so an existing ``db.sqlite`` keeps working.

Differences, all additive (the reference ignores unknown tables):
  * ``invalid_tasks`` IS created (reference defect Q1: ``db.ts:27-36`` never loads it);
  * WAL journal + one connection guarded by a lock (dispatcher, RPC server and
    GPU workers share it from threads);
  * ``job_leases``: a job taken by a worker is leased, not deleted, and is
    deleted only on completion - a crashed worker's job becomes runnable again
    after the lease expires (fixes Q4: concurrent jobs deleted before finishing);
  * ``block_cursor``: last processed block for event backfill (fixes Q8);
  * index ``jobs_method_wait`` on ``jobs(method, waituntil)``: a node at full rate holds ~2,000 s of
    future claim jobs (tens of thousands of rows); the scheduler asks per job class for the few
    runnable rows it can start, instead of scanning and sorting the whole table every pass.
"""
from __future__ import annotations

import json
import sqlite3
import threading
import time
from typing import Any, Dict, List, Optional

from ..utils.protocol import taskid2seed

SCHEMA = {
    "models": """
CREATE TABLE IF NOT EXISTS models (
    id TEXT PRIMARY KEY,
    addr TEXT,
    mineable BOOLEAN,
    cid TEXT
);""",
    "tasks": """
CREATE TABLE IF NOT EXISTS tasks (
    id TEXT PRIMARY KEY,
    modelid TEXT,
    fee TEXT,
    address TEXT,
    blocktime TEXT,
    version INT,
    cid TEXT,
    retracted BOOLEAN DEFAULT FALSE
);
CREATE INDEX IF NOT EXISTS tasks_id ON tasks(id);
CREATE INDEX IF NOT EXISTS tasks_modelid ON tasks(modelid);
CREATE INDEX IF NOT EXISTS tasks_address ON tasks(address);""",
    "task_inputs": """
CREATE TABLE IF NOT EXISTS task_inputs (
    taskid TEXT,
    cid TEXT,
    data TEXT
);
CREATE INDEX IF NOT EXISTS task_inputs_taskid ON task_inputs(taskid);
CREATE INDEX IF NOT EXISTS task_inputs_cid ON task_inputs(cid);""",
    "solutions": """
CREATE TABLE IF NOT EXISTS solutions (
    id INTEGER PRIMARY KEY AUTOINCREMENT,
    taskid TEXT,
    validator TEXT,
    blocktime TEXT,
    claimed BOOLEAN,
    cid TEXT
);
CREATE INDEX IF NOT EXISTS solutions_taskid ON solutions(taskid);
CREATE INDEX IF NOT EXISTS solutions_validator ON solutions(validator);""",
    "contestations": """
CREATE TABLE IF NOT EXISTS contestations (
    id INTEGER PRIMARY KEY AUTOINCREMENT,
    taskid TEXT,
    validator TEXT,
    blocktime TEXT,
    finish_start_index TEXT
);
CREATE INDEX IF NOT EXISTS contestations_taskid ON contestations(taskid);
CREATE INDEX IF NOT EXISTS contestations_validator ON contestations(validator);""",
    "contestation_votes": """
CREATE TABLE IF NOT EXISTS contestation_votes (
    id INTEGER PRIMARY KEY AUTOINCREMENT,
    taskid TEXT,
    validator TEXT,
    yea BOOLEAN
);
CREATE INDEX IF NOT EXISTS contestation_votes_taskid ON contestation_votes(taskid);
CREATE INDEX IF NOT EXISTS contestation_votes_validator ON contestation_votes(validator);""",
    "jobs": """
CREATE TABLE IF NOT EXISTS jobs (
    id INTEGER PRIMARY KEY AUTOINCREMENT,
    priority INTEGER,
    waituntil INTEGER,
    concurrent BOOLEAN,
    method TEXT,
    data TEXT
);""",
    "failed_jobs": """
CREATE TABLE IF NOT EXISTS failed_jobs (
    id INTEGER PRIMARY KEY AUTOINCREMENT,
    method TEXT,
    data TEXT
);""",
    "invalid_tasks": """
CREATE TABLE IF NOT EXISTS invalid_tasks (
    taskid TEXT PRIMARY KEY
);
CREATE INDEX IF NOT EXISTS invalid_tasks_taskid ON invalid_tasks(taskid);""",
    # ---- additive tables (unknown to the reference, ignored by it)
    "jobs_index": """
CREATE INDEX IF NOT EXISTS jobs_method_wait ON jobs(method, waituntil);""",
    "job_leases": """
CREATE TABLE IF NOT EXISTS job_leases (
    jobid INTEGER PRIMARY KEY,
    worker TEXT,
    expires REAL
);""",
    "block_cursor": """
CREATE TABLE IF NOT EXISTS block_cursor (
    name TEXT PRIMARY KEY,
    block INTEGER
);""",
}


class DB:
    def __init__(self, path: str = ":memory:"):
        self.path = path
        self.conn = sqlite3.connect(path, check_same_thread=False, isolation_level=None)
        self.conn.row_factory = sqlite3.Row
        self.lock = threading.RLock()
        if path != ":memory:":
            self.conn.execute("PRAGMA journal_mode=WAL")
            # WAL + NORMAL: a commit is durable against a process crash (what the lease / cursor
            # recovery needs) without an fsync per statement (~10 statements per task)
            self.conn.execute("PRAGMA synchronous=NORMAL")
        for sql in SCHEMA.values():
            self.conn.executescript(sql)

    # ------------------------------------------------------------------ helpers
    def _one(self, q, args=()) -> Optional[Dict[str, Any]]:
        with self.lock:
            r = self.conn.execute(q, args).fetchone()
        return dict(r) if r else None

    def _all(self, q, args=()) -> List[Dict[str, Any]]:
        with self.lock:
            return [dict(r) for r in self.conn.execute(q, args).fetchall()]

    def _run(self, q, args=()) -> int:
        with self.lock:
            cur = self.conn.execute(q, args)
            return cur.lastrowid

    def close(self):
        self.conn.close()

    # ------------------------------------------------------------------ getters (db.ts:55-144)
    def get_task(self, taskid):
        return self._one("SELECT * FROM tasks WHERE id=?", (taskid,))

    def get_solution(self, taskid):
        return self._one("SELECT * FROM solutions WHERE taskid=?", (taskid,))

    def get_contestation(self, taskid):
        return self._one("SELECT * FROM contestations WHERE taskid=?", (taskid,))

    def get_invalid_task(self, taskid):
        return self._one("SELECT * FROM invalid_tasks WHERE taskid=?", (taskid,))

    def get_contestation_votes(self, taskid):
        return self._all("SELECT * FROM contestation_votes WHERE taskid=?", (taskid,))

    def get_task_input(self, taskid, cid):
        """Re-applies the seed on every read (db.ts:97-117)."""
        row = self._one("SELECT * FROM task_inputs WHERE taskid=? AND cid=?", (taskid, cid))
        if row is None:
            return None
        data = json.loads(row["data"])
        data["seed"] = taskid2seed(taskid)
        row["data"] = json.dumps(data, separators=(",", ":"))
        return row

    def get_job(self, jobid):
        return self._one("SELECT * FROM jobs WHERE id=?", (jobid,))

    def get_jobs(self, limit: int = 10000):
        return self._all("SELECT * FROM jobs ORDER BY priority DESC LIMIT ?", (limit,))

    def get_failed_jobs(self):
        return self._all("SELECT * FROM failed_jobs")

    # ------------------------------------------------------------------ stores (db.ts:146-376)
    def store_task(self, taskid, modelid, fee, owner, blocktime, version, cid):
        self._run("INSERT OR IGNORE INTO tasks (id, modelid, fee, address, blocktime, version, cid) "
                  "VALUES (?, ?, ?, ?, ?, ?, ?)", (taskid, modelid, str(fee), owner, str(blocktime), version, cid))
        return {"id": taskid, "modelid": modelid, "fee": str(fee), "address": owner,
                "blocktime": str(blocktime), "version": version, "cid": cid, "retracted": False}

    def store_invalid_task(self, taskid):
        self._run("INSERT OR IGNORE INTO invalid_tasks (taskid) VALUES (?)", (taskid,))
        return {"taskid": taskid}

    def store_failed_job(self, job):
        self._run("INSERT INTO failed_jobs (method, data) VALUES (?, ?)", (job["method"], job["data"]))
        return True

    def update_task_set_retracted(self, taskid):
        self._run("UPDATE tasks SET retracted=true WHERE id = ?", (taskid,))
        return True

    def queue_job(self, method, priority, waituntil, concurrent, data) -> int:
        return self._run("INSERT INTO jobs (priority, waituntil, concurrent, method, data) VALUES (?, ?, ?, ?, ?)",
                         (int(priority), int(waituntil), bool(concurrent), method,
                          json.dumps(data, separators=(",", ":"))))

    def delete_job(self, jobid):
        with self.lock:
            self.conn.execute("DELETE FROM jobs WHERE id=?", (jobid,))
            self.conn.execute("DELETE FROM job_leases WHERE jobid=?", (jobid,))

    def clear_jobs_by_method(self, method):
        with self.lock:
            ids = [r["id"] for r in self._all("SELECT id FROM jobs WHERE method=?", (method,))]
            for i in ids:
                self.delete_job(i)

    def store_task_input(self, taskid, cid, data):
        self._run("INSERT INTO task_inputs (taskid, cid, data) VALUES (?, ?, ?)",
                  (taskid, cid, json.dumps(data, separators=(",", ":"))))
        return True

    def store_solution(self, taskid, validator, blocktime, claimed, cid):
        self._run("INSERT INTO solutions (taskid, validator, blocktime, claimed, cid) VALUES (?, ?, ?, ?, ?)",
                  (taskid, validator, str(blocktime), bool(claimed), cid))
        return True

    def store_contestation(self, taskid, validator, blocktime, finish_start_index):
        self._run("INSERT INTO contestations (taskid, validator, blocktime, finish_start_index) VALUES (?, ?, ?, ?)",
                  (taskid, validator, str(blocktime), str(finish_start_index)))
        return True

    def store_contestation_vote(self, taskid, validator, yea):
        self._run("INSERT INTO contestation_votes (taskid, validator, yea) VALUES (?, ?, ?)",
                  (taskid, validator, bool(yea)))
        return True

    # ------------------------------------------------------------------ leases (additive)
    def runnable_jobs(self, now: int, limit: int = 10000):
        """Jobs whose waituntil has passed and that are not under a live lease, priority order."""
        return self._all(
            "SELECT j.* FROM jobs j LEFT JOIN job_leases l ON l.jobid = j.id "
            "WHERE j.waituntil <= ? AND (l.jobid IS NULL OR l.expires < ?) "
            "ORDER BY j.priority DESC, j.id ASC LIMIT ?", (int(now), time.time(), limit))

    def runnable_jobs_of(self, now: int, methods, limit: int):
        """Up to ``limit`` runnable jobs of the given methods (priority order, then FIFO)."""
        if limit <= 0:
            return []
        methods = list(methods)
        marks = ",".join("?" * len(methods))
        return self._all(
            f"SELECT j.* FROM jobs j LEFT JOIN job_leases l ON l.jobid = j.id "
            f"WHERE j.method IN ({marks}) AND j.waituntil <= ? AND (l.jobid IS NULL OR l.expires < ?) "
            f"ORDER BY j.priority DESC, j.id ASC LIMIT ?", (*methods, int(now), time.time(), int(limit)))

    def job_methods(self):
        return [r["method"] for r in self._all("SELECT DISTINCT method FROM jobs")]

    def lease_job(self, jobid, worker: str, seconds: float) -> bool:
        with self.lock:
            row = self.conn.execute("SELECT expires FROM job_leases WHERE jobid=?", (jobid,)).fetchone()
            if row is not None and row[0] >= time.time():
                return False
            self.conn.execute("INSERT OR REPLACE INTO job_leases (jobid, worker, expires) VALUES (?, ?, ?)",
                              (jobid, worker, time.time() + seconds))
            return True

    def renew_lease(self, jobid, seconds: float):
        self._run("UPDATE job_leases SET expires=? WHERE jobid=?", (time.time() + seconds, jobid))

    def release_lease(self, jobid):
        self._run("DELETE FROM job_leases WHERE jobid=?", (jobid,))

    # ------------------------------------------------------------------ block cursor (additive)
    def get_cursor(self, name="events") -> Optional[int]:
        r = self._one("SELECT block FROM block_cursor WHERE name=?", (name,))
        return None if r is None else int(r["block"])

    def set_cursor(self, block: int, name="events"):
        self._run("INSERT OR REPLACE INTO block_cursor (name, block) VALUES (?, ?)", (name, int(block)))

    # ------------------------------------------------------------------ raw (rpc /api/db/*)
    def execute(self, sql: str, args=()):
        return self._all(sql, args)
