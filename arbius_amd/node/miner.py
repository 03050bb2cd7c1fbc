"""The mining node orchestrator (the role of ``miner/src/index.ts``), asyncio-native.

Chain events -> SQLite job queue -> job processors, with the reference's job
methods, priorities and delays (index.ts:506-1101):

  task (p10, concurrent) -> solve (p20) -> [commit, submit] -> claim (p50, +2120 s)
  pinTaskInput (p10, concurrent), validatorStake (p30 boot / p100 every 600 s),
  automine (p5, +delay), contestationVoteFinish (p30, +5010 s)

MI355X-first differences (all behaviour-compatible on chain):
  * ``solve`` jobs run on a pool of GPU task workers - up to one solve per GPU in
    flight (the reference serialises solves, index.ts:555-563);
  * the solution CID is computed locally from the output bytes, so the commitment
    is signalled before the IPFS pin completes; the pin runs in the background and
    its CID is checked against the local one;
  * jobs are leased, not deleted up front (fixes Q4), and the event cursor is
    persisted so missed events are back-filled after a restart (fixes Q8);
  * ``contestationVoteFinish`` is implemented (the reference processor is a stub, Q11);
  * the scheduler never awaits a job inline (index.ts:918-958 awaits every non-concurrent job one
    by one): every job runs as a leased background task under a per-method concurrency limit
    (``JOB_LIMITS``, ``mi355x.job_concurrency``), solves under the pool's GPU capacity - a solve
    holds its GPU slot only until the solution's bytes exist, not through its commit / submit
    receipts - and the event poll runs on its own timer, so due claims (one per solved task,
    2,120 s later) never delay solve dispatch or ``TaskSubmitted`` handling;
  * events of one poll window are handled concurrently per task id (in order within a task).
"""
from __future__ import annotations

import asyncio
import contextvars
import json
import logging
import time
from typing import Awaitable, Callable, Dict, Optional

from ..chain.client import ChainClient, TxError
from ..ipfs.pin import Pinner
from ..ipfs.unixfs import cid_hex_to_str
from ..store.db import DB
from ..utils.protocol import expretry, generate_commitment, taskid2seed
from .models import Model, check_model_filter, get_model_by_id, hydrate_input, hydration_modes_agree
from .solver import EVIL_CID

log = logging.getLogger("arbius.miner")
ZERO_ADDR = "0x" + "00" * 20
MAX_UINT256 = 2 ** 256 - 1
MINER_VERSION = 0
_JOB = contextvars.ContextVar("arbius_job", default=None)

# Background concurrency per job method.  1 keeps the reference's one-at-a-time semantics where they
# matter (stake top-up, automine); claims / vote finishes are independent transactions and run wide.
JOB_LIMITS = {"task": 256, "pinTaskInput": 64, "claim": 128, "contestationVoteFinish": 8,
              "validatorStake": 1, "automine": 1}


class Metrics:
    """Counters / latency samples exported on the RPC server's /metrics route: a bounded window
    of samples per latency (p50 / p99 gauges) and a cumulative Prometheus histogram."""
    BUCKETS = (0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, 30.0, 60.0, 120.0, 300.0, 900.0)

    def __init__(self):
        self.counters: Dict[str, int] = {}
        self.latencies: Dict[str, list] = {}
        self.hist: Dict[str, list] = {}        # name -> [bucket counts..., +Inf count, sum]

    def inc(self, name, n=1):
        self.counters[name] = self.counters.get(name, 0) + n

    def observe(self, name, seconds, keep: int = 10000):
        v = self.latencies.setdefault(name, [])
        v.append(seconds)
        if len(v) > keep:          # bounded window for the p50/p99 export
            del v[: len(v) - keep]
        h = self.hist.setdefault(name, [0] * (len(self.BUCKETS) + 1) + [0.0])
        for i, b in enumerate(self.BUCKETS):
            if seconds <= b:
                h[i] += 1
        h[len(self.BUCKETS)] += 1
        h[-1] += seconds

    def prometheus_histograms(self):
        lines = []
        for k in sorted(self.hist):
            h = self.hist[k]
            lines.append(f"# TYPE arbius_{k}_seconds histogram")
            for i, b in enumerate(self.BUCKETS):
                lines.append(f'arbius_{k}_seconds_bucket{{le="{b:g}"}} {h[i]}')
            lines.append(f'arbius_{k}_seconds_bucket{{le="+Inf"}} {h[len(self.BUCKETS)]}')
            lines.append(f"arbius_{k}_seconds_sum {h[-1]:.6f}")
            lines.append(f"arbius_{k}_seconds_count {h[len(self.BUCKETS)]}")
        return lines

    def p50(self, name):
        v = sorted(self.latencies.get(name, []))
        return v[len(v) // 2] if v else None


class Miner:
    def __init__(self, cfg, db: DB, chain: ChainClient, pinner: Pinner, solver_pool, models: Dict[str, Model],
                 clock: Callable[[], int] = None, sleep: Callable[[float], Awaitable] = None,
                 retry_sleep: Callable[[float], Awaitable] = None):
        self.c = cfg
        self.db = db
        self.chain = chain
        self.pinner = pinner
        self.pool = solver_pool
        self.models = models
        self.now = clock or (lambda: int(time.time()))
        self.sleep = sleep or asyncio.sleep
        self.retry_sleep = retry_sleep or asyncio.sleep
        self.metrics = Metrics()
        self.quirks = bool(getattr(cfg.mi355x, "reference_hydration_quirks", True))
        self.lease_s = float(getattr(cfg.mi355x, "job_lease_seconds", 900.0))
        self.poll_s = float(getattr(cfg.mi355x, "poll_interval_ms", 100)) / 1000.0
        self.log_window = max(1, int(getattr(cfg.mi355x, "log_window_blocks", 2000)))
        self._bg: set = set()
        self._solving: set = set()           # solve job ids holding a GPU slot
        self._running: Dict[str, int] = {}   # method -> jobs running in this process
        self._inflight: set = set()          # job ids leased and running in this process
        self.limits = dict(JOB_LIMITS)
        self.limits.update({k: max(1, int(v)) for k, v in
                            (getattr(cfg.mi355x, "job_concurrency", None) or {}).items()})
        self.event_poll_s = float(getattr(cfg.mi355x, "event_poll_ms", 1000)) / 1000.0
        self.event_concurrency = int(getattr(cfg.mi355x, "event_concurrency", 64))
        self._last_poll: Optional[float] = None
        self.max_poll_gap_s = 0.0
        self.stopped = False

    # ------------------------------------------------------------------ helpers
    @property
    def wallet(self) -> str:
        return self.chain.address

    def _spawn(self, coro):
        t = asyncio.ensure_future(coro)
        self._bg.add(t)
        t.add_done_callback(self._bg.discard)
        return t

    async def _retry(self, fn, tries=10, base=1.5):
        return await expretry(fn, tries, base, sleep=self.retry_sleep)

    def queue(self, method, priority, waituntil, concurrent, data):
        log.info("QueueJob %s %s %s %s", method, priority, waituntil, "concurrent" if concurrent else "blocking")
        return self.db.queue_job(method, priority, waituntil, concurrent, data)

    # ------------------------------------------------------------------ lookups (index.ts:82-189)
    async def lookup_and_insert_task(self, taskid: str) -> dict:
        existing = self.db.get_task(taskid)
        if existing:
            return {"model": existing["modelid"], "fee": int(existing["fee"]), "owner": existing["address"],
                    "blocktime": int(existing["blocktime"]), "version": existing["version"], "cid": existing["cid"]}
        t = await self._retry(lambda: self.chain.get_task(taskid))
        if t is None:
            raise RuntimeError(f"could not look up task {taskid}")
        self.db.store_task(taskid, t["model"], t["fee"], t["owner"], t["blocktime"], t["version"], t["cid"])
        return t

    async def lookup_and_insert_task_input(self, taskid, cid, txid, template) -> Optional[dict]:
        cached = self.db.get_task_input(taskid, cid)
        if cached is not None:
            return json.loads(cached["data"])
        raw = await self._retry(lambda: self.chain.get_submit_task_input(txid))
        if raw is None:
            # reference Q9 (index.ts:151-155 throws): the transaction is not a submitTask call (the task
            # was sent through a contract, e.g. Example/SubmitTask.sol).  The task's on-chain cid is the
            # CIDv0 of the input bytes (EngineV1.sol:681-711, IPFS.sol:38-65): fetch them by CID and
            # accept them only if they hash to it.  Unrecoverable / mismatching bytes: skip the task,
            # never mark it invalid (that would contest a valid task).
            raw = await self.recover_input_by_cid(taskid, cid)
            if raw is None:
                return None
        try:
            pre_str = raw.decode("utf-8")
            pre = json.loads(pre_str)
        except Exception:  # noqa: BLE001
            log.warning("Task (%s) request was unable to be parsed", taskid)
            self.db.store_invalid_task(taskid)
            return None
        if not hydration_modes_agree(pre, template):
            # spec-correct and reference hydration disagree: whatever we decide, part of the
            # network decides otherwise -> stay out (no solve, no invalid mark, no contest)
            log.warning("Task (%s) input validity is ambiguous (spec vs reference hydration): skipped", taskid)
            self.metrics.inc("tasks_ambiguous_input")
            return None
        inp, err, msg = hydrate_input(pre, template, self.quirks)
        if err:
            log.warning("Task (%s) hydration error %s", taskid, msg)
            self.db.store_invalid_task(taskid)
            return None
        for row in template.get("input", []):
            if row.get("type") == "file" and inp.get(row["variable"]):
                from ..utils.video_io import UndecodableVideo, VideoSourceError, check_source, probe_video
                loop = asyncio.get_running_loop()
                try:
                    await loop.run_in_executor(None, check_source, inp[row["variable"]])
                except VideoSourceError as e:
                    # untrusted source this node will not read (local file, private address, plain
                    # http): skip - not invalid, other miners may legitimately read it
                    log.warning("Task (%s) input %s refused: %s", taskid, row["variable"], e)
                    self.metrics.inc("tasks_refused_source")
                    return None
                try:
                    await loop.run_in_executor(None, probe_video, inp[row["variable"]])
                except UndecodableVideo as e:
                    # outside this node's decoder (e.g. P/B-frame H.264 without ffmpeg): skip, not
                    # invalid - a miner with a full decoder can solve it, so contesting would be wrong
                    log.warning("Task (%s) input %s not decodable here: %s", taskid, row["variable"], e)
                    self.metrics.inc("tasks_undecodable_input")
                    return None
                except Exception as e:  # noqa: BLE001 - fetch failure: the solve retries the fetch
                    log.warning("Task (%s) input %s probe fetch failed: %r", taskid, row["variable"], e)
        inp["seed"] = taskid2seed(taskid)
        self.db.store_task_input(taskid, cid, inp)
        self.queue("pinTaskInput", 10, 0, True, {"taskid": taskid, "input": pre_str})
        return inp

    async def recover_input_by_cid(self, taskid: str, cid: str) -> Optional[bytes]:
        """The bytes behind a task's on-chain input CID (<= 65536 B: IPFS.sol:39), from the pinner
        (kubo ``cat`` / the local store) or the operator's gateway, verified against the CID."""
        import os
        from ..ipfs.pin import gateway_cat
        from ..ipfs.unixfs import onchain_cid
        want = bytes.fromhex(cid[2:] if cid.startswith("0x") else cid)
        cid58 = cid_hex_to_str(cid)
        sources = [("pinner", lambda: self.pinner.cat(cid58, 65536))]
        gw = getattr(self.c.mi355x, "ipfs_gateway", None) or os.environ.get("ARBIUS_IPFS_GATEWAY")
        if gw:
            sources.append(("gateway", lambda: gateway_cat(gw, cid58, 65536)))
        for name, fetch in sources:
            try:
                data = await fetch()
            except Exception as e:  # noqa: BLE001 - unreachable source / over the size cap
                log.warning("Task (%s) input %s from %s failed: %r", taskid, cid58, name, e)
                continue
            if data is None:
                continue
            try:
                ok = len(data) <= 65536 and onchain_cid(data) == want
            except ValueError:
                ok = False
            if ok:
                self.metrics.inc("tasks_input_by_cid")
                log.info("Task (%s) input recovered by cid %s from %s", taskid, cid58, name)
                return data
            self.metrics.inc("tasks_input_cid_mismatch")
            log.warning("Task (%s) input from %s does not hash to the on-chain cid %s: ignored", taskid, name,
                        cid58)
        self.metrics.inc("tasks_input_unrecoverable")
        log.warning("Task (%s) input could not be recovered (tx not submitTask, cid %s unavailable)", taskid,
                    cid58)
        return None

    # ------------------------------------------------------------------ event handlers (index.ts:191-333)
    async def on_event(self, ev):
        a = ev.args
        if ev.name == "TaskSubmitted":
            await self.lookup_and_insert_task(a["id"])      # cached in the DB after the first read
            self.queue("task", 10, 0, True, {"taskid": a["id"], "txid": ev.tx})
            self.metrics.inc("tasks_seen")
        elif ev.name == "TaskRetracted":
            if not self.db.get_task(a["id"]):
                await self.lookup_and_insert_task(a["id"])
            self.db.update_task_set_retracted(a["id"])
        elif ev.name == "SolutionSubmitted":
            taskid = a["task"]
            if self.db.get_solution(taskid):
                return
            s = await self._retry(lambda: self.chain.get_solution(taskid))
            if self.db.get_invalid_task(taskid) is not None and s["validator"].lower() != self.wallet:
                await self.contest_solution(taskid)
            self.db.store_solution(taskid, s["validator"], s["blocktime"], s["claimed"], s["cid"])
        elif ev.name == "ContestationSubmitted":
            taskid = a["task"]
            if self.db.get_contestation(taskid):
                return
            c = await self._retry(lambda: self.chain.get_contestation(taskid))
            if self.db.get_invalid_task(taskid) is not None:
                await self.vote_on_contestation(taskid, True)
            elif c["validator"].lower() != self.wallet and self._should_verify(taskid):
                # verify mode: re-run the task and vote by comparing CIDs
                self._spawn(self._verify_and_vote(taskid))
            self.db.store_contestation(taskid, c["validator"], c["blocktime"], c["finish_start_index"])
        elif ev.name == "ContestationVote":
            taskid, validator = a["task"], a["addr"]
            if any(r["validator"] == validator for r in self.db.get_contestation_votes(taskid)):
                return
            self.db.store_contestation_vote(taskid, validator, a["yea"])
        elif ev.name == "VersionChanged":
            await self.version_check()

    async def _handle_events(self, evs):
        """Handlers of one window: events of one task in log order, different tasks concurrently
        (each handler is a few chain reads; at node rate a window holds hundreds of events)."""
        groups: Dict[str, list] = {}
        for ev in evs:
            key = ev.args.get("id") or ev.args.get("task") or ev.name
            groups.setdefault(str(key).lower(), []).append(ev)
        sem = asyncio.Semaphore(max(1, self.event_concurrency))

        async def run(group):
            async with sem:
                for ev in group:
                    try:
                        await self.on_event(ev)
                    except SystemExit:
                        raise
                    except Exception as e:  # noqa: BLE001
                        log.error("event handler %s failed: %r", ev.name, e)
        if len(groups) == 1:
            await run(next(iter(groups.values())))
        elif groups:
            await asyncio.gather(*(run(g) for g in groups.values()))

    async def poll_events(self):
        """Back-fill ``eth_getLogs`` from the persisted cursor in bounded windows (providers cap the
        block range / result size of one call; after downtime on Nova the gap is large).  The
        cursor is persisted after every window; a failing window is halved until it passes."""
        t = time.monotonic()
        if self._last_poll is not None:
            gap = t - self._last_poll
            self.max_poll_gap_s = max(self.max_poll_gap_s, gap)
            self.metrics.observe("event_poll_gap_s", gap)
        self._last_poll = t
        latest = await self.chain.block_number()
        cur = self.db.get_cursor()
        if cur is None:      # first boot: only new events (reference .on semantics)
            self.db.set_cursor(latest)
            return 0
        start = cur + 1
        n = 0
        while start <= latest:
            end = min(latest, start + self.log_window - 1)
            try:
                evs = await self.chain.get_events(start, end)
            except Exception as e:  # noqa: BLE001
                if self.log_window <= 1:
                    raise
                self.log_window = max(1, self.log_window // 2)
                log.warning("eth_getLogs %d..%d failed (%r): window -> %d blocks", start, end, e, self.log_window)
                continue
            await self._handle_events(evs)
            self.db.set_cursor(end)
            n += len(evs)
            start = end + 1
        return n

    # ------------------------------------------------------------------ processors (index.ts:379-750)
    async def process_pin_task_input(self, taskid, input_str):
        cid = await self._retry(lambda: self.pinner.pin_file(input_str.encode(), f"task-{taskid}.json"))
        log.debug("Task input %s pinned with %s", taskid, cid)

    async def process_validator_stake(self):
        eth = await self.chain.eth_balance(self.wallet)
        if eth < 10 ** 16:
            log.warning("BCHK Low Ether balance")
        staked = (await self.chain.get_validator(self.wallet))["staked"]
        vmin = await self._retry(lambda: self.chain.get_validator_minimum())
        self.queue("validatorStake", 100, self.now() + 600, False, {"validatorMinimum": str(vmin)})
        min_topup = vmin * 100 // int(100 - self.c.stake_buffer_topup_percent)
        if staked >= min_topup:
            log.debug("BCHK Have sufficient stake")
            return
        min_buffer = vmin * 100 // int(100 - self.c.stake_buffer_percent)
        deposit = min_buffer - staked
        balance = await self._retry(lambda: self.chain.token_balance(self.wallet))
        if balance < deposit:
            log.error("BCHK Balance %s less than deposit amount %s", balance, deposit)
            raise RuntimeError("unable to stake required balance")
        allowance = await self._retry(lambda: self.chain.token_allowance(self.wallet, self.chain.engine_address))
        if allowance < balance:
            await self._retry(lambda: self.chain.token_approve(self.chain.engine_address, MAX_UINT256 - allowance))
        await self._retry(lambda: self.chain.validator_deposit(self.wallet, deposit))
        self.metrics.inc("stake_deposits")

    async def process_automine(self):
        a = self.c.automine
        try:
            await self.chain.submit_task(a.version, self.wallet, a.model, int(a.fee),
                                         json.dumps(a.input, separators=(",", ":")).encode())
        except Exception as e:  # noqa: BLE001
            log.error("Automine submitTask failed %r", e)
        if a.enabled:
            self.queue("automine", 5, self.now() + a.delay, False, {})

    async def process_task(self, taskid, txid):
        t = await self.lookup_and_insert_task(taskid)
        if int(t["version"]) != 0:
            self.db.store_invalid_task(taskid)
            return
        enabled, passed, template = check_model_filter(self.models, t["model"], self.now(), int(t["fee"]),
                                                       int(t["blocktime"]), t["owner"])
        if not enabled or not passed:
            return
        inp = await self.lookup_and_insert_task_input(taskid, t["cid"], txid, template)
        if inp is None:
            return
        self.queue("solve", 20, 0, False, {"taskid": taskid})

    async def get_cid(self, model: Model, taskid: str, inp: dict) -> Optional[str]:
        """default__getcid (models.ts:34-54) with local CID + background pin."""
        if self.c.evilmode:
            return EVIL_CID
        t0 = time.perf_counter()
        sol = await self._retry(lambda: self.pool.solve(model, taskid, inp))
        if sol is None:
            raise RuntimeError("cannot get files")
        self.metrics.observe("gpu_solve_s", time.perf_counter() - t0)
        for k, v in (sol.timings or {}).items():       # per-stage spans from the worker
            if isinstance(v, (int, float)):
                self.metrics.observe(f"stage_{k}", float(v))
        self._spawn(self._pin_solution(taskid, sol))
        return sol.cid

    async def _pin_solution(self, taskid, sol):
        cid58 = await self._retry(lambda: self.pinner.pin_files(taskid, sol.files))
        if cid58 is None:
            log.error("Task (%s) pin failed", taskid)
            self.metrics.inc("pin_failures")
        elif cid58 != cid_hex_to_str(sol.cid):
            log.error("Task (%s) pinned CID %s != local CID %s", taskid, cid58, cid_hex_to_str(sol.cid))
            self.metrics.inc("pin_cid_mismatch")

    async def process_solve(self, taskid):
        t_start = time.perf_counter()
        s = await self._retry(lambda: self.chain.get_solution(taskid))
        if s["validator"] != ZERO_ADDR:
            if s["validator"].lower() != self.wallet and self._should_verify(taskid):
                return await self.verify_solution(taskid, s)
            log.debug("Task (%s) already has solution", taskid)
            return
        t = await self.lookup_and_insert_task(taskid)
        m = get_model_by_id(self.models, t["model"])
        if m is None:
            log.error("Task (%s) could not find model (%s)", taskid, t["model"])
            return
        row = self.db.get_task_input(taskid, t["cid"])
        if row is None:
            log.warning("Task (%s) input not found in db", taskid)
            return
        inp = json.loads(row["data"])
        try:
            cid = await self.get_cid(m, taskid, inp)
        finally:
            self._release_gpu()              # the bytes exist: the chain phase holds no GPU slot
        if not cid:
            return
        commitment = generate_commitment(self.wallet, taskid, cid)
        t_c = time.perf_counter()
        # wait for the commitment's receipt: submitSolution requires the commitment in an EARLIER
        # block (EngineV1.sol:797-802); the reference sends both back to back (index.ts:619-639)
        # and relies on its retry delay, paying for a reverted submit whenever both land in one
        # block.  The GPU slot was released when the solve returned, so waiting costs no throughput.
        # (a commitment already on chain - a restarted solve - is not signalled twice: the second
        # signalCommitment would revert "commitment exists", EngineV1.sol:764-768)
        blk = await self._retry(lambda: self.chain.commitment_block(commitment))
        if not blk:
            try:
                await self.chain.signal_commitment(commitment, wait=True)
            except Exception as e:  # noqa: BLE001
                # a receipt timeout or a revert does not mean the commitment is missing (a slow
                # sequencer, or an earlier attempt of this solve that landed meanwhile): ask the
                # chain; only a commitment that is really absent drops the task
                self.metrics.inc("tx_failures")
                blk = await self._retry(lambda: self.chain.commitment_block(commitment))
                if not blk:
                    log.error("Commitment submission failed %r", e)
                    return
                log.warning("Commitment wait failed (%r) but it is on chain: submitting", e)
        self.metrics.observe("commit_tx_s", time.perf_counter() - t_c)

        async def submit():
            try:
                t_s = time.perf_counter()
                await self.chain.submit_solution(taskid, cid)
                self.metrics.observe("submit_tx_s", time.perf_counter() - t_s)
                self.queue("claim", 50, self.now() + 2000 + 120, False, {"taskid": taskid})
                self.metrics.inc("solutions_submitted")
                self.metrics.observe("task_latency_s", time.perf_counter() - t_start)
                return True
            except TxError as e:
                self.metrics.inc("tx_failures")
                ex = await self._retry(lambda: self.chain.get_solution(taskid))
                if ex["validator"] == ZERO_ADDR:
                    raise RuntimeError(f"unknown error submitting solution for {taskid}: {e.reason}")
                if ex["cid"] == cid:
                    log.info("Solution found for %s matches our cid %s", taskid, cid)
                    return True
                log.info("Solution found with cid %s does not match ours %s", ex["cid"], cid)
                await self.contest_solution(taskid)
                return True

        await self._retry(submit, 3, 1.25)

    def _should_verify(self, taskid) -> bool:
        """Verify mode (reference defect Q10: solutions of others are never re-checked):
        re-solve a deterministic fraction of already-solved tasks on spare GPU capacity."""
        frac = float(getattr(self.c.mi355x, "verify_fraction", 0.0))
        if frac <= 0.0:
            return False
        return (int(taskid, 16) % 10000) < frac * 10000

    async def verify_solution(self, taskid, s):
        t = await self.lookup_and_insert_task(taskid)
        m = get_model_by_id(self.models, t["model"])
        row = self.db.get_task_input(taskid, t["cid"])
        if m is None or row is None or self.c.evilmode:
            return
        sol = await self._retry(lambda: self.pool.solve(m, taskid, json.loads(row["data"])))
        if sol is None:
            return
        self.metrics.inc("verifications")
        if sol.cid != s["cid"]:
            log.info("Verify: task %s solution cid %s != ours %s -> contest", taskid, s["cid"], sol.cid)
            await self.contest_solution(taskid)

    async def _verify_and_vote(self, taskid):
        s = await self._retry(lambda: self.chain.get_solution(taskid))
        if s["validator"] == ZERO_ADDR or s["validator"].lower() == self.wallet:
            return
        try:
            t = await self.lookup_and_insert_task(taskid)
            m = get_model_by_id(self.models, t["model"])
            row = self.db.get_task_input(taskid, t["cid"])
            if m is None or row is None:
                return
            sol = await self._retry(lambda: self.pool.solve(m, taskid, json.loads(row["data"])))
        except Exception as e:  # noqa: BLE001
            log.error("verify %s failed: %r", taskid, e)
            return
        if sol is not None:
            await self.vote_on_contestation(taskid, sol.cid != s["cid"])

    async def contest_solution(self, taskid):
        try:
            await self.chain.submit_contestation(taskid)
            self.queue("contestationVoteFinish", 30, self.now() + 5010, False, {"taskid": taskid})
            self.metrics.inc("contestations_submitted")
        except TxError:
            c = await self._retry(lambda: self.chain.get_contestation(taskid))
            if c["validator"] == ZERO_ADDR:
                log.error("An unknown error occurred when we tried to contest %s", taskid)
                return
            await self.vote_on_contestation(taskid, True)

    async def vote_on_contestation(self, taskid, yea):
        if await self._retry(lambda: self.chain.contestation_voted(taskid, self.wallet)):
            return
        try:
            await self.chain.vote_on_contestation(taskid, yea)
            self.metrics.inc("contestation_votes")
        except TxError as e:
            log.error("Failed voting on contestation %s: %s", taskid, e.reason)

    FINISH_PAGE = 32

    async def process_contestation_vote_finish(self, taskid):
        """Implemented (reference stub, index.ts:392-395): finish in pages of 32 voters, paged by
        CHAIN state.  The on-chain loop pays the winning side's voters i in [finish_start_index,
        +amnt) (EngineV1.sol:1043-1106), so pages are sent until ``finish_start_index`` covers that
        side's vote count as the contract stores it - votes cast before this node's event cursor
        existed are not in the local DB, and a DB count would stop early and strand their stakes."""
        c = await self._retry(lambda: self.chain.get_contestation(taskid))
        if c["validator"] == ZERO_ADDR:
            return
        yeas, nays = await self._retry(lambda: self.chain.contestation_vote_counts(taskid))
        need = max(1, yeas if yeas > nays else nays)     # at least one call: it settles the task
        start = int(c["finish_start_index"])
        while start < need:
            try:
                await self.chain.contestation_vote_finish(taskid, self.FINISH_PAGE)
            except TxError as e:
                log.error("contestationVoteFinish %s failed: %s", taskid, e.reason)
                return
            c = await self._retry(lambda: self.chain.get_contestation(taskid))
            nxt = int(c["finish_start_index"])
            if nxt <= start:
                log.error("contestationVoteFinish %s did not advance (%d)", taskid, nxt)
                return
            start = nxt
            self.metrics.inc("contestation_finish_pages")

    async def process_claim(self, taskid):
        async def claim():
            s = await self._retry(lambda: self.chain.get_solution(taskid))
            if s["claimed"]:
                return "already"
            await self.chain.claim_solution(taskid)
            return "ok"
        r = await self._retry(claim)
        if r is None:
            log.error("Failed claiming (%s)", taskid)
        elif r == "ok":
            self.metrics.inc("claims")

    # ------------------------------------------------------------------ boot / loop (index.ts:960-1101)
    async def version_check(self):
        v = await self.chain.version()
        if v > MINER_VERSION:
            raise SystemExit(f"version mismatch, have miner version {MINER_VERSION} and arbius is {v}")

    def _selftest_key(self) -> str:
        arch = getattr(self.pool, "hardware", None)
        arch = arch() if callable(arch) else (arch or "unknown")
        weights = getattr(self.pool, "weights_id", None)
        weights = weights() if callable(weights) else (weights or "unknown")
        return f"{arch}/{weights}"

    async def self_test(self):
        """Boot CID self-test (miner/src/index.ts:981-1001) against a per-hardware table."""
        from pathlib import Path
        path = getattr(self.c.mi355x, "selftest_table", None) or str(Path(__file__).resolve().parents[1]
                                                                       / "config" / "selftest.json")
        table = json.loads(Path(path).read_text())
        key = self._selftest_key()
        from ..numerics import NUMERICS_VERSION
        if table.get("numerics_version", NUMERICS_VERSION) != NUMERICS_VERSION:
            log.error("Self test table pinned for numerics %s, this node is %s: values not enforced (re-pin with "
                      "scripts/pin_goldens.py --selftest)", table.get("numerics_version"), NUMERICS_VERSION)
            table = {k: dict(v, expected={}) if isinstance(v, dict) else v for k, v in table.items()}
        for m in self.models.values():
            entry = table.get(m.name)
            if entry is None or not isinstance(entry, dict):
                continue
            inp, err, msg = hydrate_input(dict(entry["input"]), m.template)
            if err:
                raise SystemExit(f"self test input invalid for {m.name}: {msg}")
            inp["seed"] = entry["input"]["seed"]
            sol = await self.pool.solve(m, "selftest", inp)
            want = entry.get("expected", {}).get(key)
            if want is None:
                log.warning("Self test %s on %s: cid %s (no pinned value for this hardware/weights)", m.name, key,
                            sol.cid)
            elif want.lower() != sol.cid.lower():
                log.error("Self test %s on %s FAILED: expected %s got %s", m.name, key, want, sol.cid)
                raise SystemExit("boot self test cid mismatch")
            else:
                log.info("Self test %s on %s passed (%s)", m.name, key, sol.cid)
            self.metrics.inc("selftests_run")

    async def boot(self):
        self.db.clear_jobs_by_method("validatorStake")
        self.db.clear_jobs_by_method("automine")
        await self.version_check()
        if getattr(self.c.mi355x, "selftest", False) and not self.c.evilmode:
            await self.self_test()
        self.queue("validatorStake", 30, 0, False, {})
        if self.c.automine.enabled:
            self.queue("automine", 5, 0, False, {})

    def _dispatch(self, method: str, data: dict):
        if method == "automine":
            return self.process_automine()
        if method == "validatorStake":
            return self.process_validator_stake()
        if method == "task":
            return self.process_task(data["taskid"], data["txid"])
        if method == "solve":
            return self.process_solve(data["taskid"])
        if method == "claim":
            return self.process_claim(data["taskid"])
        if method == "pinTaskInput":
            return self.process_pin_task_input(data["taskid"], data["input"])
        if method == "contestationVoteFinish":
            return self.process_contestation_vote_finish(data["taskid"])
        raise SystemExit(f"method ({method}) has no implementation")  # index.ts:914-916

    async def _renew(self, jobid):
        """Lease heartbeat: a job that outlives ``job_lease_seconds`` (a long solve) must not be
        leased and run a second time."""
        while True:
            await asyncio.sleep(max(0.05, self.lease_s / 3.0))
            self.db.renew_lease(jobid, self.lease_s)

    def _release_gpu(self):
        jid = _JOB.get()
        if jid is not None:
            self._solving.discard(jid)

    async def _run_job(self, job):
        _JOB.set(job["id"])
        hb = asyncio.ensure_future(self._renew(job["id"]))
        method = job["method"]
        try:
            await self._dispatch(method, json.loads(job["data"]))
            self.metrics.inc(f"jobs_ok_{method}")
        except SystemExit:
            raise
        except Exception as e:  # noqa: BLE001
            log.error("Job (%s) [%s] failed: %r", job["id"], method, e)
            self.db.store_failed_job(job)
            self.metrics.inc(f"jobs_failed_{method}")
        finally:
            hb.cancel()
            self.db.delete_job(job["id"])
            self._inflight.discard(job["id"])
            self._solving.discard(job["id"])
            self._running[method] = self._running.get(method, 1) - 1

    def _start(self, job, worker: str) -> bool:
        if job["id"] in self._inflight or not self.db.lease_job(job["id"], worker, self.lease_s):
            return False
        self._inflight.add(job["id"])
        self._running[job["method"]] = self._running.get(job["method"], 0) + 1
        self._spawn(self._run_job(job))
        return True

    async def process_jobs(self) -> int:
        """One scheduler pass; it starts jobs and never awaits one.  Solves fill the GPU pool's
        capacity; every other method runs up to its concurrency limit as a leased background task."""
        # jobs already running in this process are skipped even if their lease lapsed (they renew
        # it, but a stalled event loop could still let one expire)
        now = self.now()
        n = 0
        cap = max(1, int(getattr(self.pool, "capacity", 1)))
        free = cap - len(self._solving)
        if free > 0:
            for job in self.db.runnable_jobs_of(now, ["solve"], free + len(self._inflight)):
                if len(self._solving) >= cap:
                    break
                if self._start(job, "gpu"):
                    self._solving.add(job["id"])
                    n += 1
        for method, lim in self.limits.items():
            free = lim - self._running.get(method, 0)
            if free <= 0:
                continue
            for job in self.db.runnable_jobs_of(now, [method], free + len(self._inflight)):
                if self._running.get(method, 0) >= lim:
                    break
                n += self._start(job, "node")
        return n

    async def drain(self, max_rounds=10000):
        """Run until no runnable job is left and no background work is pending (tests)."""
        for _ in range(max_rounds):
            n = await self.process_jobs()
            if self._bg:
                await asyncio.sleep(0)
                await asyncio.gather(*list(self._bg), return_exceptions=True)
                continue
            if n == 0 and not self.db.runnable_jobs(self.now()):
                return

    async def _poll_loop(self, stop: asyncio.Event):
        while not stop.is_set():
            t0 = time.monotonic()
            try:
                await self.poll_events()
            except SystemExit:
                raise
            except Exception as e:  # noqa: BLE001
                log.error("event poll failed: %r", e)
            await asyncio.sleep(max(0.0, self.event_poll_s - (time.monotonic() - t0)))

    async def run(self, stop: asyncio.Event = None):
        """Boot, then two independent loops: the event poll on its own timer and the job scheduler
        (index.ts:1078-1101 runs both in one loop and awaits blocking jobs in it)."""
        await self.boot()
        for m in self.db.job_methods():      # reference: an unknown method stops the miner (index.ts:914)
            if m not in self.limits and m != "solve":
                raise SystemExit(f"method ({m}) has no implementation")
        stop = stop or asyncio.Event()
        poller = asyncio.ensure_future(self._poll_loop(stop))
        try:
            while not stop.is_set():
                if poller.done():
                    poller.result()          # SystemExit from a handler (VersionChanged) ends the node
                    poller = asyncio.ensure_future(self._poll_loop(stop))
                n = await self.process_jobs()
                if n == 0:
                    await self.sleep(self.poll_s)
                else:
                    await asyncio.sleep(0.005)   # finishing jobs free slots continuously: bound the pass rate
        finally:
            poller.cancel()
