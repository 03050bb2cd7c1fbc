"""Pipelined transaction sender: one per wallet, local nonces, batched broadcasts and receipts,
stuck-transaction recovery.

The reference signs through an ethers v5 ``Wallet`` (``/root/reference/miner/src/blockchain.ts:22-32``),
which asks the provider for the ``pending`` nonce before every send: correct, but one send at a time,
two round trips each, and its fire-and-forget ``signalCommitment`` (``miner/src/index.ts:619-628``) relies
on the next send to heal a dropped transaction.  A node that solves tens of tasks per second per
wallet needs ~3 transactions per task (commit, submit, claim: ``EngineV1.sol:764,786,867``), so this
sender is built for a latent JSON-RPC endpoint instead:

* **local nonces** - synced once from ``eth_getTransactionCount(pending)``, then assigned in order;
* **batched broadcast** - every request queued while the previous batch was in flight goes out in
  ONE JSON-RPC batch of ``eth_sendRawTransaction`` calls in nonce order (one round trip per batch,
  not two per transaction); batches are sent one after another so nonces reach the node in order;
* **gas price cached** - refreshed every ``gas_ttl_s`` inside the receipt tracker's batch, never on
  the send path;
* **receipts by batch** - one tracker polls the receipts of every in-flight transaction plus the
  ``latest`` / ``pending`` nonces in one batch per ``poll_s``;
* **recovery** - the lowest unmined nonce is re-broadcast if the node lost it (``pending`` count does
  not cover it) and fee-bumped (same nonce, ``bump`` x price) if it sits in the mempool past
  ``stuck_s``; a ``nonce too low`` answer re-syncs and re-queues the request on a fresh nonce; a
  request the node refuses outright leaves a hole that is filled by a 0-value self-transfer so the
  nonces above it still mine.  A transaction whose nonce was mined under another hash (another
  process using the wallet) fails its waiter with ``TxError``.

Waiters get ``TxError`` for a reverted receipt, a refused broadcast or a consumed nonce; a caller's
``timeout`` only stops waiting - the tracker keeps the transaction alive.
"""
from __future__ import annotations

import asyncio
import logging
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from .client import TxError
from .tx import Tx

log = logging.getLogger("arbius.txpipe")


def _msg(e) -> str:
    return str(e).lower()


def _already_known(e) -> bool:
    m = _msg(e)
    return "already known" in m or "known transaction" in m or "already imported" in m


def _nonce_low(e) -> bool:
    m = _msg(e)
    return "nonce too low" in m or "nonce has already been used" in m or "oldnonce" in m


def _nonce_high(e) -> bool:
    m = _msg(e)
    return "nonce too high" in m or "nonce gap" in m or "futurenonce" in m


def _underpriced(e) -> bool:
    return "underpriced" in _msg(e)


@dataclass
class PendingTx:
    to: str
    data: bytes
    gas: int
    value: int
    nonce: int = -1
    price: int = 0
    raw: bytes = b""
    hashes: List[str] = field(default_factory=list)
    sent_at: float = 0.0
    attempts: int = 0
    filler: bool = False
    grace: int = 0
    hash_fut: Optional[asyncio.Future] = None
    receipt_fut: Optional[asyncio.Future] = None

    @property
    def hash(self) -> Optional[str]:
        return self.hashes[-1] if self.hashes else None


class TxPipeline:
    def __init__(self, client, *, poll_s: float = 0.25, stuck_s: float = 12.0, gas_ttl_s: float = 2.0,
                 bump: float = 1.125, max_batch: int = 64, max_receipts: int = 256,
                 clock: Callable[[], float] = time.monotonic):
        self.c = client
        self.poll_s = poll_s
        self.stuck_s = stuck_s
        self.gas_ttl_s = gas_ttl_s
        self.bump = bump
        self.max_batch = max_batch
        self.max_receipts = max_receipts
        self.clock = clock
        self._out: List[PendingTx] = []
        self._inflight: Dict[int, PendingTx] = {}
        self._by_hash: Dict[str, PendingTx] = {}
        self._next: Optional[int] = None
        self._gas: Optional[int] = None
        self._gas_t = -1e30
        self._flusher: Optional[asyncio.Task] = None
        self._tracker: Optional[asyncio.Task] = None
        self.stats = {"sent": 0, "batches": 0, "rebroadcasts": 0, "bumps": 0, "resyncs": 0, "fillers": 0,
                      "refused": 0, "replaced": 0, "mined": 0, "reverted": 0}

    # ------------------------------------------------------------------ public API
    @property
    def next_nonce(self) -> Optional[int]:
        return self._next

    def inflight(self) -> int:
        return len(self._inflight) + len(self._out)

    async def send(self, to: str, data: bytes, gas: int, value: int = 0) -> PendingTx:
        """Queue one transaction; returns once the node accepted its broadcast (``.hash``, ``.nonce``)."""
        loop = asyncio.get_running_loop()
        p = PendingTx(to, data, gas, value, hash_fut=loop.create_future(), receipt_fut=loop.create_future())
        self._out.append(p)
        self._kick()
        await asyncio.shield(p.hash_fut)
        return p

    async def wait(self, p: PendingTx, timeout: float = 300.0) -> dict:
        try:
            return await asyncio.wait_for(asyncio.shield(p.receipt_fut), timeout)
        except asyncio.TimeoutError:
            raise TxError("receipt timeout") from None

    async def wait_hash(self, txh: str, timeout: float = 300.0) -> dict:
        p = self._by_hash.get(txh)
        if p is None:                      # not ours / already resolved and forgotten: ask the node
            return await self._poll_foreign(txh, timeout)
        return await self.wait(p, timeout)

    async def close(self):
        for t in (self._flusher, self._tracker):
            if t is not None and not t.done():
                t.cancel()
                try:
                    await t
                except (asyncio.CancelledError, Exception):  # noqa: BLE001
                    pass

    # ------------------------------------------------------------------ internals
    def _kick(self):
        if self._flusher is None or self._flusher.done():
            self._flusher = asyncio.ensure_future(self._flush())

    def _kick_tracker(self):
        if self._tracker is None or self._tracker.done():
            self._tracker = asyncio.ensure_future(self._track())

    async def _poll_foreign(self, txh, timeout):
        t_end = self.clock() + timeout
        while self.clock() < t_end:
            rc = await self.c.rpc("eth_getTransactionReceipt", [txh])
            if rc:
                if int(rc["status"], 16) != 1:
                    raise TxError(rc.get("revertReason") or "transaction reverted")
                return rc
            await asyncio.sleep(self.poll_s)
        raise TxError("receipt timeout")

    async def _ensure_ready(self):
        c = self.c
        calls = []
        if c.chain_id is None:
            calls.append(("eth_chainId", []))
        if self._next is None:
            calls.append(("eth_getTransactionCount", [c.address, "pending"]))
        if self._gas is None or self.clock() - self._gas_t > 10 * self.gas_ttl_s:   # idle sender: stale price
            calls.append(("eth_gasPrice", []))
        if not calls:
            return
        out = await c.rpc_batch(calls)
        for (m, _), r in zip(calls, out):
            if isinstance(r, Exception):
                raise TxError(f"{m}: {r}")
            if m == "eth_chainId":
                c.chain_id = int(r, 16)
            elif m == "eth_getTransactionCount":
                self._next = int(r, 16)
            else:
                self._gas, self._gas_t = int(r, 16), self.clock()

    def _sign(self, p: PendingTx):
        c = self.c
        if c.eip1559:
            tx = Tx(p.nonce, p.to, p.data, p.gas, c.chain_id, p.value, None, p.price * 2, 0)
        else:
            tx = Tx(p.nonce, p.to, p.data, p.gas, c.chain_id, p.value, p.price)
        p.raw = tx.sign(c.priv)
        from ..utils.keccak import keccak256
        h = "0x" + keccak256(p.raw).hex()
        p.hashes.append(h)
        self._by_hash[h] = p
        return h

    def _resolve(self, p: PendingTx, exc: Optional[BaseException] = None, receipt: Optional[dict] = None):
        for f in (p.hash_fut, p.receipt_fut):
            if f is not None and not f.done():
                if exc is not None:
                    f.set_exception(exc)
                    f.exception()            # retrieved: no "never retrieved" warning for unawaited futures
                elif f is p.hash_fut:
                    f.set_result(p.hash)
                else:
                    f.set_result(receipt)
        self._inflight.pop(p.nonce, None) if self._inflight.get(p.nonce) is p else None
        for h in p.hashes:
            self._by_hash.pop(h, None)

    async def _flush(self):
        """Broadcast queued requests in nonce-ordered batches, one batch in flight at a time."""
        while self._out:
            try:
                await self._ensure_ready()
            except Exception as e:  # noqa: BLE001 - endpoint down: fail the waiting senders
                batch, self._out = self._out, []
                for p in batch:
                    self._resolve(p, TxError(str(e)))
                return
            batch, self._out = self._out[: self.max_batch], self._out[self.max_batch:]
            for p in batch:
                if p.nonce < 0:
                    p.nonce = self._next
                    self._next += 1
                p.price = max(p.price, self._gas)
                self._sign(p)
                p.attempts += 1
                p.sent_at = self.clock()
            try:
                out = await self.c.rpc_batch([("eth_sendRawTransaction", ["0x" + p.raw.hex()]) for p in batch])
            except Exception as e:  # noqa: BLE001 - transport failure: the node may or may not hold them
                log.warning("broadcast of nonces %d..%d failed in transport (%r): tracking them", batch[0].nonce,
                            batch[-1].nonce, e)
                out = [None] * len(batch)
            self.stats["batches"] += 1
            requeue, resync = [], False
            for p, r in zip(batch, out):
                if not isinstance(r, Exception) or _already_known(r):
                    self._accept(p)
                elif _nonce_high(r):
                    # a lower nonce is missing at the node: keep ours, the tracker re-broadcasts in order
                    self._accept(p, stale=True)
                elif _nonce_low(r):
                    resync = True
                    self._by_hash.pop(p.hashes.pop(), None)
                    if not p.filler:
                        p.nonce = -1
                        requeue.append(p)
                else:
                    self.stats["refused"] += 1
                    log.warning("transaction nonce %d refused by the node: %s", p.nonce, r)
                    self._hole(p.nonce)
                    self._resolve(p, TxError(str(r)))
            if resync:
                self.stats["resyncs"] += 1
                try:
                    pend = int(await self.c.rpc("eth_getTransactionCount", [self.c.address, "pending"]), 16)
                    self._next = max(self._next, pend)
                except Exception as e:  # noqa: BLE001
                    log.warning("nonce re-sync failed: %r", e)
                self._out[:0] = requeue
            if self._inflight:
                self._kick_tracker()

    def _accept(self, p: PendingTx, stale: bool = False):
        if stale:
            p.sent_at = -1e30                 # eligible for re-broadcast at the tracker's next pass
        self._inflight[p.nonce] = p
        self.stats["sent"] += 1
        if p.hash_fut is not None and not p.hash_fut.done():
            p.hash_fut.set_result(p.hash)

    def _hole(self, nonce: int):
        """The node refused nonce ``nonce`` outright: give it back if it was the last one handed
        out, else fill it with a 0-value self-transfer so the nonces above it can still mine."""
        if self._next == nonce + 1 and not any(q.nonce > nonce for q in self._out):
            self._next = nonce
            return
        f = PendingTx(self.c.address, b"", 21000, 0, nonce=nonce, filler=True)
        self.stats["fillers"] += 1
        self._out.insert(0, f)

    async def _track(self):
        """Receipts, nonce state and gas price in one batch per ``poll_s`` while anything is in flight."""
        c = self.c
        while self._inflight:
            await asyncio.sleep(self.poll_s)
            low = sorted(self._inflight)[: self.max_receipts]
            calls = [("eth_getTransactionCount", [c.address, "latest"]),
                     ("eth_getTransactionCount", [c.address, "pending"])]
            refresh_gas = self.clock() - self._gas_t >= self.gas_ttl_s
            if refresh_gas:
                calls.append(("eth_gasPrice", []))
            slots = []
            for n in low:
                for h in self._inflight[n].hashes:
                    calls.append(("eth_getTransactionReceipt", [h]))
                    slots.append((n, h))
            try:
                out = await c.rpc_batch(calls)
            except Exception as e:  # noqa: BLE001 - transient endpoint failure: next pass
                log.warning("receipt poll failed: %r", e)
                continue
            if isinstance(out[0], Exception) or isinstance(out[1], Exception):
                continue
            latest, pending = int(out[0], 16), int(out[1], 16)
            k = 2
            if refresh_gas:
                if not isinstance(out[2], Exception):
                    self._gas, self._gas_t = int(out[2], 16), self.clock()
                k = 3
            seen = set()
            for (n, h), rc in zip(slots, out[k:]):
                p = self._inflight.get(n)
                if p is None or isinstance(rc, Exception) or not rc:
                    continue
                seen.add(n)
                if int(rc["status"], 16) == 1:
                    self.stats["mined"] += 1
                    self._resolve(p, receipt=rc)
                else:
                    self.stats["reverted"] += 1
                    self._resolve(p, TxError(rc.get("revertReason") or "transaction reverted"))
            for n in low:
                p = self._inflight.get(n)
                if p is None or n in seen or n >= latest:
                    continue
                p.grace += 1                   # mined nonce, none of our hashes has a receipt (yet)
                if p.grace >= 3:
                    self.stats["replaced"] += 1
                    log.error("nonce %d was mined by another transaction: %s lost", n, p.hash)
                    self._resolve(p, TxError("nonce consumed by another transaction"))
            await self._recover(latest, pending)

    async def _recover(self, latest: int, pending: int):
        if not self._inflight:
            return
        n0 = min(self._inflight)
        p0 = self._inflight[n0]
        now = self.clock()
        if n0 < latest or now - p0.sent_at < self.stuck_s:
            return
        if pending <= n0:
            # the node does not hold nonce n0 (dropped by the sequencer / mempool eviction, or a
            # broadcast refused as a gap): re-broadcast it and everything above, in nonce order
            redo = [self._inflight[n] for n in sorted(self._inflight)]
            self.stats["rebroadcasts"] += len(redo)
            log.warning("nonce %d not held by the node (latest %d, pending %d): re-broadcasting %d transactions",
                        n0, latest, pending, len(redo))
            for i in range(0, len(redo), self.max_batch):
                part = redo[i:i + self.max_batch]
                out = await self.c.rpc_batch([("eth_sendRawTransaction", ["0x" + p.raw.hex()]) for p in part])
                for p, r in zip(part, out):
                    p.sent_at = self.clock()
                    if isinstance(r, Exception) and not (_already_known(r) or _nonce_low(r) or _nonce_high(r)):
                        log.warning("re-broadcast of nonce %d failed: %s", p.nonce, r)
            return
        # held but not mined: outbid ourselves on the same nonce
        p0.price = max(int(p0.price * self.bump) + 1, self._gas or 0)
        self._sign(p0)
        p0.attempts += 1
        p0.sent_at = now
        self.stats["bumps"] += 1
        log.warning("nonce %d stuck for %.0f s: fee bump to %d (attempt %d)", n0, self.stuck_s, p0.price, p0.attempts)
        r, = await self.c.rpc_batch([("eth_sendRawTransaction", ["0x" + p0.raw.hex()])])
        if isinstance(r, Exception) and not _already_known(r):
            if _underpriced(r):
                p0.sent_at = now - self.stuck_s          # bump again next pass
            log.warning("fee bump of nonce %d refused: %s", n0, r)
