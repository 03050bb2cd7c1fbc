"""ChainClient over Ethereum JSON-RPC (Arbitrum Nova in production): eth_call
reads, locally signed transactions through a pipelined sender, receipts, and
``eth_getLogs`` event back-fill (replaces ethers v5 ``.on`` polling, fixes Q8).

One RpcChainClient owns the wallet; GPU workers never sign.
Transport for a node that runs tens of tasks per second over a latent endpoint:

* reads issued in the same event-loop turn go out as ONE JSON-RPC batch (``batch=True``;
  ``max_batch`` calls per POST) - concurrent task / solution / claim lookups share round trips;
* transactions go through ``txpipe.TxPipeline``: local nonces, nonce-ordered batched broadcasts,
  batched receipt polling, cached gas price, re-broadcast / fee-bump of a stuck nonce.
"""
from __future__ import annotations

import asyncio
import itertools
import logging
from typing import List, Optional, Sequence, Tuple

from . import abi, secp256k1
from .client import ChainClient, ChainEvent
from .engine_abi import FUNCS, TOPIC_TO_EVENT, decode_log
from .txpipe import PendingTx, TxPipeline

log = logging.getLogger("arbius.chain")

GAS = {  # explicit gas limits of the reference (index.ts:620-739, 476-485)
    "signalCommitment": 450_000, "submitSolution": 500_000, "claimSolution": 300_000,
    "submitTask": 2_500_000, "submitContestation": 900_000, "voteOnContestation": 500_000,
    "contestationVoteFinish": 3_000_000, "validatorDeposit": 400_000, "approve": 100_000,
}


class RpcError(Exception):
    def __init__(self, message: str, code: Optional[int] = None):
        super().__init__(message)
        self.code = code

    @property
    def is_revert(self) -> bool:
        """An EVM revert / invalid opcode / panic (the call itself failed), as opposed to a transport,
        rate-limit or node error that says nothing about the call."""
        m = str(self).lower()
        return self.code == 3 or "revert" in m or "invalid opcode" in m or "panic" in m


def _err(e: dict) -> RpcError:
    return RpcError(e.get("message", str(e)), e.get("code"))


class RpcChainClient(ChainClient):
    def __init__(self, url: str, private_key: str, engine_address: str, token_address: str,
                 chain_id: Optional[int] = None, timeout: float = 30.0, receipt_poll: float = 0.25,
                 eip1559: bool = False, batch: bool = True, max_batch: int = 50, stuck_s: float = 12.0):
        import httpx
        self.url = url
        self.priv = private_key
        self.address = secp256k1.address_from_priv(private_key)
        self._engine = engine_address.lower()
        self.token = token_address.lower()
        self.chain_id = chain_id
        self.http = httpx.AsyncClient(timeout=timeout,
                                      limits=httpx.Limits(max_connections=64, max_keepalive_connections=64))
        self._ids = itertools.count(1)
        self.receipt_poll = receipt_poll
        self.eip1559 = eip1559
        self.batch = batch
        self.max_batch = max(1, int(max_batch))
        self._reads: List[Tuple[str, list, asyncio.Future]] = []
        self._read_flush = False
        self.txs = TxPipeline(self, poll_s=receipt_poll, stuck_s=stuck_s)
        self.rpc_stats = {"posts": 0, "calls": 0}

    @property
    def engine_address(self) -> str:
        return self._engine

    @property
    def token_address(self) -> str:
        return self.token

    # ------------------------------------------------------------------ transport
    async def _post(self, body):
        r = await self.http.post(self.url, json=body)
        r.raise_for_status()
        self.rpc_stats["posts"] += 1
        self.rpc_stats["calls"] += len(body) if isinstance(body, list) else 1
        return r.json()

    async def _rpc_one(self, method: str, params: list):
        j = await self._post({"jsonrpc": "2.0", "id": next(self._ids), "method": method, "params": params})
        if "error" in j:
            raise _err(j["error"])
        return j["result"]

    async def _post_batch(self, calls: Sequence[Tuple[str, list]]) -> list:
        """One POST carrying ``calls`` as a JSON-RPC batch: results (or RpcError) in call order."""
        if len(calls) == 1:
            try:
                return [await self._rpc_one(*calls[0])]
            except RpcError as e:
                return [e]
        ids = [next(self._ids) for _ in calls]
        out = await self._post([{"jsonrpc": "2.0", "id": i, "method": m, "params": p}
                                for i, (m, p) in zip(ids, calls)])
        if isinstance(out, dict):          # a node that refuses batches answers with one error object
            raise _err(out.get("error", {"message": "batch refused"}))
        by_id = {r.get("id"): r for r in out}
        res = []
        for i in ids:
            r = by_id.get(i)
            if r is None:
                res.append(RpcError("missing response in batch"))
            elif "error" in r:
                res.append(_err(r["error"]))
            else:
                res.append(r["result"])
        return res

    async def rpc_batch(self, calls: Sequence[Tuple[str, list]]) -> list:
        """Results (or RpcError instances) of ``calls``, sent in order.  Batched in one POST per
        ``max_batch`` calls unless batching is off (or ``rpc`` was replaced by a test stub)."""
        if not self.batch or "rpc" in self.__dict__:
            res = []
            for m, p in calls:
                try:
                    res.append(await self.rpc(m, p))
                except RpcError as e:
                    res.append(e)
            return res
        res = []
        for i in range(0, len(calls), self.max_batch):
            res.extend(await self._post_batch(calls[i:i + self.max_batch]))
        return res

    async def rpc(self, method: str, params: list):
        """One JSON-RPC call; with batching on, it rides in the batch of this event-loop turn."""
        if not self.batch:
            return await self._rpc_one(method, params)
        fut = asyncio.get_running_loop().create_future()
        self._reads.append((method, params, fut))
        if not self._read_flush:
            self._read_flush = True
            asyncio.get_running_loop().call_soon(self._flush_reads)
        return await fut

    def _flush_reads(self):
        self._read_flush = False
        q, self._reads = self._reads, []
        for i in range(0, len(q), self.max_batch):
            asyncio.ensure_future(self._serve(q[i:i + self.max_batch]))

    async def _serve(self, part):
        try:
            out = await self._post_batch([(m, p) for m, p, _ in part])
        except Exception as e:  # noqa: BLE001 - transport failure: every caller in the batch sees it
            for _, _, f in part:
                if not f.done():
                    f.set_exception(e)
            return
        for (_, _, f), r in zip(part, out):
            if f.done():
                continue
            if isinstance(r, Exception):
                f.set_exception(r)
            else:
                f.set_result(r)

    async def _call(self, to: str, name: str, *args):
        sig, rets = FUNCS[name]
        data = abi.encode_call(sig, *args)
        out = await self.rpc("eth_call", [{"to": to, "data": "0x" + data.hex()}, "latest"])
        raw = bytes.fromhex(out[2:])
        return abi.decode(rets, raw) if rets else []

    # ------------------------------------------------------------------ reads
    async def get_task(self, taskid):
        model, fee, owner, blocktime, version, cid = await self._call(self._engine, "tasks", taskid)
        return {"model": model, "fee": fee, "owner": owner, "blocktime": blocktime, "version": version, "cid": cid}

    async def get_solution(self, taskid):
        validator, blocktime, claimed, cid = await self._call(self._engine, "solutions", taskid)
        return {"validator": validator, "blocktime": blocktime, "claimed": claimed, "cid": cid}

    async def get_contestation(self, taskid):
        validator, blocktime, fsi, slash = await self._call(self._engine, "contestations", taskid)
        return {"validator": validator, "blocktime": blocktime, "finish_start_index": fsi, "slashAmount": slash}

    async def contestation_voted(self, taskid, addr):
        return (await self._call(self._engine, "contestationVoted", taskid, addr))[0]

    async def get_validator(self, addr):
        staked, since, a = await self._call(self._engine, "validators", addr)
        return {"staked": staked, "since": since, "addr": a}

    async def get_validator_minimum(self):
        return (await self._call(self._engine, "getValidatorMinimum"))[0]

    async def version(self):
        return (await self._call(self._engine, "version"))[0]

    async def token_balance(self, addr):
        return (await self._call(self.token, "balanceOf", addr))[0]

    async def token_allowance(self, owner, spender):
        return (await self._call(self.token, "allowance", owner, spender))[0]

    async def eth_balance(self, addr):
        return int(await self.rpc("eth_getBalance", [addr, "latest"]), 16)

    async def block_number(self):
        return int(await self.rpc("eth_blockNumber", []), 16)

    async def commitment_block(self, commitment):
        return (await self._call(self._engine, "commitments", commitment))[0]

    async def contestation_vote_counts(self, taskid):
        """Lengths of ``contestationVoteYeas/Nays[taskid]``: the public array getters revert past the
        end, so each length is found by an exponential + binary search over indices (O(log n) calls)."""
        async def has(name, i):
            try:
                await self._call(self._engine, name, taskid, i)
                return True
            except RpcError as e:
                if e.is_revert:          # array getter past the end: Panic(0x32) / revert
                    return False
                raise                    # rate limit / node error: not an answer (caller retries)

        async def length(name):
            if not await has(name, 0):
                return 0
            hi = 1
            while await has(name, hi):
                hi *= 2
            lo = hi // 2                     # has(lo), not has(hi)
            while hi - lo > 1:
                mid = (lo + hi) // 2
                if await has(name, mid):
                    lo = mid
                else:
                    hi = mid
            return hi
        return await length("contestationVoteYeas"), await length("contestationVoteNays")

    async def get_submit_task_input(self, txid):
        tx = await self.rpc("eth_getTransactionByHash", [txid])
        if not tx:
            return None
        data = bytes.fromhex(tx["input"][2:])
        sig = FUNCS["submitTask"][0]
        if data[:4] != abi.selector(sig):
            return None  # task submitted through a contract (reference Q9)
        return bytes.fromhex(abi.decode_call(sig, data)[4][2:])

    # ------------------------------------------------------------------ transactions
    async def call_sig(self, to: str, sig: str, rets: List[str], *args):
        """Generic eth_call by signature string (operator CLI: admin/governance reads)."""
        out = await self.rpc("eth_call", [{"to": to, "data": "0x" + abi.encode_call(sig, *args).hex()}, "latest"])
        raw = bytes.fromhex(out[2:])
        return abi.decode(rets, raw) if rets else []

    async def send_sig(self, to: str, sig: str, *args, value: int = 0, gas: int = 1_000_000, wait: bool = True):
        """Generic signed transaction by signature string ("" = plain value transfer)."""
        data = abi.encode_call(sig, *args) if sig else b""
        return await self._send_raw(to, data, gas, value, wait)

    async def _send(self, to: str, name: str, *args, wait: bool = True) -> str:
        sig, _ = FUNCS[name]
        data = abi.encode_call(sig, *args)
        return await self._send_raw(to, data, GAS.get(name, 1_000_000), 0, wait)

    async def submit_tx(self, to: str, data: bytes, gas: int, value: int = 0) -> PendingTx:
        """Broadcast through the pipelined sender; the returned handle carries ``hash`` and ``nonce``."""
        return await self.txs.send(to, data, gas, value)

    async def _send_raw(self, to: str, data: bytes, gas: int, value: int, wait: bool) -> str:
        p = await self.txs.send(to, data, gas, value)
        if wait:
            await self.txs.wait(p)
        return p.hash

    async def wait_receipt(self, txh: str, timeout: float = 300.0):
        return await self.txs.wait_hash(txh, timeout)

    async def signal_commitment(self, commitment, wait=False):
        return await self._send(self._engine, "signalCommitment", commitment, wait=wait)

    async def submit_solution(self, taskid, cid):
        return await self._send(self._engine, "submitSolution", taskid, cid)

    async def claim_solution(self, taskid):
        return await self._send(self._engine, "claimSolution", taskid)

    async def submit_contestation(self, taskid):
        return await self._send(self._engine, "submitContestation", taskid)

    async def vote_on_contestation(self, taskid, yea):
        return await self._send(self._engine, "voteOnContestation", taskid, bool(yea))

    async def contestation_vote_finish(self, taskid, amnt):
        return await self._send(self._engine, "contestationVoteFinish", taskid, int(amnt))

    async def validator_deposit(self, validator, amount):
        return await self._send(self._engine, "validatorDeposit", validator, int(amount))

    async def token_approve(self, spender, amount):
        return await self._send(self.token, "approve", spender, int(amount))

    async def submit_task(self, version, owner, model, fee, input_):
        return await self._send(self._engine, "submitTask", int(version), owner, model, int(fee), input_)

    async def register_model(self, addr, fee, template: bytes):
        return await self._send(self._engine, "registerModel", addr, int(fee), template)

    async def signal_support(self, model, support: bool):
        return await self._send(self._engine, "signalSupport", model, bool(support))

    # ------------------------------------------------------------------ logs
    async def get_events(self, from_block, to_block) -> List[ChainEvent]:
        logs = await self.rpc("eth_getLogs", [{"address": self._engine, "fromBlock": hex(from_block),
                                               "toBlock": hex(to_block), "topics": [list(TOPIC_TO_EVENT)]}])
        out = []
        for lg in logs:
            name, args = decode_log(lg["topics"], bytes.fromhex(lg["data"][2:]))
            if name is None:
                continue
            out.append(ChainEvent(name, args, int(lg["blockNumber"], 16), lg["transactionHash"],
                                  int(lg["logIndex"], 16)))
        out.sort(key=lambda e: (e.block, e.log_index))
        return out

    async def close(self):
        await self.txs.close()
        await self.http.aclose()
