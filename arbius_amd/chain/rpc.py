"""ChainClient over Ethereum JSON-RPC (Arbitrum Nova in production): eth_call
reads, locally signed transactions with a single nonce manager, receipts, and
``eth_getLogs`` event back-fill (replaces ethers v5 ``.on`` polling, fixes Q8).

One RpcChainClient owns the wallet; GPU workers never sign:
concurrent solves serialise only on the nonce lock, not on inference.
"""
from __future__ import annotations

import asyncio
import itertools
import logging
from typing import List, Optional

from . import abi, secp256k1
from .client import ChainClient, ChainEvent, TxError
from .engine_abi import FUNCS, TOPIC_TO_EVENT, decode_log
from .tx import Tx

log = logging.getLogger("arbius.chain")

GAS = {  # explicit gas limits of the reference (index.ts:620-739, 476-485)
    "signalCommitment": 450_000, "submitSolution": 500_000, "claimSolution": 300_000,
    "submitTask": 2_500_000, "submitContestation": 900_000, "voteOnContestation": 500_000,
    "contestationVoteFinish": 3_000_000, "validatorDeposit": 400_000, "approve": 100_000,
}


class RpcError(Exception):
    pass


class RpcChainClient(ChainClient):
    def __init__(self, url: str, private_key: str, engine_address: str, token_address: str,
                 chain_id: Optional[int] = None, timeout: float = 30.0, receipt_poll: float = 0.25,
                 eip1559: bool = False):
        import httpx
        self.url = url
        self.priv = private_key
        self.address = secp256k1.address_from_priv(private_key)
        self._engine = engine_address.lower()
        self.token = token_address.lower()
        self.chain_id = chain_id
        self.http = httpx.AsyncClient(timeout=timeout)
        self._ids = itertools.count(1)
        self._nonce: Optional[int] = None
        self._nonce_lock = asyncio.Lock()
        self.receipt_poll = receipt_poll
        self.eip1559 = eip1559

    @property
    def engine_address(self) -> str:
        return self._engine

    @property
    def token_address(self) -> str:
        return self.token

    async def rpc(self, method: str, params: list):
        r = await self.http.post(self.url, json={"jsonrpc": "2.0", "id": next(self._ids), "method": method,
                                                 "params": params})
        r.raise_for_status()
        j = r.json()
        if "error" in j:
            raise RpcError(j["error"].get("message", str(j["error"])))
        return j["result"]

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
            except RpcError:
                return False

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

    async def _send_raw(self, to: str, data: bytes, gas: int, value: int, wait: bool) -> str:
        async with self._nonce_lock:
            if self.chain_id is None:
                self.chain_id = int(await self.rpc("eth_chainId", []), 16)
            if self._nonce is None:
                self._nonce = int(await self.rpc("eth_getTransactionCount", [self.address, "pending"]), 16)
            gas_price = int(await self.rpc("eth_gasPrice", []), 16)
            if self.eip1559:
                tx = Tx(self._nonce, to, data, gas, self.chain_id, value, None, gas_price * 2, 0)
            else:
                tx = Tx(self._nonce, to, data, gas, self.chain_id, value, gas_price)
            raw = tx.sign(self.priv)
            try:
                txh = await self.rpc("eth_sendRawTransaction", ["0x" + raw.hex()])
            except RpcError as e:
                self._nonce = None  # resync on next send
                raise TxError(str(e)) from None
            self._nonce += 1
        if wait:
            await self.wait_receipt(txh)
        return txh

    async def wait_receipt(self, txh: str, timeout: float = 120.0):
        for _ in range(int(timeout / self.receipt_poll)):
            rc = await self.rpc("eth_getTransactionReceipt", [txh])
            if rc:
                if int(rc["status"], 16) != 1:
                    raise TxError(rc.get("revertReason", "transaction reverted"))
                return rc
            await asyncio.sleep(self.receipt_poll)
        raise TxError("receipt timeout")

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
        await self.http.aclose()
