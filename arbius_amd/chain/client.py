"""Chain access layer used by the node (the role of ``miner/src/blockchain.ts`` +
the ethers ``arbius``/``token`` contract objects).

``ChainClient`` is the interface; ``MockChainClient`` binds it to the in-process
``MockEngine`` (tests, the CPU plumbing config) and ``rpc.RpcChainClient`` binds
it to a real JSON-RPC endpoint (Arbitrum Nova) with local signing.

All ids / cids / addresses are lowercase 0x-hex strings; amounts are ints (wei).
"""
from __future__ import annotations

import abc
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

from .mock_engine import MockEngine, Revert


@dataclass
class ChainEvent:
    name: str
    args: dict
    block: int
    tx: str
    log_index: int


class TxError(Exception):
    """A transaction that reverted / failed; ``reason`` is the revert string when known."""

    def __init__(self, reason: str):
        super().__init__(reason)
        self.reason = reason


class ChainClient(abc.ABC):
    address: str

    # ---- reads (eth_call)
    @abc.abstractmethod
    async def get_task(self, taskid: str) -> dict: ...          # model, fee, owner, blocktime, version, cid

    @abc.abstractmethod
    async def get_solution(self, taskid: str) -> dict: ...      # validator, blocktime, claimed, cid

    @abc.abstractmethod
    async def get_contestation(self, taskid: str) -> dict: ...  # validator, blocktime, finish_start_index, slashAmount

    @abc.abstractmethod
    async def contestation_voted(self, taskid: str, addr: str) -> bool: ...

    @abc.abstractmethod
    async def get_validator(self, addr: str) -> dict: ...       # staked, since, addr

    @abc.abstractmethod
    async def get_validator_minimum(self) -> int: ...

    @abc.abstractmethod
    async def version(self) -> int: ...

    @abc.abstractmethod
    async def token_balance(self, addr: str) -> int: ...

    @abc.abstractmethod
    async def token_allowance(self, owner: str, spender: str) -> int: ...

    @abc.abstractmethod
    async def eth_balance(self, addr: str) -> int: ...

    @abc.abstractmethod
    async def block_number(self) -> int: ...

    @abc.abstractmethod
    async def commitment_block(self, commitment: str) -> int: ...   # commitments(bytes32): 0 = none

    @abc.abstractmethod
    async def contestation_vote_counts(self, taskid: str) -> Tuple[int, int]: ...   # (yeas, nays) on chain

    @abc.abstractmethod
    async def get_submit_task_input(self, txid: str) -> Optional[bytes]:
        """Decode ``submitTask`` calldata of ``txid`` -> ``input_`` bytes (index.ts:151-159)."""

    # ---- transactions
    @abc.abstractmethod
    async def signal_commitment(self, commitment: str, wait: bool = False) -> str: ...

    @abc.abstractmethod
    async def submit_solution(self, taskid: str, cid: str) -> str: ...

    @abc.abstractmethod
    async def claim_solution(self, taskid: str) -> str: ...

    @abc.abstractmethod
    async def submit_contestation(self, taskid: str) -> str: ...

    @abc.abstractmethod
    async def vote_on_contestation(self, taskid: str, yea: bool) -> str: ...

    @abc.abstractmethod
    async def contestation_vote_finish(self, taskid: str, amnt: int) -> str: ...

    @abc.abstractmethod
    async def validator_deposit(self, validator: str, amount: int) -> str: ...

    @abc.abstractmethod
    async def token_approve(self, spender: str, amount: int) -> str: ...

    @abc.abstractmethod
    async def submit_task(self, version: int, owner: str, model: str, fee: int, input_: bytes) -> str: ...

    # ---- logs
    @abc.abstractmethod
    async def get_events(self, from_block: int, to_block: int) -> List[ChainEvent]: ...

    @property
    @abc.abstractmethod
    def engine_address(self) -> str: ...


class MockChainClient(ChainClient):
    """ChainClient over an in-process MockEngine, acting as ``address``."""

    def __init__(self, engine: MockEngine, address: str, eth_balance: int = 10 ** 18, batch_blocks: bool = False):
        self.engine = engine
        self.address = address.lower()
        self._eth = eth_balance
        self.sent: List[Tuple[str, tuple]] = []  # tx log for tests / fault injection
        self.fail_next: Dict[str, str] = {}       # method -> revert reason (fault injection)
        self.reverted: List[Tuple[str, tuple, str]] = []   # (method, args, reason) of reverted txs
        # batch_blocks: a transaction sent without waiting for its receipt stays pending and is mined
        # in ONE block together with the next transaction (a real chain's sequencing); hardhat
        # automine (every transaction its own block) otherwise
        self.batch_blocks = batch_blocks
        self._pending: List[Tuple[str, tuple]] = []

    @property
    def engine_address(self) -> str:
        return self.engine.address

    def _call(self, method, *args):
        if method in self.fail_next:
            raise TxError(self.fail_next.pop(method))
        try:
            fn = getattr(self.engine, method)
            fn(self.address, *args)
        except Revert as e:
            self.reverted.append((method, args, str(e)))
            raise TxError(str(e)) from None
        self.sent.append((method, args))
        ev = self.engine.events[-1] if self.engine.events else None
        return ev.tx if ev else "0x"

    def _send(self, method, *args, wait: bool = True):
        if not self.batch_blocks:
            return self._call(method, *args)
        self._pending.append((method, args))
        if not wait:
            return "0x"
        return self.flush()

    def flush(self):
        """Mine the pending transactions in one block; raises the LAST one's revert (the caller
        waits on that one's receipt; earlier ones fail silently, as unawaited sends do)."""
        pend, self._pending = self._pending, []
        if not pend:
            return "0x"
        out = None
        with self.engine.one_block():
            for i, (m, a) in enumerate(pend):
                try:
                    out = self._call(m, *a)
                except TxError:
                    if i == len(pend) - 1:
                        raise
        return out

    async def get_task(self, taskid):
        t = self.engine.get_task(taskid)
        return {"model": t.model, "fee": t.fee, "owner": t.owner, "blocktime": t.blocktime, "version": t.version,
                "cid": t.cid}

    async def get_solution(self, taskid):
        s = self.engine.get_solution(taskid)
        return {"validator": s.validator, "blocktime": s.blocktime, "claimed": s.claimed, "cid": s.cid}

    async def get_contestation(self, taskid):
        c = self.engine.get_contestation(taskid)
        return {"validator": c.validator, "blocktime": c.blocktime, "finish_start_index": c.finish_start_index,
                "slashAmount": c.slash_amount}

    async def contestation_voted(self, taskid, addr):
        return bool(self.engine.contestation_voted.get((taskid.lower(), addr.lower())))

    async def get_validator(self, addr):
        v = self.engine.get_validator(addr)
        return {"staked": v.staked, "since": v.since, "addr": v.addr}

    async def get_validator_minimum(self):
        return self.engine.get_validator_minimum()

    async def version(self):
        return self.engine.version

    async def token_balance(self, addr):
        return self.engine.token.balance_of(addr)

    async def token_allowance(self, owner, spender):
        return self.engine.token.allowance(owner, spender)

    async def eth_balance(self, addr):
        return self._eth

    async def block_number(self):
        self.flush() if self.batch_blocks else None
        return self.engine.block_number

    async def commitment_block(self, commitment):
        return self.engine.commitments.get(commitment.lower(), 0)

    async def contestation_vote_counts(self, taskid):
        t = taskid.lower()
        return len(self.engine.vote_yeas.get(t, [])), len(self.engine.vote_nays.get(t, []))

    async def get_submit_task_input(self, txid):
        r = self.engine.get_transaction(txid)
        if r is None or r[0] != "submitTask":
            return None
        return r[1][4]

    async def signal_commitment(self, commitment, wait=False):
        return self._send("signal_commitment", commitment, wait=wait)

    async def submit_solution(self, taskid, cid):
        return self._send("submit_solution", taskid, cid)

    async def claim_solution(self, taskid):
        return self._send("claim_solution", taskid)

    async def submit_contestation(self, taskid):
        return self._send("submit_contestation", taskid)

    async def vote_on_contestation(self, taskid, yea):
        return self._send("vote_on_contestation", taskid, yea)

    async def contestation_vote_finish(self, taskid, amnt):
        return self._send("contestation_vote_finish", taskid, amnt)

    async def validator_deposit(self, validator, amount):
        return self._send("validator_deposit", validator, amount)

    async def token_approve(self, spender, amount):
        self.engine.token.approve(self.address, spender, amount)
        self.sent.append(("approve", (spender, amount)))
        return "0x"

    async def submit_task(self, version, owner, model, fee, input_):
        if "submit_task" in self.fail_next:
            raise TxError(self.fail_next.pop("submit_task"))
        try:
            self.engine.submit_task(self.address, version, owner, model, fee, input_)
        except Revert as e:
            raise TxError(str(e)) from None
        self.sent.append(("submit_task", (version, owner, model, fee)))
        return self.engine.events[-1].tx

    async def get_events(self, from_block, to_block):
        return [ChainEvent(e.name, dict(e.args), e.block, e.tx, e.index) for e in self.engine.events
                if from_block <= e.block <= to_block]
