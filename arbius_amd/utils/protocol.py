"""Byte-compatibility invariants of the Arbius protocol.

* seed        = taskid mod 0x1FFFFFFFFFFFF0          (miner/src/utils.ts:15-19, paper.tex:83)
* commitment  = keccak256(abi.encode(address, bytes32, bytes))
                                                     (miner/src/utils.ts:42-48 == EngineV1.sol:537-543)
* task id     = keccak256(abi.encode(sender, prevhash, model, fee, cid))  (EngineV1.sol:431-438)
* model id    = keccak256(abi.encode(sender, addr, fee, cid))        (EngineV1.sol:419-424)
"""
from __future__ import annotations

import asyncio
import logging
import time
from typing import Awaitable, Callable, Optional, TypeVar

from ..chain import abi
from .keccak import keccak256

SEED_MOD = 0x1FFFFFFFFFFFF0
T = TypeVar("T")
log = logging.getLogger("arbius")


def _b(v) -> bytes:
    if isinstance(v, (bytes, bytearray)):
        return bytes(v)
    return bytes.fromhex(v[2:] if v.startswith("0x") else v)


def taskid2seed(taskid) -> int:
    return int.from_bytes(_b(taskid), "big") % SEED_MOD if not isinstance(taskid, int) else taskid % SEED_MOD


def generate_commitment(address, taskid, cid) -> str:
    enc = abi.encode(["address", "bytes32", "bytes"], [_b(address), _b(taskid), _b(cid)])
    return "0x" + keccak256(enc).hex()


def hash_task(sender, prevhash, model, fee: int, cid) -> str:
    enc = abi.encode(["address", "bytes32", "bytes32", "uint256", "bytes"],
                     [_b(sender), _b(prevhash), _b(model), int(fee), _b(cid)])
    return "0x" + keccak256(enc).hex()


def hash_model(sender, addr, fee: int, cid) -> str:
    # EngineV1.hashModel (EngineV1.sol:419-424) encodes (sender, o.addr, o.fee, o.cid); rate is not hashed
    enc = abi.encode(["address", "address", "uint256", "bytes"], [_b(sender), _b(addr), int(fee), _b(cid)])
    return "0x" + keccak256(enc).hex()


def now() -> int:
    return int(time.time())


async def expretry(fn: Callable[[], Awaitable[T]], tries: int = 10, base: float = 1.5,
                   sleep=asyncio.sleep) -> Optional[T]:
    """Exponential-backoff retry returning None after ``tries`` failures
    (``miner/src/utils.ts:21-39``)."""
    for retry in range(tries):
        try:
            return await fn()
        except Exception as e:  # noqa: BLE001 - mirror reference semantics
            seconds = base ** retry
            log.warning("retry request failed, retrying in %s", seconds)
            log.debug("%r", e)
            await sleep(seconds)
    log.error("retry request failed %d times", tries)
    return None
