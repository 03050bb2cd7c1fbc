"""The pipelined transaction sender (chain/txpipe.py) against the mock node in mempool / block mode:
batched nonce-ordered broadcasts, a dropped transaction re-broadcast, a held transaction fee-bumped,
a nonce used by another process re-synced, a refused nonce filled, and revert-only vote-count probes."""
import asyncio

import pytest
from aiohttp.test_utils import TestServer

from arbius_amd.chain.client import TxError
from arbius_amd.chain.mock_engine import E18, MockEngine, MockToken
from arbius_amd.chain.mock_node import TOKEN_ADDRESS, MockNode
from arbius_amd.chain.rpc import RpcChainClient, RpcError
from arbius_amd.chain.secp256k1 import address_from_priv

KEY = "0x" + "11" * 32
OTHER = "0x" + "99" * 20


def _node(**kw):
    tok = MockToken()
    e = MockEngine(tok, owner="0x" + "0e" * 20, chain_id=42170)
    e.token_address = TOKEN_ADDRESS
    tok.mint(address_from_priv(KEY), 10 * E18)
    return MockNode(e, TOKEN_ADDRESS, **kw)


def _run(node, body):
    async def go():
        server = TestServer(node.app())
        await server.start_server()
        url = str(server.make_url("/"))
        clients = []

        def client(**kw):
            c = RpcChainClient(url, KEY, node.engine.address, TOKEN_ADDRESS, receipt_poll=0.02, **kw)
            clients.append(c)
            return c
        try:
            return await body(client)
        finally:
            for c in clients:
                await c.close()
            await server.close()
    return asyncio.run(go())


def _approve(c, i):
    return c.token_approve(OTHER, i + 1)


def test_concurrent_sends_batch_in_nonce_order_and_all_mine():
    node = _node(block_time_s=0.05, latency_s=0.01)

    async def body(client):
        c = client(stuck_s=5.0)
        await asyncio.gather(*(_approve(c, i) for i in range(60)))
        return c
    c = _run(node, body)
    me = address_from_priv(KEY)
    assert node.nonces[me] == 60 and c.txs.stats["mined"] == 60
    assert c.txs.stats["batches"] < 20                      # 60 transactions, a handful of round trips
    assert c.txs.stats["rebroadcasts"] == c.txs.stats["bumps"] == 0


def test_dropped_transaction_is_rebroadcast_and_later_nonces_mine():
    node = _node(block_time_s=0.05)

    async def body(client):
        c = client(stuck_s=0.3)
        await _approve(c, 0)
        node.drop_next = 1                                   # the sequencer loses the next one
        await asyncio.gather(*(_approve(c, i) for i in range(1, 8)))
        return c
    c = _run(node, body)
    me = address_from_priv(KEY)
    assert len(node.dropped) == 1 and node.nonces[me] == 8    # no permanent gap
    assert c.txs.stats["rebroadcasts"] >= 1 and c.txs.stats["mined"] == 8
    assert node.engine.token.allowance(me, OTHER) > 0


def test_held_transaction_is_fee_bumped():
    node = _node(block_time_s=0.05)

    async def body(client):
        c = client(stuck_s=0.3)
        c.txs.gas_ttl_s = 0.05
        await _approve(c, 0)
        node.min_gas_price = 3 * 10 ** 8                     # base fee rises: our 1e8 tx is held, unmined
        await _approve(c, 1)
        return c
    c = _run(node, body)
    me = address_from_priv(KEY)
    assert node.nonces[me] == 2 and c.txs.stats["bumps"] >= 1 and node.stats["replaced"] >= 1


def test_nonce_used_by_another_process_resyncs():
    node = _node(block_time_s=0.02)

    async def body(client):
        a, b = client(), client()
        await _approve(a, 0)                                 # a: nonce 0
        await _approve(b, 1)                                 # b (same key, own pipeline): nonces 1, 2
        await _approve(b, 2)
        await _approve(a, 3)                                 # a believes 1: "nonce too low" -> re-sync -> 3
        return a
    a = _run(node, body)
    assert node.nonces[address_from_priv(KEY)] == 4 and a.txs.stats["resyncs"] == 1


def test_refused_broadcast_fails_its_waiter_and_leaves_no_gap():
    node = _node(block_time_s=0.05)
    orig = node._to_mempool

    def refuse_one(f, sender):
        if f["nonce"] == 1 and f["data"] and not getattr(node, "_refused", False):
            node._refused = True
            raise ValueError("insufficient funds for gas * price + value")
        return orig(f, sender)
    node._to_mempool = refuse_one

    async def body(client):
        c = client(stuck_s=0.3)
        res = await asyncio.gather(*(_approve(c, i) for i in range(4)), return_exceptions=True)
        return c, res
    c, res = _run(node, body)
    assert sum(isinstance(r, TxError) for r in res) == 1    # only the refused request fails
    assert node.nonces[address_from_priv(KEY)] == 4 and c.txs.stats["fillers"] == 1   # hole filled


def test_vote_count_probe_reraises_non_revert_errors():
    """only a revert ends the index search; a rate limit must not shorten it."""
    class Fake(RpcChainClient):
        def __init__(self, n, flaky_at):
            self.n, self.flaky_at, self.calls = n, flaky_at, 0
            self._engine = "0x" + "11" * 20

        async def _call(self, to, name, taskid, i):
            self.calls += 1
            if self.calls == self.flaky_at:
                raise RpcError("daily request count exceeded, request rate limited", -32005)
            if i >= self.n:
                raise RpcError("execution reverted", 3)
            return ["0x" + "22" * 20]

    with pytest.raises(RpcError, match="rate limited"):
        asyncio.run(Fake(41, 4).contestation_vote_counts("0x" + "33" * 32))
    assert asyncio.run(Fake(41, 10 ** 6).contestation_vote_counts("0x" + "33" * 32)) == (41, 41)


def test_reads_share_batches():
    node = _node(latency_s=0.01)

    async def body(client):
        c = client()
        vals = await asyncio.gather(*(c.token_balance(address_from_priv(KEY)) for _ in range(40)))
        return c, vals
    c, vals = _run(node, body)
    assert set(vals) == {10 * E18}
    assert c.rpc_stats["calls"] == 40 and c.rpc_stats["posts"] <= 2
