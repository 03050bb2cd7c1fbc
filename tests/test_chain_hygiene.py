"""Chain-path hygiene, MockEngine on CPU:

* contract-submitted tasks (Example/SubmitTask.sol): the input is recovered by the
  task's on-chain CID and solved; bytes that do not hash to the CID are rejected and the task is
  skipped, never marked invalid;
* the commitment is mined in a block before ``submitSolution`` (EngineV1.sol:797-802): on a chain
  that batches unawaited transactions into one block, 50 solves send zero reverted submits;
* ``contestationVoteFinish`` pages by chain state: votes cast before the node's event cursor
  existed are still finished (EngineV1.sol:1026-1106).
"""
import asyncio
import json

from arbius_amd.chain import examples as ex
from arbius_amd.chain.client import MockChainClient
from arbius_amd.chain.mock_engine import E18
from arbius_amd.config.mining_config import MiningConfig
from arbius_amd.ipfs.pin import LocalPinner
from arbius_amd.node.miner import Miner
from arbius_amd.node.models import default_models
from arbius_amd.node.pool import FakeSolverPool
from arbius_amd.store.db import DB
from arbius_amd.utils.protocol import generate_commitment

from test_node_e2e import DEPLOYER, MINER, MINER2, make_world, submit

INPUT = {"prompt": "a lighthouse at dusk", "negative_prompt": "blurry"}


def _miner(e, mid, pinner=None, client=None, addr=MINER, **mi):
    cfg = MiningConfig.from_dict({"db_path": ":memory:", "mi355x": {"selftest": False, **mi}})
    return Miner(cfg, DB(":memory:"), client or MockChainClient(e, addr), pinner or LocalPinner(), FakeSolverPool(),
                 default_models({"anythingv3": mid}), clock=lambda: e.timestamp,
                 retry_sleep=lambda s: asyncio.sleep(0))


async def _boot(m):
    await m.boot()
    await m.poll_events()
    await m.drain()


def _contract_task(e, tok, mid, raw):
    sub = ex.SubmitTask(e, tok, mid, raw)
    tok.transfer(DEPLOYER, sub.address, E18)
    return sub.submit_task()


def test_contract_submitted_task_is_recovered_by_cid_and_solved():
    e, tok, mid = make_world()
    raw = json.dumps(INPUT).encode()
    pinner = LocalPinner()
    asyncio.run(pinner.pin_file(raw, "input.json"))      # the task's input is on IPFS (any pinner)
    m = _miner(e, mid, pinner)

    async def go():
        await _boot(m)
        tid = _contract_task(e, tok, mid, raw)
        # the transaction is the contract call, not the engine's submitTask: no input in calldata
        assert await m.chain.get_submit_task_input(e.events[-1].tx) is None
        await m.poll_events()
        await m.drain()
        return tid

    tid = asyncio.run(go())
    assert e.solutions[tid].validator == MINER.lower()
    assert m.metrics.counters.get("tasks_input_by_cid") == 1
    (_, ctid, inp), = m.pool.calls
    assert ctid == tid and inp["prompt"] == INPUT["prompt"] and inp["seed"] == int(tid, 16) % 0x1FFFFFFFFFFFF0
    e.increase_time(2200)
    asyncio.run(m.drain())
    assert e.solutions[tid].claimed


def test_tampered_gateway_bytes_are_rejected_and_the_task_skipped(monkeypatch):
    e, tok, mid = make_world()
    raw = json.dumps(INPUT).encode()
    fetched = []

    async def evil_gateway(gw, cid, max_bytes, **kw):
        fetched.append((gw, cid))
        return json.dumps({"prompt": "something else entirely", "negative_prompt": "x"}).encode()

    monkeypatch.setattr("arbius_amd.ipfs.pin.gateway_cat", evil_gateway)
    m = _miner(e, mid, ipfs_gateway="https://gateway.example")      # the pinner does not have it

    async def go():
        await _boot(m)
        tid = _contract_task(e, tok, mid, raw)
        await m.poll_events()
        await m.drain()
        return tid

    tid = asyncio.run(go())
    assert fetched and fetched[0][0] == "https://gateway.example"
    assert e.solutions.get(tid) is None and m.pool.calls == []
    assert m.db.get_invalid_task(tid) is None              # skipped, NOT invalid (no contest)
    assert m.metrics.counters.get("tasks_input_cid_mismatch") == 1
    assert m.metrics.counters.get("tasks_input_unrecoverable") == 1


def test_gateway_bytes_matching_the_cid_are_accepted(monkeypatch):
    e, tok, mid = make_world()
    raw = json.dumps(INPUT).encode()

    async def gateway(gw, cid, max_bytes, **kw):
        return raw

    monkeypatch.setattr("arbius_amd.ipfs.pin.gateway_cat", gateway)
    m = _miner(e, mid, ipfs_gateway="https://gateway.example")

    async def go():
        await _boot(m)
        tid = _contract_task(e, tok, mid, raw)
        await m.poll_events()
        await m.drain()
        return tid

    tid = asyncio.run(go())
    assert e.solutions[tid].validator == MINER.lower()


class _NoWaitClient(MockChainClient):
    """The reference's ordering (index.ts:619-639): the commitment is sent without waiting."""

    async def signal_commitment(self, commitment, wait=False):
        return await super().signal_commitment(commitment, wait=False)


def _solve_many(client_cls, n):
    e, tok, mid = make_world()
    client = client_cls(e, MINER, batch_blocks=True)
    m = _miner(e, mid, client=client)

    async def go():
        await _boot(m)
        tids = []
        for i in range(n):
            tids.append(submit(e, mid, dict(INPUT, prompt=f"task {i}")))
            await m.poll_events()
            await m.drain()
        return tids

    tids = asyncio.run(go())
    solved = sum(1 for t in tids if e.solutions.get(t) is not None and e.solutions[t].validator == MINER.lower())
    submits_reverted = [r for r in client.reverted if r[0] == "submit_solution"]
    return solved, submits_reverted


def test_commitment_is_mined_before_submit_no_reverted_submits():
    solved, reverted = _solve_many(MockChainClient, 50)
    assert solved == 50 and reverted == []


def test_unawaited_commitment_reverts_submits_on_a_batching_chain():
    """Control for the test above: with the reference's unawaited commitment, commitment and submit
    land in one block and every first submit reverts ("commitment must be in past")."""
    solved, reverted = _solve_many(_NoWaitClient, 5)
    assert solved == 5
    assert len(reverted) == 5 and all("commitment must be in past" in r[2] for r in reverted)


def test_restarted_solve_does_not_resignal_an_existing_commitment():
    """A solve that dies after its commitment was mined (submit never sent) and runs again must not
    signal the same commitment twice (it would revert "commitment exists", EngineV1.sol:764-768)."""
    e, tok, mid = make_world()

    class Crashy(MockChainClient):
        crash = True

        async def submit_solution(self, taskid, cid):
            if self.crash:
                raise ConnectionError("node lost before submitSolution")
            return await super().submit_solution(taskid, cid)

    client = Crashy(e, MINER)
    m = _miner(e, mid, client=client)

    async def go():
        await _boot(m)
        tid = submit(e, mid, INPUT)
        await m.poll_events()
        await m.drain()                                   # commitment mined, submit lost
        assert e.solutions.get(tid) is None and len(e.commitments) == 1
        client.crash = False
        m.queue("solve", 20, 0, False, {"taskid": tid})   # the solve runs again
        await m.drain()
        return tid

    tid = asyncio.run(go())
    assert e.solutions[tid].validator == MINER.lower()
    assert [r for r in client.reverted if r[0] == "signal_commitment"] == []
    assert sum(1 for meth, _ in client.sent if meth == "signal_commitment") == 1


def _stake(e, tok, addr, amount):
    tok.transfer(DEPLOYER, addr, amount)
    tok.approve(addr, e.address, 2 ** 256 - 1)
    e.validator_deposit(addr, addr, amount)


def test_vote_finish_pages_by_chain_state_with_votes_before_the_cursor():
    e, tok, mid = make_world()
    tok.mint(DEPLOYER, 1000 * E18)
    voters = ["0x" + f"{0xb000 + i:040x}" for i in range(40)]
    solver, contester = MINER2, "0x" + f"{0xc0de:040x}"
    for a in [solver, contester] + voters:
        _stake(e, tok, a, 3 * E18)
    e.increase_time(200)                                  # validators' stake is older than 120 s
    tid = submit(e, mid, INPUT)
    cid = "0x1220" + "ab" * 32
    e.signal_commitment(solver, generate_commitment(solver, tid, cid))
    e.mine(1)
    e.submit_solution(solver, tid, cid)
    e.submit_contestation(contester, tid)                 # yea (contester) + nay (solver)
    for v in voters:                                      # 40 more yeas, all before the node boots
        e.vote_on_contestation(v, tid, True)
    staked_before = {v: e.validators[v].staked for v in voters}
    yeas = 1 + len(voters)
    assert len(e.vote_yeas[tid]) == yeas and len(e.vote_nays[tid]) == 1

    m = _miner(e, mid)                                    # boots now: its cursor starts after the votes

    async def go():
        await _boot(m)
        assert m.db.get_contestation_votes(tid) == []     # the node never saw those votes
        e.increase_time(4100)
        await m.process_contestation_vote_finish(tid)

    asyncio.run(go())
    c = e.contestations[tid]
    assert c.finish_start_index >= yeas                   # 41 yeas: two pages of 32
    assert m.metrics.counters.get("contestation_finish_pages") == 2
    slash = c.slash_amount
    assert all(e.validators[v].staked == staked_before[v] + slash for v in voters)   # every stake returned
    assert e.validators[contester.lower()].staked == 3 * E18


def test_rpc_vote_counts_by_index_search():
    """RpcChainClient finds the on-chain array lengths with reverting index getters."""
    from arbius_amd.chain.rpc import RpcChainClient, RpcError

    class Fake(RpcChainClient):
        def __init__(self, ny, nn):
            self.n = {"contestationVoteYeas": ny, "contestationVoteNays": nn}
            self._engine = "0x" + "11" * 20
            self.calls = 0

        async def _call(self, to, name, taskid, i):
            self.calls += 1
            if i >= self.n[name]:
                raise RpcError("execution reverted")
            return ["0x" + "22" * 20]

    for ny, nn in ((0, 0), (1, 0), (41, 1), (64, 65), (1000, 3)):
        f = Fake(ny, nn)
        assert asyncio.run(f.contestation_vote_counts("0x" + "33" * 32)) == (ny, nn)
        assert f.calls < 60
