"""End-to-end plumbing on CPU (BASELINE config #1): MockEngine chain + MockIPFS +
the real orchestrator, with a fake GPU pool and with the real SD pipeline."""
import asyncio
import json

import pytest

from arbius_amd.chain.client import MockChainClient
from arbius_amd.chain.mock_engine import E18, MockEngine, MockToken
from arbius_amd.config.mining_config import MiningConfig
from arbius_amd.ipfs.pin import LocalPinner
from arbius_amd.ipfs.unixfs import cid_hex_to_str
from arbius_amd.node.miner import Miner
from arbius_amd.node.models import default_models, template_bytes
from arbius_amd.node.pool import FakeSolverPool, LocalSolverPool
from arbius_amd.store.db import DB

DEPLOYER, USER, MINER, MINER2, MINER3 = ("0x" + f"{i:040x}" for i in (1, 2, 3, 4, 5))


def make_world(model="anythingv3", supply_engine=597000):
    tok = MockToken()
    e = MockEngine(tok, owner=DEPLOYER)
    tok.mint(DEPLOYER, 2000 * E18)
    tok.mint(e.address, supply_engine * E18)
    tok.transfer(DEPLOYER, MINER, 10 * E18)
    tok.transfer(DEPLOYER, MINER2, 10 * E18)
    tok.transfer(DEPLOYER, MINER3, 10 * E18)
    tok.approve(USER, e.address, 2 ** 256 - 1)
    mid = e.register_model(USER, USER, 0, template_bytes(model))
    return e, tok, mid


def make_miner(e, mid, pool, addr=MINER, model="anythingv3", **cfg_over):
    cfg_over.setdefault("mi355x", {"selftest": False})
    cfg = MiningConfig.from_dict({"db_path": ":memory:", "evilmode": False, **cfg_over})
    m = Miner(cfg, DB(":memory:"), MockChainClient(e, addr), LocalPinner(), pool,
              default_models({model: mid}), clock=lambda: e.timestamp, retry_sleep=lambda s: asyncio.sleep(0))
    return m


def submit(e, mid, inp):
    return e.submit_task(USER, 0, USER, mid, 0, json.dumps(inp).encode())


async def _full_cycle(e, mid, miner, inp):
    await miner.boot()
    await miner.poll_events()          # first poll pins the cursor
    await miner.drain()                # validatorStake -> deposit
    assert e.validators[MINER.lower()].staked >= e.get_validator_minimum() > 0
    tid = submit(e, mid, inp)
    await miner.poll_events()
    await miner.drain()
    sol = e.solutions[tid]
    assert sol.validator == MINER.lower()
    e.increase_time(2200)
    await miner.drain()
    assert e.solutions[tid].claimed
    return tid


def test_e2e_fake_gpu():
    e, tok, mid = make_world()
    pool = FakeSolverPool()
    m = make_miner(e, mid, pool)
    tid = asyncio.run(_full_cycle(e, mid, m, {"prompt": "a cat", "negative_prompt": "x"}))
    # hydrated input: template defaults + seed (index.ts:174)
    (_, ctid, inp), = pool.calls
    assert ctid == tid and inp["width"] == 768 and inp["seed"] == int(tid, 16) % 0x1FFFFFFFFFFFF0
    # solution CID pinned to (mock) IPFS, same CID as on chain
    assert cid_hex_to_str(e.solutions[tid].cid) in m.pinner.pins
    # pinTaskInput pinned the raw input
    assert len(m.pinner.pins) == 2
    # our own SolutionSubmitted event is recorded like any other (index.ts:236-266)
    asyncio.run(m.poll_events())
    row = m.db.get_solution(tid)
    assert row is not None and row["validator"].lower() == MINER.lower() and row["cid"] == e.solutions[tid].cid
    assert m.metrics.counters.get("claims") == 1


def test_invalid_input_marked_and_not_solved():
    e, tok, mid = make_world()
    pool = FakeSolverPool()
    m = make_miner(e, mid, pool)

    async def go():
        await m.boot()
        await m.poll_events()
        await m.drain()
        tid = e.submit_task(USER, 0, USER, mid, 0, b"{not json")
        tid2 = submit(e, mid, {"negative_prompt": "x"})  # missing required prompt
        await m.poll_events()
        await m.drain()
        return tid, tid2

    tid, tid2 = asyncio.run(go())
    assert m.db.get_invalid_task(tid) and m.db.get_invalid_task(tid2)
    assert pool.calls == []


def test_evil_solution_gets_contested_and_slashed():
    """Miner2 in evilmode submits the bogus CID; honest miner re-solves, sees a different
    CID, contests; after the vote period the contestation succeeds."""
    e, tok, mid = make_world()
    honest = make_miner(e, mid, FakeSolverPool(), MINER, mi355x={"verify_fraction": 1.0})
    evil = make_miner(e, mid, FakeSolverPool(), MINER2, evilmode=True)
    voter = make_miner(e, mid, FakeSolverPool(), MINER3, mi355x={"verify_fraction": 1.0})

    async def go():
        for m in (honest, evil, voter):
            await m.boot()
            await m.poll_events()
            await m.drain()
        tid = submit(e, mid, {"prompt": "p", "negative_prompt": "n"})
        await evil.poll_events()
        await evil.drain()                 # evil solves first
        assert e.solutions[tid].cid == "0x1220" + "66" * 32
        await honest.poll_events()
        await honest.drain()               # honest: submit fails -> CID mismatch -> contest
        assert e.contestations[tid].validator == MINER.lower()
        await voter.poll_events()
        await voter.drain()                # third miner verifies and votes yea
        assert e.contestation_voted.get((tid, MINER3.lower()))
        e.increase_time(5100)
        await honest.drain()               # contestationVoteFinish job
        return tid

    tid = asyncio.run(go())
    c = e.contestations[tid]
    assert c.finish_start_index >= 1
    # 2 yeas vs 1 nay: contestation succeeds, the evil solver is slashed, yeas refunded + rewarded
    assert e.validators[MINER.lower()].staked > e.validators[MINER2.lower()].staked
    assert tok.balance_of(MINER) > 0


def test_solve_failure_goes_to_failed_jobs():
    e, tok, mid = make_world()
    pool = FakeSolverPool()
    pool.fail_next = 100
    m = make_miner(e, mid, pool)

    async def go():
        await m.boot()
        await m.poll_events()
        await m.drain()
        submit(e, mid, {"prompt": "p", "negative_prompt": "n"})
        await m.poll_events()
        await m.drain()

    asyncio.run(go())
    assert [j["method"] for j in m.db.get_failed_jobs()] == ["solve"]


def test_e2e_real_pipeline_tiny_cpu():
    """The real SD-architecture pipeline (tiny widths) through the whole node."""
    e, tok, mid = make_world()
    pool = LocalSolverPool("cpu", tiny=True)
    m = make_miner(e, mid, pool)
    inp = {"prompt": "arbius test cat", "negative_prompt": "n", "width": 128, "height": 128,
           "num_inference_steps": 2, "scheduler": "DDIM"}
    tid = asyncio.run(_full_cycle(e, mid, m, inp))
    # determinism: re-solving the same task gives the same CID
    model = m.models[mid.lower()]
    row = json.loads(m.db.get_task_input(tid, e.tasks[tid].cid)["data"])
    assert pool.solve_sync(model, tid, row).cid == e.solutions[tid].cid


@pytest.mark.slow
def test_config1_full_arch_64px_2step_ddim_cpu():
    """BASELINE config #1: anythingv3 (full SD1.5 architecture) 64x64, 2-step DDIM on CPU."""
    e, tok, mid = make_world()
    pool = LocalSolverPool("cpu", tiny=False)
    m = make_miner(e, mid, pool)
    inp = {"prompt": "arbius test cat", "negative_prompt": "n", "width": 128, "height": 128,
           "num_inference_steps": 2, "scheduler": "DDIM"}
    # template enum has no 64 -> smallest legal 128x128 image (latent 16x16)
    asyncio.run(_full_cycle(e, mid, m, inp))


def test_concurrent_forks_match_solo():
    """Pipeline forks solving tasks concurrently (threads; private streams on GPU) give the
    same bytes as a solo solve - concurrency never changes a CID."""
    from concurrent.futures import ThreadPoolExecutor
    from arbius_amd.models.registry import build_pipeline
    from arbius_amd.node.solver import solve_image
    pipe = build_pipeline("anythingv3", tiny=True)
    inps = [{"prompt": f"cat {i}", "negative_prompt": "", "width": 128, "height": 128, "num_inference_steps": 2,
             "guidance_scale": 7.5, "scheduler": "DDIM", "seed": 10 + i} for i in range(3)]
    solo = [solve_image(pipe, inp).cid for inp in inps]
    forks = [pipe.fork() for _ in range(3)]
    with ThreadPoolExecutor(3) as ex:
        conc = list(ex.map(lambda a: solve_image(a[0], a[1]).cid, zip(forks, inps)))
    assert conc == solo


def test_boot_selftest_pins_per_hardware_cid(tmp_path):
    """Boot self-test: unknown hardware/weights key -> computed CID logged; pinned key with a
    wrong CID -> the node refuses to start (miner/src/index.ts:995-1000)."""
    e, tok, mid = make_world("kandinsky2")
    pool = FakeSolverPool()
    m = make_miner(e, mid, pool, model="kandinsky2", mi355x={"selftest": True})
    asyncio.run(m.boot())
    assert m.metrics.counters["selftests_run"] == 1
    got = pool.calls[-1]
    assert got[2]["prompt"] == "arbius test cat" and got[2]["seed"] == 1337 and got[2]["width"] == 768
    table = {"kandinsky2": {"input": {"prompt": "arbius test cat", "seed": 1337},
                            "expected": {"fake/synthetic": "0x1220" + "00" * 32}}}
    p = tmp_path / "t.json"
    p.write_text(json.dumps(table))
    m2 = make_miner(e, mid, FakeSolverPool(), model="kandinsky2",
                    mi355x={"selftest": True, "selftest_table": str(p)})
    with pytest.raises(SystemExit):
        asyncio.run(m2.boot())


def test_lockstep_group_matches_solo_on_cpu_reference():
    """run_group's bookkeeping (per-task noise, sampler state, guidance, VAE) on the CPU fp32
    reference path: images equal the solo ones up to CPU GEMM batch rounding (<= 1 level)."""
    import numpy as np
    from arbius_amd.models.registry import build_pipeline
    pipe = build_pipeline("anythingv3", tiny=True)
    inps = [{"prompt": f"cat {i}", "negative_prompt": "", "width": 64, "height": 64, "num_inference_steps": 3,
             "guidance_scale": 7.5 + i, "scheduler": "DPMSolverMultistep", "seed": 10 + i} for i in range(3)]
    solo = [pipe(prompt=i["prompt"], negative_prompt="", width=64, height=64, num_inference_steps=3,
                 guidance_scale=i["guidance_scale"], scheduler="DPMSolverMultistep", seed=i["seed"]) for i in inps]
    grp = pipe.run_group(inps)
    for a, b in zip(solo, grp):
        assert np.abs(a.astype(int) - b.astype(int)).max() <= 1
    import pytest
    with pytest.raises(ValueError):
        pipe.run_group([inps[0], dict(inps[1], num_inference_steps=4)])
