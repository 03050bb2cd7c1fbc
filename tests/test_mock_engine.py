"""MockEngine scenarios re-created from the reference contract tests
(contract/test/base.test.ts, reward.test.ts) - run
against the Python twin of EngineV1 with hardhat-style time travel."""
import pytest

from arbius_amd.chain.mock_engine import E18, MockEngine, MockToken, Revert
from arbius_amd.utils.protocol import generate_commitment

TESTBUF = bytes.fromhex("746573740a")  # base.test.ts:10
TESTCID = "0x1220f4ad8a3bd3189da2ad909ee41148d6893d8c629c410f7f2c7e3fae75aade79c8"


def A(n):
    return "0x" + f"{n:040x}"


DEPLOYER, USER1, USER2, V1, V2, V3, V4, TREASURY, MODEL1 = (A(i) for i in range(1, 10))


def eth(x):
    from decimal import Decimal
    return int(Decimal(str(x)) * E18)


@pytest.fixture
def env():
    tok = MockToken()
    e = MockEngine(tok, treasury=TREASURY, owner=DEPLOYER)
    tok.mint(DEPLOYER, eth(2000))
    for a in (USER1, USER2, V1, V2, V3, V4):
        tok.approve(a, e.address, 2 ** 256 - 1)
    return e, tok


def bootstrap_model(e, fee=0):
    return e.register_model(USER1, USER1, fee, TESTBUF)


def bootstrap_validator(e, tok, v=V1, mint=eth(599990), amount=eth(2.4)):
    if mint:
        tok.mint(e.address, mint)
    tok.transfer(DEPLOYER, v, amount)
    e.validator_deposit(v, v, amount)


def bootstrap_task(e, modelid, fee=0):
    return e.submit_task(USER1, 0, USER1, modelid, fee, TESTBUF)


def solve(e, v, taskid, cid=TESTCID):
    e.signal_commitment(v, generate_commitment(v, taskid, cid))
    e.submit_solution(v, taskid, cid)


def test_reinitialize_reverts(env):
    e, _ = env
    with pytest.raises(Revert, match="already initialized"):
        e.initialize()


def test_model_register_id(env):
    e, _ = env
    mid = bootstrap_model(e)
    assert mid == MockEngine.hash_model(USER1, 0, TESTCID, USER1)
    assert e.models[mid].cid == TESTCID
    assert e.events[-1].name == "ModelRegistered"
    with pytest.raises(Revert, match="model already registered"):
        bootstrap_model(e)
    e.set_paused(DEPLOYER, True)
    with pytest.raises(Revert, match="paused"):
        e.register_model(USER2, USER2, 0, b"x")


def test_validator_deposit_and_exit(env):
    e, tok = env
    bootstrap_validator(e, tok)
    assert e.validators[V1.lower()].staked == eth(2.4)
    e.set_paused(DEPLOYER, True)
    with pytest.raises(Revert, match="paused"):
        e.initiate_validator_withdraw(V1, eth(1))
    e.set_paused(DEPLOYER, False)
    cnt = e.initiate_validator_withdraw(V1, eth(1))
    with pytest.raises(Revert, match="wait longer"):
        e.validator_withdraw(V1, cnt, V1)
    e.increase_time(86400)
    e.validator_withdraw(V1, cnt, V1)
    assert tok.balance_of(V1) == eth(1)
    with pytest.raises(Revert, match="request not exist"):
        e.validator_withdraw(V1, cnt, V1)


def test_task_lifecycle_and_claim(env):
    e, tok = env
    bootstrap_validator(e, tok)
    mid = bootstrap_model(e)
    tid = bootstrap_task(e, mid)
    assert e.events[-1].name == "TaskSubmitted" and e.events[-1].args["id"] == tid
    # commitment must be in a strictly earlier block
    c = generate_commitment(V1, tid, TESTCID)
    with pytest.raises(Revert, match="non existent commitment"):
        e.submit_solution(V1, tid, TESTCID)
    e.signal_commitment(V1, c)
    with pytest.raises(Revert, match="commitment exists"):
        e.signal_commitment(V1, c)
    e.submit_solution(V1, tid, TESTCID)
    with pytest.raises(Revert, match="solution already submitted"):
        e.submit_solution(V1, tid, TESTCID)
    with pytest.raises(Revert, match="not enough delay"):
        e.claim_solution(V1, tid)
    e.increase_time(3600)
    e.set_paused(DEPLOYER, True)
    with pytest.raises(Revert, match="paused"):
        e.claim_solution(V1, tid)
    e.set_paused(DEPLOYER, False)
    e.claim_solution(V1, tid)
    assert e.events[-1].name == "SolutionClaimed"
    with pytest.raises(Revert, match="already claimed"):
        e.claim_solution(V1, tid)


def test_retract(env):
    e, tok = env
    mid = bootstrap_model(e)
    tid = bootstrap_task(e, mid)
    with pytest.raises(Revert, match="did not wait long enough"):
        e.retract_task(USER1, tid)
    with pytest.raises(Revert, match="not owner"):
        e.retract_task(USER2, tid)
    e.increase_time(10010)
    e.retract_task(USER1, tid)
    assert e.events[-1].name == "TaskRetracted"


def test_fee_split_golden(env):
    # base.test.ts:911-981: task fee 4, model fee 3 -> model 3, solver 0.9, accrued 0.1
    e, tok = env
    bootstrap_validator(e, tok)
    mid = e.register_model(USER1, MODEL1, eth(3), TESTBUF)
    tok.transfer(DEPLOYER, USER1, eth(4))
    with pytest.raises(Revert, match="lower fee than model fee"):
        e.submit_task(USER1, 0, USER1, mid, eth(2), bytes.fromhex(TESTCID[2:]))
    tid = e.submit_task(USER1, 0, USER1, mid, eth(4), bytes.fromhex(TESTCID[2:]))
    solve(e, V1, tid)
    e.increase_time(3600)
    e.claim_solution(V1, tid)
    assert tok.balance_of(USER1) == 0
    assert tok.balance_of(MODEL1) == eth(3)
    assert tok.balance_of(V1) == eth(0.9)
    assert e.accrued_fees == eth(0.1)


def test_claim_with_reward_golden():
    # reward.test.ts:189-231: rate 0.1 -> validator 8.999999999999999999, treasury 1
    tok = MockToken()
    e = MockEngine(tok, treasury=TREASURY, owner=DEPLOYER)
    tok.mint(e.address, eth("599999.999999999999999999"))
    tok.mint(DEPLOYER, eth(2000))
    tok.approve(V1, e.address, 2 ** 256 - 1)
    e.validator_deposit(V1, V1, 0)
    mid = e.register_model(USER1, USER1, 0, TESTBUF)
    tid = e.submit_task(USER1, 0, USER1, mid, 0, TESTBUF)
    e.set_solution_mineable_rate(DEPLOYER, mid, eth(0.1))
    solve(e, V1, tid)
    e.increase_time(3600)
    assert tok.balance_of(V1) == 0
    e.claim_solution(V1, tid)
    assert tok.balance_of(V1) == eth("8.999999999999999999")
    assert tok.balance_of(TREASURY) == eth(1)


def _slashing_setup(env, n_validators=4):
    e, tok = env
    tok.mint(e.address, eth(597000))  # deployBootstrapEngineSlashingReached
    mid = bootstrap_model(e)
    tid = bootstrap_task(e, mid)
    e.set_solution_mineable_rate(DEPLOYER, mid, eth(1))
    vs = [V1, V2, V3, V4][:n_validators]
    for v in vs:
        tok.transfer(DEPLOYER, v, eth(2.4))
        e.validator_deposit(v, v, eth(2.4))
    solve(e, V1, tid)
    return e, tok, tid


def test_contestation_paginated_finish_golden(env):
    # base.test.ts:2931-3070 (3 yeas vs 1 nay, slashing reached): originator 0.14952, others 0.07476
    e, tok, tid = _slashing_setup(env)
    assert e.get_slash_amount() == eth(0.29904)
    e.submit_contestation(V2, tid)
    e.vote_on_contestation(V3, tid, True)
    e.vote_on_contestation(V4, tid, True)
    assert e.validators[V1.lower()].staked == eth(2.10096)
    with pytest.raises(Revert, match="voting period not ended"):
        e.contestation_vote_finish(V1, tid, 1)
    e.increase_time(4000)
    with pytest.raises(Revert, match="amnt too small"):
        e.contestation_vote_finish(V1, tid, 0)
    e.contestation_vote_finish(V1, tid, 1)
    assert tok.balance_of(V2) == eth(0.14952)
    assert e.validators[V2.lower()].staked == eth(2.4)
    assert e.validators[V3.lower()].staked == eth(2.10096)
    assert e.contestations[tid].finish_start_index == 1
    e.contestation_vote_finish(V1, tid, 1)
    assert tok.balance_of(V3) == eth(0.07476)
    e.contestation_vote_finish(V1, tid, 1)
    assert tok.balance_of(V4) == eth(0.07476)
    assert e.validators[V4.lower()].staked == eth(2.4)
    e.contestation_vote_finish(V1, tid, 1)  # fourth iteration does nothing
    assert e.contestations[tid].finish_start_index == 4
    assert tok.balance_of(V1) == 0 and e.validators[V1.lower()].staked == eth(2.10096)


def test_contestation_blocks_claim_and_failed_contestation_pays_solver(env):
    e, tok, tid = _slashing_setup(env, 3)
    e.submit_contestation(V2, tid)
    e.vote_on_contestation(V3, tid, False)  # 1 yea vs 2 nays -> contestation fails
    e.increase_time(3600)
    with pytest.raises(Revert, match="has contestation"):
        e.claim_solution(V1, tid)
    assert e.validator_can_vote(V3, tid) == 3  # already voted
    with pytest.raises(Revert, match="min staked too low"):  # vote debited the slash: below minimum now
        e.vote_on_contestation(V3, tid, False)
    e.increase_time(4000)
    e.contestation_vote_finish(V1, tid, 10)
    slash = e.contestations[tid].slash_amount
    # accused (nays[0]) gets yea*slash/2, other nay the rest; solver also claims normally (reward, rate 1)
    assert e.validators[V1.lower()].staked == eth(2.4)
    assert e.validators[V2.lower()].staked == eth(2.4) - slash
    assert tok.balance_of(V3) == slash - slash // 2


def test_validator_can_vote_codes(env):
    e, tok, tid = _slashing_setup(env, 2)
    assert e.validator_can_vote(V3, tid) == 1  # no contestation
    e.submit_contestation(V2, tid)
    assert e.validator_can_vote(V2, tid) == 3  # already voted
    assert e.validator_can_vote(V3, tid) == 4  # never staked
    e.increase_time(4001)
    assert e.validator_can_vote(V3, tid) == 2  # period ended


def test_contest_errors(env):
    e, tok, tid = _slashing_setup(env, 2)
    with pytest.raises(Revert, match="solution does not exist"):
        e.submit_contestation(V2, "0x" + "ab" * 32)
    with pytest.raises(Revert, match="min staked too low"):
        e.submit_contestation(USER2, tid)
    e.increase_time(2001)
    with pytest.raises(Revert, match="too late"):
        e.submit_contestation(V2, tid)


def test_admin_setters(env):
    e, _ = env
    with pytest.raises(Revert, match="not the owner"):
        e.set_version(USER1, 1)
    e.set_version(DEPLOYER, 2)
    assert e.version == 2 and e.events[-1].name == "VersionChanged"
    for name in MockEngine._PARAMS:
        e.set_param(DEPLOYER, name, 7)
        assert getattr(e, name) == 7
        with pytest.raises(Revert):
            e.set_param(USER1, name, 8)
    with pytest.raises(Revert, match="not pauser"):
        e.set_paused(USER1, True)
    e.transfer_pauser(DEPLOYER, USER2)
    e.set_paused(USER2, True)
    assert e.paused
