"""The 13 Engine example integrations (contract/contracts/Example/*.sol) against MockEngine:
each twin is msg.sender for its call, as the example contract is on chain."""
import pytest

from arbius_amd.chain import examples as ex
from arbius_amd.chain.mock_engine import E18, MockEngine, MockToken, Revert
from arbius_amd.utils.protocol import generate_commitment

TEMPLATE = b'{"meta":{"title":"t"}}'
INPUT = b'{"prompt":"arbius test cat"}'
CID = "0x1220f4ad8a3bd3189da2ad909ee41148d6893d8c629c410f7f2c7e3fae75aade79c8"
DEPLOYER, TREASURY = "0x" + "01" * 20, "0x" + "02" * 20


@pytest.fixture
def env():
    tok = MockToken()
    e = MockEngine(tok, treasury=TREASURY, owner=DEPLOYER)
    tok.mint(DEPLOYER, 2000 * E18)
    tok.mint(e.address, 599990 * E18)     # engine holds the emission: pseudo supply 10 AIUS (base.test.ts:115-131)
    return e, tok


def _stake(e, tok, who, amount=int(2.4 * E18)):
    tok.transfer(DEPLOYER, who.address, amount)
    tok.approve(who.address, e.address, 2 ** 256 - 1)
    e.validator_deposit(who.address, who.address, amount)


def test_all_thirteen_examples_present():
    assert len(ex.ALL) == 13


def test_lifecycle_through_examples(env):
    e, tok = env
    reg = ex.RegisterModel(e)
    mid = reg.register_model(TEMPLATE)
    assert ex.LookupModelAddress(e).lookup_model_address(mid) == reg.address

    sub = ex.SubmitTask(e, tok, mid, INPUT)
    tok.transfer(DEPLOYER, sub.address, E18)
    tid = sub.submit_task()
    assert ex.LookupTaskCID(e).lookup_task_cid(tid) == e.get_task(tid).cid != "0x"

    solver = ex.SubmitSolution(e)
    _stake(e, tok, solver)
    assert ex.LookupValidatorStakedBalance(e).lookup_staked(solver.address) == int(2.4 * E18)
    solver.signal_commitment(generate_commitment(solver.address, tid, CID))
    solver.submit_solution(tid, CID)
    assert ex.LookupSolutionCID(e).lookup_solution_cid(tid) == CID

    claimer = ex.ClaimSolution(e)
    with pytest.raises(Revert):
        claimer.claim_solution(tid)                       # before minClaimSolutionTime
    e.increase_time(2001)
    claimer.claim_solution(tid)                           # anyone may trigger the claim
    assert e.get_solution(tid).claimed
    # the model fee (0.1 AIUS to the model contract, minus the treasury cut) reached it
    assert tok.balance_of(reg.address) > 0


def test_contestation_through_examples(env):
    e, tok = env
    mid = ex.RegisterModel(e).register_model(TEMPLATE)
    sub = ex.SubmitTask(e, tok, mid, INPUT)
    tok.transfer(DEPLOYER, sub.address, E18)
    tid = sub.submit_task()
    solver, contestor, voter = ex.SubmitSolution(e), ex.SubmitContestation(e), ex.VoteOnContestation(e)
    for v in (solver, contestor, voter):
        _stake(e, tok, v)
    solver.signal_commitment(generate_commitment(solver.address, tid, CID))
    solver.submit_solution(tid, CID)
    contestor.submit_contestation(tid)
    assert ex.LookupContestationValidator(e).lookup_contestation_validator(tid) == contestor.address
    voter.vote_on_contestation(tid, True)
    e.increase_time(4000)
    ex.FinishContestationVote(e).finish_vote(tid, 3)
    assert e.get_contestation(tid).finish_start_index == 3


def test_retract_through_example(env):
    e, tok = env
    mid = ex.RegisterModel(e).register_model(TEMPLATE)
    sub = ex.SubmitTask(e, tok, mid, INPUT)
    tok.transfer(DEPLOYER, sub.address, E18)
    tid = sub.submit_task()
    # RetractTask.sol calls retractTask from ITS address: only the task owner may retract
    with pytest.raises(Revert):
        ex.RetractTask(e).retract_task(tid)
    e.increase_time(10001)
    before = tok.balance_of(sub.address)
    ex.RetractTask(e, address=sub.address).retract_task(tid)
    assert e.get_task(tid).owner == "0x" + "00" * 20              # task deleted
    assert tok.balance_of(sub.address) - before == E18 // 10 - E18 // 100   # fee minus 10% retraction fee
