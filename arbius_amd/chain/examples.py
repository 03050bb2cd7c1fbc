"""Engine integrations: the 13 minimal caller contracts of ``contract/contracts/Example/*.sol``
 as Python objects with their own address, driving an in-process ``MockEngine``
(or anything with the same method surface).  Each mirrors one Solidity example: the object is
``msg.sender`` for the engine, exactly as the example contract is on chain.

=============================  ===========================================================
Example contract               Python twin
=============================  ===========================================================
SubmitTask.sol:6-33            ``SubmitTask(engine, token, model, input).submit_task()``
RegisterModel.sol              ``RegisterModel(engine).register_model(template)`` (fee 0.1)
RetractTask.sol                ``RetractTask(engine).retract_task(taskid)``
SubmitSolution.sol             ``SubmitSolution(engine).signal_commitment / submit_solution``
ClaimSolution.sol              ``ClaimSolution(engine).claim_solution(taskid)``
SubmitContestation.sol         ``SubmitContestation(engine).submit_contestation(taskid)``
VoteOnContestation.sol         ``VoteOnContestation(engine).vote_on_contestation(taskid, agree)``
FinishContestationVote.sol     ``FinishContestationVote(engine).finish_vote(taskid, iterations)``
LookupModelAddress.sol         ``LookupModelAddress(engine).lookup_model_address(modelid)``
LookupTaskCID.sol              ``LookupTaskCID(engine).lookup_task_cid(taskid)``
LookupSolutionCID.sol          ``LookupSolutionCID(engine).lookup_solution_cid(taskid)``
LookupContestationValidator    ``LookupContestationValidator(engine).lookup_contestation_validator``
LookupValidatorStakedBalance   ``LookupValidatorStakedBalance(engine).lookup_staked(validator)``
=============================  ===========================================================
"""
from __future__ import annotations

import itertools

E18 = 10 ** 18
_ids = itertools.count(0xE000)


class _Integration:
    """A caller contract: a fresh address of its own (CREATE), the engine handle."""

    def __init__(self, engine, address: str | None = None):
        self.engine = engine
        self.address = address or "0x" + f"{next(_ids):040x}"


class SubmitTask(_Integration):
    """SubmitTask.sol:6-33: approves the engine for max, submits version 0 with fee 0.1 AIUS.

    The transaction that carries it is an EOA's call of the contract's ``submitTask()``, not of the
    engine's ``submitTask(uint8,address,bytes32,uint256,bytes)``: its calldata holds no task input
    (the reference miner throws on it).  The engine's transaction record is
    rewritten to that outer call, so a node has to recover the input by the task's on-chain CID."""

    SELECTOR_SIG = "submitTask()"

    def __init__(self, engine, token, model: str, input_: bytes, address: str | None = None,
                 caller: str = "0x" + "ca" * 20):
        super().__init__(engine, address)
        self.token, self.model, self.input, self.caller = token, model, input_, caller

    def submit_task(self) -> str:
        self.token.approve(self.address, self.engine.address, 2 ** 256 - 1)
        tid = self.engine.submit_task(self.address, 0, self.address, self.model, E18 // 10, self.input)
        txin = getattr(self.engine, "_tx_inputs", None)
        if txin is not None:
            tx = next(ev.tx for ev in reversed(self.engine.events) if ev.name == "TaskSubmitted")
            txin[tx] = (self.SELECTOR_SIG, (self.address,), self.caller)
        return tid


class RegisterModel(_Integration):
    def register_model(self, template: bytes) -> str:
        return self.engine.register_model(self.address, self.address, E18 // 10, template)


class RetractTask(_Integration):
    def retract_task(self, taskid: str):
        return self.engine.retract_task(self.address, taskid)


class SubmitSolution(_Integration):
    def signal_commitment(self, commitment: str):
        return self.engine.signal_commitment(self.address, commitment)

    def submit_solution(self, taskid: str, cid: str):
        return self.engine.submit_solution(self.address, taskid, cid)


class ClaimSolution(_Integration):
    def claim_solution(self, taskid: str):
        return self.engine.claim_solution(self.address, taskid)


class SubmitContestation(_Integration):
    def submit_contestation(self, taskid: str):
        return self.engine.submit_contestation(self.address, taskid)


class VoteOnContestation(_Integration):
    def vote_on_contestation(self, taskid: str, agree: bool):
        return self.engine.vote_on_contestation(self.address, taskid, agree)


class FinishContestationVote(_Integration):
    def finish_vote(self, taskid: str, iterations: int):
        return self.engine.contestation_vote_finish(self.address, taskid, iterations)


class LookupModelAddress(_Integration):
    def lookup_model_address(self, modelid: str) -> str:
        m = self.engine.models.get(modelid)
        return m.addr if m is not None else "0x" + "00" * 20


class LookupTaskCID(_Integration):
    def lookup_task_cid(self, taskid: str) -> str:
        return self.engine.get_task(taskid).cid


class LookupSolutionCID(_Integration):
    def lookup_solution_cid(self, taskid: str) -> str:
        return self.engine.get_solution(taskid).cid


class LookupContestationValidator(_Integration):
    def lookup_contestation_validator(self, taskid: str) -> str:
        return self.engine.get_contestation(taskid).validator


class LookupValidatorStakedBalance(_Integration):
    def lookup_staked(self, validator: str) -> int:
        return self.engine.get_validator(validator).staked


ALL = (SubmitTask, RegisterModel, RetractTask, SubmitSolution, ClaimSolution, SubmitContestation,
       VoteOnContestation, FinishContestationVote, LookupModelAddress, LookupTaskCID, LookupSolutionCID,
       LookupContestationValidator, LookupValidatorStakedBalance)
