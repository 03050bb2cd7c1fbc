"""The subset of the EngineV1 / BaseToken ABI the node uses:
function signatures, return tuples and event layouts (indexed/non-indexed)."""
from __future__ import annotations

from typing import Dict, List, Tuple

from . import abi

# name -> (signature, return types)
FUNCS: Dict[str, Tuple[str, List[str]]] = {
    "tasks": ("tasks(bytes32)", ["bytes32", "uint256", "address", "uint64", "uint8", "bytes"]),
    "solutions": ("solutions(bytes32)", ["address", "uint64", "bool", "bytes"]),
    "contestations": ("contestations(bytes32)", ["address", "uint64", "uint32", "uint256"]),
    "contestationVoted": ("contestationVoted(bytes32,address)", ["bool"]),
    "validators": ("validators(address)", ["uint256", "uint256", "address"]),
    "getValidatorMinimum": ("getValidatorMinimum()", ["uint256"]),
    "version": ("version()", ["uint256"]),
    "paused": ("paused()", ["bool"]),
    "getReward": ("getReward()", ["uint256"]),
    "getPsuedoTotalSupply": ("getPsuedoTotalSupply()", ["uint256"]),
    "generateCommitment": ("generateCommitment(address,bytes32,bytes)", ["bytes32"]),
    "generateIPFSCID": ("generateIPFSCID(bytes)", ["bytes"]),
    "models": ("models(bytes32)", ["uint256", "address", "uint256", "bytes"]),
    "accruedFees": ("accruedFees()", ["uint256"]),
    "validatorCanVote": ("validatorCanVote(address,bytes32)", ["uint256"]),
    # transactions
    "submitTask": ("submitTask(uint8,address,bytes32,uint256,bytes)", ["bytes32"]),
    "signalCommitment": ("signalCommitment(bytes32)", []),
    "submitSolution": ("submitSolution(bytes32,bytes)", []),
    "claimSolution": ("claimSolution(bytes32)", []),
    "submitContestation": ("submitContestation(bytes32)", []),
    "voteOnContestation": ("voteOnContestation(bytes32,bool)", []),
    "contestationVoteFinish": ("contestationVoteFinish(bytes32,uint32)", []),
    "validatorDeposit": ("validatorDeposit(address,uint256)", []),
    "registerModel": ("registerModel(address,uint256,bytes)", ["bytes32"]),
    "signalSupport": ("signalSupport(bytes32,bool)", []),
    "retractTask": ("retractTask(bytes32)", []),
    "withdrawAccruedFees": ("withdrawAccruedFees()", []),
    "setPaused": ("setPaused(bool)", []),
    "initiateValidatorWithdraw": ("initiateValidatorWithdraw(uint256)", ["uint256"]),
    "validatorWithdraw": ("validatorWithdraw(uint256,address)", []),
    "cancelValidatorWithdraw": ("cancelValidatorWithdraw(uint256)", []),
    # owner / admin (EngineV1.sol:264-383; contract/tasks/index.ts admin:* tasks)
    "transferOwnership": ("transferOwnership(address)", []),
    "transferTreasury": ("transferTreasury(address)", []),
    "transferPauser": ("transferPauser(address)", []),
    "setSolutionMineableRate": ("setSolutionMineableRate(bytes32,uint256)", []),
    "setVersion": ("setVersion(uint256)", []),
    "owner": ("owner()", ["address"]),
    "treasury": ("treasury()", ["address"]),
    "pauser": ("pauser()", ["address"]),
    # ERC20 (base token)
    "balanceOf": ("balanceOf(address)", ["uint256"]),
    "allowance": ("allowance(address,address)", ["uint256"]),
    "approve": ("approve(address,uint256)", ["bool"]),
    "transfer": ("transfer(address,uint256)", ["bool"]),
}


# the 10 uint256 parameter setters / getters (EngineV1.sol:313-383)
ENGINE_PARAMS = ['validatorMinimumPercentage', 'slashAmountPercentage', 'solutionFeePercentage', 'retractionFeePercentage', 'treasuryRewardPercentage', 'minClaimSolutionTime', 'minRetractionWaitTime', 'minContestationVotePeriodTime', 'maxContestationValidatorStakeSince', 'exitValidatorMinUnlockTime']
for _p in ENGINE_PARAMS:
    FUNCS["set" + _p[0].upper() + _p[1:]] = ("set" + _p[0].upper() + _p[1:] + "(uint256)", [])
    FUNCS[_p] = (_p + "()", ["uint256"])

# event -> (signature, [(name, type, indexed)])
EVENTS: Dict[str, Tuple[str, List[Tuple[str, str, bool]]]] = {
    "TaskSubmitted": ("TaskSubmitted(bytes32,bytes32,uint256,address)",
                      [("id", "bytes32", True), ("model", "bytes32", True), ("fee", "uint256", False),
                       ("sender", "address", True)]),
    "TaskRetracted": ("TaskRetracted(bytes32)", [("id", "bytes32", True)]),
    "SignalCommitment": ("SignalCommitment(address,bytes32)", [("addr", "address", True),
                                                                ("commitment", "bytes32", True)]),
    "SolutionSubmitted": ("SolutionSubmitted(address,bytes32)", [("addr", "address", True),
                                                                  ("task", "bytes32", True)]),
    "SolutionClaimed": ("SolutionClaimed(address,bytes32)", [("addr", "address", True), ("task", "bytes32", True)]),
    "ContestationSubmitted": ("ContestationSubmitted(address,bytes32)", [("addr", "address", True),
                                                                          ("task", "bytes32", True)]),
    "ContestationVote": ("ContestationVote(address,bytes32,bool)", [("addr", "address", True),
                                                                     ("task", "bytes32", True),
                                                                     ("yea", "bool", False)]),
    "ContestationVoteFinish": ("ContestationVoteFinish(bytes32,uint32,uint32)",
                               [("id", "bytes32", True), ("start_idx", "uint32", True), ("end_idx", "uint32", False)]),
    "VersionChanged": ("VersionChanged(uint256)", [("version", "uint256", False)]),
    "ModelRegistered": ("ModelRegistered(bytes32)", [("id", "bytes32", True)]),
    "ValidatorDeposit": ("ValidatorDeposit(address,address,uint256)",
                         [("addr", "address", True), ("validator", "address", True), ("amount", "uint256", False)]),
}

TOPIC_TO_EVENT = {abi.topic(sig): name for name, (sig, _) in EVENTS.items()}


def _word(t: str, v) -> bytes:
    return abi.encode([t], [v])


def encode_log(name: str, args: dict) -> Tuple[List[str], bytes]:
    sig, fields = EVENTS[name]
    topics = [abi.topic(sig)]
    data_t, data_v = [], []
    for fname, t, indexed in fields:
        v = args[fname]
        if t in ("address", "bytes32") and isinstance(v, str):
            v = bytes.fromhex(v[2:])
        if indexed:
            topics.append("0x" + _word(t, v).hex())
        else:
            data_t.append(t)
            data_v.append(v)
    return topics, abi.encode(data_t, data_v)


def decode_log(topics: List[str], data: bytes):
    name = TOPIC_TO_EVENT.get(topics[0].lower())
    if name is None:
        return None, None
    _, fields = EVENTS[name]
    args, ti = {}, 1
    data_fields = [(n, t) for n, t, ix in fields if not ix]
    dvals = abi.decode([t for _, t in data_fields], data) if data_fields else []
    di = 0
    for fname, t, indexed in fields:
        if indexed:
            raw = bytes.fromhex(topics[ti][2:])
            args[fname] = abi.decode([t], raw)[0]
            ti += 1
        else:
            args[fname] = dvals[di]
            di += 1
    return name, args
