"""The EngineV1 ABI (all 77 functions and 31 events of
``miner/src/artifacts/contracts/EngineV1.sol/EngineV1.json``; events declared at
``contract/contracts/EngineV1.sol:141-206`` plus OpenZeppelin's ``Initialized`` /
``OwnershipTransferred``) and the BaseToken ERC20 calls the node makes:
function signatures, return tuples and event layouts (indexed/non-indexed).
``tests/test_engine_abi.py`` checks every selector, return list and topic against the artifact."""
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
    # remaining public getters / pure helpers / init (EngineV1.sol:70-137, 387-543)
    "baseToken": ("baseToken()", ["address"]),
    "prevhash": ("prevhash()", ["bytes32"]),
    "startBlockTime": ("startBlockTime()", ["uint64"]),
    "commitments": ("commitments(bytes32)", ["uint256"]),
    "contestationVoteYeas": ("contestationVoteYeas(bytes32,uint256)", ["address"]),
    "contestationVoteNays": ("contestationVoteNays(bytes32,uint256)", ["address"]),
    "contestationVotedIndex": ("contestationVotedIndex(bytes32)", ["uint256"]),
    "pendingValidatorWithdrawRequests": ("pendingValidatorWithdrawRequests(address,uint256)", ["uint256", "uint256"]),
    "pendingValidatorWithdrawRequestsCount": ("pendingValidatorWithdrawRequestsCount(address)", ["uint256"]),
    "validatorWithdrawPendingAmount": ("validatorWithdrawPendingAmount(address)", ["uint256"]),
    "getSlashAmount": ("getSlashAmount()", ["uint256"]),
    "diffMul": ("diffMul(uint256,uint256)", ["uint256"]),
    "reward": ("reward(uint256,uint256)", ["uint256"]),
    "targetTs": ("targetTs(uint256)", ["uint256"]),
    "hashModel": ("hashModel((uint256,address,uint256,bytes),address)", ["bytes32"]),
    "hashTask": ("hashTask((bytes32,uint256,address,uint64,uint8,bytes),address,bytes32)", ["bytes32"]),
    "initialize": ("initialize(address,address)", []),
    "renounceOwnership": ("renounceOwnership()", []),
    # ERC20 (base token)
    "balanceOf": ("balanceOf(address)", ["uint256"]),
    "allowance": ("allowance(address,address)", ["uint256"]),
    "approve": ("approve(address,uint256)", ["bool"]),
    "transfer": ("transfer(address,uint256)", ["bool"]),
}


# the 10 uint256 parameter setters / getters (EngineV1.sol:313-383)
ENGINE_PARAMS = [
    'validatorMinimumPercentage',
    'slashAmountPercentage',
    'solutionFeePercentage',
    'retractionFeePercentage',
    'treasuryRewardPercentage',
    'minClaimSolutionTime',
    'minRetractionWaitTime',
    'minContestationVotePeriodTime',
    'maxContestationValidatorStakeSince',
    'exitValidatorMinUnlockTime',
]
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
    "ValidatorWithdrawInitiated": ("ValidatorWithdrawInitiated(address,uint256,uint256,uint256)",
                                   [("addr", "address", True), ("count", "uint256", True),
                                    ("unlockTime", "uint256", False), ("amount", "uint256", False)]),
    "ValidatorWithdrawCancelled": ("ValidatorWithdrawCancelled(address,uint256)",
                                   [("addr", "address", True), ("count", "uint256", True)]),
    "ValidatorWithdraw": ("ValidatorWithdraw(address,address,uint256,uint256)",
                          [("addr", "address", True), ("to", "address", True), ("count", "uint256", True),
                           ("amount", "uint256", False)]),
    "SignalSupport": ("SignalSupport(address,bytes32,bool)",
                      [("addr", "address", True), ("model", "bytes32", True), ("supported", "bool", False)]),
    "TreasuryTransferred": ("TreasuryTransferred(address)", [("to", "address", True)]),
    "PauserTransferred": ("PauserTransferred(address)", [("to", "address", True)]),
    "PausedChanged": ("PausedChanged(bool)", [("paused", "bool", True)]),
    "SolutionMineableRateChange": ("SolutionMineableRateChange(bytes32,uint256)",
                                   [("id", "bytes32", True), ("rate", "uint256", False)]),
    "Initialized": ("Initialized(uint8)", [("version", "uint8", False)]),
    "OwnershipTransferred": ("OwnershipTransferred(address,address)",
                             [("previousOwner", "address", True), ("newOwner", "address", True)]),
}
# the 10 parameter setters emit <Param>Changed(uint256 indexed amount) (EngineV1.sol:193-206)
for _p in ENGINE_PARAMS:
    _e = _p[0].upper() + _p[1:] + "Changed"
    EVENTS[_e] = (_e + "(uint256)", [("amount", "uint256", True)])

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
