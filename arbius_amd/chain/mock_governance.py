"""Governance twins: ``BaseTokenV1`` (ERC20 + Permit + Votes, bridge mint/burn),
``TimelockV1`` (OZ 4.9 ``TimelockController``) and ``GovernorV1`` (OZ 4.9 Governor +
GovernorCompatibilityBravo + Settings + VotesQuorumFraction + TimelockControl).

Reference contracts: ``contract/contracts/BaseTokenV1.sol:11-99``,
``contract/contracts/TimelockV1.sol:6-17``, ``contract/contracts/GovernorV1.sol:12-184``;
scenarios: ``contract/test/governance.test.ts:27-444`` (tests/test_governance.py).

The three share the MockEngine's clock (block number for Governor/Votes snapshots,
block timestamp for Timelock ETAs): ``engine.mine(n)`` is ``hardhat_mine``,
``engine.increase_time(s)`` is ``evm_increaseTime`` + ``evm_mine``; every state-changing call
mines one block (hardhat automine).  Calls scheduled through the Timelock are real ABI
calldata, dispatched by selector to whichever mock owns the target address, with
``msg.sender`` = the timelock - exactly how ``setSolutionMineableRate`` reaches the Engine
after a successful vote.  Revert strings are OZ 4.9's.
"""
from __future__ import annotations

import bisect
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from ..ipfs.unixfs import onchain_cid
from ..utils.keccak import keccak256
from . import abi
from .mock_engine import ZERO, ZERO32, Event, MockEngine, MockToken, Revert, _addr, _h32
from .secp256k1 import recover_address

MAX_UINT256 = 2 ** 256 - 1


def tx(fn):
    """A state-changing entry point: mines one block (hardhat automine) unless it runs inside
    another transaction (a Timelock/Governor call chain), and marks the clock as "in a tx" so
    views evaluate ``block.number`` as the tx's block instead of the pending block."""
    def wrapped(self, *a, **k):
        clock = self.clock
        if clock is None:
            return fn(self, *a, **k)
        depth = getattr(clock, "_txdepth", 0)
        if depth == 0:
            clock._tx()
        clock._txdepth = depth + 1
        try:
            return fn(self, *a, **k)
        finally:
            clock._txdepth = depth
    wrapped.__name__, wrapped.__doc__ = fn.__name__, fn.__doc__
    return wrapped


def view_block(clock) -> int:
    """``block.number`` as a view sees it: the tx's block inside a tx, else hardhat's pending
    block (eth_call runs on top of the latest block)."""
    return clock.block_number + (0 if getattr(clock, "_txdepth", 0) else 1)


def _role(name: str) -> str:
    return "0x" + keccak256(name.encode()).hex()


TIMELOCK_ADMIN_ROLE = _role("TIMELOCK_ADMIN_ROLE")
PROPOSER_ROLE = _role("PROPOSER_ROLE")
EXECUTOR_ROLE = _role("EXECUTOR_ROLE")
CANCELLER_ROLE = _role("CANCELLER_ROLE")
DEFAULT_ADMIN_ROLE = ZERO32
_DONE_TIMESTAMP = 1


class Registry:
    """Address -> mock contract, for calls made by the Timelock (``_execute`` low-level call)."""

    def __init__(self, clock: MockEngine):
        self.clock = clock
        self.contracts: Dict[str, object] = {clock.address: clock}

    def add(self, c):
        self.contracts[_addr(c.address)] = c
        return c

    def call(self, sender: str, target: str, value: int, data: bytes):
        c = self.contracts.get(_addr(target))
        if c is None:
            if data:
                raise Revert("Address: call to non-contract")
            return None            # plain value transfer to an EOA
        return dispatch(c, sender, data)


# selector table per contract class: signature -> (method name, arg adapter)
_ENGINE_ABI = {
    "setSolutionMineableRate(bytes32,uint256)": "set_solution_mineable_rate",
    "setPaused(bool)": "set_paused",
    "setVersion(uint256)": "set_version",
    "transferOwnership(address)": "transfer_ownership",
    "transferTreasury(address)": "transfer_treasury",
    "transferPauser(address)": "transfer_pauser",
    "withdrawAccruedFees()": "withdraw_accrued_fees",
}
_ENGINE_PARAMS = ("validatorMinimumPercentage", "slashAmountPercentage", "solutionFeePercentage",
                  "retractionFeePercentage", "treasuryRewardPercentage", "minClaimSolutionTime",
                  "minRetractionWaitTime", "minContestationVotePeriodTime",
                  "maxContestationValidatorStakeSince", "exitValidatorMinUnlockTime")


def dispatch(contract, sender: str, data: bytes):
    """Decode ``data`` against the contract's ABI table and run the method as ``sender``."""
    table = getattr(contract, "ABI", None)
    if table is None and isinstance(contract, MockEngine):
        table = dict(_ENGINE_ABI)
        for p in _ENGINE_PARAMS:
            table[f"set{p[0].upper()}{p[1:]}(uint256)"] = ("set_param", p)
    sel = bytes(data[:4])
    for sig, meth in (table or {}).items():
        if abi.selector(sig) == sel:
            args = abi.decode_call(sig, bytes(data))
            if isinstance(meth, tuple):          # MockEngine.set_param(sender, name, amount)
                name, pname = meth
                return getattr(contract, name)(sender, _snake(pname), *args)
            return getattr(contract, meth)(sender, *args)
    raise Revert("function selector was not recognized and there's no fallback function")


def call_view(contract, data: bytes) -> bytes:
    """eth_call against a twin's ``VIEWS`` table: signature -> (method, return types)."""
    sel = bytes(data[:4])
    for sig, (meth, rets) in getattr(contract, "VIEWS", {}).items():
        if abi.selector(sig) == sel:
            out = getattr(contract, meth)(*abi.decode_call(sig, bytes(data)))
            return abi.encode(rets, list(out) if isinstance(out, tuple) else [out])
    raise Revert("unsupported view")


def _snake(camel: str) -> str:
    return "".join("_" + ch.lower() if ch.isupper() else ch for ch in camel)


# ---------------------------------------------------------------------------------------------
@dataclass
class Checkpoint:
    from_block: int
    votes: int


class MockBaseToken(MockToken):
    """BaseTokenV1: OZ ERC20Upgradeable + ERC20PermitUpgradeable + ERC20VotesUpgradeable +
    Ownable; ``bridgeMint``/``bridgeBurn`` only from the L2 gateway (BaseTokenV1.sol:53-68)."""

    ADDRESS = "0xe3dbc4f88eaa632ddf9708732e2832eeaa6688ab"
    ABI = {
        "transfer(address,uint256)": "transfer_call",
        "approve(address,uint256)": "approve_call",
        "transferFrom(address,address,uint256)": "transfer_from_call",
        "delegate(address)": "delegate",
        "bridgeMint(address,uint256)": "bridge_mint",
        "bridgeBurn(address,uint256)": "bridge_burn",
        "transferOwnership(address)": "transfer_ownership",
    }

    VIEWS = {
        "balanceOf(address)": ("balance_of", ["uint256"]),
        "allowance(address,address)": ("allowance", ["uint256"]),
        "totalSupply()": ("_total_supply", ["uint256"]),
        "getVotes(address)": ("get_votes", ["uint256"]),
        "getPastVotes(address,uint256)": ("get_past_votes", ["uint256"]),
        "getPastTotalSupply(uint256)": ("get_past_total_supply", ["uint256"]),
        "delegates(address)": ("delegates_of", ["address"]),
        "nonces(address)": ("nonce_of", ["uint256"]),
    }

    def _total_supply(self):
        return self.total_supply

    def delegates_of(self, account):
        return self.delegates.get(_addr(account), ZERO)

    def nonce_of(self, account):
        return self.nonces.get(_addr(account), 0)

    def __init__(self, clock: Optional[MockEngine] = None, l2_gateway: str = ZERO, l1_address: str = ZERO,
                 owner: str = "0x" + "0e" * 20, address: Optional[str] = None, chain_id: int = 31337):
        super().__init__("Arbius", "AIUS")
        self.clock = clock
        self.address = _addr(address or self.ADDRESS)
        self.owner = _addr(owner)
        self.l2_gateway = _addr(l2_gateway)
        self.l1_address = _addr(l1_address)
        self.chain_id = chain_id
        self.delegates: Dict[str, str] = {}
        self.checkpoints: Dict[str, List[Checkpoint]] = {}
        self.total_supply_checkpoints: List[Checkpoint] = []
        self.nonces: Dict[str, int] = {}
        self.events: List[Event] = []

    # -------------------------------------------------------------- clock / events
    def _block(self) -> int:
        return self.clock.block_number if self.clock is not None else 0

    def _emit(self, name, **args):
        self.events.append(Event(name, args, self._block(), "", len(self.events)))

    # -------------------------------------------------------------- ERC20 hooks -> votes
    def mint(self, to, amount):
        super().mint(to, amount)
        if self.total_supply > 2 ** 224 - 1:
            raise Revert("ERC20Votes: total supply risks overflowing votes")
        self._write(self.total_supply_checkpoints, lambda v: v + amount)
        self._move_voting_power(ZERO, self.delegates.get(_addr(to), ZERO), amount)
        self._emit("Transfer", **{"from": ZERO, "to": _addr(to), "value": amount})

    def burn(self, account, amount):
        a = _addr(account)
        if self.balances.get(a, 0) < amount:
            raise Revert("ERC20: burn amount exceeds balance")
        self.balances[a] -= amount
        self.total_supply -= amount
        self._write(self.total_supply_checkpoints, lambda v: v - amount)
        self._move_voting_power(self.delegates.get(a, ZERO), ZERO, amount)
        self._emit("Transfer", **{"from": a, "to": ZERO, "value": amount})

    def transfer(self, frm, to, amount):
        if _addr(frm) == ZERO:
            raise Revert("ERC20: transfer from the zero address")
        super().transfer(frm, to, amount)
        self._move_voting_power(self.delegates.get(_addr(frm), ZERO), self.delegates.get(_addr(to), ZERO), amount)
        self._emit("Transfer", **{"from": _addr(frm), "to": _addr(to), "value": amount})

    # ABI entry points (msg.sender first)
    @tx
    def transfer_call(self, sender, to, amount):
        self.transfer(sender, to, amount)
        return True

    @tx
    def approve_call(self, sender, spender, amount):
        self.approve(sender, spender, amount)
        return True

    @tx
    def transfer_from_call(self, sender, frm, to, amount):
        self.transfer_from(sender, frm, to, amount)
        return True

    # -------------------------------------------------------------- bridge / ownership
    @tx
    def bridge_mint(self, sender, account, amount):
        if _addr(sender) != self.l2_gateway:
            raise Revert("NOT_GATEWAY")
        self.mint(account, amount)

    @tx
    def bridge_burn(self, sender, account, amount):
        if _addr(sender) != self.l2_gateway:
            raise Revert("NOT_GATEWAY")
        self.burn(account, amount)

    @tx
    def transfer_ownership(self, sender, to):
        if _addr(sender) != self.owner:
            raise Revert("Ownable: caller is not the owner")
        if _addr(to) == ZERO:
            raise Revert("Ownable: new owner is the zero address")
        self.owner = _addr(to)

    # -------------------------------------------------------------- ERC20Votes
    def _write(self, ckpts: List[Checkpoint], op: Callable[[int], int]) -> Tuple[int, int]:
        old = ckpts[-1].votes if ckpts else 0
        new = op(old)
        blk = self._block()
        if ckpts and ckpts[-1].from_block == blk:
            ckpts[-1].votes = new
        else:
            ckpts.append(Checkpoint(blk, new))
        return old, new

    def _move_voting_power(self, src: str, dst: str, amount: int):
        if src == dst or amount == 0:
            return
        if src != ZERO:
            old, new = self._write(self.checkpoints.setdefault(src, []), lambda v: v - amount)
            self._emit("DelegateVotesChanged", delegate=src, previousBalance=old, newBalance=new)
        if dst != ZERO:
            old, new = self._write(self.checkpoints.setdefault(dst, []), lambda v: v + amount)
            self._emit("DelegateVotesChanged", delegate=dst, previousBalance=old, newBalance=new)

    @tx
    def delegate(self, sender, delegatee):
        self._delegate(_addr(sender), _addr(delegatee))

    def _delegate(self, delegator: str, delegatee: str):
        cur = self.delegates.get(delegator, ZERO)
        self.delegates[delegator] = delegatee
        self._emit("DelegateChanged", delegator=delegator, fromDelegate=cur, toDelegate=delegatee)
        self._move_voting_power(cur, delegatee, self.balance_of(delegator))

    def get_votes(self, account) -> int:
        c = self.checkpoints.get(_addr(account), [])
        return c[-1].votes if c else 0

    @staticmethod
    def _lookup(ckpts: List[Checkpoint], timepoint: int) -> int:
        i = bisect.bisect_right([c.from_block for c in ckpts], timepoint)
        return ckpts[i - 1].votes if i else 0

    def get_past_votes(self, account, timepoint: int) -> int:
        if self.clock is not None and timepoint >= view_block(self.clock):
            raise Revert("ERC20Votes: future lookup")
        return self._lookup(self.checkpoints.get(_addr(account), []), timepoint)

    def get_past_total_supply(self, timepoint: int) -> int:
        if self.clock is not None and timepoint >= view_block(self.clock):
            raise Revert("ERC20Votes: future lookup")
        return self._lookup(self.total_supply_checkpoints, timepoint)

    # -------------------------------------------------------------- EIP-2612 permit
    def domain_separator(self) -> bytes:
        th = keccak256(b"EIP712Domain(string name,string version,uint256 chainId,address verifyingContract)")
        return keccak256(abi.encode(["bytes32", "bytes32", "bytes32", "uint256", "address"],
                                    [th, keccak256(b"Arbius"), keccak256(b"1"), self.chain_id, self.address]))

    def permit_digest(self, owner, spender, value: int, nonce: int, deadline: int) -> bytes:
        th = keccak256(b"Permit(address owner,address spender,uint256 value,uint256 nonce,uint256 deadline)")
        sh = keccak256(abi.encode(["bytes32", "address", "address", "uint256", "uint256", "uint256"],
                                  [th, _addr(owner), _addr(spender), value, nonce, deadline]))
        return keccak256(b"\x19\x01" + self.domain_separator() + sh)

    @tx
    def permit(self, sender, owner, spender, value: int, deadline: int, v: int, r: int, s: int):
        now = self.clock.timestamp if self.clock is not None else 0
        if now > deadline:
            raise Revert("ERC20Permit: expired deadline")
        owner = _addr(owner)
        digest = self.permit_digest(owner, spender, value, self.nonces.get(owner, 0), deadline)
        if recover_address(digest, r, s, v - 27 if v >= 27 else v).lower() != owner:
            raise Revert("ERC20Permit: invalid signature")
        self.nonces[owner] = self.nonces.get(owner, 0) + 1
        self.approve(owner, spender, value)


# ---------------------------------------------------------------------------------------------
class MockTimelock:
    """TimelockV1 = OZ 4.9 TimelockController (AccessControl roles, min delay, batched ops)."""

    ADDRESS = "0x" + "71" * 20
    ABI = {
        "updateDelay(uint256)": "update_delay",
        "grantRole(bytes32,address)": "grant_role",
        "revokeRole(bytes32,address)": "revoke_role",
    }

    def __init__(self, registry: Registry, min_delay: int, proposers: Sequence[str], executors: Sequence[str],
                 admin: str = ZERO, address: Optional[str] = None):
        self.registry = registry
        self.clock = registry.clock
        self.address = _addr(address or self.ADDRESS)
        self.roles: Dict[str, set] = {}
        self.role_admin = {PROPOSER_ROLE: TIMELOCK_ADMIN_ROLE, EXECUTOR_ROLE: TIMELOCK_ADMIN_ROLE,
                           CANCELLER_ROLE: TIMELOCK_ADMIN_ROLE, TIMELOCK_ADMIN_ROLE: TIMELOCK_ADMIN_ROLE}
        self.timestamps: Dict[str, int] = {}
        self.events: List[Event] = []
        self._grant(TIMELOCK_ADMIN_ROLE, self.address)
        if _addr(admin) != ZERO:
            self._grant(TIMELOCK_ADMIN_ROLE, admin)
        for p in proposers:
            self._grant(PROPOSER_ROLE, p)
            self._grant(CANCELLER_ROLE, p)
        for e in executors:
            self._grant(EXECUTOR_ROLE, e)
        self.min_delay = int(min_delay)
        self._emit("MinDelayChange", oldDuration=0, newDuration=self.min_delay)
        registry.add(self)

    def _emit(self, name, **args):
        self.events.append(Event(name, args, self.clock.block_number, "", len(self.events)))

    # -------------------------------------------------------------- AccessControl
    def has_role(self, role, account) -> bool:
        return _addr(account) in self.roles.get(_h32(role), set())

    def _check_role(self, role, account):
        if not self.has_role(role, account):
            raise Revert(f"AccessControl: account {_addr(account)} is missing role {_h32(role)}")

    def _grant(self, role, account):
        role, account = _h32(role), _addr(account)
        if account not in self.roles.setdefault(role, set()):
            self.roles[role].add(account)
            self._emit("RoleGranted", role=role, account=account)

    @tx
    def grant_role(self, sender, role, account):
        self._check_role(self.role_admin.get(_h32(role), DEFAULT_ADMIN_ROLE), sender)
        self._grant(role, account)

    @tx
    def revoke_role(self, sender, role, account):
        self._check_role(self.role_admin.get(_h32(role), DEFAULT_ADMIN_ROLE), sender)
        self.roles.get(_h32(role), set()).discard(_addr(account))
        self._emit("RoleRevoked", role=_h32(role), account=_addr(account))

    @tx
    def renounce_role(self, sender, role, account):
        if _addr(account) != _addr(sender):
            raise Revert("AccessControl: can only renounce roles for self")
        self.roles.get(_h32(role), set()).discard(_addr(account))
        self._emit("RoleRevoked", role=_h32(role), account=_addr(account))

    def _only_role_or_open(self, role, sender):
        if not self.has_role(role, ZERO):
            self._check_role(role, sender)

    # -------------------------------------------------------------- operations
    @staticmethod
    def hash_operation(target, value, data, predecessor, salt) -> str:
        return "0x" + keccak256(abi.encode(["address", "uint256", "bytes", "bytes32", "bytes32"],
                                           [_addr(target), value, data, predecessor, salt])).hex()

    @staticmethod
    def hash_operation_batch(targets, values, payloads, predecessor, salt) -> str:
        return "0x" + keccak256(abi.encode(["address[]", "uint256[]", "bytes[]", "bytes32", "bytes32"],
                                           [[_addr(t) for t in targets], list(values), list(payloads),
                                            predecessor, salt])).hex()

    def get_timestamp(self, op_id) -> int:
        return self.timestamps.get(_h32(op_id), 0)

    def is_operation(self, op_id) -> bool:
        return self.get_timestamp(op_id) > 0

    def is_operation_pending(self, op_id) -> bool:
        return self.get_timestamp(op_id) > _DONE_TIMESTAMP

    def is_operation_ready(self, op_id) -> bool:
        t = self.get_timestamp(op_id)
        return t > _DONE_TIMESTAMP and t <= self.clock.timestamp

    def is_operation_done(self, op_id) -> bool:
        return self.get_timestamp(op_id) == _DONE_TIMESTAMP

    def _schedule(self, op_id, delay):
        if self.is_operation(op_id):
            raise Revert("TimelockController: operation already scheduled")
        if delay < self.min_delay:
            raise Revert("TimelockController: insufficient delay")
        self.timestamps[_h32(op_id)] = self.clock.timestamp + delay

    @tx
    def schedule(self, sender, target, value, data, predecessor, salt, delay):
        self._check_role(PROPOSER_ROLE, sender)
        op = self.hash_operation(target, value, data, predecessor, salt)
        self._schedule(op, delay)
        self._emit("CallScheduled", id=op, index=0, target=_addr(target), value=value, data=data,
                   predecessor=predecessor, delay=delay)
        if salt != ZERO32:
            self._emit("CallSalt", id=op, salt=salt)
        return op

    @tx
    def schedule_batch(self, sender, targets, values, payloads, predecessor, salt, delay):
        self._check_role(PROPOSER_ROLE, sender)
        if not (len(targets) == len(values) == len(payloads)):
            raise Revert("TimelockController: length mismatch")
        op = self.hash_operation_batch(targets, values, payloads, predecessor, salt)
        self._schedule(op, delay)
        for i, (t, v, d) in enumerate(zip(targets, values, payloads)):
            self._emit("CallScheduled", id=op, index=i, target=_addr(t), value=v, data=d,
                       predecessor=predecessor, delay=delay)
        if salt != ZERO32:
            self._emit("CallSalt", id=op, salt=salt)
        return op

    @tx
    def cancel(self, sender, op_id):
        self._check_role(CANCELLER_ROLE, sender)
        if not self.is_operation_pending(op_id):
            raise Revert("TimelockController: operation cannot be cancelled")
        del self.timestamps[_h32(op_id)]
        self._emit("Cancelled", id=_h32(op_id))

    def _before_call(self, op_id, predecessor):
        if not self.is_operation_ready(op_id):
            raise Revert("TimelockController: operation is not ready")
        if predecessor != ZERO32 and not self.is_operation_done(predecessor):
            raise Revert("TimelockController: missing dependency")

    def _call(self, target, value, data):
        try:
            return self.registry.call(self.address, target, value, bytes(abi._to_bytes(data)))
        except Revert as e:
            raise Revert("TimelockController: underlying transaction reverted") from e

    @tx
    def execute(self, sender, target, value, payload, predecessor, salt):
        self._only_role_or_open(EXECUTOR_ROLE, sender)
        op = self.hash_operation(target, value, payload, predecessor, salt)
        self._before_call(op, predecessor)
        self._call(target, value, payload)
        self._emit("CallExecuted", id=op, index=0, target=_addr(target), value=value, data=payload)
        self.timestamps[op] = _DONE_TIMESTAMP
        return op

    @tx
    def execute_batch(self, sender, targets, values, payloads, predecessor, salt):
        self._only_role_or_open(EXECUTOR_ROLE, sender)
        if not (len(targets) == len(values) == len(payloads)):
            raise Revert("TimelockController: length mismatch")
        op = self.hash_operation_batch(targets, values, payloads, predecessor, salt)
        self._before_call(op, predecessor)
        for i, (t, v, d) in enumerate(zip(targets, values, payloads)):
            self._call(t, v, d)
            self._emit("CallExecuted", id=op, index=i, target=_addr(t), value=v, data=d)
        self.timestamps[op] = _DONE_TIMESTAMP
        return op

    def update_delay(self, sender, new_delay):
        if _addr(sender) != self.address:
            raise Revert("TimelockController: caller must be timelock")
        self._emit("MinDelayChange", oldDuration=self.min_delay, newDuration=int(new_delay))
        self.min_delay = int(new_delay)


# ---------------------------------------------------------------------------------------------
PENDING, ACTIVE, CANCELED, DEFEATED, SUCCEEDED, QUEUED, EXPIRED, EXECUTED = range(8)
STATE_NAMES = ("Pending", "Active", "Canceled", "Defeated", "Succeeded", "Queued", "Expired", "Executed")


@dataclass
class Proposal:
    proposer: str
    vote_start: int
    vote_end: int
    executed: bool = False
    canceled: bool = False
    for_votes: int = 0
    against_votes: int = 0
    abstain_votes: int = 0
    eta: int = 0
    receipts: Dict[str, Tuple[int, int]] = field(default_factory=dict)   # voter -> (support, weight)
    details: tuple = ()          # (targets, values, calldatas, descriptionHash): Bravo id overloads


class MockGovernor:
    """GovernorV1 (GovernorV1.sol:12-184): votingDelay = votingPeriod = 6575 blocks, threshold
    1e18, quorum 4 % of past total supply, Bravo counting (quorum counts FOR votes only), proposals
    executed through the Timelock; stores proposal ids, description hashes and description CIDs."""

    ADDRESS = "0x" + "60" * 20
    ABI = {
        "propose(address[],uint256[],bytes[],string)": "propose",
        "castVote(uint256,uint8)": "cast_vote",
        "castVoteWithReason(uint256,uint8,string)": "cast_vote",
        "queue(address[],uint256[],bytes[],bytes32)": "queue",
        "execute(address[],uint256[],bytes[],bytes32)": "execute",
        "cancel(address[],uint256[],bytes[],bytes32)": "cancel",
        "queue(uint256)": "queue_id",
        "execute(uint256)": "execute_id",
        "cancel(uint256)": "cancel_id",
    }
    VIEWS = {
        "state(uint256)": ("state", ["uint8"]),
        "proposalSnapshot(uint256)": ("proposal_snapshot", ["uint256"]),
        "proposalDeadline(uint256)": ("proposal_deadline", ["uint256"]),
        "proposalEta(uint256)": ("proposal_eta", ["uint256"]),
        "proposalVotes(uint256)": ("proposal_votes", ["uint256", "uint256", "uint256"]),
        "hasVoted(uint256,address)": ("has_voted", ["bool"]),
        "quorum(uint256)": ("quorum", ["uint256"]),
        "getVotes(address,uint256)": ("get_votes", ["uint256"]),
        "proposalsCreatedLength()": ("proposals_created_length", ["uint256"]),
        "proposalsCreated(uint256)": ("proposal_created_at", ["uint256"]),
        "descriptionHashes(uint256)": ("description_hash_of", ["bytes32"]),
        "descriptionCids(uint256)": ("description_cid_of", ["bytes"]),
        "votingDelay()": ("get_voting_delay", ["uint256"]),
        "votingPeriod()": ("get_voting_period", ["uint256"]),
        "proposalThreshold()": ("get_proposal_threshold", ["uint256"]),
    }

    def proposal_created_at(self, i):
        return self.proposals_created[int(i)]

    def description_hash_of(self, pid):
        return self.description_hashes.get(int(pid), ZERO32)

    def description_cid_of(self, pid):
        return self.description_cids.get(int(pid), "0x")

    def get_voting_delay(self):
        return self.voting_delay

    def get_voting_period(self):
        return self.voting_period

    def get_proposal_threshold(self):
        return self.proposal_threshold

    # GovernorCompatibilityBravo id-only overloads (the CLI's governance queue/execute/cancel)
    def queue_id(self, sender, pid):
        return self.queue(sender, *self._proposal(pid).details)

    def execute_id(self, sender, pid):
        return self.execute(sender, *self._proposal(pid).details)

    def cancel_id(self, sender, pid):
        return self.cancel(sender, *self._proposal(pid).details)

    def __init__(self, registry: Registry, token: MockBaseToken, timelock: MockTimelock,
                 voting_delay: int = 6575, voting_period: int = 6575, proposal_threshold: int = 10 ** 18,
                 quorum_numerator: int = 4, address: Optional[str] = None):
        self.registry = registry
        self.clock = registry.clock
        self.token, self.timelock = token, timelock
        self.address = _addr(address or self.ADDRESS)
        self.name = "Governor"
        self.voting_delay, self.voting_period = voting_delay, voting_period
        self.proposal_threshold = proposal_threshold
        self.quorum_numerator, self.quorum_denominator = quorum_numerator, 100
        self.proposals: Dict[int, Proposal] = {}
        self.timelock_ids: Dict[int, str] = {}
        self.proposals_created: List[int] = []
        self.description_hashes: Dict[int, str] = {}
        self.description_cids: Dict[int, str] = {}
        self.events: List[Event] = []
        registry.add(self)

    def _emit(self, name, **args):
        self.events.append(Event(name, args, self.clock.block_number, "", len(self.events)))

    def clock_now(self) -> int:
        return view_block(self.clock)

    @staticmethod
    def hash_proposal(targets, values, calldatas, description_hash) -> int:
        return int.from_bytes(keccak256(abi.encode(
            ["address[]", "uint256[]", "bytes[]", "bytes32"],
            [[_addr(t) for t in targets], list(values), list(calldatas), description_hash])), "big")

    @staticmethod
    def description_hash(description: str) -> str:
        return "0x" + keccak256(description.encode()).hex()

    def quorum(self, timepoint: int) -> int:
        return self.token.get_past_total_supply(timepoint) * self.quorum_numerator // self.quorum_denominator

    def get_votes(self, account, timepoint: int) -> int:
        return self.token.get_past_votes(account, timepoint)

    def _proposal(self, pid) -> Proposal:
        p = self.proposals.get(int(pid))
        if p is None:
            raise Revert("Governor: unknown proposal id")
        return p

    def proposal_snapshot(self, pid) -> int:
        return self._proposal(pid).vote_start

    def proposal_deadline(self, pid) -> int:
        return self._proposal(pid).vote_end

    def _quorum_reached(self, p: Proposal) -> bool:
        return self.quorum(p.vote_start) <= p.for_votes

    @staticmethod
    def _vote_succeeded(p: Proposal) -> bool:
        return p.for_votes > p.against_votes

    def state(self, pid) -> int:
        p = self._proposal(pid)
        if p.executed:
            st = EXECUTED
        elif p.canceled:
            st = CANCELED
        else:
            now = self.clock_now()
            if p.vote_start >= now:
                return PENDING
            if p.vote_end >= now:
                return ACTIVE
            st = SUCCEEDED if (self._quorum_reached(p) and self._vote_succeeded(p)) else DEFEATED
        if st != SUCCEEDED:
            return st
        qid = self.timelock_ids.get(int(pid))             # GovernorTimelockControl.state
        if qid is None:
            return SUCCEEDED
        if self.timelock.is_operation_done(qid):
            return EXECUTED
        if self.timelock.is_operation_pending(qid):
            return QUEUED
        return CANCELED

    # -------------------------------------------------------------- lifecycle
    @tx
    def propose(self, sender, targets, values, calldatas, description: str) -> int:
        sender = _addr(sender)
        now = self.clock_now()
        if self.get_votes(sender, now - 1) < self.proposal_threshold:
            raise Revert("Governor: proposer votes below proposal threshold")
        dh = self.description_hash(description)
        pid = self.hash_proposal(targets, values, calldatas, dh)
        if not (len(targets) == len(values) == len(calldatas)):
            raise Revert("Governor: invalid proposal length")
        if not targets:
            raise Revert("Governor: empty proposal")
        if int(pid) in self.proposals:
            raise Revert("Governor: proposal already exists")
        snapshot = now + self.voting_delay
        self.proposals[pid] = Proposal(sender, snapshot, snapshot + self.voting_period,
                                       details=(list(targets), list(values), list(calldatas), dh))
        self._emit("ProposalCreated", proposalId=pid, proposer=sender, targets=list(targets), values=list(values),
                   calldatas=list(calldatas), voteStart=snapshot, voteEnd=snapshot + self.voting_period,
                   description=description)
        self.proposals_created.append(pid)                                   # GovernorV1.sol:124-128
        self.description_hashes[pid] = dh
        self.description_cids[pid] = "0x" + onchain_cid(description.encode()).hex()
        return pid

    @tx
    def cast_vote(self, sender, pid, support: int, reason: str = "") -> int:
        sender = _addr(sender)
        p = self._proposal(pid)
        if self.state(pid) != ACTIVE:
            raise Revert("Governor: vote not currently active")
        weight = self.get_votes(sender, p.vote_start)
        if sender in p.receipts:
            raise Revert("GovernorCompatibilityBravo: vote already cast")
        if support == 0:
            p.against_votes += weight
        elif support == 1:
            p.for_votes += weight
        elif support == 2:
            p.abstain_votes += weight
        else:
            raise Revert("GovernorCompatibilityBravo: invalid vote type")
        p.receipts[sender] = (support, weight)
        self._emit("VoteCast", voter=sender, proposalId=pid, support=support, weight=weight, reason=reason)
        return weight

    def has_voted(self, pid, account) -> bool:
        return _addr(account) in self._proposal(pid).receipts

    def proposal_votes(self, pid) -> Tuple[int, int, int]:
        p = self._proposal(pid)
        return p.against_votes, p.for_votes, p.abstain_votes

    def _timelock_salt(self, description_hash) -> str:
        """OZ 4.9 GovernorTimelockControl: bytes20(address(this)) ^ descriptionHash."""
        a = bytes.fromhex(self.address[2:]) + b"\0" * 12
        d = abi._to_bytes(description_hash)
        return "0x" + bytes(x ^ y for x, y in zip(a, d)).hex()

    @tx
    def queue(self, sender, targets, values, calldatas, description_hash) -> int:
        pid = self.hash_proposal(targets, values, calldatas, description_hash)
        if self.state(pid) != SUCCEEDED:
            raise Revert("Governor: proposal not successful")
        delay = self.timelock.min_delay
        salt = self._timelock_salt(description_hash)
        self.timelock.schedule_batch(self.address, targets, values, calldatas, ZERO32, salt, delay)
        self.timelock_ids[pid] = self.timelock.hash_operation_batch(targets, values, calldatas, ZERO32, salt)
        eta = self.clock.timestamp + delay
        self.proposals[pid].eta = eta
        self._emit("ProposalQueued", proposalId=pid, eta=eta)
        return pid

    def proposal_eta(self, pid) -> int:
        qid = self.timelock_ids.get(int(pid))
        if qid is None:
            return 0
        t = self.timelock.get_timestamp(qid)
        return 0 if t == _DONE_TIMESTAMP else t

    @tx
    def execute(self, sender, targets, values, calldatas, description_hash) -> int:
        pid = self.hash_proposal(targets, values, calldatas, description_hash)
        st = self.state(pid)
        if st not in (SUCCEEDED, QUEUED):
            raise Revert("Governor: proposal not successful")
        # the timelock call runs first here: a Python Revert rolls nothing back, so no state
        # is written before the last call that can revert (Solidity would undo it all)
        self.timelock.execute_batch(self.address, targets, values, calldatas, ZERO32,
                                    self._timelock_salt(description_hash))
        self.proposals[pid].executed = True
        self._emit("ProposalExecuted", proposalId=pid)
        return pid

    @tx
    def cancel(self, sender, targets, values, calldatas, description_hash) -> int:
        """GovernorCompatibilityBravo.cancel: the proposer, or anyone once the proposer's votes
        fell below the threshold; then Governor._cancel + GovernorTimelockControl._cancel."""
        pid = self.hash_proposal(targets, values, calldatas, description_hash)
        p = self._proposal(pid)
        if _addr(sender) != p.proposer and not (
                self.get_votes(p.proposer, self.clock_now() - 1) < self.proposal_threshold):
            raise Revert("GovernorBravo: proposer above threshold")
        st = self.state(pid)
        if st in (CANCELED, EXPIRED, EXECUTED):
            raise Revert("Governor: proposal not active")
        qid = self.timelock_ids.get(pid)
        if qid is not None:
            self.timelock.cancel(self.address, qid)
            del self.timelock_ids[pid]
        p.canceled = True
        self._emit("ProposalCanceled", proposalId=pid)
        return pid

    def proposals_created_length(self) -> int:
        return len(self.proposals_created)


def deploy_governance(engine: MockEngine, deployer: str, extra_admin: Optional[str] = None,
                      min_delay: int = 3 * 86400) -> Tuple[MockBaseToken, MockTimelock, MockGovernor, Registry]:
    """The governance fixture of contract/test/governance.test.ts:27-125: BaseToken (deployer
    is the gateway so tests can bridgeMint), Timelock(0, [deployer, extra], [deployer, extra],
    deployer), Engine ownership -> Timelock, Governor(token, timelock) granted PROPOSER and
    EXECUTOR, Timelock delay raised to 3 days through its own schedule/execute, deployer renounces
    PROPOSER and TIMELOCK_ADMIN."""
    reg = Registry(engine)
    token = engine.token
    if not isinstance(token, MockBaseToken):
        raise TypeError("deploy_governance needs an engine built on MockBaseToken")
    token.clock = engine
    reg.add(token)
    members = [deployer] + ([extra_admin] if extra_admin else [])
    tl = MockTimelock(reg, 0, members, members, admin=deployer)
    engine.transfer_ownership(engine.owner, tl.address)
    gov = MockGovernor(reg, token, tl)
    tl.grant_role(deployer, PROPOSER_ROLE, gov.address)
    tl.grant_role(deployer, EXECUTOR_ROLE, gov.address)
    upd = abi.encode_call("updateDelay(uint256)", min_delay)
    tl.schedule(deployer, tl.address, 0, upd, ZERO32, ZERO32, 0)
    tl.execute(deployer, tl.address, 0, upd, ZERO32, ZERO32)
    tl.renounce_role(deployer, PROPOSER_ROLE, deployer)
    tl.renounce_role(deployer, TIMELOCK_ADMIN_ROLE, deployer)
    return token, tl, gov, reg
