"""MockEngine: an in-process Python twin of ``EngineV1`` + its ERC20 base token.

Every state transition, revert string, event and fixed-point formula follows
``contract/contracts/EngineV1.sol`` (line refs inline) so the node's chain
logic can be exercised end-to-end without a chain (SURVEY.md §4 "MockEngine",
Appendix A-C).  Time travel mirrors hardhat's ``evm_increaseTime``/``evm_mine``;
every transaction mines one block (hardhat automine).

Amounts are integers in wei (18 decimals).  Addresses are lowercase 0x-hex.
"""
from __future__ import annotations

import contextlib

import itertools
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

from ..utils.keccak import keccak256
from ..utils.protocol import generate_commitment, hash_model, hash_task
from ..ipfs.unixfs import onchain_cid
from . import prbmath as pm

E18 = 10 ** 18
MAX_SUPPLY_BASE_TOKEN = 1_000_000 * E18
STARTING_ENGINE_TOKEN_AMOUNT = 600_000 * E18
BASE_TOKEN_STARTING_REWARD = E18
MIN_SUPPLY_FOR_VALIDATOR_DEPOSITS = 1_000 * E18
MIN_SUPPLY_FOR_SLASHING = 2_000 * E18
ARBITRUM_CHAINIDS = (0xA4BA, 0x66EED, 0x66EEE)
ZERO = "0x" + "00" * 20
ZERO32 = "0x" + "00" * 32


class Revert(Exception):
    """A reverted call; ``str(e)`` is the Solidity revert string."""


def _addr(a: str) -> str:
    a = a.lower()
    if not a.startswith("0x") or len(a) != 42:
        raise ValueError(f"bad address {a}")
    return a


def _h32(x) -> str:
    if isinstance(x, bytes):
        return "0x" + x.hex()
    return x.lower()


@dataclass
class Model:
    fee: int = 0
    addr: str = ZERO
    rate: int = 0
    cid: str = "0x"


@dataclass
class Validator:
    staked: int = 0
    since: int = 0
    addr: str = ZERO


@dataclass
class Task:
    model: str = ZERO32
    fee: int = 0
    owner: str = ZERO
    blocktime: int = 0
    version: int = 0
    cid: str = "0x"


@dataclass
class Solution:
    validator: str = ZERO
    blocktime: int = 0
    claimed: bool = False
    cid: str = "0x"


@dataclass
class Contestation:
    validator: str = ZERO
    blocktime: int = 0
    finish_start_index: int = 0
    slash_amount: int = 0


@dataclass
class Event:
    name: str
    args: dict
    block: int
    tx: str
    index: int


class MockToken:
    """Minimal OZ ERC20 (revert strings of OZ 4.x)."""

    def __init__(self, name="Arbius", symbol="AIUS"):
        self.name, self.symbol = name, symbol
        self.balances: Dict[str, int] = {}
        self.allowances: Dict[Tuple[str, str], int] = {}
        self.total_supply = 0

    def balance_of(self, a):
        return self.balances.get(_addr(a), 0)

    def mint(self, to, amount):
        to = _addr(to)
        self.balances[to] = self.balances.get(to, 0) + amount
        self.total_supply += amount

    def transfer(self, frm, to, amount):
        frm, to = _addr(frm), _addr(to)
        if to == ZERO:
            raise Revert("ERC20: transfer to the zero address")
        if self.balances.get(frm, 0) < amount:
            raise Revert("ERC20: transfer amount exceeds balance")
        self.balances[frm] = self.balances.get(frm, 0) - amount
        self.balances[to] = self.balances.get(to, 0) + amount

    def approve(self, owner, spender, amount):
        self.allowances[(_addr(owner), _addr(spender))] = amount

    def allowance(self, owner, spender):
        return self.allowances.get((_addr(owner), _addr(spender)), 0)

    def transfer_from(self, spender, frm, to, amount):
        key = (_addr(frm), _addr(spender))
        cur = self.allowances.get(key, 0)
        if cur != 2 ** 256 - 1:
            if cur < amount:
                raise Revert("ERC20: insufficient allowance")
            self.allowances[key] = cur - amount
        self.transfer(frm, to, amount)


class MockEngine:
    """State + semantics of EngineV1 (version 0)."""

    ADDRESS = "0x399511edeb7ca4a8328e801b1b3d0fe232abc996"

    def __init__(self, token: Optional[MockToken] = None, treasury: str = "0x" + "7e" * 20,
                 owner: str = "0x" + "0e" * 20, chain_id: int = 31337, start_time: int = 1_700_000_000):
        self.token = token or MockToken()
        self.chain_id = chain_id
        self.timestamp = start_time
        self.block_number = 1
        self.arb_block_number = 1
        self.events: List[Event] = []
        self._txc = itertools.count(1)
        self.address = self.ADDRESS
        # initialize (EngineV1.sol:240-260)
        self.owner = _addr(owner)
        self.treasury = _addr(treasury)
        self.pauser = self.owner
        self.paused = False
        self.accrued_fees = 0
        self.prevhash = ZERO32
        self.start_block_time = start_time
        self.version = 0
        self.validator_minimum_percentage = 8 * 10 ** 14
        self.slash_amount_percentage = 10 ** 14
        self.solution_fee_percentage = 10 ** 17
        self.retraction_fee_percentage = 10 ** 17
        self.treasury_reward_percentage = 10 ** 17
        self.min_claim_solution_time = 2000
        self.min_retraction_wait_time = 10000
        self.min_contestation_vote_period_time = 4000
        self.max_contestation_validator_stake_since = 120
        self.exit_validator_min_unlock_time = 86400
        self.models: Dict[str, Model] = {}
        self.validators: Dict[str, Validator] = {}
        self.pending_withdraw_count: Dict[str, int] = {}
        self.pending_withdraws: Dict[Tuple[str, int], Tuple[int, int]] = {}
        self.withdraw_pending_amount: Dict[str, int] = {}
        self.tasks: Dict[str, Task] = {}
        self.commitments: Dict[str, int] = {}
        self.solutions: Dict[str, Solution] = {}
        self.contestations: Dict[str, Contestation] = {}
        self.contestation_voted: Dict[Tuple[str, str], bool] = {}
        self.vote_yeas: Dict[str, List[str]] = {}
        self.vote_nays: Dict[str, List[str]] = {}
        self._initialized = True
        self.listeners = []

    # ------------------------------------------------------------------ chain mechanics
    def _tx(self) -> str:
        """Mine one block for a transaction (hardhat automine); inside ``one_block()`` every
        transaction lands in the block that context opened (a real chain's batching)."""
        if not getattr(self, "_open_block", False):
            self.block_number += 1
            self.arb_block_number += 1
        return "0x" + keccak256(f"tx{next(self._txc)}".encode()).hex()

    @contextlib.contextmanager
    def one_block(self):
        """Execute the enclosed transactions in ONE new block (the same ``block.number`` /
        ``arbBlockNumber``), as a sequencer does with transactions that arrive together."""
        self.block_number += 1
        self.arb_block_number += 1
        prev, self._open_block = getattr(self, "_open_block", False), True
        try:
            yield
        finally:
            self._open_block = prev

    def _current_block(self) -> int:
        """``getBlockNumberNow()`` as seen by the executing transaction: the block it is mined in."""
        return self.get_block_number_now() + (0 if getattr(self, "_open_block", False) else 1)

    def increase_time(self, seconds: int):
        """evm_increaseTime + evm_mine."""
        self.timestamp += int(seconds)
        self.block_number += 1
        self.arb_block_number += 1

    def mine(self, n: int = 1):
        self.block_number += n
        self.arb_block_number += n
        self.timestamp += n

    def _emit(self, name, tx, **args):
        ev = Event(name, args, self.block_number, tx, len(self.events))
        self.events.append(ev)
        for cb in list(self.listeners):
            cb(ev)
        return ev

    def get_block_number_now(self) -> int:
        """EngineV1.sol:740-755: ArbSys.arbBlockNumber on Arbitrum chain ids, else block.number."""
        return self.arb_block_number if self.chain_id in ARBITRUM_CHAINIDS else self.block_number

    def initialize(self, *a, **k):
        if self._initialized:
            raise Revert("Initializable: contract is already initialized")

    # ------------------------------------------------------------------ modifiers
    def _not_paused(self):
        if self.paused:
            raise Revert("paused")

    def _only_owner(self, sender):
        if _addr(sender) != self.owner:
            raise Revert("Ownable: caller is not the owner")

    def _only_validator(self, sender):
        s = _addr(sender)
        v = self.validators.get(s, Validator())
        if v.staked - self.withdraw_pending_amount.get(s, 0) < self.get_validator_minimum():
            raise Revert("min staked too low")

    # ------------------------------------------------------------------ views / math (EngineV1.sol:387-543)
    def get_psuedo_total_supply(self) -> int:
        b = self.token.balance_of(self.address)
        return 0 if b >= STARTING_ENGINE_TOKEN_AMOUNT else STARTING_ENGINE_TOKEN_AMOUNT - b

    def get_slash_amount(self) -> int:
        ts = self.get_psuedo_total_supply()
        if ts < MIN_SUPPLY_FOR_SLASHING:
            return 0
        return ts - (ts * (E18 - self.slash_amount_percentage)) // E18

    def get_validator_minimum(self) -> int:
        ts = self.get_psuedo_total_supply()
        if ts < MIN_SUPPLY_FOR_VALIDATOR_DEPOSITS:
            return 0
        return ts - (ts * (E18 - self.validator_minimum_percentage)) // E18

    @staticmethod
    def generate_ipfs_cid(content: bytes) -> str:
        return "0x" + onchain_cid(content).hex()

    @staticmethod
    def target_ts(t: int) -> int:
        if t > 3153600000:
            return STARTING_ENGINE_TOKEN_AMOUNT
        e = pm.ud_exp2(pm.ud_div(t, 60 * 60 * 24 * 365))
        return STARTING_ENGINE_TOKEN_AMOUNT - ((STARTING_ENGINE_TOKEN_AMOUNT * E18 * E18) // e // E18)

    @classmethod
    def diff_mul(cls, t: int, ts: int) -> int:
        if not (t > 0 and ts > 0):
            raise Revert("min vals")
        e = cls.target_ts(t)
        d = pm.sd_div(ts, e)
        if d < 933561438102252700:
            return 100 * E18
        one, onehundred = E18, 100 * E18
        c = one + (pm.sd_mul(d - one, onehundred) - one)
        if c >= 20 * E18:
            return 0
        if c < 0:
            return pm.sd_exp2(abs(c))
        return pm.sd_div(one, pm.sd_exp2(c))

    @classmethod
    def reward(cls, t: int, ts: int) -> int:
        if ts == 0:
            return BASE_TOKEN_STARTING_REWARD
        return ((STARTING_ENGINE_TOKEN_AMOUNT - ts) * BASE_TOKEN_STARTING_REWARD) * cls.diff_mul(t, ts) \
            // STARTING_ENGINE_TOKEN_AMOUNT // E18

    def get_reward(self) -> int:
        return self.reward(self.timestamp - self.start_block_time, self.get_psuedo_total_supply())

    @staticmethod
    def generate_commitment(sender, taskid, cid) -> str:
        return generate_commitment(sender, taskid, cid)

    @staticmethod
    def hash_model(addr, fee, cid, sender) -> str:
        return hash_model(sender, addr, fee, cid)

    @staticmethod
    def hash_task(task: Task, sender, prevhash) -> str:
        return hash_task(sender, prevhash, task.model, task.fee, task.cid)

    # ------------------------------------------------------------------ owner / pauser (EngineV1.sol:264-383)
    def transfer_ownership(self, sender, to):
        self._only_owner(sender)
        if _addr(to) == ZERO:
            raise Revert("Ownable: new owner is the zero address")
        self.owner = _addr(to)
        self._emit("OwnershipTransferred", self._tx(), previousOwner=_addr(sender), newOwner=_addr(to))

    def renounce_ownership(self, sender):
        self._only_owner(sender)
        self.owner = ZERO

    def transfer_treasury(self, sender, to):
        self._only_owner(sender)
        self.treasury = _addr(to)
        self._emit("TreasuryTransferred", self._tx(), to=_addr(to))

    def transfer_pauser(self, sender, to):
        self._only_owner(sender)
        self.pauser = _addr(to)
        self._emit("PauserTransferred", self._tx(), to=_addr(to))

    def set_paused(self, sender, paused: bool):
        if _addr(sender) != self.pauser:
            raise Revert("not pauser")
        self.paused = bool(paused)
        self._emit("PausedChanged", self._tx(), paused=bool(paused))

    def set_solution_mineable_rate(self, sender, model, rate):
        self._only_owner(sender)
        model = _h32(model)
        if self.models.get(model, Model()).addr == ZERO:
            raise Revert("model does not exist")
        self.models[model].rate = int(rate)
        self._emit("SolutionMineableRateChange", self._tx(), id=model, rate=int(rate))

    def set_version(self, sender, version):
        self._only_owner(sender)
        self.version = int(version)
        self._emit("VersionChanged", self._tx(), version=int(version))

    _PARAMS = {
        "validator_minimum_percentage": "ValidatorMinimumPercentageChanged",
        "slash_amount_percentage": "SlashAmountPercentageChanged",
        "solution_fee_percentage": "SolutionFeePercentageChanged",
        "retraction_fee_percentage": "RetractionFeePercentageChanged",
        "treasury_reward_percentage": "TreasuryRewardPercentageChanged",
        "min_claim_solution_time": "MinClaimSolutionTimeChanged",
        "min_retraction_wait_time": "MinRetractionWaitTimeChanged",
        "min_contestation_vote_period_time": "MinContestationVotePeriodTimeChanged",
        "max_contestation_validator_stake_since": "MaxContestationValidatorStakeSinceChanged",
        "exit_validator_min_unlock_time": "ExitValidatorMinUnlockTimeChanged",
    }

    def set_param(self, sender, name: str, amount: int):
        """The 10 ``set<Param>`` owner setters (EngineV1.sol:313-383)."""
        self._only_owner(sender)
        if name not in self._PARAMS:
            raise ValueError(name)
        setattr(self, name, int(amount))
        self._emit(self._PARAMS[name], self._tx(), amount=int(amount))

    # ------------------------------------------------------------------ treasury
    def withdraw_accrued_fees(self, sender):
        self._not_paused()
        self.token.transfer(self.address, self.treasury, self.accrued_fees)
        self.accrued_fees = 0
        self._tx()

    # ------------------------------------------------------------------ models (EngineV1.sol:557-575)
    def register_model(self, sender, addr, fee: int, template: bytes) -> str:
        self._not_paused()
        if _addr(addr) == ZERO:
            raise Revert("address must be non-zero")
        cid = self.generate_ipfs_cid(template)
        mid = hash_model(_addr(sender), _addr(addr), int(fee), cid)
        if self.models.get(mid, Model()).addr != ZERO:
            raise Revert("model already registered")
        self.models[mid] = Model(int(fee), _addr(addr), 0, cid)
        self._emit("ModelRegistered", self._tx(), id=mid)
        return mid

    # ------------------------------------------------------------------ validators (EngineV1.sol:581-672)
    def validator_deposit(self, sender, validator, amount: int):
        self._not_paused()
        validator = _addr(validator)
        self.token.transfer_from(self.address, sender, self.address, amount)
        mn = self.get_validator_minimum()
        v = self.validators.get(validator, Validator())
        since = v.since
        if v.staked <= mn and v.staked + amount >= mn:
            since = self.timestamp
        self.validators[validator] = Validator(v.staked + amount, since, validator)
        self._emit("ValidatorDeposit", self._tx(), addr=_addr(sender), validator=validator, amount=int(amount))

    def initiate_validator_withdraw(self, sender, amount: int) -> int:
        self._not_paused()
        s = _addr(sender)
        v = self.validators.get(s, Validator())
        if v.staked - self.withdraw_pending_amount.get(s, 0) < amount:
            raise Revert("")
        unlock = self.timestamp + self.exit_validator_min_unlock_time
        cnt = self.pending_withdraw_count.get(s, 0) + 1
        self.pending_withdraw_count[s] = cnt
        self.pending_withdraws[(s, cnt)] = (unlock, int(amount))
        self.withdraw_pending_amount[s] = self.withdraw_pending_amount.get(s, 0) + int(amount)
        self._emit("ValidatorWithdrawInitiated", self._tx(), addr=s, count=cnt, unlockTime=unlock, amount=int(amount))
        return cnt

    def cancel_validator_withdraw(self, sender, count: int):
        self._not_paused()
        s = _addr(sender)
        unlock, amount = self.pending_withdraws.get((s, count), (0, 0))
        if unlock == 0:
            raise Revert("request not exist")
        self.withdraw_pending_amount[s] -= amount
        del self.pending_withdraws[(s, count)]
        self._emit("ValidatorWithdrawCancelled", self._tx(), addr=s, count=count)

    def validator_withdraw(self, sender, count: int, to):
        self._not_paused()
        s = _addr(sender)
        unlock, amount = self.pending_withdraws.get((s, count), (0, 0))
        if unlock == 0:
            raise Revert("request not exist")
        if self.timestamp < unlock:
            raise Revert("wait longer")
        v = self.validators.get(s, Validator())
        if v.staked < amount:
            raise Revert("stake insufficient")
        self.token.transfer(self.address, to, amount)
        v.staked -= amount
        self.withdraw_pending_amount[s] -= amount
        del self.pending_withdraws[(s, count)]
        self._emit("ValidatorWithdraw", self._tx(), addr=s, to=_addr(to), count=count, amount=amount)

    # ------------------------------------------------------------------ tasks (EngineV1.sol:681-736)
    def submit_task(self, sender, version: int, owner, model, fee: int, input_: bytes) -> str:
        self._not_paused()
        model = _h32(model)
        m = self.models.get(model, Model())
        if m.addr == ZERO:
            raise Revert("model does not exist")
        if fee < m.fee:
            raise Revert("lower fee than model fee")
        cid = self.generate_ipfs_cid(input_)
        task = Task(model, int(fee), _addr(owner), self.timestamp, int(version), cid)
        tid = self.hash_task(task, _addr(sender), self.prevhash)
        self.token.transfer_from(self.address, sender, self.address, fee)  # atomic: raises before mutating
        tx = self._tx()
        self._emit("TaskSubmitted", tx, id=tid, model=model, fee=int(fee), sender=_addr(sender))
        self.tasks[tid] = task
        self.prevhash = tid
        args = (int(version), _addr(owner), model, int(fee), bytes(input_))
        self._tx_inputs[tx] = ("submitTask", args, _addr(sender))
        return tid

    @property
    def _tx_inputs(self):
        if not hasattr(self, "_txin"):
            self._txin = {}
        return self._txin

    def get_transaction(self, tx: str):
        """-> (method, args, from) of a mined submitTask tx (eth_getTransactionByHash + decode)."""
        return self._tx_inputs.get(tx)

    def retract_task(self, sender, taskid):
        self._not_paused()
        taskid = _h32(taskid)
        t = self.tasks.get(taskid, Task())
        if t.owner != _addr(sender):
            raise Revert("not owner")
        if self.solutions.get(taskid, Solution()).validator != ZERO:
            raise Revert("has solution")
        if not self.timestamp - t.blocktime > self.min_retraction_wait_time:
            raise Revert("did not wait long enough")
        amount_minus_fee = (t.fee * (E18 - self.retraction_fee_percentage)) // E18
        fee = t.fee - amount_minus_fee
        self.token.transfer(self.address, sender, amount_minus_fee)
        self.accrued_fees += fee
        del self.tasks[taskid]
        self._emit("TaskRetracted", self._tx(), id=taskid)

    # ------------------------------------------------------------------ commitments / solutions (EngineV1.sol:764-889)
    def signal_commitment(self, sender, commitment):
        self._not_paused()
        commitment = _h32(commitment)
        if self.commitments.get(commitment, 0) != 0:
            raise Revert("commitment exists")
        tx = self._tx()
        self.commitments[commitment] = self.get_block_number_now()
        self._emit("SignalCommitment", tx, addr=_addr(sender), commitment=commitment)

    def signal_support(self, sender, model, support: bool):
        self._only_validator(sender)
        model = _h32(model)
        if self.models.get(model, Model()).addr == ZERO:
            raise Revert("model does not exist")
        self._emit("SignalSupport", self._tx(), addr=_addr(sender), model=model, supported=bool(support))

    def submit_solution(self, sender, taskid, cid):
        self._not_paused()
        self._only_validator(sender)
        taskid = _h32(taskid)
        cid = _h32(cid)
        if self.tasks.get(taskid, Task()).model == ZERO32:
            raise Revert("task does not exist")
        if self.solutions.get(taskid, Solution()).validator != ZERO:
            raise Revert("solution already submitted")
        commitment = generate_commitment(_addr(sender), taskid, cid)
        blk = self.commitments.get(commitment, 0)
        if blk == 0:
            raise Revert("non existent commitment")
        if not blk < self._current_block():  # EngineV1.sol:797-802
            raise Revert("commitment must be in past")
        tx = self._tx()
        self.solutions[taskid] = Solution(_addr(sender), self.timestamp, False, cid)
        self._emit("SolutionSubmitted", tx, addr=_addr(sender), task=taskid)

    def _claim_solution_fees_and_reward(self, taskid):
        t = self.tasks[taskid]
        m = self.models.get(t.model, Model())
        model_fee = m.fee
        if model_fee > t.fee:
            model_fee = 0
        if model_fee > 0:
            self.token.transfer(self.address, m.addr, model_fee)
        remaining = t.fee - model_fee
        treasury_fee = remaining - (remaining * (E18 - self.solution_fee_percentage)) // E18
        self.accrued_fees += treasury_fee
        validator_fee = remaining - treasury_fee
        sol = self.solutions[taskid]
        if validator_fee > 0:
            self.token.transfer(self.address, sol.validator, validator_fee)
        if m.rate > 0:
            total = (self.get_reward() * m.rate) // E18
            if total > 0:
                treasury_reward = total - (total * (E18 - self.treasury_reward_percentage)) // E18
                self.token.transfer(self.address, sol.validator, total - treasury_reward)
                self.token.transfer(self.address, self.treasury, treasury_reward)

    def claim_solution(self, sender, taskid):
        self._not_paused()
        taskid = _h32(taskid)
        sol = self.solutions.get(taskid, Solution())
        if sol.validator == ZERO:
            raise Revert("solution not found")
        if self.contestations.get(taskid, Contestation()).validator != ZERO:
            raise Revert("has contestation")
        if not sol.blocktime < self.timestamp - self.min_claim_solution_time:
            raise Revert("not enough delay")
        if sol.claimed:
            raise Revert("already claimed")
        sol.claimed = True
        self._emit("SolutionClaimed", self._tx(), addr=sol.validator, task=taskid)
        self._claim_solution_fees_and_reward(taskid)

    # ------------------------------------------------------------------ contestations (EngineV1.sol:893-1106)
    def submit_contestation(self, sender, taskid):
        self._not_paused()
        self._only_validator(sender)
        taskid = _h32(taskid)
        s = _addr(sender)
        sol = self.solutions.get(taskid, Solution())
        if sol.validator == ZERO:
            raise Revert("solution does not exist")
        if self.contestations.get(taskid, Contestation()).validator != ZERO:
            raise Revert("contestation already exists")
        if not self.timestamp < sol.blocktime + self.min_claim_solution_time:
            raise Revert("too late")
        if sol.claimed:
            raise Revert("wtf")
        slash = self.get_slash_amount()
        if self.validators.get(s, Validator()).staked < slash:
            raise Revert("Arithmetic operation underflowed or overflowed outside of an unchecked block")
        self.contestations[taskid] = Contestation(s, self.timestamp, 0, slash)
        tx = self._tx()
        self._emit("ContestationSubmitted", tx, addr=s, task=taskid)
        self._vote(taskid, True, s, tx)
        if self.validators.get(sol.validator, Validator()).staked >= slash:
            self._vote(taskid, False, sol.validator, tx)

    def validator_can_vote(self, addr, taskid) -> int:
        taskid = _h32(taskid)
        a = _addr(addr)
        c = self.contestations.get(taskid, Contestation())
        if c.validator == ZERO:
            return 0x01
        if self.timestamp > c.blocktime + self.min_contestation_vote_period_time:
            return 0x02
        if self.contestation_voted.get((taskid, a)):
            return 0x03
        v = self.validators.get(a, Validator())
        if v.since == 0:
            return 0x04
        if v.since < self.max_contestation_validator_stake_since:
            return 0x05
        if v.since - self.max_contestation_validator_stake_since > c.blocktime:
            return 0x06
        return 0x00

    def _vote(self, taskid, yea, addr, tx):
        self.contestation_voted[(taskid, addr)] = True
        (self.vote_yeas if yea else self.vote_nays).setdefault(taskid, []).append(addr)
        v = self.validators.setdefault(addr, Validator(0, 0, addr))
        slash = self.contestations[taskid].slash_amount
        if v.staked < slash:
            raise Revert("Arithmetic operation underflowed or overflowed outside of an unchecked block")
        v.staked -= slash
        self._emit("ContestationVote", tx, addr=addr, task=taskid, yea=bool(yea))

    def vote_on_contestation(self, sender, taskid, yea: bool):
        self._not_paused()
        self._only_validator(sender)
        taskid = _h32(taskid)
        if self.validator_can_vote(sender, taskid) != 0:
            raise Revert("not allowed")
        self._vote(taskid, bool(yea), _addr(sender), self._tx())

    def contestation_vote_finish(self, sender, taskid, amnt: int):
        self._not_paused()
        taskid = _h32(taskid)
        c = self.contestations.get(taskid, Contestation())
        if c.validator == ZERO:
            raise Revert("contestation doesn't exist")
        if not self.timestamp >= c.blocktime + self.min_contestation_vote_period_time:
            raise Revert("voting period not ended")
        if not amnt > 0:
            raise Revert("amnt too small")
        yeas = self.vote_yeas.get(taskid, [])
        nays = self.vote_nays.get(taskid, [])
        ya, na = len(yeas), len(nays)
        start, end = c.finish_start_index, c.finish_start_index + amnt
        slash = c.slash_amount
        if ya > na:
            total = na * slash
            to_orig = total if ya == 1 else total - total // 2
            to_other = 0 if ya == 1 else (total - to_orig) // (ya - 1)
            for i in range(start, end):
                if i < ya:
                    a = yeas[i]
                    self.validators[a].staked += slash
                    self.token.transfer(self.address, a, to_orig if i == 0 else to_other)
            if c.finish_start_index == 0:
                t = self.tasks[taskid]
                self.token.transfer(self.address, t.owner, t.fee)
        else:
            total = ya * slash
            to_acc = total if na == 1 else total // 2
            to_other = 0 if na == 1 else (total - to_acc) // (na - 1)
            for i in range(start, end):
                if i < na:
                    a = nays[i]
                    self.validators[a].staked += slash
                    self.token.transfer(self.address, a, to_acc if i == 0 else to_other)
            if c.finish_start_index == 0:
                self._claim_solution_fees_and_reward(taskid)
        c.finish_start_index = end
        self._emit("ContestationVoteFinish", self._tx(), id=taskid, start_idx=start, end_idx=end)

    # ------------------------------------------------------------------ getters mirroring the ABI tuples
    def get_task(self, taskid):
        t = self.tasks.get(_h32(taskid), Task())
        return t

    def get_solution(self, taskid):
        return self.solutions.get(_h32(taskid), Solution())

    def get_contestation(self, taskid):
        return self.contestations.get(_h32(taskid), Contestation())

    def get_validator(self, addr):
        return self.validators.get(_addr(addr), Validator())
