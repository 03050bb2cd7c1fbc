"""A local Ethereum JSON-RPC node backed by MockEngine (the role of the reference's
``npx hardhat node`` + ``setup_local.sh`` for manual end-to-end runs).

Speaks enough of the JSON-RPC API for ``RpcChainClient`` and any ethers/web3
client: chainId, blockNumber, getBalance, getTransactionCount, gasPrice,
estimateGas, call, sendRawTransaction (signature recovered, nonce checked),
getTransactionReceipt, getTransactionByHash, getLogs, plus hardhat's
``evm_increaseTime`` / ``evm_mine``.

    python -m arbius_amd.chain.mock_node --port 8545

Production-shaped mode (``block_time_s`` > 0): transactions enter a per-sender mempool (future
nonces are held, a same-nonce replacement must outbid by 10 %, ``pending`` nonces count the
consecutive run) and a block producer mines everything executable every ``block_time_s`` in ONE
block.  ``latency_s`` delays every HTTP request (one delay per JSON-RPC batch), ``clock`` drives
block timestamps (accelerated simulations), ``drop_next`` silently loses accepted transactions
(a sequencer / mempool drop) and ``load_rate`` submits tasks from a user account every block
(the offered load of a node benchmark).  JSON-RPC batches (arrays) are answered element-wise.
"""
from __future__ import annotations

import argparse
import asyncio
import bisect
import json
from typing import Callable, Dict, List, Optional

from aiohttp import web

from . import abi
import re

from .engine_abi import ENGINE_PARAMS, FUNCS, encode_log
from .mock_engine import MockEngine, Revert
from .tx import decode_raw_tx

TOKEN_ADDRESS = "0xe3dbc4f88eaa632ddf9708732e2832eeaa6688ab"
DEFAULT_ETH = 10 * 10 ** 18      # every account starts funded (hardhat-node style)


def _snake(name: str) -> str:
    return re.sub(r"(?<!^)(?=[A-Z])", "_", name).lower()


def _h(b: bytes) -> str:
    return "0x" + b.hex()


class MockNode:
    def __init__(self, engine: MockEngine = None, token_address: str = TOKEN_ADDRESS, latency_s: float = 0.0,
                 block_time_s: float = 0.0, clock: Optional[Callable[[], float]] = None):
        from .mock_governance import MockBaseToken
        self.engine = engine or MockEngine(MockBaseToken(address=token_address))
        if getattr(self.engine.token, "clock", False) is None:
            self.engine.token.clock = self.engine
        self.token_address = token_address.lower()
        self.nonces: Dict[str, int] = {}
        self.eth: Dict[str, int] = {}
        self.receipts: Dict[str, dict] = {}
        self.txs: Dict[str, dict] = {}
        self.by_selector = {abi.selector(sig): (name, sig, rets) for name, (sig, rets) in FUNCS.items()}
        self.contracts: Dict[str, object] = {}     # extra twins by address (governance: deploy_basic)
        self.latency_s = latency_s
        self.block_time_s = block_time_s
        self.clock = clock
        self.mempool: Dict[str, Dict[int, tuple]] = {}   # sender -> nonce -> (fields, hash)
        self.drop_next = 0
        self.dropped: List[str] = []
        self.min_gas_price = 0                          # mempool txs priced below it are held, not mined
        self.load: Optional[dict] = None                # {"rate", "model", "user", "input", "acc", "n"}
        self.stats = {"requests": 0, "calls": 0, "blocks": 0, "mined_txs": 0, "replaced": 0}
        self._ev_blocks: List[int] = []                 # block of engine.events[i] (getLogs bisect)

    # ------------------------------------------------------------------ views
    def _view(self, to: str, data: bytes) -> bytes:
        e, tok = self.engine, self.engine.token
        from .mock_governance import call_view
        if to in self.contracts:
            return call_view(self.contracts[to], data)
        if to == self.token_address and hasattr(tok, "VIEWS") and data[:4] not in self.by_selector:
            return call_view(tok, data)
        name, sig, rets = self.by_selector[data[:4]]
        args = abi.decode_call(sig, data)
        b32 = lambda x: x  # noqa: E731
        if to == self.token_address:
            if name == "balanceOf":
                return abi.encode(rets, [tok.balance_of(args[0])])
            if name == "allowance":
                return abi.encode(rets, [tok.allowance(args[0], args[1])])
            raise Revert(f"unsupported token view {name}")
        if name == "tasks":
            t = e.get_task(b32(args[0]))
            return abi.encode(rets, [t.model, t.fee, t.owner, t.blocktime, t.version, t.cid])
        if name == "solutions":
            s = e.get_solution(args[0])
            return abi.encode(rets, [s.validator, s.blocktime, s.claimed, s.cid])
        if name == "contestations":
            c = e.get_contestation(args[0])
            return abi.encode(rets, [c.validator, c.blocktime, c.finish_start_index, c.slash_amount])
        if name == "contestationVoted":
            return abi.encode(rets, [bool(e.contestation_voted.get((args[0].lower(), args[1].lower())))])
        if name == "validators":
            v = e.get_validator(args[0])
            return abi.encode(rets, [v.staked, v.since, v.addr])
        if name == "getValidatorMinimum":
            return abi.encode(rets, [e.get_validator_minimum()])
        if name == "version":
            return abi.encode(rets, [e.version])
        if name == "paused":
            return abi.encode(rets, [e.paused])
        if name == "getReward":
            return abi.encode(rets, [e.get_reward()])
        if name == "getPsuedoTotalSupply":
            return abi.encode(rets, [e.get_psuedo_total_supply()])
        if name == "accruedFees":
            return abi.encode(rets, [e.accrued_fees])
        if name == "generateCommitment":
            return abi.encode(rets, [e.generate_commitment(*args)])
        if name == "generateIPFSCID":
            return abi.encode(rets, [e.generate_ipfs_cid(bytes.fromhex(args[0][2:]))])
        if name == "validatorCanVote":
            return abi.encode(rets, [e.validator_can_vote(args[0], args[1])])
        if name in ("owner", "treasury", "pauser"):
            return abi.encode(rets, [getattr(e, name)])
        if name in ENGINE_PARAMS:
            return abi.encode(rets, [int(getattr(e, _snake(name)))])
        if name == "commitments":
            return abi.encode(rets, [e.commitments.get(args[0].lower(), 0)])
        if name in ("contestationVoteYeas", "contestationVoteNays"):
            lst = (e.vote_yeas if name.endswith("Yeas") else e.vote_nays).get(args[0].lower(), [])
            if args[1] >= len(lst):
                raise Revert("index out of bounds")      # solidity array getter: Panic(0x32)
            return abi.encode(rets, [lst[args[1]]])
        if name == "models":
            m = e.models.get(args[0].lower())
            return abi.encode(rets, [m.fee, m.addr, m.rate, m.cid] if m else [0, "0x" + "00" * 20, 0, b""])
        raise Revert(f"unsupported view {name}")

    # ------------------------------------------------------------------ transactions
    def _exec(self, sender: str, to: str, data: bytes):
        e, tok = self.engine, self.engine.token
        from .mock_governance import dispatch
        if to in self.contracts:
            dispatch(self.contracts[to], sender, data)
            return
        if to == self.token_address and hasattr(tok, "ABI") and data[:4] not in self.by_selector:
            dispatch(tok, sender, data)             # delegate / bridgeMint / ... (BaseTokenV1)
            return
        name, sig, rets = self.by_selector[data[:4]]
        args = abi.decode_call(sig, data)
        raw = lambda x: bytes.fromhex(x[2:])  # noqa: E731
        if to == self.token_address:
            if name == "approve":
                tok.approve(sender, args[0], args[1])
            elif name == "transfer":
                tok.transfer(sender, args[0], args[1])
            else:
                raise Revert(f"unsupported token method {name}")
            e.mine(1)
            return
        dispatch = {
            "submitTask": lambda: e.submit_task(sender, args[0], args[1], args[2], args[3], raw(args[4])),
            "signalCommitment": lambda: e.signal_commitment(sender, args[0]),
            "submitSolution": lambda: e.submit_solution(sender, args[0], args[1]),
            "claimSolution": lambda: e.claim_solution(sender, args[0]),
            "submitContestation": lambda: e.submit_contestation(sender, args[0]),
            "voteOnContestation": lambda: e.vote_on_contestation(sender, args[0], args[1]),
            "contestationVoteFinish": lambda: e.contestation_vote_finish(sender, args[0], args[1]),
            "validatorDeposit": lambda: e.validator_deposit(sender, args[0], args[1]),
            "registerModel": lambda: e.register_model(sender, args[0], args[1], raw(args[2])),
            "signalSupport": lambda: e.signal_support(sender, args[0], args[1]),
            "retractTask": lambda: e.retract_task(sender, args[0]),
            "withdrawAccruedFees": lambda: e.withdraw_accrued_fees(sender),
            "setPaused": lambda: e.set_paused(sender, args[0]),
            "initiateValidatorWithdraw": lambda: e.initiate_validator_withdraw(sender, args[0]),
            "validatorWithdraw": lambda: e.validator_withdraw(sender, args[0], args[1]),
            "cancelValidatorWithdraw": lambda: e.cancel_validator_withdraw(sender, args[0]),
            "transferOwnership": lambda: e.transfer_ownership(sender, args[0]),
            "transferTreasury": lambda: e.transfer_treasury(sender, args[0]),
            "transferPauser": lambda: e.transfer_pauser(sender, args[0]),
            "setSolutionMineableRate": lambda: e.set_solution_mineable_rate(sender, args[0], args[1]),
            "setVersion": lambda: e.set_version(sender, args[0]),
        }
        for p in ENGINE_PARAMS:
            setter = "set" + p[0].upper() + p[1:]
            dispatch[setter] = (lambda p=p: e.set_param(sender, _snake(p), args[0]))
        if name not in dispatch:
            raise Revert(f"unsupported method {name}")
        dispatch[name]()

    def send_raw(self, raw_hex: str) -> str:
        raw = bytes.fromhex(raw_hex[2:])
        f, sender = decode_raw_tx(raw)
        if self.block_time_s > 0:
            return self._to_mempool(f, sender)
        if not f["data"]:                      # plain value transfer (send-eth)
            return self._value_transfer(f, sender)
        if f["chain_id"] != self.engine.chain_id:
            raise ValueError("invalid chain id")
        expected = self.nonces.get(sender, 0)
        if f["nonce"] != expected:
            raise ValueError(f"nonce too {'low' if f['nonce'] < expected else 'high'}")
        return self._apply(f, sender)

    def _apply(self, f, sender) -> str:
        self.nonces[sender] = f["nonce"] + 1
        txh = f["hash"]
        n_ev = len(self.engine.events)
        status, reason = 1, None
        try:
            self._exec(sender, f["to"].lower(), f["data"])
        except Revert as ex:
            status, reason = 0, str(ex)
            if not getattr(self.engine, "_open_block", False):
                self.engine.mine(1)
        new = self.engine.events[n_ev:]
        for ev in new:
            ev.tx = txh
        blk = self.engine.block_number
        logs = []
        for ev in new:
            topics, data = encode_log(ev.name, ev.args) if ev.name in _LOGGABLE else ([], b"")
            if topics:
                logs.append({"address": self.engine.address, "topics": topics, "data": _h(data),
                             "blockNumber": hex(ev.block), "transactionHash": txh, "logIndex": hex(ev.index)})
        self.receipts[txh] = {"transactionHash": txh, "status": hex(status), "blockNumber": hex(blk), "logs": logs,
                              "revertReason": reason}
        self.txs[txh] = {"hash": txh, "from": sender, "to": f["to"], "input": _h(f["data"]),
                         "nonce": hex(f["nonce"]), "blockNumber": hex(blk)}
        return txh

    # ------------------------------------------------------------------ mempool + blocks
    def _price(self, f) -> int:
        return int(f.get("gas_price") or f.get("max_fee") or 0)

    def _to_mempool(self, f, sender) -> str:
        if f["chain_id"] is not None and f["chain_id"] != self.engine.chain_id:
            raise ValueError("invalid chain id")
        mined = self.nonces.get(sender, 0)
        if f["nonce"] < mined:
            raise ValueError("nonce too low")
        pool = self.mempool.setdefault(sender, {})
        old = pool.get(f["nonce"])
        if old is not None:
            if old[1] == f["hash"]:
                raise ValueError("already known")
            if self._price(f) * 10 < self._price(old[0]) * 11:
                raise ValueError("replacement transaction underpriced")
            self.stats["replaced"] += 1
        if self.drop_next > 0:                 # accepted, then lost by the sequencer
            self.drop_next -= 1
            self.dropped.append(f["hash"])
            return f["hash"]
        pool[f["nonce"]] = (f, f["hash"])
        return f["hash"]

    def pending_nonce(self, sender: str) -> int:
        n = self.nonces.get(sender, 0)
        pool = self.mempool.get(sender, {})
        while n in pool:
            n += 1
        return n

    def produce_block(self):
        """Mine every executable mempool transaction (consecutive nonces per sender) in ONE block,
        plus this block's share of the offered task load."""
        e = self.engine
        if self.clock is not None:
            e.timestamp = max(e.timestamp + 1, int(self.clock()))
        else:
            e.timestamp += max(1, int(round(self.block_time_s)))
        with e.one_block():
            self._load_block()
            for sender in list(self.mempool):
                pool = self.mempool[sender]
                n = self.nonces.get(sender, 0)
                for k in [k for k in pool if k < n]:
                    del pool[k]
                while n in pool and self._price(pool[n][0]) >= self.min_gas_price:
                    f, _ = pool.pop(n)
                    if not f["data"]:
                        self._value_transfer(f, sender, mine=False)
                    else:
                        self._apply(f, sender)
                    self.stats["mined_txs"] += 1
                    n += 1
                if not pool:
                    del self.mempool[sender]
        self.stats["blocks"] += 1

    def _load_block(self):
        ld = self.load
        if not ld:
            return
        ld["acc"] += ld["rate"] * self.block_time_s
        sig = FUNCS["submitTask"][0]
        while ld["acc"] >= 1.0:
            ld["acc"] -= 1.0
            i = ld["n"]
            ld["n"] += 1
            inp = json.dumps(dict(ld["input"], prompt=f"{ld['input'].get('prompt', 'task')} #{i}")).encode()
            data = abi.encode_call(sig, 0, ld["user"], ld["model"], 0, inp)
            from ..utils.keccak import keccak256
            txh = "0x" + keccak256(b"load" + i.to_bytes(8, "big") + data).hex()
            n_ev = len(self.engine.events)
            self._exec(ld["user"], self.engine.address, data)
            for ev in self.engine.events[n_ev:]:
                ev.tx = txh
            blk = self.engine.block_number
            self.receipts[txh] = {"transactionHash": txh, "status": "0x1", "blockNumber": hex(blk), "logs": [],
                                  "revertReason": None}
            self.txs[txh] = {"hash": txh, "from": ld["user"], "to": self.engine.address, "input": _h(data),
                             "nonce": hex(i), "blockNumber": hex(blk)}

    async def block_loop(self):
        while True:
            await asyncio.sleep(self.block_time_s)
            self.produce_block()

    def _value_transfer(self, f, sender, mine: bool = True):
        expected = self.nonces.get(sender, 0)
        if f["nonce"] != expected:
            raise ValueError("nonce mismatch")
        self.nonces[sender] = expected + 1
        bal = self.eth.get(sender, DEFAULT_ETH)
        if bal < f["value"]:
            raise ValueError("insufficient funds")
        to = f["to"].lower()
        self.eth[sender] = bal - f["value"]
        self.eth[to] = self.eth.get(to, DEFAULT_ETH) + f["value"]
        if mine:
            self.engine.mine(1)
        txh = f["hash"]
        self.receipts[txh] = {"transactionHash": txh, "status": "0x1", "blockNumber": hex(self.engine.block_number),
                              "logs": [], "revertReason": None}
        self.txs[txh] = {"hash": txh, "from": sender, "to": f["to"], "input": "0x", "value": hex(f["value"]),
                         "nonce": hex(f["nonce"]), "blockNumber": hex(self.engine.block_number)}
        return txh

    def get_logs(self, flt: dict):
        lo = int(flt.get("fromBlock", "0x0"), 16)
        hi_raw = flt.get("toBlock", "latest")
        hi = self.engine.block_number if hi_raw == "latest" else int(hi_raw, 16)
        evs = self.engine.events
        blocks = self._ev_blocks
        if len(blocks) > len(evs):
            blocks.clear()
        blocks.extend(ev.block for ev in evs[len(blocks):])    # events append in block order
        start = bisect.bisect_left(blocks, lo)
        out = []
        for ev in evs[start:]:
            if ev.block > hi:
                break
            if lo <= ev.block and ev.name in _LOGGABLE:
                topics, data = encode_log(ev.name, ev.args)
                out.append({"address": self.engine.address, "topics": topics, "data": _h(data),
                            "blockNumber": hex(ev.block), "transactionHash": ev.tx, "logIndex": hex(ev.index)})
        return out

    # ------------------------------------------------------------------ JSON-RPC
    def handle(self, method: str, params: list):
        e = self.engine
        if method == "eth_chainId":
            return hex(e.chain_id)
        if method == "net_version":
            return str(e.chain_id)
        if method == "eth_blockNumber":
            return hex(e.block_number)
        if method == "eth_getBalance":
            return hex(self.eth.get(params[0].lower(), DEFAULT_ETH))
        if method == "eth_getTransactionCount":
            a = params[0].lower()
            if len(params) > 1 and params[1] == "pending" and self.block_time_s > 0:
                return hex(self.pending_nonce(a))
            return hex(self.nonces.get(a, 0))
        if method == "eth_gasPrice":
            return hex(max(10 ** 8, self.min_gas_price))
        if method == "eth_estimateGas":
            return hex(500_000)
        if method == "eth_call":
            c = params[0]
            return _h(self._view(c["to"].lower(), bytes.fromhex(c["data"][2:])))
        if method == "eth_sendRawTransaction":
            return self.send_raw(params[0])
        if method == "eth_getTransactionReceipt":
            return self.receipts.get(params[0])
        if method == "eth_getTransactionByHash":
            return self.txs.get(params[0])
        if method == "eth_getLogs":
            return self.get_logs(params[0])
        if method == "evm_increaseTime":
            e.timestamp += int(params[0])
            return hex(int(params[0]))
        if method == "evm_mine":
            if self.block_time_s > 0:
                self.produce_block()
            else:
                e.mine(1)
            return "0x0"
        if method == "arbius_dropNext":          # test hook: lose the next N accepted transactions
            self.drop_next += int(params[0])
            return hex(self.drop_next)
        if method == "arbius_minGasPrice":       # test hook: the base fee rises (held txs need a bump)
            self.min_gas_price = int(params[0])
            return hex(self.min_gas_price)
        if method == "arbius_load":              # test hook: offered task load (tasks/s, model id, user)
            rate, model, user = float(params[0]), params[1], params[2].lower()
            self.load = {"rate": rate, "model": model, "user": user, "acc": 0.0,
                         "n": (self.load or {}).get("n", 0), "input": params[3] if len(params) > 3 else {}}
            return "0x1"
        if method == "arbius_stats":
            return dict(self.stats, dropped=list(self.dropped), tasks=len(e.tasks), solutions=len(e.solutions),
                        claimed=sum(1 for x in e.solutions.values() if x.claimed),
                        mempool=sum(len(v) for v in self.mempool.values()), block=e.block_number,
                        timestamp=e.timestamp)
        raise KeyError(method)

    def _answer(self, body):
        self.stats["calls"] += 1
        rid = body.get("id") if isinstance(body, dict) else None
        try:
            res = self.handle(body["method"], body.get("params", []))
            return {"jsonrpc": "2.0", "id": rid, "result": res}
        except Revert as ex:
            return {"jsonrpc": "2.0", "id": rid, "error": {"code": 3, "message": f"execution reverted: {ex}"}}
        except Exception as ex:  # noqa: BLE001
            return {"jsonrpc": "2.0", "id": rid, "error": {"code": -32000, "message": str(ex)}}

    def app(self) -> web.Application:
        app = web.Application()

        async def rpc(req):
            body = await req.json()
            self.stats["requests"] += 1
            if self.latency_s > 0:
                await asyncio.sleep(self.latency_s)
            if isinstance(body, list):
                return web.json_response([self._answer(b) for b in body])
            return web.json_response(self._answer(body))

        async def start_blocks(app_):
            if self.block_time_s > 0:
                app_[_BLOCKS] = asyncio.ensure_future(self.block_loop())

        async def stop_blocks(app_):
            t = app_.get(_BLOCKS)
            if t is not None:
                t.cancel()

        app.on_startup.append(start_blocks)
        app.on_cleanup.append(stop_blocks)
        app.router.add_post("/", rpc)
        return app


_BLOCKS = web.AppKey("blocks", asyncio.Task)
_LOGGABLE = {"TaskSubmitted", "TaskRetracted", "SignalCommitment", "SolutionSubmitted", "SolutionClaimed",
             "ContestationSubmitted", "ContestationVote", "ContestationVoteFinish", "VersionChanged",
             "ModelRegistered", "ValidatorDeposit"}


def deploy_basic(node: "MockNode", deployer: str, engine_supply: int = 597_000 * 10 ** 18,
                 governance: bool = False) -> dict:
    """``scripts/003-deploy-core-basic.ts`` on the mock chain: the deployer owns the
    engine and is treasury, the engine holds the mining supply, and kandinsky2 is
    registered as a FREE mineable model (addr 0x..01, fee 0) with rate 1e18."""
    from ..node.models import template_bytes
    e, tok = node.engine, node.engine.token
    deployer = deployer.lower()
    e.owner = e.treasury = e.pauser = deployer
    tok.mint(e.address, engine_supply)
    addr = "0x" + "00" * 19 + "01"
    mid = e.register_model(deployer, addr, 0, template_bytes("kandinsky2"))
    e.set_solution_mineable_rate(deployer, mid, 10 ** 18)
    out = {"engineAddress": e.address, "baseTokenAddress": node.token_address,
           "models": {"kandinsky2": {"id": mid, "mineable": True,
                                     "params": {"addr": addr, "fee": "0", "rate": str(10 ** 18)}}}}
    if governance:      # governance.test.ts fixture: Timelock (3 days) owns the Engine, Governor proposes
        from .mock_governance import deploy_governance
        tok.l2_gateway = deployer
        _, tl, gov, reg = deploy_governance(e, deployer)
        node.contracts.update({tl.address: tl, gov.address: gov})
        out.update(timelockAddress=tl.address, governorAddress=gov.address)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description="local mock Arbius chain (JSON-RPC)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8545)
    ap.add_argument("--deploy", default=None, metavar="DEPLOYER",
                    help="run the 003-deploy-core-basic equivalent for this deployer address")
    ap.add_argument("--governance", action="store_true",
                    help="with --deploy: also deploy Timelock + Governor (the engine's owner becomes the timelock)")
    a = ap.parse_args(argv)
    node = MockNode()
    if a.deploy:
        import json
        print(json.dumps(deploy_basic(node, a.deploy, governance=a.governance), indent=2), flush=True)  # noqa: T201
    web.run_app(node.app(), host=a.host, port=a.port)


if __name__ == "__main__":
    main()
