"""A local Ethereum JSON-RPC node backed by MockEngine (the role of the reference's
``npx hardhat node`` + ``setup_local.sh`` for manual end-to-end runs).

Speaks enough of the JSON-RPC API for ``RpcChainClient`` and any ethers/web3
client: chainId, blockNumber, getBalance, getTransactionCount, gasPrice,
estimateGas, call, sendRawTransaction (signature recovered, nonce checked),
getTransactionReceipt, getTransactionByHash, getLogs, plus hardhat's
``evm_increaseTime`` / ``evm_mine``.

    python -m arbius_amd.chain.mock_node --port 8545
"""
from __future__ import annotations

import argparse
from typing import Dict

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
    def __init__(self, engine: MockEngine = None, token_address: str = TOKEN_ADDRESS):
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
        if not f["data"]:                      # plain value transfer (send-eth)
            return self._value_transfer(f, sender)
        if f["chain_id"] != self.engine.chain_id:
            raise ValueError("invalid chain id")
        expected = self.nonces.get(sender, 0)
        if f["nonce"] != expected:
            raise ValueError(f"nonce too {'low' if f['nonce'] < expected else 'high'}")
        self.nonces[sender] = expected + 1
        txh = f["hash"]
        n_ev = len(self.engine.events)
        status, reason = 1, None
        try:
            self._exec(sender, f["to"].lower(), f["data"])
        except Revert as ex:
            status, reason = 0, str(ex)
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

    def _value_transfer(self, f, sender):
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
        out = []
        for ev in self.engine.events:
            if lo <= ev.block <= hi and ev.name in _LOGGABLE:
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
            return hex(self.nonces.get(params[0].lower(), 0))
        if method == "eth_gasPrice":
            return hex(10 ** 8)
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
            e.mine(1)
            return "0x0"
        raise KeyError(method)

    def app(self) -> web.Application:
        app = web.Application()

        async def rpc(req):
            body = await req.json()
            try:
                res = self.handle(body["method"], body.get("params", []))
                return web.json_response({"jsonrpc": "2.0", "id": body.get("id"), "result": res})
            except Revert as ex:
                return web.json_response({"jsonrpc": "2.0", "id": body.get("id"),
                                          "error": {"code": 3, "message": f"execution reverted: {ex}"}})
            except Exception as ex:  # noqa: BLE001
                return web.json_response({"jsonrpc": "2.0", "id": body.get("id"),
                                          "error": {"code": -32000, "message": str(ex)}})

        app.router.add_post("/", rpc)
        return app


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
