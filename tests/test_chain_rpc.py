"""The real JSON-RPC chain client (signing, nonces, eth_call/getLogs decoding)
against the local mock node, and the whole miner over JSON-RPC."""
import asyncio
import json

from aiohttp.test_utils import TestServer

from arbius_amd.chain import abi
from arbius_amd.chain.engine_abi import decode_log, encode_log
from arbius_amd.chain.mock_engine import E18, MockEngine, MockToken
from arbius_amd.chain.mock_node import TOKEN_ADDRESS, MockNode
from arbius_amd.chain.rpc import RpcChainClient
from arbius_amd.chain.secp256k1 import address_from_priv
from arbius_amd.config.mining_config import MiningConfig
from arbius_amd.ipfs.pin import LocalPinner
from arbius_amd.node.miner import Miner
from arbius_amd.node.models import default_models, template_bytes
from arbius_amd.node.pool import FakeSolverPool
from arbius_amd.store.db import DB

MINER_KEY = "0x" + "11" * 32
USER_KEY = "0x" + "22" * 32


def test_log_codec_roundtrip():
    args = {"id": "0x" + "ab" * 32, "model": "0x" + "cd" * 32, "fee": 7, "sender": "0x" + "12" * 20}
    topics, data = encode_log("TaskSubmitted", args)
    assert topics[0] == abi.topic("TaskSubmitted(bytes32,bytes32,uint256,address)")
    name, dec = decode_log(topics, data)
    assert name == "TaskSubmitted" and dec == args


def _world():
    tok = MockToken()
    e = MockEngine(tok, owner="0x" + "0e" * 20, chain_id=42170)  # Nova: ArbSys block numbers
    miner, user = address_from_priv(MINER_KEY), address_from_priv(USER_KEY)
    tok.mint(e.address, 597000 * E18)
    tok.mint(miner, 10 * E18)
    tok.mint(user, 10 * E18)
    mid = e.register_model(user, user, 0, template_bytes("anythingv3"))
    return e, mid, miner, user


def test_miner_over_jsonrpc():
    e, mid, miner_addr, user_addr = _world()
    node = MockNode(e, TOKEN_ADDRESS)
    # the node's token contract address is a separate namespace from MockToken addresses
    e.token_address = TOKEN_ADDRESS

    async def go():
        server = TestServer(node.app())
        await server.start_server()
        url = str(server.make_url("/"))
        try:
            mc = RpcChainClient(url, MINER_KEY, e.address, TOKEN_ADDRESS, receipt_poll=0.001)
            uc = RpcChainClient(url, USER_KEY, e.address, TOKEN_ADDRESS, receipt_poll=0.001)
            assert mc.address == miner_addr
            assert await mc.version() == 0
            assert await mc.token_balance(miner_addr) == 10 * E18
            cfg = MiningConfig.from_dict({})
            m = Miner(cfg, DB(":memory:"), mc, LocalPinner(), FakeSolverPool(), default_models({"anythingv3": mid}),
                      clock=lambda: e.timestamp, retry_sleep=lambda s: asyncio.sleep(0))
            await m.boot()
            await m.poll_events()
            await m.drain()  # validatorStake: approve + deposit through signed txs
            assert e.validators[miner_addr].staked > 0
            await uc.token_approve(e.address, 2 ** 256 - 1)
            await uc.submit_task(0, user_addr, mid, 0, json.dumps({"prompt": "p", "negative_prompt": "n"}).encode())
            tid = e.prevhash
            await m.poll_events()
            await m.drain()
            s = await mc.get_solution(tid)
            assert s["validator"] == miner_addr and s["cid"].startswith("0x1220")
            node.handle("evm_increaseTime", [2200])
            node.handle("evm_mine", [])
            await m.drain()
            assert (await mc.get_solution(tid))["claimed"]
            # nonces are sequential per sender and the node saw every tx signed by us
            assert node.nonces[miner_addr] == len([t for t in node.txs.values() if t["from"] == miner_addr])
            await mc.close()
            await uc.close()
        finally:
            await server.close()

    asyncio.run(go())


def test_operator_cli_against_mock_node(tmp_path, capsys):
    """contract/tasks/index.ts operator tasks over JSON-RPC: deploy, accounts, params,
    admin setters, pause, send-eth, transfer, timetravel, explorer, task."""
    import json as _json
    import threading
    import time as _time

    from aiohttp import web as _web

    from arbius_amd import cli
    from arbius_amd.chain.mock_node import MockNode, deploy_basic
    from arbius_amd.chain.secp256k1 import address_from_priv

    key = "0x" + "42" * 32
    me = address_from_priv(key)
    node = MockNode()
    info = deploy_basic(node, me)
    node.engine.token.mint(me, 100 * 10 ** 18)
    port = _free()
    loop = asyncio.new_event_loop()
    runner = _web.AppRunner(node.app())

    def serve():
        asyncio.set_event_loop(loop)
        loop.run_until_complete(runner.setup())
        loop.run_until_complete(_web.TCPSite(runner, "127.0.0.1", port).start())
        loop.run_forever()

    th = threading.Thread(target=serve, daemon=True)
    th.start()
    _time.sleep(0.5)
    cfgp = tmp_path / "cfg.json"
    cfgp.write_text(_json.dumps({"blockchain": {"private_key": key, "rpc_url": f"http://127.0.0.1:{port}"},
                                 "mi355x": {"chain_id": node.engine.chain_id}}))
    import arbius_amd.node.models as nm
    old = dict(nm.CHAIN_CONFIG)
    nm.CHAIN_CONFIG["engineAddress"] = node.engine.address
    nm.CHAIN_CONFIG["baseTokenAddress"] = node.token_address
    try:
        c = ["-c", str(cfgp)]
        cli.main(["params"] + c)
        params = _json.loads(capsys.readouterr().out)
        assert params["minClaimSolutionTime"] == "2000" and params["owner"].lower() == me.lower()
        cli.main(["admin", "setMinClaimSolutionTime", "1500"] + c)
        cli.main(["admin", "setVersion", "3"] + c)
        assert node.engine.min_claim_solution_time == 1500 and node.engine.version == 3
        cli.main(["engine-pause", "true"] + c)
        assert node.engine.paused
        cli.main(["engine-pause", "false"] + c)
        other = "0x" + "99" * 20
        cli.main(["send-eth", other, "1.5"] + c)
        assert node.eth[other] == 10 * 10 ** 18 + 15 * 10 ** 17
        cli.main(["transfer", other, "2"] + c)
        assert node.engine.token.balance_of(other) == 2 * 10 ** 18
        t0 = node.engine.timestamp
        cli.main(["timetravel", "100"] + c)
        assert node.engine.timestamp >= t0 + 100
        capsys.readouterr()
        cli.main(["explorer", "1000"] + c)
        evs = [_json.loads(x) for x in capsys.readouterr().out.splitlines()]
        assert any(e["event"] == "VersionChanged" for e in evs)
        mid = info["models"]["kandinsky2"]["id"]
        assert node.engine.models[mid.lower()].rate == 10 ** 18
    finally:
        nm.CHAIN_CONFIG.clear()
        nm.CHAIN_CONFIG.update(old)
        loop.call_soon_threadsafe(loop.stop)


def _free():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p
