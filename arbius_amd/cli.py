"""Command line: the miner (``yarn start MiningConfig.json``, miner/src/start.ts) and
the operator tasks of ``contract/tasks/index.ts`` that a miner needs.

    python -m arbius_amd start MiningConfig.json
    python -m arbius_amd mock-node --port 8545          # local chain (hardhat node analog)
    python -m arbius_amd gen-wallet
    python -m arbius_amd cid FILE [--wrap NAME]         # CIDv0 without a daemon
    python -m arbius_amd decode-calldata 0x08745dd1...  # submitTask input (decode-tx)
    python -m arbius_amd decode-tx TXHASH -c cfg.json
    python -m arbius_amd model-register TEMPLATE --fee 0 -c cfg.json
    python -m arbius_amd validator-stake AMOUNT -c cfg.json
    python -m arbius_amd balance -c cfg.json
    python -m arbius_amd claim TASKID -c cfg.json
    python -m arbius_amd signal-support MODEL true -c cfg.json
    python -m arbius_amd is-paused -c cfg.json
    python -m arbius_amd submit-task MODEL '{"prompt":"..."}' --fee 0 -c cfg.json
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import secrets
import subprocess
import sys
from pathlib import Path

log = logging.getLogger("arbius")
E18 = 10 ** 18


def _fmt(wei: int) -> str:
    return f"{wei / E18:.6f}"


def _chain(cfg):
    from .chain.rpc import RpcChainClient
    from .node.models import CHAIN_CONFIG
    return RpcChainClient(cfg.blockchain.rpc_url, cfg.blockchain.private_key, CHAIN_CONFIG["engineAddress"],
                          CHAIN_CONFIG["baseTokenAddress"], chain_id=cfg.mi355x.chain_id)


def _cfg(path):
    from .config.mining_config import MiningConfig
    return MiningConfig.load(path)


def build_pool(cfg, models):
    """Solver pool from MiningConfig: cog/replicate (reference strategies) or the
    in-process MI355X engine (one worker process per GPU)."""
    if cfg.ml.strategy == "cog" and cfg.ml.cog and any(e.url and e.url != "CHANGEME" for e in cfg.ml.cog.values()):
        from .node.external import CogSolverPool
        return CogSolverPool({k: e.url for k, e in cfg.ml.cog.items()})
    if cfg.ml.strategy == "replicate" and cfg.ml.replicate.api_token:
        from .node.external import ReplicateSolverPool
        return ReplicateSolverPool(cfg.ml.replicate.api_token)
    import torch
    names = sorted({m.name for m in models.values()})
    n = cfg.mi355x.gpus if cfg.mi355x.gpus is not None else (torch.cuda.device_count() if torch.cuda.is_available() else 0)
    if n > 1:
        from .parallel.workers import MultiGPUSolverPool
        return MultiGPUSolverPool(n, names, "cuda")
    from .node.pool import LocalSolverPool
    return LocalSolverPool("cuda:0" if n == 1 else "cpu", weights_dir=cfg.mi355x.weights_dir)


async def _start(path: str):
    from .config.mining_config import MiningConfig
    from .ipfs.pin import make_pinner
    from .node.miner import Miner
    from .node.models import default_models
    from .node.rpc import start_rpc
    from .store.db import DB
    from .utils.log import init_logging

    try:
        cfg = MiningConfig.load(path)
    except Exception as e:  # noqa: BLE001
        print(f"unable to parse {path}: {e}", file=sys.stderr)
        sys.exit(1)
    init_logging(cfg.log_path)
    if cfg.evilmode:
        for _ in range(20):
            log.warning("YOU HAVE EVIL MODE ENABLED, YOU WILL BE SLASHED")
            log.warning("KILL YOUR MINER IMMEDIATELY IF NOT ON TESTNET")
    try:
        rev = subprocess.check_output(["git", "rev-parse", "HEAD"], cwd=os.path.dirname(__file__),
                                      stderr=subprocess.DEVNULL).decode().strip()
        log.info("Arbius Miner (MI355X) %s starting", rev[:8])
    except Exception:  # noqa: BLE001
        log.warning('Could not run "git rev-parse HEAD" do you have git in PATH?')
    db = DB(cfg.db_path)
    if cfg.mi355x.mock_chain:
        from .chain.client import MockChainClient
        from .chain.mock_engine import MockEngine
        from .chain.secp256k1 import address_from_priv
        chain = MockChainClient(MockEngine(), address_from_priv(cfg.blockchain.private_key))
    else:
        chain = _chain(cfg)
    log.debug("Loaded wallet (%s)", chain.address)
    ids = dict(getattr(cfg.mi355x, "model_ids", {}) or {})
    models = {k: v for k, v in default_models(ids).items() if v.name in set(cfg.mi355x.models)}
    pool = build_pool(cfg, models)
    miner = Miner(cfg, db, chain, make_pinner(cfg), pool, models)
    runner = await start_rpc(db, cfg.rpc.host, cfg.rpc.port, miner)
    try:
        await miner.run()
    finally:
        await runner.cleanup()


def main(argv=None):
    ap = argparse.ArgumentParser(prog="arbius_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("start"); p.add_argument("config")
    p = sub.add_parser("mock-node"); p.add_argument("--host", default="127.0.0.1"); p.add_argument("--port", type=int, default=8545)
    sub.add_parser("gen-wallet")
    p = sub.add_parser("cid"); p.add_argument("file"); p.add_argument("--wrap", default=None)
    p = sub.add_parser("decode-calldata"); p.add_argument("data")
    for name, extra in [("decode-tx", ["txid"]), ("model-register", ["template"]), ("validator-stake", ["amount"]),
                        ("balance", []), ("claim", ["taskid"]), ("signal-support", ["model", "support"]),
                        ("is-paused", []), ("submit-task", ["model", "input"])]:
        p = sub.add_parser(name)
        for e in extra:
            p.add_argument(e)
        p.add_argument("-c", "--config", default="MiningConfig.json")
        if name in ("model-register", "submit-task"):
            p.add_argument("--fee", default="0")
    a = ap.parse_args(argv)

    if a.cmd == "start":
        asyncio.run(_start(a.config))
        return
    if a.cmd == "mock-node":
        from .chain.mock_node import main as node_main
        node_main(["--host", a.host, "--port", str(a.port)])
        return
    if a.cmd == "gen-wallet":
        from .chain.secp256k1 import address_from_priv
        k = "0x" + secrets.token_bytes(32).hex()
        print(json.dumps({"address": address_from_priv(k), "private_key": k}))
        return
    if a.cmd == "cid":
        from .ipfs.unixfs import add_file, wrap_directory
        data = Path(a.file).read_bytes()
        r = wrap_directory([(a.wrap, data)]) if a.wrap else add_file(data)
        print(json.dumps({"cid": r.cid_str, "hex": r.cid_hex}))
        return
    if a.cmd == "decode-calldata":
        from .chain import abi
        raw = bytes.fromhex(a.data[2:] if a.data.startswith("0x") else a.data)
        v, owner, model, fee, inp = abi.decode_call("submitTask(uint8,address,bytes32,uint256,bytes)", raw)
        print(json.dumps({"version": v, "owner": owner, "model": model, "fee": str(fee),
                          "input": bytes.fromhex(inp[2:]).decode("utf-8", "replace")}))
        return

    cfg = _cfg(a.config)

    async def run():
        c = _chain(cfg)
        try:
            if a.cmd == "decode-tx":
                inp = await c.get_submit_task_input(a.txid)
                print(inp.decode() if inp is not None else "not a submitTask transaction")
            elif a.cmd == "model-register":
                from .node.models import template_bytes
                tpl = Path(a.template).read_bytes() if os.path.exists(a.template) else template_bytes(a.template)
                if len(tpl) > 262144:
                    raise SystemExit("template too large")
                print(await c.register_model(c.address, int(a.fee), tpl))
            elif a.cmd == "validator-stake":
                amt = int(float(a.amount) * E18)
                await c.token_approve(c.engine_address, 2 ** 256 - 1)
                print(await c.validator_deposit(c.address, amt))
            elif a.cmd == "balance":
                v = await c.get_validator(c.address)
                print(json.dumps({"address": c.address, "eth": _fmt(await c.eth_balance(c.address)),
                                  "aius": _fmt(await c.token_balance(c.address)), "staked": _fmt(v["staked"]),
                                  "validator_minimum": _fmt(await c.get_validator_minimum())}))
            elif a.cmd == "claim":
                print(await c.claim_solution(a.taskid))
            elif a.cmd == "signal-support":
                print(await c.signal_support(a.model, a.support.lower() in ("1", "true", "yes")))
            elif a.cmd == "is-paused":
                print((await c._call(c.engine_address, "paused"))[0])
            elif a.cmd == "submit-task":
                print(await c.submit_task(0, c.address, a.model, int(a.fee), a.input.encode()))
        finally:
            await c.close()

    asyncio.run(run())


if __name__ == "__main__":
    main()
