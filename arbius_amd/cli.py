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
    python -m arbius_amd accounts | mine [N] | timetravel SECONDS -c cfg.json
    python -m arbius_amd send-eth TO AMOUNT | transfer TO AMOUNT -c cfg.json
    python -m arbius_amd engine-pause true|false | withdraw-fees | params -c cfg.json
    python -m arbius_amd admin setVersion 1 | admin setSolutionMineableRate MODEL RATE -c cfg.json
    python -m arbius_amd validator-withdraw initiate AMOUNT | cancel COUNT | withdraw COUNT -c cfg.json
    python -m arbius_amd governance delegate|propose|vote|cancel|queue|execute|proposal ... --governor ADDR
    python -m arbius_amd call TO 'sig(types)' 'ret,types' ARGS... | send TO 'sig(types)' ARGS... [--value ETH]
    python -m arbius_amd explorer [--blocks 128] | task TASKID -c cfg.json
    python -m arbius_amd pinata-gc -c cfg.json          # unpin Pinata files older than 2 h
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
    x = cfg.mi355x
    return RpcChainClient(cfg.blockchain.rpc_url, cfg.blockchain.private_key, CHAIN_CONFIG["engineAddress"],
                          CHAIN_CONFIG["baseTokenAddress"], chain_id=x.chain_id, batch=x.rpc_batch,
                          max_batch=x.rpc_max_batch, stuck_s=x.tx_stuck_s)


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
    # device_count() does not initialise HIP: the dispatcher process stays GPU-free
    n = cfg.mi355x.gpus if cfg.mi355x.gpus is not None else torch.cuda.device_count()
    if n > 1 or (n == 1 and cfg.mi355x.worker_processes):
        from .parallel.cpu_budget import model_gpu_caps
        from .parallel.workers import MultiGPUSolverPool
        caps = model_gpu_caps(names, n, cfg.mi355x.host_cores) if cfg.mi355x.cpu_admission else {}
        return MultiGPUSolverPool(n, names, "cuda", streams_per_gpu=cfg.mi355x.workers_per_gpu,
                                  model_streams=cfg.mi355x.model_streams,
                                  lockstep=cfg.mi355x.lockstep_group, weights_dir=cfg.mi355x.weights_dir,
                                  hang_timeout=cfg.mi355x.hang_timeout_s, force_group=n == 1,
                                  dispatch=cfg.mi355x.dispatch_policy, model_lockstep=cfg.mi355x.model_lockstep,
                                  model_gpu_cap=caps)
    from .node.pool import LocalSolverPool
    return LocalSolverPool("cuda:0" if n == 1 else "cpu", capacity=cfg.mi355x.workers_per_gpu,
                           model_streams=cfg.mi355x.model_streams, model_lockstep=cfg.mi355x.model_lockstep,
                           lockstep=cfg.mi355x.lockstep_group, weights_dir=cfg.mi355x.weights_dir)


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
    from .numerics import NUMERICS_VERSION, check_mining_env
    check_mining_env()                 # A/B knobs would produce non-consensus CIDs
    log.info("numerics version %s", NUMERICS_VERSION)
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
    models = {k: v for k, v in default_models(ids, int(cfg.mi355x.min_model_filter_fee)).items()
              if v.name in set(cfg.mi355x.models)}
    pool = build_pool(cfg, models)
    miner = Miner(cfg, db, chain, make_pinner(cfg), pool, models)
    runner = await start_rpc(db, cfg.rpc.host, cfg.rpc.port, miner)
    try:
        await miner.run()
    finally:
        await runner.cleanup()


def _arg(v: str):
    """CLI argument -> ABI value: JSON for arrays/numbers/bools, else the string itself."""
    try:
        return json.loads(v)
    except ValueError:
        return v


GOV = {  # GovernorV1 (OZ Governor + Bravo) / token votes: contract/tasks/index.ts:234-465
    "delegate": ("token", "delegate(address)"),
    "propose": ("governor", "propose(address[],uint256[],bytes[],string)"),
    "vote": ("governor", "castVote(uint256,uint8)"),
    "cancel": ("governor", "cancel(uint256)"),
    "queue": ("governor", "queue(uint256)"),
    "execute": ("governor", "execute(uint256)"),
}


async def _operator(a, c):
    """contract/tasks/index.ts operator tasks beyond the miner's own needs."""
    from .chain.engine_abi import ENGINE_PARAMS, FUNCS
    eng = c.engine_address
    if a.cmd == "accounts":
        print(json.dumps({"address": c.address, "eth": _fmt(await c.eth_balance(c.address)),
                          "aius": _fmt(await c.token_balance(c.address))}))
    elif a.cmd == "mine":
        for _ in range(a.n):
            await c.rpc("evm_mine", [])
        print(await c.block_number())
    elif a.cmd == "timetravel":
        await c.rpc("evm_increaseTime", [int(a.seconds)])
        await c.rpc("evm_mine", [])
        print(await c.block_number())
    elif a.cmd == "send-eth":
        print(await c.send_sig(a.to, "", value=int(float(a.amount) * E18), gas=21000))
    elif a.cmd == "transfer":
        print(await c.send_sig(c.token_address, "transfer(address,uint256)", a.to, int(float(a.amount) * E18)))
    elif a.cmd == "engine-pause":
        print(await c.send_sig(eng, "setPaused(bool)", a.paused.lower() in ("1", "true", "yes")))
    elif a.cmd == "withdraw-fees":
        print(await c.send_sig(eng, "withdrawAccruedFees()"))
    elif a.cmd == "params":
        out = {}
        for p in ENGINE_PARAMS + ["version", "owner", "treasury", "pauser", "paused", "accruedFees"]:
            sig, rets = FUNCS[p]
            out[p] = str((await c.call_sig(eng, sig, rets))[0])
        print(json.dumps(out, indent=1))
    elif a.cmd == "admin":
        if a.setter not in FUNCS:
            raise SystemExit(f"unknown admin function {a.setter}")
        print(await c.send_sig(eng, FUNCS[a.setter][0], *[_arg(x) for x in a.args]))
    elif a.cmd == "validator-withdraw":
        sig = {"initiate": "initiateValidatorWithdraw(uint256)", "cancel": "cancelValidatorWithdraw(uint256)",
               "withdraw": "validatorWithdraw(uint256,address)"}[a.action]
        args = [int(float(a.args[0]) * E18)] if a.action == "initiate" else [int(a.args[0])]
        if a.action == "withdraw":
            args.append(a.args[1] if len(a.args) > 1 else c.address)
        print(await c.send_sig(eng, sig, *args))
    elif a.cmd == "governance":
        if a.action == "proposal":
            gov = a.governor or _need_gov()
            st = await c.call_sig(gov, "state(uint256)", ["uint8"], int(a.args[0]))
            names = ["Pending", "Active", "Canceled", "Defeated", "Succeeded", "Queued", "Expired", "Executed"]
            print(json.dumps({"id": a.args[0], "state": names[st[0]] if st[0] < len(names) else st[0]}))
            return
        target, sig = GOV[a.action]
        to = c.token_address if target == "token" else (a.governor or _need_gov())
        print(await c.send_sig(to, sig, *[_arg(x) for x in a.args]))
    elif a.cmd == "call":
        rets = [t for t in a.rets.split(",") if t]
        print(json.dumps([str(v) for v in await c.call_sig(a.to, a.sig, rets, *[_arg(x) for x in a.args])]))
    elif a.cmd == "send":
        print(await c.send_sig(a.to, a.sig, *[_arg(x) for x in a.args], value=int(float(a.value) * E18)))
    elif a.cmd == "explorer":
        head = await c.block_number()
        for ev in await c.get_events(max(0, head - a.n), head):
            print(json.dumps({"block": ev.block, "event": ev.name, **{k: str(v) for k, v in ev.args.items()}}))
    elif a.cmd == "task":
        from .ipfs.unixfs import cid_hex_to_str
        t = await c.get_task(a.taskid)
        s = await c.get_solution(a.taskid)
        k = await c.get_contestation(a.taskid)
        out = {"task": {k2: str(v) for k2, v in t.items()}, "solution": {k2: str(v) for k2, v in s.items()},
               "contestation": {k2: str(v) for k2, v in k.items()}}
        cid = s.get("cid")
        if cid and cid not in ("0x", b""):
            h = cid if isinstance(cid, str) else "0x" + cid.hex()
            out["solution_cid"] = cid_hex_to_str(h)
        print(json.dumps(out, indent=1))
    elif a.cmd == "deploy":
        from .chain.deploy import deploy
        print(json.dumps(await deploy(c, a.artifact, [_arg(x) for x in a.args])))
    elif a.cmd == "deploy-core":
        # contract/scripts/003-deploy-core-basic.ts: Engine behind a transparent proxy + free kandinsky2
        from .chain.deploy import deploy_core
        from .node.models import template_bytes
        tpl = None if a.no_model else (Path(a.template).read_bytes() if os.path.exists(a.template)
                                       else template_bytes(a.template))
        rec = await deploy_core(c, a.engine_artifact, a.proxy_artifact, a.token or c.token_address,
                                a.treasury, tpl, proxy_admin_artifact=a.proxy_admin_artifact,
                                proxy_admin=a.proxy_admin)
        if a.out:
            Path(a.out).write_text(json.dumps(rec, indent=2))
        print(json.dumps(rec, indent=1))
    elif a.cmd == "pinata-gc":
        from .ipfs.pin import pinata_gc
        print(json.dumps(await pinata_gc(_cfg(a.config).ipfs.pinata.jwt)))
    else:
        raise SystemExit(f"unknown command {a.cmd}")


def _need_gov():
    raise SystemExit("--governor ADDRESS is required for governance commands")


def main(argv=None):
    ap = argparse.ArgumentParser(prog="arbius_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("start"); p.add_argument("config")
    p = sub.add_parser("mock-node")
    p.add_argument("--host", default="127.0.0.1")
    p.add_argument("--port", type=int, default=8545)
    sub.add_parser("gen-wallet")
    p = sub.add_parser("cid"); p.add_argument("file"); p.add_argument("--wrap", default=None)
    p = sub.add_parser("decode-calldata"); p.add_argument("data")
    for name, extra in [("decode-tx", ["txid"]), ("model-register", ["template"]), ("validator-stake", ["amount"]),
                        ("balance", []), ("claim", ["taskid"]), ("signal-support", ["model", "support"]),
                        ("is-paused", []), ("submit-task", ["model", "input"]), ("accounts", []),
                        ("timetravel", ["seconds"]), ("send-eth", ["to", "amount"]), ("transfer", ["to", "amount"]),
                        ("engine-pause", ["paused"]), ("withdraw-fees", []), ("params", []),
                        ("task", ["taskid"]), ("pinata-gc", [])]:
        p = sub.add_parser(name)
        for e in extra:
            p.add_argument(e)
        p.add_argument("-c", "--config", default="MiningConfig.json")
        if name in ("model-register", "submit-task"):
            p.add_argument("--fee", default="0")
    for name in ("mine", "explorer"):
        p = sub.add_parser(name)
        p.add_argument("n", nargs="?", type=int, default=1 if name == "mine" else 128)
        p.add_argument("-c", "--config", default="MiningConfig.json")
    for name, first in (("admin", "setter"), ("validator-withdraw", "action"), ("governance", "action")):
        p = sub.add_parser(name)
        p.add_argument(first)
        p.add_argument("args", nargs="*")
        p.add_argument("-c", "--config", default="MiningConfig.json")
        p.add_argument("--governor", default=None)
    p = sub.add_parser("call")
    p.add_argument("to"); p.add_argument("sig"); p.add_argument("rets"); p.add_argument("args", nargs="*")
    p.add_argument("-c", "--config", default="MiningConfig.json")
    p = sub.add_parser("deploy", help="contract creation from a compiled Hardhat artifact")
    p.add_argument("artifact"); p.add_argument("args", nargs="*")
    p.add_argument("-c", "--config", default="MiningConfig.json")
    p = sub.add_parser("deploy-core", help="003-deploy-core-basic: Engine proxy + free mineable model")
    p.add_argument("--engine-artifact", required=True)
    p.add_argument("--proxy-artifact", required=True, help="TransparentUpgradeableProxy artifact")
    g = p.add_mutually_exclusive_group(required=True)
    g.add_argument("--proxy-admin-artifact", help="ProxyAdmin artifact (deployed, owned by the deployer)")
    g.add_argument("--proxy-admin", help="existing ProxyAdmin contract address")
    p.add_argument("--token", default=None, help="BaseToken address (default: the config's)")
    p.add_argument("--treasury", default=None)
    p.add_argument("--template", default="kandinsky2")
    p.add_argument("--no-model", action="store_true")
    p.add_argument("--out", default=None, help="write the deployment record (scripts/config.json analog)")
    p.add_argument("-c", "--config", default="MiningConfig.json")
    p = sub.add_parser("send")
    p.add_argument("to"); p.add_argument("sig"); p.add_argument("args", nargs="*")
    p.add_argument("--value", default="0")
    p.add_argument("-c", "--config", default="MiningConfig.json")
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
            else:
                await _operator(a, c)
        finally:
            await c.close()

    asyncio.run(run())


if __name__ == "__main__":
    main()
