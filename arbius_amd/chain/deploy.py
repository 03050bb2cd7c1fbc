"""Real-chain contract deployment: the ``contract/scripts/003-deploy-core-basic.ts``
flow over plain JSON-RPC with the node's own signer, instead of Hardhat + OZ upgrades.

The EngineV1 implementation disables initializers in its constructor
(``contract/contracts/EngineV1.sol:231-233``), so it must sit behind a proxy exactly like
``upgrades.deployProxy`` does (``003-deploy-core-basic.ts:20-26``):

1. deploy the Engine implementation (contract creation, no constructor arguments);
2. deploy a ProxyAdmin owned by the deployer (or use ``proxy_admin=`` an existing one), then a
   TransparentUpgradeableProxy(implementation, proxyAdmin, initialize(baseToken, treasury)) - the
   proxy's constructor runs the initializer in the proxy's storage.  The admin must NOT be the
   deployer's own address: OZ 4.9's transparent proxy refuses to forward any call from its admin
   ("admin cannot fallback to proxy target"), so the deployer's registerModel below would revert -
   ``upgrades.deployProxy`` uses a ProxyAdmin contract for the same reason;
3. ``registerModel(0x..01, 0, kandinsky2 template)`` on the proxy and ``setSolutionMineableRate(id,
   1e18)`` (``deployFreeMineableModel``, ``:60-100``);
4. write the deployment record (the reference rewrites ``scripts/config.json``).

Bytecode comes from Hardhat artifacts the OPERATOR compiled (``{"abi": [...], "bytecode": "0x.."}``):
this repository ships no EVM bytecode.  The mock chain is a behavioural twin without an EVM, so
``mock-node --deploy`` (``chain/mock_node.py deploy_basic``) stays the local path; here the tests pin
the transaction encoding (contract creation RLP, constructor ABI tail, CREATE address).
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Any, Dict, List, Sequence, Tuple

from ..ipfs.unixfs import onchain_cid
from ..utils.keccak import keccak256
from ..utils.protocol import hash_model
from . import abi
from .tx import rlp_encode

FREE_MODEL_ADDR = "0x0000000000000000000000000000000000000001"   # 003-deploy-core-basic.ts:64


def load_artifact(path) -> Tuple[list, bytes]:
    """Hardhat artifact JSON -> (abi, creation bytecode).  Unlinked libraries are refused."""
    d = json.loads(Path(path).read_text())
    code = d.get("bytecode")
    if isinstance(code, dict):                     # solc standard-json {"object": ...}
        code = code.get("object", "")
    if not isinstance(code, str) or not code:
        raise ValueError(f"{path}: no creation bytecode")
    code = code[2:] if code.startswith("0x") else code
    if "__" in code:
        raise ValueError(f"{path}: bytecode has unlinked library placeholders")
    return d.get("abi", []), bytes.fromhex(code)


def constructor_types(abi_json: list) -> List[str]:
    for item in abi_json:
        if item.get("type") == "constructor":
            return [_abi_type(i) for i in item.get("inputs", [])]
    return []


def _abi_type(inp: dict) -> str:
    t = inp["type"]
    if t.startswith("tuple"):
        inner = ",".join(_abi_type(c) for c in inp.get("components", []))
        return f"({inner})" + t[len("tuple"):]
    return t


def creation_data(abi_json: list, bytecode: bytes, args: Sequence[Any] = ()) -> bytes:
    types = constructor_types(abi_json)
    if len(types) != len(args):
        raise ValueError(f"constructor takes {len(types)} argument(s) {types}, got {len(args)}")
    return bytecode + (abi.encode(types, list(args)) if types else b"")


def create_address(sender: str, nonce: int) -> str:
    """Address of the contract created by ``sender``'s transaction with ``nonce`` (CREATE)."""
    h = keccak256(rlp_encode([bytes.fromhex(sender[2:] if sender.startswith("0x") else sender), nonce]))
    return "0x" + h[12:].hex()


async def deploy(client, artifact, args: Sequence[Any] = (), gas: int = 8_000_000) -> Dict[str, str]:
    """Contract creation from an artifact; returns {"tx", "address"} (receipt's contractAddress,
    checked against the CREATE address of the signer's nonce)."""
    abi_json, code = load_artifact(artifact)
    data = creation_data(abi_json, code, args)
    p = await client.submit_tx("", data, gas, 0)
    expect = create_address(client.address, p.nonce)
    rc = await client.wait_receipt(p.hash)
    addr = (rc or {}).get("contractAddress") or expect
    if addr.lower() != expect.lower():
        raise RuntimeError(f"contract created at {addr}, expected {expect} (nonce {p.nonce})")
    return {"tx": p.hash, "address": addr}


async def deploy_core(client, engine_artifact, proxy_artifact, base_token: str, treasury: str = None,
                      template: bytes = None, rate: int = 10 ** 18, proxy_admin_artifact=None,
                      proxy_admin: str = None) -> Dict[str, Any]:
    """003-deploy-core-basic: Engine behind a transparent proxy + one free mineable model.

    Exactly one of ``proxy_admin_artifact`` (a ProxyAdmin to deploy, owned by the deployer) and
    ``proxy_admin`` (an existing admin contract) is required; the deployer itself is refused as admin."""
    if (proxy_admin_artifact is None) == (proxy_admin is None):
        raise ValueError("deploy_core needs exactly one of proxy_admin_artifact / proxy_admin")
    if proxy_admin is not None and proxy_admin.lower() == client.address.lower():
        raise ValueError("the proxy admin must not be the deployer: OZ transparent proxies do not forward "
                         "the admin's calls, so the deployer's registerModel would revert")
    treasury = treasury or client.address
    impl = await deploy(client, engine_artifact)
    if proxy_admin_artifact is not None:
        # OZ 4.x ProxyAdmin: no constructor arguments, owner = msg.sender; OZ 5.x: ProxyAdmin(initialOwner)
        admin_abi, _ = load_artifact(proxy_admin_artifact)
        admin_args = [client.address] if constructor_types(admin_abi) == ["address"] else []
        proxy_admin = (await deploy(client, proxy_admin_artifact, admin_args))["address"]
    init = abi.encode_call("initialize(address,address)", base_token, treasury)
    proxy = await deploy(client, proxy_artifact, [impl["address"], proxy_admin, init])
    engine = proxy["address"]
    out: Dict[str, Any] = {"baseTokenAddress": base_token, "engineAddress": engine,
                           "engineImplementation": impl["address"], "proxyAdmin": proxy_admin, "models": {}}
    if template is not None:
        # both ids are pure functions (EngineV1.sol:409-424), so compute them here rather than eth_call:
        # hashModel(Model{fee, addr, rate, cid}, sender) = keccak(abi.encode(sender, addr, fee, cid))
        cid_hex = "0x" + onchain_cid(template).hex()
        mid_hex = hash_model(client.address, FREE_MODEL_ADDR, 0, cid_hex)
        await client.send_sig(engine, "registerModel(address,uint256,bytes)", FREE_MODEL_ADDR, 0, template,
                              gas=3_000_000)
        await client.send_sig(engine, "setSolutionMineableRate(bytes32,uint256)", mid_hex, rate)
        out["models"]["kandinsky2"] = {"id": mid_hex, "mineable": True,
                                       "params": {"addr": FREE_MODEL_ADDR, "fee": "0", "rate": str(rate),
                                                  "cid": cid_hex}}
    return out
