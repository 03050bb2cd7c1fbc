"""Real-chain deployment path (``contract/scripts/003-deploy-core-basic.ts``):
contract-creation transactions built and signed by the node, against a recording JSON-RPC stub
(the mock chain has no EVM).  No EVM bytecode ships with the repo: the artifacts here are dummies."""
import asyncio
import json

import pytest

from arbius_amd.chain import abi
from arbius_amd.chain.deploy import FREE_MODEL_ADDR, create_address, creation_data, deploy, deploy_core
from arbius_amd.chain.rpc import RpcChainClient as RpcClient
from arbius_amd.chain.tx import decode_raw_tx
from arbius_amd.ipfs.unixfs import onchain_cid
from arbius_amd.utils.keccak import keccak256

KEY = "0x" + "42" * 32


def test_create_address_vectors():
    # the CREATE address vectors of the Ethereum yellow-paper derivation keccak(rlp([sender, nonce]))[12:]
    s = "0x6ac7ea33f8831ea9dcc53393aaa88b25a785dbf0"
    assert create_address(s, 0) == "0xcd234a471b72ba2f1ccf0a70fcaba648a5eecd8d"
    assert create_address(s, 1) == "0x343c43a37d37dff08ae8c4a11544c718abb4fcf8"
    assert create_address(s, 2) == "0xf778b86fa74e846c4f0a1fbd1335fe81c00a0c91"


def _artifact(tmp_path, name, inputs, code="0x6080604052348015600f57600080fd5b50"):
    p = tmp_path / f"{name}.json"
    p.write_text(json.dumps({"contractName": name, "abi": [{"type": "constructor", "inputs": inputs}],
                             "bytecode": code}))
    return p


class _Chain:
    """eth_* stub: records raw transactions, answers receipts with the CREATE address."""
    def __init__(self):
        self.raw, self.nonce = [], 0

    async def rpc(self, method, params):
        if method == "eth_chainId":
            return hex(42170)
        if method == "eth_getTransactionCount":
            return hex(self.nonce)
        if method == "eth_gasPrice":
            return hex(10 ** 8)
        if method == "eth_sendRawTransaction":
            raw = bytes.fromhex(params[0][2:])
            f, sender = decode_raw_tx(raw)
            self.raw.append((f, sender))
            created = create_address(sender, f["nonce"]) if f["to"] == "0x" else None
            self.nonce += 1
            self.last = {"status": "0x1", "contractAddress": created}
            return f["hash"]
        if method == "eth_getTransactionReceipt":
            return self.last
        raise AssertionError(f"unexpected JSON-RPC call {method}")   # no eth_call: ids are computed locally


def _client(chain):
    c = RpcClient("http://127.0.0.1:1", KEY, "0x" + "00" * 20, "0x" + "00" * 20, receipt_poll=0.001)
    c.rpc = chain.rpc
    return c


def test_contract_creation_tx(tmp_path):
    art = _artifact(tmp_path, "Box", [{"name": "v", "type": "uint256"}, {"name": "o", "type": "address"}])
    chain = _Chain()
    c = _client(chain)
    out = asyncio.run(deploy(c, art, [7, c.address]))
    (f, sender), = chain.raw
    assert sender.lower() == c.address.lower() and f["to"] == "0x" and f["chain_id"] == 42170
    code = bytes.fromhex("6080604052348015600f57600080fd5b50")
    assert f["data"] == code + abi.encode(["uint256", "address"], [7, c.address])
    assert out["address"] == create_address(c.address, 0)
    with pytest.raises(ValueError, match="constructor takes 2"):
        creation_data(json.loads(art.read_text())["abi"], code, [1])


def _proxy_artifacts(tmp_path):
    eng = _artifact(tmp_path, "EngineV1", [])
    prx = _artifact(tmp_path, "TransparentUpgradeableProxy",
                    [{"name": "_logic", "type": "address"}, {"name": "admin_", "type": "address"},
                     {"name": "_data", "type": "bytes"}])
    adm = _artifact(tmp_path, "ProxyAdmin", [])            # OZ 4.9: owner = msg.sender
    return eng, prx, adm


def test_deploy_core_flow(tmp_path):
    """impl -> ProxyAdmin -> TransparentUpgradeableProxy(impl, proxyAdmin, initialize(token, treasury)) ->
    registerModel -> setSolutionMineableRate, each signed by the deployer, nonces consecutive."""
    eng, prx, adm = _proxy_artifacts(tmp_path)
    chain = _Chain()
    c = _client(chain)
    token = "0x" + "ab" * 20
    tpl = b'{"meta": {}}'
    rec = asyncio.run(deploy_core(c, eng, prx, token, template=tpl, proxy_admin_artifact=adm))
    kinds = [f["to"] for f, _ in chain.raw]
    impl, admin, proxy = (create_address(c.address, n) for n in range(3))
    assert kinds == ["0x", "0x", "0x", proxy, proxy]
    assert [f["nonce"] for f, _ in chain.raw] == [0, 1, 2, 3, 4]
    init = abi.encode_call("initialize(address,address)", token, c.address)
    assert chain.raw[2][0]["data"].endswith(abi.encode(["address", "address", "bytes"], [impl, admin, init]))
    # the transparent proxy never forwards its admin's calls: the admin must not be the tx sender
    assert admin.lower() != c.address.lower() and rec["proxyAdmin"] == admin
    reg = abi.decode_call("registerModel(address,uint256,bytes)", chain.raw[3][0]["data"])
    assert reg[0].lower() == FREE_MODEL_ADDR and reg[1] == 0 and reg[2] == "0x" + tpl.hex()
    rate = abi.decode_call("setSolutionMineableRate(bytes32,uint256)", chain.raw[4][0]["data"])
    assert rate[1] == 10 ** 18
    assert rec["engineAddress"] == proxy and rec["engineImplementation"] == impl
    # EngineV1.hashModel(Model{fee, addr, rate, cid}, sender) = keccak(abi.encode(sender, addr, fee, cid))
    cid = onchain_cid(tpl)
    want = "0x" + keccak256(abi.encode(["address", "address", "uint256", "bytes"],
                                       [c.address, FREE_MODEL_ADDR, 0, cid])).hex()
    assert rec["models"]["kandinsky2"]["id"] == want
    assert "0x" + bytes(rate[0]).hex() == want if not isinstance(rate[0], str) else rate[0] == want


def test_deploy_core_refuses_deployer_as_admin(tmp_path):
    eng, prx, _ = _proxy_artifacts(tmp_path)
    c = _client(_Chain())
    with pytest.raises(ValueError, match="must not be the deployer"):
        asyncio.run(deploy_core(c, eng, prx, "0x" + "ab" * 20, proxy_admin=c.address))
    with pytest.raises(ValueError, match="exactly one"):
        asyncio.run(deploy_core(c, eng, prx, "0x" + "ab" * 20))
