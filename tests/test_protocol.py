"""Golden vectors and byte-compat invariants."""
import json
import os

import pytest

from arbius_amd.chain import abi
from arbius_amd.chain.mock_engine import MockEngine
from arbius_amd.ipfs.unixfs import (add_file, b58decode, b58encode, cid_hex_to_str, cid_str_to_hex, onchain_cid,
                                    wrap_directory)
from arbius_amd.node.models import (KANDINSKY2_ID, KANDINSKY2_TEMPLATE_CID, check_model_filter, default_models,
                                    hydrate_input, load_template, template_cid)
from arbius_amd.utils.keccak import keccak256, keccak256_py
from arbius_amd.utils.protocol import generate_commitment, hash_task, taskid2seed

FIX = os.path.join(os.path.dirname(__file__), "fixtures")

# contract/test/ipfs.ts:52-55 and miner/test/ipfs.test.ts:106-109
CID_VECTORS = {
    "a": "0x1220e844b8764c00d4a76ac03930a3d8f32f3df59aea3ed0ade4c3bc38a3b23a31d9",
    "b": "0x1220f782bf27d7dfa16c5556ae0e19d41a73fc380a28455abcedecd70460505f022b",
    "c": "0x1220c32cae42b7d6ed6efd2512fd7dac6530cbd96cbcc19a3d1c336ace8e401f1c3a",
    "d": "0x1220f4ad8a3bd3189da2ad909ee41148d6893d8c629c410f7f2c7e3fae75aade79c8",
}


@pytest.mark.parametrize("name", sorted(CID_VECTORS))
def test_cid_vectors(name):
    data = open(os.path.join(FIX, f"ipfs_{name}.bin"), "rb").read()
    assert "0x" + onchain_cid(data).hex() == CID_VECTORS[name]
    assert add_file(data).cid_hex == CID_VECTORS[name]  # kubo single-chunk add == on-chain CID


def test_template_cid():
    # miner/src/config.json:15
    assert template_cid("kandinsky2") == KANDINSKY2_TEMPLATE_CID


def test_base58_roundtrip():
    h = CID_VECTORS["a"]
    s = cid_hex_to_str(h)
    assert s.startswith("Qm") and len(s) == 46
    assert cid_str_to_hex(s) == h
    assert b58decode(b58encode(b"\0\0abc")) == b"\0\0abc"


def test_multichunk_file_and_directory_structure():
    import random
    data = random.Random(0).randbytes(768000)  # 3 distinct chunks
    r = add_file(data)
    assert r.filesize == len(data)
    assert len(r.blocks) == 4  # 3 leaves + root
    root = r.root
    assert root.count(b"\x12\x00") >= 3  # empty link names
    d = wrap_directory([("out-1.png", data)])
    assert d.cid != r.cid and d.tsize > r.tsize
    assert d.root.endswith(b"\x0a\x02\x08\x01")  # UnixFS Directory data
    assert b"out-1.png" in d.root


def test_keccak_vectors():
    assert keccak256_py(b"").hex() == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"
    assert keccak256(b"abc").hex() == keccak256_py(b"abc").hex()
    long = os.urandom(1000)
    assert keccak256(long) == keccak256_py(long)


def test_commitment_vector():
    # miner/test/utils.test.ts:61-63 (value re-derived)
    c = generate_commitment("0x1A320E53A25f518B893F286f3600cc204c181a8E",
                            "0xdc6a147f2cd937a1b290b0dc4eff49a084ad72468fcb36df6d8ddb00c5ff6f7b",
                            "0x122002e2550d45270ed9c0df80be9a331940d391bcb138e0edfce4d2ff20168d6691")
    assert c == "0xb5fa4a5b4a1febe1ac696ace872867f629cfbed3996c128a25f1aafd56b7cb50"


def test_seed():
    assert taskid2seed("0x00") == 0
    assert taskid2seed(hex(0x1FFFFFFFFFFFF0 + 5)) == 5
    assert taskid2seed("0x" + "ff" * 32) == (2 ** 256 - 1) % 0x1FFFFFFFFFFFF0


@pytest.mark.parametrize("sig,topic", [
    ("TaskSubmitted(bytes32,bytes32,uint256,address)",
     "0xc3d3e0544c80e3bb83f62659259ae1574f72a91515ab3cae3dd75cf77e1b0aea"),
])
def test_event_topics(sig, topic):
    assert abi.topic(sig) == topic


@pytest.mark.parametrize("sig,sel", [
    ("submitTask(uint8,address,bytes32,uint256,bytes)", "08745dd1"),
    ("signalCommitment(bytes32)", "506ea7de"),
    ("submitSolution(bytes32,bytes)", "56914caf"),
    ("claimSolution(bytes32)", "77286d17"),
    ("submitContestation(bytes32)", "671f8152"),
    ("voteOnContestation(bytes32,bool)", "1825c20e"),
    ("validatorDeposit(address,uint256)", "93a090ec"),
    ("tasks(bytes32)", "e579f500"),
    ("solutions(bytes32)", "75c70509"),
    ("contestations(bytes32)", "d33b2ef5"),
    ("contestationVoted(bytes32,address)", "d2780940"),
    ("validators(address)", "fa52c7d8"),
    ("getValidatorMinimum()", "2258d105"),
    ("version()", "54fd4d50"),
    ("balanceOf(address)", "70a08231"),
    ("allowance(address,address)", "dd62ed3e"),
    ("approve(address,uint256)", "095ea7b3"),
])
def test_selectors(sig, sel):
    # SURVEY.md §2.7 message table (verified against the deployed bytecode)
    assert abi.selector(sig).hex() == sel


def test_abi_roundtrip_submit_task():
    inp = json.dumps({"prompt": "arbius test cat"}).encode()
    data = abi.encode_call("submitTask(uint8,address,bytes32,uint256,bytes)", 0, "0x" + "11" * 20,
                           KANDINSKY2_ID, 10 ** 18, inp)
    v, owner, model, fee, raw = abi.decode_call("submitTask(uint8,address,bytes32,uint256,bytes)", data)
    assert (v, owner, model, fee) == (0, "0x" + "11" * 20, KANDINSKY2_ID, 10 ** 18)
    assert bytes.fromhex(raw[2:]) == inp
    out = abi.encode(["(address,uint64,bool,bytes)"], [("0x" + "22" * 20, 5, True, b"\x12\x20")])
    assert abi.decode(["(address,uint64,bool,bytes)"], out)[0] == ("0x" + "22" * 20, 5, True, "0x1220")


# ------------------------------------------------------------------ hydration (Appendix D)
def test_hydrate_defaults_and_order():
    tpl = load_template("anythingv3")
    inp, err, msg = hydrate_input({"prompt": "x", "negative_prompt": "n", "foo": 1}, tpl)
    assert not err, msg
    assert list(inp) == [r["variable"] for r in tpl["input"]]
    assert "foo" not in inp and inp["width"] == 768 and inp["scheduler"] == "DPMSolverMultistep"


def test_hydrate_errors():
    tpl = load_template("anythingv3")
    assert hydrate_input({"negative_prompt": "n"}, tpl)[2] == "input missing required field (prompt)"
    assert hydrate_input({"prompt": 1, "negative_prompt": "n"}, tpl)[2] == "input wrong type (prompt)"
    assert hydrate_input({"prompt": "p", "negative_prompt": "n", "width": 100}, tpl)[2] == "input not in enum (width)"
    assert hydrate_input({"prompt": "p", "negative_prompt": "n", "num_inference_steps": 0}, tpl)[2] == \
        "input out of bounds (num_inference_steps)"
    assert hydrate_input({"prompt": "p", "negative_prompt": "n", "num_inference_steps": 2.5}, tpl)[1]


def test_hydrate_quirks():
    tpl = load_template("anythingv3")
    base = {"prompt": "p", "negative_prompt": "n"}
    # spec-correct: decimal 7.5 ok, max enforced
    assert not hydrate_input({**base, "guidance_scale": 7.5}, tpl)[1]
    assert hydrate_input({**base, "guidance_scale": 25}, tpl)[1]
    # reference quirks Q2/Q3 (models.ts:185-194)
    assert hydrate_input({**base, "guidance_scale": 7.5}, tpl, quirks=True)[1]
    assert not hydrate_input({**base, "guidance_scale": 25}, tpl, quirks=True)[1]


def test_model_filter():
    models = default_models()
    assert check_model_filter(models, KANDINSKY2_ID, 100, 0, 50, "0x" + "00" * 20) == (True, True,
                                                                                      models[KANDINSKY2_ID].template)
    assert check_model_filter(models, "0x" + "ab" * 32, 100, 0, 50, "0x" + "00" * 20)[0] is False


def test_hash_task_matches_engine():
    e = MockEngine()
    assert hash_task("0x" + "11" * 20, "0x" + "00" * 32, KANDINSKY2_ID, 5, "0x1220" + "ab" * 32).startswith("0x")


# ------------------------------------------------------------------ protocol math goldens (reward.test.ts:152-231)
@pytest.mark.parametrize("t,expected", [
    (0, 0), (15768000, 175735931288071485118987), (31536000, 300000 * 10 ** 18), (63072000, 450000 * 10 ** 18),
    (94608000, 525000 * 10 ** 18), (126144000, 562500 * 10 ** 18), (157680000, 581250 * 10 ** 18),
    (315360000, 599414062500000000000000), (3153600000, 600000 * 10 ** 18), (31536000000, 600000 * 10 ** 18)])
def test_target_ts(t, expected):
    assert MockEngine.target_ts(t) == expected


@pytest.mark.parametrize("ts,expected", [
    (100000, 100 * 10 ** 18), (250000, 100 * 10 ** 18), (300000, 10 ** 18), (305000, 314980262473718305),
    (350000, 9612434767874), (355000, 3027727226196), (360000, 0), (400000, 0), (500000, 0), (600000, 0)])
def test_diff_mul(ts, expected):
    assert MockEngine.diff_mul(31536000, ts * 10 ** 18) == expected
