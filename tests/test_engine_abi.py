"""The node's Engine binding covers the reference ABI completely: every function (77) with its
return types and every event (31) with its indexed layout, against the signatures extracted from
``miner/src/artifacts/contracts/EngineV1.sol/EngineV1.json`` (tests/fixtures)."""
import json
import os

from arbius_amd.chain import abi
from arbius_amd.chain.engine_abi import EVENTS, FUNCS, TOPIC_TO_EVENT, decode_log, encode_log

REF = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "engine_v1_abi_signatures.json")))


def test_every_reference_function_bound_with_its_returns():
    bound = {sig: rets for sig, rets in FUNCS.values()}
    assert len(REF["functions"]) == 77
    for sig, rets in REF["functions"].items():
        assert sig in bound, f"unbound Engine function {sig}"
        assert bound[sig] == rets, (sig, bound[sig], rets)
        assert len(abi.selector(sig)) == 4


def test_every_reference_event_decodable():
    assert len(REF["events"]) == 31
    mine = {sig: [(n, t, ix) for n, t, ix in fields] for sig, fields in EVENTS.values()}
    for sig, fields in REF["events"].items():
        assert sig in mine, f"event {sig} invisible to get_events"
        assert [(t, ix) for _, t, ix in fields] == [(t, ix) for _, t, ix in mine[sig]], sig
        assert TOPIC_TO_EVENT[abi.topic(sig)]


def test_known_selectors_and_topics():
    # SURVEY.md §2.7 / §2.8.5 verified values
    assert abi.selector("submitTask(uint8,address,bytes32,uint256,bytes)").hex() == "08745dd1"
    assert abi.selector("signalCommitment(bytes32)").hex() == "506ea7de"
    assert abi.topic("TaskSubmitted(bytes32,bytes32,uint256,address)").startswith("0xc3d3e054")


def test_roundtrip_new_events():
    a = "0x" + "ab" * 20
    for name, args in [("ValidatorWithdrawInitiated", {"addr": a, "count": 3, "unlockTime": 99, "amount": 7}),
                       ("SignalSupport", {"addr": a, "model": "0x" + "11" * 32, "supported": True}),
                       ("MinClaimSolutionTimeChanged", {"amount": 2000}),
                       ("PausedChanged", {"paused": True})]:
        topics, data = encode_log(name, args)
        got_name, got = decode_log(topics, data)
        assert got_name == name
        for k, v in args.items():
            assert (got[k].lower() if isinstance(got[k], str) else got[k]) == (v.lower() if isinstance(v, str) else v)
