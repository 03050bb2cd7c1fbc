"""Consensus pinning on gfx950: each golden task's CID must equal the value pinned for this
NUMERICS_VERSION (arbius_amd/numerics.py).  A kernel / plan / sampler / encoder change that flips
one output bit fails here by name; re-pin with scripts/pin_goldens.py AND bump NUMERICS_VERSION.
The 2-stream x lock-step-4 case also checks that the benched configuration reproduces every
task's solo CID bit for bit."""
import json
import os

import pytest

from arbius_amd.numerics import NUMERICS_VERSION, golden_cases

pytestmark = pytest.mark.gpu
GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden_cids.json")))


def test_golden_file_matches_numerics_version():
    assert GOLDEN["numerics_version"] == NUMERICS_VERSION, (
        "NUMERICS_VERSION changed: re-pin tests/golden_cids.json with scripts/pin_goldens.py")


@pytest.fixture(scope="module")
def cases(cuda):
    return dict(golden_cases(cuda))


@pytest.mark.parametrize("name", sorted(GOLDEN["cases"]))
def test_golden_cid(cases, name):
    from arbius_amd.node.pool import hardware_id
    import torch
    key = f"{hardware_id(torch.device('cuda', 0))}/random-init-seed0"
    assert key == GOLDEN["key"], f"goldens are pinned for {GOLDEN['key']}, this box is {key}"
    got = cases[name]()
    assert got == GOLDEN["cases"][name], (
        f"{name}: output bytes changed under NUMERICS_VERSION {NUMERICS_VERSION} "
        f"(got {got}, pinned {GOLDEN['cases'][name]}): bump the version and re-pin")


def test_boot_selftest_table_matches_this_gpu(cuda):
    """Every config/selftest.json task recomputed on this GPU equals its pinned gfx950 value (the
    node refuses to start on a mismatch, miner/src/index.ts:981-1001)."""
    import torch
    from pathlib import Path

    from arbius_amd.node.pool import hardware_id
    from arbius_amd.numerics import selftest_cids
    table = json.loads((Path(__file__).resolve().parents[1] / "arbius_amd" / "config" / "selftest.json").read_text())
    assert table["numerics_version"] == NUMERICS_VERSION, "re-pin config/selftest.json (scripts/pin_goldens.py)"
    key = f"{hardware_id(torch.device('cuda', 0))}/random-init-seed0"
    got = selftest_cids(cuda)
    for name, cid in got.items():
        assert table[name]["expected"].get(key) == cid, f"self test {name}: got {cid}, pinned {table[name]['expected']}"
