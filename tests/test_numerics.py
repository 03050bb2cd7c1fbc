"""Consensus guard rails that need no GPU: the numerics-changing env knobs are refused by
``start`` and the golden-CID table is versioned."""
import json
import os

import pytest

from arbius_amd import numerics


def test_mining_refuses_numerics_knobs():
    numerics.check_mining_env({"PATH": "/bin", "ARBIUS_PLAN_CANON": ""})     # empty = unset
    for k in ("ARBIUS_PLAN_CANON", "ARB_CONV_PLANS", "ARB_GN_GROUP", "ARBIUS_NORM_PROLOGUE",
              "ARBIUS_KERNEL_LIB", "ARBIUS_EXPERIMENT_SKIP", "ARBIUS_REFERENCE_OPS"):
        with pytest.raises(SystemExit, match=k):
            numerics.check_mining_env({k: "1"})


def test_start_refuses_knobs_before_touching_chain(tmp_path, monkeypatch):
    from arbius_amd import cli
    cfg = tmp_path / "MiningConfig.json"
    cfg.write_text(json.dumps({"db_path": str(tmp_path / "db.sqlite"), "mi355x": {"mock_chain": True}}))
    monkeypatch.setenv("ARB_CONV_PLANS", "/tmp/other_plans.txt")
    with pytest.raises(SystemExit, match="ARB_CONV_PLANS"):
        cli.main(["start", str(cfg)])


def test_golden_table_is_versioned():
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden_cids.json")))
    assert {"numerics_version", "key", "cases"} <= set(g)


def test_selftest_table_pinned_for_this_numerics_version():
    from arbius_amd.node import miner
    t = json.load(open(os.path.join(os.path.dirname(miner.__file__), "..", "config", "selftest.json")))
    assert t["numerics_version"] == numerics.NUMERICS_VERSION
    assert t["kandinsky2"]["expected"]["gfx950/random-init-seed0"].startswith("0x1220")


def test_repository_lint_clean():
    """scripts/lint.py (the CI lint step): syntax, unused imports, whitespace, line length."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "lint.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:]


def test_family_table_well_formed():
    """csrc/conv_family.inc (scripts/tune_family.py): unique (M, N, K, split, ratio) keys, ratios of the
    canonical batch 8 over the actual batch (4 solo, 2 groups of 2, 1 groups of 4, 0 groups larger than
    4 - keyed by their own M), known tile cfgs and no family that lacks split-K at a split > 1
    (persistent kernels 24-27)."""
    import os
    import re
    path = os.path.join(os.path.dirname(__file__), "..", "arbius_amd", "ops", "csrc", "conv_family.inc")
    rows = [tuple(int(v) for v in m.groups()) for m in
            re.finditer(r"\{(\d+), (\d+), (\d+), (\d+), (\d+), (\d+)\},", open(path).read())]
    assert len(rows) > 100
    keys = [r[:5] for r in rows]
    assert len(keys) == len(set(keys))
    for M, N, K, split, ratio, cfg in rows:
        assert ratio in (0, 1, 2, 4) and split >= 1 and K % 64 == 0
        assert 0 <= cfg < 46 and not (24 <= cfg < 28 and split > 1)   # 0..45: conv.hip tile cfgs


def test_plan_rows_is_batch_invariant():
    """Size-dependent kernel choices use the canonical batch's rows under ops.plan_batch, so a
    lock-step group (batch 2k) makes the same choice as each solo CFG pair (batch 2)."""
    import torch
    from arbius_amd import ops
    solo, group = torch.empty(2, 1024, 320), torch.empty(8, 1024, 320)
    with ops.plan_batch(2):
        assert ops._plan_rows(solo) == ops._plan_rows(group) == ops.PLAN_CANON * 1024
    assert ops._plan_rows(solo) == 2 * 1024 and ops._plan_rows(group) == 8 * 1024


def test_every_kernel_env_knob_is_refused_when_mining():
    """Every environment variable the HIP kernel library reads (std::getenv in csrc/) selects a kernel,
    plan or layout: ``start`` must refuse to mine with any of them set."""
    import re
    from pathlib import Path

    from arbius_amd.numerics import NUMERICS_ENV_KNOBS
    csrc = Path(__file__).resolve().parents[1] / "arbius_amd" / "ops" / "csrc"
    names = set()
    for f in csrc.glob("*.hip"):
        names |= set(re.findall(r'getenv\("([A-Z0-9_]+)"\)', f.read_text()))
    assert names, "no getenv found"
    missing = sorted(n for n in names if n not in NUMERICS_ENV_KNOBS)
    assert missing == [], missing
