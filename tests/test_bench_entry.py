"""bench.py contract on CPU (gloo ranks): ``--gpus N`` without torchrun spawns N rank processes,
rank 0 broadcasts the weights, every rank solves its tasks, one JSON line with whole-node numbers;
a ``--gpus`` that disagrees with the launcher's world size fails loudly."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--device", "cpu", "--tiny", "--steps", "1", "--warmup", "0", "--denoise-steps", "2", "--res", "64",
        "--concurrent", "1", "--group", "2"]


def _run(args, env=None, timeout=600):
    e = dict(os.environ, **(env or {}))
    e.pop("WORLD_SIZE", None) if env is None else None
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


def _json(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.timeout(900)
def test_bench_spawns_gpus_ranks_and_broadcasts():
    r = _run(["--gpus", "2", *TINY])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 4                 # 2 ranks x 1 stream x group 2
    assert [p["rank"] for p in d["per_rank"]] == [0, 1]
    assert all(p["tasks"] == 2 for p in d["per_rank"])      # every rank solved its tasks
    assert d["weight_broadcast"]["bytes"] > 0 and d["weight_broadcast"]["backend"] == "gloo"
    assert d["value"] == pytest.approx(2 * 2 * 3600e3 / d["ms_per_step"], rel=1e-3)


@pytest.mark.timeout(600)
def test_bench_single_rank_unchanged():
    r = _run(["--gpus", "1", *TINY])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r.stdout)
    assert d["n_gpus"] == 1 and d["weight_broadcast"]["bytes"] == 0 and len(d["per_rank"]) == 1


@pytest.mark.timeout(600)
def test_bench_gpus_must_match_launcher_world():
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29599"}
    r = _run(["--gpus", "2", *TINY], env=env)
    assert r.returncode != 0 and "--gpus 2" in (r.stderr + r.stdout)


@pytest.mark.timeout(900)
def test_node_bench_through_the_node_stack_gloo():
    """``--node``: tasks are submitted to the MockEngine and solved by the orchestrator + a 2-worker
    MultiGPUSolverPool (gloo ranks, weights broadcast); every solution is accepted on chain."""
    r = _run(["--node", "--gpus", "2", "--device", "cpu", "--tiny", "--steps", "2", "--warmup", "0",
              "--denoise-steps", "2", "--res", "128", "--scheduler", "DDIM", "--concurrent", "1", "--group", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r.stdout)
    assert d["config"]["mode"] == "node" and d["n_gpus"] == 2 and d["pool_capacity"] == 2
    assert d["tasks_timed"] == 4 and d["pins_ok"]
    assert d["jobs"]["jobs_ok_solve"] == 4 and d["jobs"]["jobs_ok_task"] == 4
    assert d["p50_task_latency_ms"] > 0
    assert d["value"] == pytest.approx(4 * 3600e3 / (2 * d["ms_per_step"]), rel=1e-3)


@pytest.mark.timeout(300)
def test_bench_exits_nonzero_when_a_rank_dies_in_the_broadcast():
    import time
    t0 = time.time()
    r = _run(["--gpus", "2", *TINY], env={"ARBIUS_FAULT_INJECTION": "1", "ARBIUS_FAULT_BCAST_DIE_RANK": "1",
                                          "WORLD_SIZE": "0"}, timeout=240)
    assert r.returncode != 0
    assert time.time() - t0 < 200


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(1200)
def test_bench_eight_ranks_through_torchrun_gloo():
    """The driver's 8-GPU launch line (torch.distributed.run, 8 ranks, 127.0.0.1) at the real world
    size, on gloo: rank 0 broadcasts to 7 ranks, every rank solves, one JSON line for the node."""
    args = ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr", "127.0.0.1",
            "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "8", *TINY]
    e = dict(os.environ, OMP_NUM_THREADS="1")
    e.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, *args], capture_output=True, text=True, timeout=1100, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r.stdout)
    assert d["n_gpus"] == 8 and d["config"]["parallelism"] == "dp8" and d["config"]["global_batch"] == 16
    assert [p["rank"] for p in d["per_rank"]] == list(range(8)) and all(p["tasks"] == 2 for p in d["per_rank"])
    assert d["world"]["world_size"] == 8 and len(d["world"]["ranks"]) == 8
    assert d["weight_broadcast"]["backend"] == "gloo" and d["weight_broadcast"]["bytes"] > 0
    assert all(p["weight_broadcast_bytes"] == d["weight_broadcast"]["bytes"] for p in d["per_rank"])


@pytest.mark.timeout(1200)
def test_node_bench_eight_workers_gloo():
    """``--node --gpus 8``: the orchestrator drives an 8-worker MultiGPUSolverPool (gloo ranks)."""
    r = _run(["--node", "--gpus", "8", "--device", "cpu", "--tiny", "--steps", "2", "--warmup", "0",
              "--denoise-steps", "2", "--res", "128", "--scheduler", "DDIM", "--concurrent", "1", "--group", "1"],
             env={"OMP_NUM_THREADS": "1", "WORLD_SIZE": "0"}, timeout=1100)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r.stdout)
    assert d["config"]["mode"] == "node" and d["n_gpus"] == 8 and d["pool_capacity"] == 8
    assert d["tasks_timed"] == 16 and d["pins_ok"] and d["jobs"]["jobs_ok_solve"] == 16


@pytest.mark.timeout(600)
def test_bench_one_rank_group_runs_the_broadcast_path():
    """``--rccl-group`` at N = 1: a one-rank process group (gloo here, RCCL on a GPU) carries the
    weight broadcast - the multi-GPU path, exercised without a second device."""
    r = _run(["--gpus", "1", "--rccl-group", *TINY])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r.stdout)
    assert d["weight_broadcast"]["backend"] == "gloo" and d["weight_broadcast"]["bytes"] > 0
    assert d["world"]["world_size"] == 1
