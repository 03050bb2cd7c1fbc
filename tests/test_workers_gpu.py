"""The shipped multi-GPU worker path ON a GPU (parallel/workers.py): spawned worker processes that
build their pipelines on ``cuda:r``, a one-rank RCCL communicator carrying the weight broadcast,
lock-step groups on pipeline forks inside the worker, ``Solution`` objects over ``mp.Queue``, and a
respawn of a killed GPU worker as a fresh spawned child - every CID equal to the solo solve in this
process.  (The driver's 8-GPU node runs the same code at world size 8.)"""
import asyncio
import json
import os
import subprocess
import sys

import pytest

from arbius_amd.node.models import Model, load_template

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODEL = Model("0x" + "ab" * 32, "anythingv3", load_template("anythingv3"), True, [], "image")


def _inps(n, steps=3):
    return [{"prompt": f"harbour {i}", "negative_prompt": "blurry", "width": 128, "height": 128,
             "num_inference_steps": steps, "guidance_scale": 7.5, "scheduler": "DPMSolverMultistep", "seed": 900 + i}
            for i in range(n)]


@pytest.mark.timeout(900)
def test_multigpu_pool_on_gpu_lockstep_rccl_and_respawn(cuda):
    from arbius_amd.models.registry import build_pipeline
    from arbius_amd.node.solver import solve_image
    from arbius_amd.parallel.workers import MultiGPUSolverPool
    inps = _inps(8)
    pipe = build_pipeline("anythingv3", device=cuda)
    solo = [solve_image(pipe, i).cid for i in inps]
    del pipe

    async def go():
        pool = MultiGPUSolverPool(1, ["anythingv3"], "cuda", streams_per_gpu=2, lockstep=4, force_group=True,
                                  start_timeout=600)
        try:
            assert pool.world["backend"] == "nccl" and pool.world["world_size"] == 1
            assert pool.broadcast_stats[0]["bytes"] > 1 << 30        # the whole SD1.5 went through RCCL
            assert pool.hardware() == "gfx950"                      # reported by the worker
            assert pool.capacity == 2 * 4 * 2
            sols = await asyncio.wait_for(asyncio.gather(*[pool.solve(MODEL, f"t{i}", x)
                                                           for i, x in enumerate(inps)]), 600)
            assert [s.cid for s in sols] == solo
            assert max(s.timings.get("group", 1) for s in sols) > 1   # lock-step groups formed
            pool.kill_worker(0)
            again = await asyncio.wait_for(asyncio.gather(*[pool.solve(MODEL, f"r{i}", x)
                                                            for i, x in enumerate(inps[:4])]), 600)
            assert pool.restarts == 1 and [s.cid for s in again] == solo[:4]
        finally:
            await pool.close()

    asyncio.run(go())


@pytest.mark.timeout(600)
def test_bench_one_rank_rccl_group_reports_nccl(cuda, tmp_path):
    """``bench.py --rccl-group`` at N = 1: the weight broadcast runs through a one-rank RCCL
    communicator and the bench JSON says so."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--rccl-group", "--steps", "1",
                          "--warmup", "1", "--res", "128", "--denoise-steps", "3", "--concurrent", "1", "--group", "2"],
                         capture_output=True, text=True, timeout=500, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    js = json.loads(out.stdout.strip().splitlines()[-1])
    assert js["weight_broadcast"]["backend"] == "nccl" and js["weight_broadcast"]["bytes"] > 1 << 30
    assert js["world"]["backend"] == "nccl" and js["native_kernels_loaded"]
