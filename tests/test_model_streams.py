"""Per-model task-stream caps (mi355x.model_streams): a capped model gets fewer pipeline forks /
concurrently solving worker slots than the GPU's stream count."""
import threading
import time

from arbius_amd.config.mining_config import DEFAULT_MODEL_LOCKSTEP, DEFAULT_MODEL_STREAMS, MI355XConfig
from arbius_amd.node.pool import LocalSolverPool


class _Pipe:
    forks = 0

    def fork(self):
        _Pipe.forks += 1
        return _Pipe()


class _Model:
    def __init__(self, name):
        self.name = name


def test_defaults():
    cfg = MI355XConfig()
    assert cfg.workers_per_gpu == 4
    assert cfg.model_streams == DEFAULT_MODEL_STREAMS and cfg.model_streams["kandinsky2"] == 2
    assert MI355XConfig(model_streams={"kandinsky2": 3}).model_streams == {"kandinsky2": 3}
    # SD1.5 (anythingv3): 3 streams x lock-step groups of 8 (profiles/sd_groups_r5.md), Kandinsky2 2 x 8
    # (profiles/r6/k2/); others groups of 4
    assert cfg.model_streams["anythingv3"] == 3 and cfg.model_lockstep == DEFAULT_MODEL_LOCKSTEP
    assert cfg.model_lockstep["anythingv3"] == 8 and cfg.model_lockstep["kandinsky2"] == 8
    assert cfg.lockstep_group == 4


def test_pool_group_size_per_model(monkeypatch):
    """mi355x.model_lockstep: the pool forms each model's lock-step groups at that model's size and sizes
    its capacity for the largest group (GPU only - the CPU reference path never groups)."""
    import arbius_amd.node.solver as solver
    seen = []
    monkeypatch.setattr(solver, "take_group", lambda jobs, first, n, *a: seen.append(n) or [first])
    gpu = LocalSolverPool.__new__(LocalSolverPool)
    LocalSolverPool.__init__(gpu, "cuda:0", pipeline_factory=lambda name, **kw: _Pipe(), capacity=3, lockstep=4,
                             model_lockstep={"anythingv3": 8})
    assert gpu.capacity == 3 * 8 * 2 and gpu.model_lockstep == {"anythingv3": 8}
    cpu = LocalSolverPool("cpu", pipeline_factory=lambda name, **kw: _Pipe(), capacity=3, lockstep=4,
                          model_lockstep={"anythingv3": 8})
    assert cpu.lockstep == 1 and cpu.model_lockstep == {} and cpu.capacity == 3


def test_local_pool_caps_forks_per_model():
    pool = LocalSolverPool("cpu", pipeline_factory=lambda name, **kw: _Pipe(), capacity=4,
                           model_streams={"kandinsky2": 2})
    _Pipe.forks = 0
    assert pool._pipe(_Model("kandinsky2")).qsize() == 2 and _Pipe.forks == 2
    _Pipe.forks = 0
    assert pool._pipe(_Model("anythingv3")).qsize() == 4 and _Pipe.forks == 4


def test_capped_model_solves_at_most_cap_at_once(monkeypatch):
    """Four concurrent solve requests for a model capped at 2: never more than 2 in flight."""
    import arbius_amd.node.pool as P
    live, peak, lock = [0], [0], threading.Lock()

    def fake_infer(model, pipe, inp):      # the GPU part (holds the fork); the tail is free
        with lock:
            live[0] += 1
            peak[0] = max(peak[0], live[0])
        time.sleep(0.05)
        with lock:
            live[0] -= 1
        return lambda: inp

    monkeypatch.setattr(P, "infer_task", fake_infer)
    pool = LocalSolverPool("cpu", pipeline_factory=lambda name, **kw: _Pipe(), capacity=4,
                           model_streams={"kandinsky2": 2})
    ts = [threading.Thread(target=pool.solve_sync, args=(_Model("kandinsky2"), i, {"i": i})) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert peak[0] == 2


def test_two_phase_solve_releases_fork_before_tail(monkeypatch):
    """A pipeline with ``infer`` / static ``finish`` (RVM): the fork goes back to the pool before the
    CPU tail runs, so a second solve's GPU part overlaps the first one's tail; same result as solve."""
    import arbius_amd.node.pool as P
    events, lock = [], threading.Lock()

    class _Split:
        def fork(self):
            return _Split()

        def infer(self, inp):
            with lock:
                events.append(("infer", inp["i"]))
            return inp["i"]

        @staticmethod
        def finish(raw):
            time.sleep(0.1)
            with lock:
                events.append(("finish", raw))
            return raw * 10

        def solve(self, inp):
            return self.finish(self.infer(inp))

    pool = P.LocalSolverPool("cpu", pipeline_factory=lambda name, **kw: _Split(), capacity=1)
    out = {}
    ts = [threading.Thread(target=lambda i=i: out.__setitem__(i, pool.solve_sync(_Model("rvm"), i, {"i": i})))
          for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert out == {0: 0, 1: 10}
    # one fork: the second infer ran before the first tail finished
    assert [e[0] for e in events][:2] == ["infer", "infer"]


def test_encode_mp4_array_equals_frame_list():
    """``encode_mp4`` on one [F, H, W, 3] array (no stack copy) writes the frame list's bytes."""
    import numpy as np

    from arbius_amd import native
    from arbius_amd.utils.mp4 import encode_mp4
    if not native.loaded:
        import pytest
        pytest.skip("native runtime not built")
    rng = np.random.default_rng(3)
    clip = rng.integers(0, 256, (3, 48, 64, 3), dtype=np.uint8)
    assert encode_mp4(clip, 12) == encode_mp4(list(clip), 12)
    assert encode_mp4(clip, 12, codec="avc") == encode_mp4(list(clip), 12, codec="avc")
