"""Per-model task-stream caps (mi355x.model_streams): a capped model gets fewer pipeline forks /
concurrently solving worker slots than the GPU's stream count."""
import threading
import time

from arbius_amd.config.mining_config import DEFAULT_MODEL_STREAMS, MI355XConfig
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

    def fake_solve(model, pipe, inp):
        with lock:
            live[0] += 1
            peak[0] = max(peak[0], live[0])
        time.sleep(0.05)
        with lock:
            live[0] -= 1
        return inp

    monkeypatch.setattr(P, "solve_task", fake_solve)
    pool = LocalSolverPool("cpu", pipeline_factory=lambda name, **kw: _Pipe(), capacity=4,
                           model_streams={"kandinsky2": 2})
    ts = [threading.Thread(target=pool.solve_sync, args=(_Model("kandinsky2"), i, {"i": i})) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert peak[0] == 2
