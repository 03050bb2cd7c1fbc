"""Lock-step grouping keys (node/solver.py): tasks share launches only when every setting the
pipeline fills in - with the model family's own defaults - is equal."""
import queue

from arbius_amd.node.solver import group_key, take_group


def test_group_key_uses_family_defaults():
    a = {"prompt": "x", "width": 768, "height": 768}
    b = dict(a, num_inference_steps=20)
    # SD family: a missing step count is the template default 20
    assert group_key(a, "anythingv3") == group_key(b, "anythingv3")
    # Kandinsky2: a missing step count is the container default 100, not 20
    assert group_key(a, "kandinsky2") != group_key(b, "kandinsky2")
    assert group_key(a, "kandinsky2") == group_key(dict(a, num_inference_steps=100, scheduler="p_sampler"),
                                                   "kandinsky2")


def test_take_group_separates_k2_default_steps():
    jobs = queue.Queue()
    mk = lambda inp: ("kandinsky2", inp)   # noqa: E731
    first = mk({"prompt": "a"})
    jobs.put(mk({"prompt": "b", "num_inference_steps": 20}))
    jobs.put(mk({"prompt": "c", "num_inference_steps": 100}))
    batch = take_group(jobs, first, 4, lambda r: "image", lambda r: r[1], lambda r: r[0])
    assert [r[1]["prompt"] for r in batch] == ["a", "c"]
    assert jobs.get_nowait()[1]["prompt"] == "b"
