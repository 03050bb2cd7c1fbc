"""Video families (BASELINE config #4 zeroscopev2xl, damo) and the deterministic
MP4 writer, on CPU: bitstream/container structure, lossless PCM round trip,
tiny UNet3D pipeline determinism and a node round trip with out-1.mp4."""
import asyncio
import json

import numpy as np
import torch

from arbius_amd.models.video import VideoConfig, VideoPipeline
from arbius_amd.utils.mp4 import _ep, encode_mp4, read_mp4_pcm, rgb_to_yuv420, sps_pps
from arbius_amd.node.pool import LocalSolverPool

from test_node_e2e import _full_cycle, make_miner, make_world


class _Reader:
    def __init__(self, data):
        self.bits = "".join(f"{b:08b}" for b in data)
        self.i = 0

    def u(self, n):
        v = int(self.bits[self.i:self.i + n], 2) if n else 0
        self.i += n
        return v

    def ue(self):
        z = 0
        while self.bits[self.i] == "0":
            z += 1
            self.i += 1
        return self.u(z + 1) - 1

    def se(self):
        k = self.ue()
        return (k + 1) // 2 if k % 2 else -(k // 2)


def test_sps_fields_and_cropping():
    sps, pps = sps_pps(1920, 1080)
    assert sps[0] == 0x67 and pps[0] == 0x68
    r = _Reader(sps[1:])
    assert (r.u(8), r.u(8), r.u(8)) == (66, 0xC0, 51)
    assert r.ue() == 0 and r.ue() == 0 and r.ue() == 2 and r.ue() == 1 and r.u(1) == 0
    assert r.ue() + 1 == 120 and r.ue() + 1 == 68          # 1920/16, 1088/16
    assert r.u(1) == 1 and r.u(1) == 1
    assert r.u(1) == 1 and [r.ue() for _ in range(4)] == [0, 0, 0, 4]   # crop 8 rows (CropUnitY = 2)
    assert r.u(1) == 0 and r.u(1) == 1                        # no VUI, stop bit


def test_emulation_prevention():
    assert _ep(b"\x00\x00\x01\x00\x00\x00\x00") == b"\x00\x00\x03\x01\x00\x00\x03\x00\x00"


def test_mp4_pcm_roundtrip_lossless_and_deterministic():
    rng = np.random.default_rng(0)
    frames = [rng.integers(0, 256, (40, 72, 3), dtype=np.uint8) for _ in range(4)]
    a, b = encode_mp4(frames, 24), encode_mp4(frames, 24)
    assert a == b and a[4:8] == b"ftyp" and a[a.index(b"moov") - 4:].startswith(a[a.index(b"moov") - 4:][:4])
    fps, planes = read_mp4_pcm(a)
    assert fps == 24 and len(planes) == 4
    for f, (y, cb, cr) in zip(frames, planes):
        ey, ecb, ecr = rgb_to_yuv420(np.pad(f, ((0, 8), (0, 8), (0, 0)), mode="edge"))
        assert (y == ey).all() and (cb == ecb).all() and (cr == ecr).all()
        assert y.min() >= 1 and cb.min() >= 1      # no start-code emulation possible in PCM bytes


def test_video_tiny_deterministic():
    pipe = VideoPipeline(VideoConfig.tiny(), device="cpu")
    kw = dict(num_frames=5, width=64, height=64, num_inference_steps=2, seed=3)
    a, b = pipe("arbius test cat", **kw), pipe("arbius test cat", **kw)
    assert a.shape == (5, 64, 64, 3) and (a == b).all()
    assert not (a == pipe("arbius test cat", **{**kw, "seed": 4})).all()


def test_temporal_ops_reference_semantics():
    """TemporalConv/TemporalTransformer mix information across frames only."""
    from arbius_amd.models.layers import init_weights
    from arbius_amd.models.unet3d import TemporalConv
    tc = init_weights(torch.nn.ModuleDict({"t": TemporalConv(64, 8, 1e-5)}), 0)["t"].eval()
    x = torch.randn(2 * 4, 3, 3, 64)
    y = tc(x, frames=4)
    x2 = x.clone()
    x2[4:] += 1.0                      # perturb the second video only
    y2 = tc(x2, frames=4)
    assert torch.allclose(y[:4], y2[:4]) and not torch.allclose(y[4:], y2[4:])


def test_damo_tiny_through_node():
    e, tok, mid = make_world("damo")
    pool = LocalSolverPool("cpu", tiny=True)
    m = make_miner(e, mid, pool, model="damo")
    inp = {"prompt": "arbius test cat", "num_frames": 3, "num_inference_steps": 2, "fps": 8}
    tid = asyncio.run(_full_cycle(e, mid, m, inp))
    model = m.models[mid.lower()]
    row = json.loads(m.db.get_task_input(tid, e.tasks[tid].cid)["data"])
    sol = pool.solve_sync(model, tid, row)
    assert sol.files[0][0] == "out-1.mp4" and sol.cid == e.solutions[tid].cid
