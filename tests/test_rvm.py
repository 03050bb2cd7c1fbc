"""Robust video matting (BASELINE config #5) on CPU: recurrence semantics,
time-batched chunks == frame-by-frame, output types, MP4 input/output, node run."""
import os
import pytest
import asyncio
import json

import numpy as np
import torch

from arbius_amd.models.rvm import ConvGRU, RVMConfig, RVMPipeline
from arbius_amd.utils.mp4 import encode_mp4
from arbius_amd.utils.video_io import load_video
from arbius_amd.node.pool import LocalSolverPool

from test_node_e2e import _full_cycle, make_miner, make_world


def test_convgru_matches_formula():
    torch.manual_seed(0)
    g = ConvGRU(8).eval()
    x = torch.randn(1, 3, 8, 5, 6)
    out, h = g(x, None)
    hh = torch.zeros(1, 8, 5, 6)
    for t in range(3):
        rz = torch.sigmoid(g.ih(torch.cat([x[:, t], hh], 1)))
        r, z = rz[:, :8], rz[:, 8:]
        c = torch.tanh(g.hh(torch.cat([x[:, t], r * hh], 1)))
        hh = (1 - z) * hh + z * c
        assert torch.allclose(out[:, t], hh, atol=1e-5)
    assert torch.allclose(h, hh, atol=1e-5)


def test_chunking_does_not_change_output():
    frames = np.random.default_rng(1).integers(0, 256, (7, 72, 128, 3), dtype=np.uint8)
    a = RVMPipeline(RVMConfig.tiny())
    b = RVMPipeline(RVMConfig.tiny())
    b.cfg.chunk = 1
    oa, ob = a(frames), b(frames)
    assert oa.shape == frames.shape
    assert np.abs(oa.astype(int) - ob.astype(int)).max() <= 1


def test_output_types_and_mp4_io(tmp_path):
    frames = np.random.default_rng(2).integers(0, 256, (3, 64, 96, 3), dtype=np.uint8)
    import base64
    src = "data:video/mp4;base64," + base64.b64encode(encode_mp4(list(frames), 10)).decode()
    dec, fps = load_video(src)
    assert dec.shape == frames.shape and fps == 10
    pipe = RVMPipeline(RVMConfig.tiny())
    alpha = pipe(dec, "alpha-mask")
    assert (alpha[..., 0] == alpha[..., 1]).all()
    sol = pipe.solve({"input_video": src, "output_type": "green-screen"})
    sol2 = pipe.solve({"input_video": src, "output_type": "green-screen"})
    assert sol.files[0][0] == "out-1.mp4" and sol.cid == sol2.cid


def test_rvm_through_node(tmp_path):
    frames = np.random.default_rng(3).integers(0, 256, (2, 48, 64, 3), dtype=np.uint8)
    import base64
    src = "data:video/mp4;base64," + base64.b64encode(encode_mp4(list(frames), 5)).decode()
    e, tok, mid = make_world("robust_video_matting")
    pool = LocalSolverPool("cpu", tiny=True)
    m = make_miner(e, mid, pool, model="robust_video_matting")
    tid = asyncio.run(_full_cycle(e, mid, m, {"input_video": src, "output_type": "alpha-mask"}))
    row = json.loads(m.db.get_task_input(tid, e.tasks[tid].cid)["data"])
    assert pool.solve_sync(m.models[mid.lower()], tid, row).cid == e.solutions[tid].cid


@pytest.mark.parametrize("ref", ["/etc/passwd", "file:///etc/passwd", "http://example.com/a.mp4",
                                 "https://127.0.0.1/a.mp4", "https://localhost:8335/api/jobs/get",
                                 "https://169.254.169.254/latest/meta-data", "https://10.1.2.3/v.mp4",
                                 "https://[::1]/v.mp4", "https://user:pw@example.com/v.mp4", "ipfs://not-a-cid", ""])
def test_untrusted_video_sources_refused(ref):
    from arbius_amd.utils.video_io import VideoSourceError, check_source, fetch
    with pytest.raises(VideoSourceError):
        check_source(ref)
    with pytest.raises(VideoSourceError):
        fetch(ref)


def test_allowed_video_sources_classified():
    from arbius_amd.utils.video_io import check_source
    assert check_source("ipfs://QmYwAPJzv5CZsnA625s3Xf2nemtYgPpHdWEz79ojWnPbdG") == "ipfs"
    assert check_source("QmYwAPJzv5CZsnA625s3Xf2nemtYgPpHdWEz79ojWnPbdG") == "ipfs"
    assert check_source("data:video/mp4;base64,AAAA") == "data"


def test_miner_skips_task_with_refused_video_source():
    """An on-chain input_video pointing at a local file / private host is neither solved nor
    marked invalid (no contest on a source-policy decision)."""
    import asyncio
    from arbius_amd.node.pool import FakeSolverPool
    from test_node_e2e import make_miner, make_world, submit
    e, tok, mid = make_world("robust_video_matting")
    pool = FakeSolverPool()
    m = make_miner(e, mid, pool, model="robust_video_matting")

    async def go():
        await m.boot()
        await m.poll_events()
        await m.drain()
        tid = submit(e, mid, {"input_video": "https://169.254.169.254/latest/meta-data"})
        await m.poll_events()
        await m.drain()
        return tid

    tid = asyncio.run(go())
    assert pool.calls == [] and m.db.get_invalid_task(tid) is None
    assert m.metrics.counters.get("tasks_refused_source") == 1


@pytest.mark.gpu
def test_rvm_forks_concurrent_bitwise_equal_solo():
    """Two forks (shared weights, private HIP streams) matting different clips on two threads give
    exactly the solo outputs - what lets the node overlap one clip's matting with another's encode."""
    import threading
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    pipe = RVMPipeline(RVMConfig(), device="cuda")
    rng = np.random.default_rng(4)
    clips = [rng.integers(0, 256, (6, 144, 256, 3), dtype=np.uint8) for _ in range(2)]
    solo = [pipe(c, "green-screen") for c in clips]
    forks = [pipe.fork(), pipe.fork()]
    out = [None, None]

    def run(i):
        out[i] = forks[i](clips[i], "green-screen")
    ts = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert all((a == b).all() for a, b in zip(out, solo))


def test_https_fetch_connects_to_the_validated_address(monkeypatch):
    """DNS rebinding: the host is resolved once, every address must be public, and the request goes
    to that address (Host header + TLS SNI carry the name) - the client never re-resolves."""
    import socket

    from arbius_amd.utils import video_io as V
    calls = []

    def fake(host, port, *a, **k):
        calls.append(host)
        return [(socket.AF_INET, socket.SOCK_STREAM, 6, "", ("93.184.216.34", port))]
    monkeypatch.setattr(socket, "getaddrinfo", fake)
    target, host, sni = V.pinned_request("https://videos.example.com:8443/a/clip.mp4?x=1")
    assert target == "https://93.184.216.34:8443/a/clip.mp4?x=1"
    assert host == "videos.example.com:8443" and sni == "videos.example.com" and calls == ["videos.example.com"]

    def mixed(host, port, *a, **k):
        return [(socket.AF_INET, socket.SOCK_STREAM, 6, "", ("93.184.216.34", port)),
                (socket.AF_INET, socket.SOCK_STREAM, 6, "", ("10.0.0.5", port))]
    monkeypatch.setattr(socket, "getaddrinfo", mixed)
    with pytest.raises(V.VideoSourceError):
        V.pinned_request("https://videos.example.com/a.mp4")


def test_gateway_fetch_is_capped_while_streaming_and_cached(monkeypatch, tmp_path):
    import http.server
    import threading

    from arbius_amd.utils import video_io as V
    hits = []

    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            hits.append(self.path)
            body = b"\0" * (4096 if "big" not in self.path else 1 << 20)
            self.send_response(200)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        monkeypatch.setenv("ARBIUS_IPFS_GATEWAY", f"http://127.0.0.1:{srv.server_address[1]}")
        monkeypatch.setattr(V, "_CACHE_DIR", str(tmp_path / "cache"))
        monkeypatch.setattr(V, "MAX_VIDEO_BYTES", 64 << 10)
        from arbius_amd.ipfs.unixfs import add_file
        cid = add_file(b"\0" * 4096).cid_str
        assert len(V.fetch(cid)) == 4096
        assert len(V.fetch("ipfs://" + cid)) == 4096 and len(V.fetch(cid)) == 4096
        assert len(hits) == 2            # "ipfs://X" and "X" are two refs; the repeat came from the cache
        assert (os.stat(tmp_path / "cache").st_mode & 0o777) == 0o700
        # a cache entry whose bytes do not hash to the CID is never used (re-fetched instead)
        with open(V._cache_path(cid), "wb") as f:
            f.write(b"planted")
        assert V.fetch(cid) == b"\0" * 4096 and len(hits) == 3
        # a cache dir other users can write to is not used at all
        os.chmod(tmp_path / "cache", 0o777)
        assert V._cache_get(cid) is None
        os.chmod(tmp_path / "cache", 0o700)
        with pytest.raises(V.VideoSourceError):
            V.fetch(cid + "/big")
    finally:
        srv.shutdown()


@pytest.mark.gpu
def test_rvm_pinned_result_equals_staged_download(monkeypatch):
    """The composites downloaded straight into one pinned result array (default) are bitwise the
    double-buffered staging path's; the array stays valid after the pipeline's next clip."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import arbius_amd.models.rvm as R
    pipe = RVMPipeline(RVMConfig(), device="cuda")
    rng = np.random.default_rng(9)
    clips = [rng.integers(0, 256, (26, 144, 256, 3), dtype=np.uint8) for _ in range(2)]   # 3 chunks
    monkeypatch.setattr(R, "_PINNED_OUT", False)
    staged = [pipe(c, "green-screen") for c in clips]
    monkeypatch.setattr(R, "_PINNED_OUT", True)
    first = pipe(clips[0], "green-screen")
    second = pipe(clips[1], "green-screen")
    assert np.array_equal(first, staged[0]) and np.array_equal(second, staged[1])
