"""Graph-replay check of the split-K conv (in-launch reduction) vs eager."""
import torch
from arbius_amd.ops import _lib

torch.manual_seed(0)
dev = torch.device("cuda")
x = torch.randn(2, 16, 16, 640, device=dev).bfloat16()
w = (torch.randn(1280, 3, 3, 640, device=dev) / 76).bfloat16()
b = torch.randn(1280, device=dev).bfloat16()
for cfg in (13, 15):
    ref = _lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1, cfg, 4)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            out = _lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1, cfg, 4)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = _lib.conv2d_nhwc(x, w, b, 1, False, None, None, 1, cfg, 4)
    for i in range(4):
        g.replay()
        torch.cuda.synchronize()
        print(cfg, i, torch.equal(out, ref), (out.float() - ref.float()).abs().max().item(), flush=True)
