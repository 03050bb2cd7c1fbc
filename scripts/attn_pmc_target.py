"""PMC target: the batched SD level-0 self-attention (B=8, 4096 tokens, 8 heads, d=40) x 20."""
import math
import sys

import torch

sys.path.insert(0, ".")
from arbius_amd.ops import _lib  # noqa: E402

B, N, H, D = 8, 4096, 8, 40
qkv = torch.randn(B, N, 3, H, D, device="cuda").bfloat16()
q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
for _ in range(20):
    _lib.flash_attention(q, k, v, 1 / math.sqrt(D), False)
torch.cuda.synchronize()
print("done")
