"""CPU paths of the GLIDE resampling ops (ops.pool2 / ops.upsample2): the fp32 references the HIP
kernels (csrc/elementwise.hip norm_pool2 / upsample2) are tested against on the GPU."""
import torch
import torch.nn.functional as F

from arbius_amd import ops


def test_pool2_raw_and_normalised():
    torch.manual_seed(0)
    x = torch.randn(2, 6, 10, 16)
    table = torch.randn(2, 16, 2)
    yn, yx = ops.pool2(x, (table, True))
    rx = F.avg_pool2d(x.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
    xn = F.silu(x * table[:, None, None, :, 0] + table[:, None, None, :, 1])
    rn = F.avg_pool2d(xn.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
    assert torch.allclose(yx, rx, atol=1e-6) and torch.allclose(yn, rn, atol=1e-5)
    none, yx2 = ops.pool2(x)
    assert none is None and torch.equal(yx2, yx)


def test_upsample2_nearest():
    x = torch.randn(2, 3, 5, 8)
    assert torch.equal(ops.upsample2(x), F.interpolate(x.permute(0, 3, 1, 2), scale_factor=2.0,
                                                          mode="nearest").permute(0, 2, 3, 1))
