"""Every legal operating point of every template lands on the HIP kernels (ops/audit.py): the
models' forward passes run on the META device through the real host-side op code (eligibility,
zero-padding onto the kernels, validation, batch-invariant plan selection from the built library's
pinned tables); a shape with no HIP kernel would raise ``ops.LibraryFallback``.  For the image
templates lock-step groups of 4 and 8 (the shipped SD / K2 group) are checked launch by launch against
the solo task (same split-K
for every conv / GEMM whose rows grow with the group: the reduction order of each output)."""
import pytest
import torch

from arbius_amd import ops
from arbius_amd.ops import audit


@pytest.mark.timeout(900)
@pytest.mark.parametrize("g", [4, 8])
def test_anythingv3_every_resolution_solo_and_group(g):
    for w in audit.SD_SIZES:
        for h in audit.SD_SIZES:
            solo, group = audit.sd15(w, h, 1), audit.sd15(w, h, g)
            assert audit.launches(solo), (w, h)
            assert audit.check_invariance(solo, group) == [], (w, h)


@pytest.mark.parametrize("g", [4, 8])
def test_kandinsky2_every_resolution_solo_and_group(g):
    for w in audit.K2_SIZES:
        for h in audit.K2_SIZES:
            solo, group = audit.kandinsky2(w, h, 1), audit.kandinsky2(w, h, g)
            assert audit.check_invariance(solo, group) == [], (w, h)


@pytest.mark.timeout(900)
def test_zeroscope_every_resolution():
    for w in audit.ZS_WIDTHS:
        for h in audit.ZS_HEIGHTS:
            for f in (1, 24, 96):
                assert audit.launches(audit.video("zeroscopev2xl", w, h, f)), (w, h, f)


def test_damo_frame_counts_past_the_register_kernel():
    """damo's num_frames is not capped under the reference hydration quirks: clips past the
    register-resident temporal kernel's 96 frames take the flash kernel (no ValueError, no library)."""
    for f in (1, 16, 96, 97, 500):
        assert audit.launches(audit.video("damo", 256, 256, f)), f


def test_audit_catches_a_shape_without_kernel():
    x = torch.empty(1, 16, 16, 64, dtype=torch.bfloat16, device="meta")
    w = torch.empty(64, 5, 5, 64, dtype=torch.bfloat16, device="meta")     # 5x5: no implicit-GEMM taps
    with audit.audit():
        with pytest.raises(ops.LibraryFallback):
            ops.conv2d(x, w, padding=2)
        # a linear whose K / N the kernel does not tile is zero-padded onto it instead
        y = ops.linear(torch.empty(4, 77, 100, dtype=torch.bfloat16, device="meta"),
                       torch.empty(30, 100, dtype=torch.bfloat16, device="meta"))
        assert y.shape == (4, 77, 30)
