"""Robust Video Matting (``templates/robust_video_matting.json``; SURVEY.md §2.6(d),
BASELINE config #5: 1080p stream, recurrent ConvGRU as CDNA4 HIP, fp16).

    frames -> (downsample to <= 512 px, ratio ~0.27 at 1080p)
    MobileNetV3-Large encoder (dilated last stage) -> LR-ASPP        [time-batched]
    recurrent decoder: 4 x {upsample, concat skip + pooled source, conv, ConvGRU
                            on half the channels}                      [GRU sequential]
    projection -> (fgr residual, alpha) -> Deep Guided Filter -> full resolution
    output_type: "" / green-screen (composite on RVM's green), alpha-mask,
                 foreground-mask -> deterministic MP4 (utils/mp4.py)

MI355X mapping: fp16 channels-last throughout.  Everything that is not
recurrent runs on a CHUNK of T frames at once (batch = T), so the encoder and
the per-stage convs are wide launches; only the ConvGRU state update walks the
time axis, as two library 3x3 convs around the fused HIP gate kernels
(csrc/convgru.hip) - the concat(x, r*h) input of the second conv is written in
place by the gate kernel.  BatchNorm is folded into conv biases (inference).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import List, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..utils.progress import beat

def _host_copy(dst: np.ndarray, src: "torch.Tensor"):
    """Pinned staging buffer -> result array.  A numpy assignment: an ATen copy (GIL released, but
    OpenMP-parallel) measured 4-7 % slower on the 2-stream bench, its worker threads competing with
    the encode (profiles/bench_r4_rvm/staging_copy_ab.md)."""
    dst[...] = src.numpy().reshape(dst.shape)


# download the composites straight into a pinned result array (A/B switch; same bytes)
_PINNED_OUT = os.environ.get("ARB_RVM_PINNED_OUT", "1") == "1"
# largest clip (output bytes) downloaded into one page-locked array: ~100 frames of 1080p; longer clips
# take the staged path (two reusable pinned chunk buffers + a pageable result)
_PINNED_OUT_MAX = int(os.environ.get("ARB_RVM_PINNED_OUT_MAX", str(640 << 20)))
# the solve path downloads GPU-converted 4:2:0 planes instead of RGB (ARB_RVM_GPU_YUV=0: RGB + host
# conversion, A/B; same bytes)
_GPU_YUV = os.environ.get("ARB_RVM_GPU_YUV", "1") != "0"
# ... and encodes them on the GPU too (ops/csrc/h264_intra.hip, the native encoder's bytes): only the
# compressed slices come back, the host keeps emulation prevention + the MP4 mux
# (ARB_RVM_GPU_H264=0: download the planes and encode on the host, A/B)
_GPU_H264 = os.environ.get("ARB_RVM_GPU_H264", "1") != "0"
# the slot thread's waits on its uploads / downloads yield the CPU (hipEventBlockingSync) instead of
# spinning: RVM is host-bound (profiles/cpu_budget_r5.md) and a spinning wait takes a core from the
# H.264 encoders of the other slots' tails (ARB_RVM_BLOCKING_SYNC=0: spin, A/B)
_BLOCKING = os.environ.get("ARB_RVM_BLOCKING_SYNC", "1") != "0"


def _event():
    return torch.cuda.Event(blocking=_BLOCKING)

# the input chunk's copy into its pinned staging buffer as a numpy assignment (A/B switch)
_NUMPY_IN = os.environ.get("ARB_RVM_NUMPY_IN", "1") == "1"

# CPU priority of the output encode's threads (RVMPipeline.finish); 0 = same as the caller
ENCODE_NICE = int(os.environ.get("ARB_ENCODE_NICE", "10"))
from .graphs import PipelineBase

CL = torch.channels_last
GREEN = (120 / 255, 255 / 255, 155 / 255)     # RVM's green-screen background
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)

# MobileNetV3-Large inverted residual table: kernel, expand, out, SE, hardswish, stride, dilation
MBV3_LARGE = [
    (3, 16, 16, False, False, 1, 1), (3, 64, 24, False, False, 2, 1), (3, 72, 24, False, False, 1, 1),
    (5, 72, 40, True, False, 2, 1), (5, 120, 40, True, False, 1, 1), (5, 120, 40, True, False, 1, 1),
    (3, 240, 80, False, True, 2, 1), (3, 200, 80, False, True, 1, 1), (3, 184, 80, False, True, 1, 1),
    (3, 184, 80, False, True, 1, 1), (3, 480, 112, True, True, 1, 1), (3, 672, 112, True, True, 1, 1),
    (5, 672, 160, True, True, 1, 2), (5, 960, 160, True, True, 1, 2), (5, 960, 160, True, True, 1, 2),
]


def _conv(conv: nn.Conv2d, x):
    """Dense 1x1 / 3x3 convs on the MFMA implicit-GEMM kernel (its fp16 twin), channels-last in
    and out (an NCHW channels-last tensor IS the NHWC buffer, and so is the weight); depthwise,
    dilated and 5x5 convs stay on the library path.  MIOpen's deterministic mode runs its naive
    direct kernel for these shapes: 1.1 ms per call, 97 % of the matting time before."""
    k = conv.kernel_size
    if (x.is_cuda and conv.groups == 1 and conv.dilation == (1, 1) and k[0] == k[1] and k[0] in (1, 3)
            and conv.padding == (k[0] // 2, k[0] // 2) and conv.stride[0] == conv.stride[1]
            and conv.stride[0] in (1, 2) and not ops.reference_ops()):
        xh = x.permute(0, 2, 3, 1)
        w = conv.weight.permute(0, 2, 3, 1)
        y = ops.conv2d(xh.contiguous(), w.contiguous(), conv.bias, stride=conv.stride[0], padding=k[0] // 2)
        return y.permute(0, 3, 1, 2)
    return conv(x)


def _div8(v):
    return max(8, int(v + 4) // 8 * 8)


@dataclass
class RVMConfig:
    width_mult: float = 1.0
    decoder_channels: Tuple[int, ...] = (80, 40, 32, 16)
    aspp_channels: int = 128
    max_side: int = 512              # auto downsample ratio = min(1, max_side / max(H, W))
    chunk: int = 12                  # frames per time-batched chunk
    dgf_hidden: int = 16

    @staticmethod
    def tiny():
        return RVMConfig(width_mult=0.5, decoder_channels=(32, 16, 16, 16), aspp_channels=32, max_side=64, chunk=4)


class ConvAct(nn.Module):
    def __init__(self, cin, cout, k=1, stride=1, groups=1, act="relu", dilation=1, bias=True):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, stride, dilation * (k // 2), dilation=dilation, groups=groups, bias=bias)
        self.act = act

    def forward(self, x):
        c = self.conv
        if c.groups > 1 and c.groups == c.in_channels == c.out_channels:     # depthwise: fused HIP pass
            return ops.depthwise_conv(x, c.weight, c.bias, c.stride[0], c.dilation[0], self.act)
        x = _conv(c, x)
        if self.act == "relu":
            return F.relu(x)
        if self.act == "hs":
            return F.hardswish(x)
        return x


class SE(nn.Module):
    def __init__(self, c):
        super().__init__()
        s = _div8(c // 4)
        self.fc1 = nn.Conv2d(c, s, 1)
        self.fc2 = nn.Conv2d(s, c, 1)

    def forward(self, x):
        w = F.adaptive_avg_pool2d(x, 1)
        return x * F.hardsigmoid(_conv(self.fc2, F.relu(_conv(self.fc1, w))))


class InvertedResidual(nn.Module):
    def __init__(self, cin, k, exp, cout, se, hs, stride, dil):
        super().__init__()
        act = "hs" if hs else "relu"
        self.expand = ConvAct(cin, exp, 1, act=act) if exp != cin else None
        self.dw = ConvAct(exp, exp, k, stride, groups=exp, act=act, dilation=dil)
        self.se = SE(exp) if se else None
        self.project = ConvAct(exp, cout, 1, act=None)
        self.res = stride == 1 and cin == cout

    def forward(self, x):
        h = self.expand(x) if self.expand is not None else x
        h = self.dw(h)
        if self.se is not None:
            h = self.se(h)
        h = self.project(h)
        return x + h if self.res else h


class MobileNetV3Encoder(nn.Module):
    def __init__(self, width_mult=1.0):
        super().__init__()
        c = lambda v: _div8(v * width_mult)
        layers: List[nn.Module] = [ConvAct(3, c(16), 3, 2, act="hs")]
        cin = c(16)
        for (k, e, o, se, hs, s, d) in MBV3_LARGE:
            layers.append(InvertedResidual(cin, k, c(e), c(o), se, hs, s, d))
            cin = c(o)
        layers.append(ConvAct(cin, c(960) if width_mult != 1.0 else 960, 1, act="hs"))
        self.features = nn.ModuleList(layers)
        self.out_channels = (c(16), c(24), c(40), c(960) if width_mult != 1.0 else 960)

    def forward(self, x):
        f = self.features
        for i in range(0, 2):
            x = f[i](x)
        f1 = x
        for i in range(2, 4):
            x = f[i](x)
        f2 = x
        for i in range(4, 7):
            x = f[i](x)
        f3 = x
        for i in range(7, 17):
            x = f[i](x)
        return f1, f2, f3, x


class LRASPP(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.aspp1 = ConvAct(cin, cout, 1, act="relu")
        self.aspp2 = nn.Conv2d(cin, cout, 1, bias=False)

    def forward(self, x):
        return self.aspp1(x) * torch.sigmoid(_conv(self.aspp2, F.adaptive_avg_pool2d(x, 1)))


class ConvGRU(nn.Module):
    """h' = (1-z) h + z tanh(W_hh * [x, r h]);  [r, z] = sigmoid(W_ih * [x, h])."""

    def __init__(self, c):
        super().__init__()
        self.c = c
        self.ih = nn.Conv2d(2 * c, 2 * c, 3, padding=1)
        self.hh = nn.Conv2d(2 * c, c, 3, padding=1)

    def forward(self, x, h):
        """x [B, T, C, H, W] (time-batched chunk), h [B, C, H, W] or None -> (out [B,T,C,H,W], h)."""
        B, T, C, H, W = x.shape
        if h is None:
            h = torch.zeros(B, C, H, W, dtype=x.dtype, device=x.device).contiguous(memory_format=CL)
        outs = []
        for t in range(T):
            buf = torch.cat([x[:, t], h], dim=1).contiguous(memory_format=CL)   # [x | h]
            z = ops.convgru_gates1(_conv(self.ih, buf).contiguous(memory_format=CL), h, buf, C)   # buf -> [x | r h]
            h = ops.convgru_gates2(_conv(self.hh, buf).contiguous(memory_format=CL), h, z)
            outs.append(h)
        return torch.stack(outs, dim=1), h


class _GRUHalf(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.half = c // 2
        self.gru = ConvGRU(c // 2)

    def forward(self, x, h):          # x [B, T, C, H, W]
        a, b = x[:, :, : self.half], x[:, :, self.half:]
        b, h = self.gru(b, h)
        return torch.cat([a, b], dim=2), h


def _bt(x):    # [B, T, C, H, W] -> [B*T, C, H, W] channels-last
    B, T = x.shape[:2]
    return x.reshape(B * T, *x.shape[2:]).contiguous(memory_format=CL)


def _ubt(x, B):
    return x.reshape(B, x.shape[0] // B, *x.shape[1:])


class UpBlock(nn.Module):
    def __init__(self, cin, cskip, csrc, cout):
        super().__init__()
        self.conv = ConvAct(cin + cskip + csrc, cout, 3, act="relu")
        self.gru = _GRUHalf(cout)

    def forward(self, x, f, s, h, B):
        x = F.interpolate(x, scale_factor=2.0, mode="bilinear", align_corners=False)
        x = x[:, :, : s.shape[2], : s.shape[3]]
        x = self.conv(torch.cat([x, f, s], dim=1).contiguous(memory_format=CL))
        x, h = self.gru(_ubt(x, B), h)
        return _bt(x), h


class RecurrentDecoder(nn.Module):
    def __init__(self, feat: Tuple[int, ...], aspp: int, dec: Tuple[int, ...]):
        super().__init__()
        self.decode4 = _GRUHalf(aspp)
        self.decode3 = UpBlock(aspp, feat[2], 3, dec[0])
        self.decode2 = UpBlock(dec[0], feat[1], 3, dec[1])
        self.decode1 = UpBlock(dec[1], feat[0], 3, dec[2])
        self.out0 = ConvAct(dec[2] + 3, dec[3], 3, act="relu")
        self.out1 = ConvAct(dec[3], dec[3], 3, act="relu")

    def forward(self, s0, f1, f2, f3, f4, rec, B):
        s1 = F.avg_pool2d(s0, 2, 2, ceil_mode=True)
        s2 = F.avg_pool2d(s1, 2, 2, ceil_mode=True)
        s3 = F.avg_pool2d(s2, 2, 2, ceil_mode=True)
        x4, r4 = self.decode4(_ubt(f4, B), rec[0])
        x3, r3 = self.decode3(_bt(x4), f3, s3, rec[1], B)
        x2, r2 = self.decode2(x3, f2, s2, rec[2], B)
        x1, r1 = self.decode1(x2, f1, s1, rec[3], B)
        x = F.interpolate(x1, scale_factor=2.0, mode="bilinear", align_corners=False)
        x = x[:, :, : s0.shape[2], : s0.shape[3]]
        x = self.out1(self.out0(torch.cat([x, s0], dim=1).contiguous(memory_format=CL)))
        return x, [r4, r3, r2, r1]


class DeepGuidedFilter(nn.Module):
    def __init__(self, hid=16):
        super().__init__()
        self.c1 = ConvAct(4 * 2 + hid, hid, 1, act="relu", bias=True)
        self.c2 = ConvAct(hid, hid, 1, act="relu", bias=True)
        self.c3 = nn.Conv2d(hid, 4, 1)

    def _boxf(self, x):
        # 3x3 mean with zero padding (RVM's box filter: a ones/9 depthwise conv) as a count-including
        # average pool: a native NHWC kernel instead of MIOpen's naive path for this 4-channel
        # depthwise conv (80 us per call at 512x288, profiles/rocprof_r2_rvm.md)
        return F.avg_pool2d(x, 3, stride=1, padding=1, count_include_pad=True)

    def forward(self, fine_src, base_src, base_fgr, base_pha, base_hid):
        fine_x = torch.cat([fine_src, fine_src.mean(1, keepdim=True)], dim=1)
        base_x = torch.cat([base_src, base_src.mean(1, keepdim=True)], dim=1)
        base_y = torch.cat([base_fgr, base_pha], dim=1)
        mean_x, mean_y = self._boxf(base_x), self._boxf(base_y)
        cov_xy = self._boxf(base_x * base_y) - mean_x * mean_y
        var_x = self._boxf(base_x * base_x) - mean_x * mean_x
        A = _conv(self.c3, self.c2(self.c1(torch.cat([cov_xy, var_x, base_hid], dim=1).contiguous(memory_format=CL))))
        b = mean_y - A * mean_x
        H, W = fine_src.shape[2:]
        A = F.interpolate(A, (H, W), mode="bilinear", align_corners=False)
        b = F.interpolate(b, (H, W), mode="bilinear", align_corners=False)
        out = A * fine_x + b
        return out[:, :3], out[:, 3:]


class MattingNetwork(nn.Module):
    def __init__(self, cfg: RVMConfig):
        super().__init__()
        self.backbone = MobileNetV3Encoder(cfg.width_mult)
        feat = self.backbone.out_channels
        self.aspp = LRASPP(feat[3], cfg.aspp_channels)
        self.decoder = RecurrentDecoder(feat, cfg.aspp_channels, cfg.decoder_channels)
        self.project = nn.Conv2d(cfg.decoder_channels[3], 4, 1)
        self.refiner = DeepGuidedFilter(cfg.decoder_channels[3])
        self.register_buffer("mean", torch.tensor(IMAGENET_MEAN).view(1, 3, 1, 1))
        self.register_buffer("std", torch.tensor(IMAGENET_STD).view(1, 3, 1, 1))

    def forward(self, src, rec, ratio: float):
        """src [B, T, 3, H, W] in [0,1] -> fgr, pha [B, T, *, H, W], new recurrent state."""
        B, T = src.shape[:2]
        fine = _bt(src)
        if ratio < 1.0:
            H, W = fine.shape[2:]
            small = F.interpolate(fine, (int(round(H * ratio)), int(round(W * ratio))), mode="bilinear",
                                  align_corners=False, antialias=False).contiguous(memory_format=CL)
        else:
            small = fine
        x = ((small - self.mean.to(small.dtype)) / self.std.to(small.dtype)).contiguous(memory_format=CL)
        f1, f2, f3, f4 = self.backbone(x)
        f4 = self.aspp(f4)
        hid, rec = self.decoder(small, f1, f2, f3, f4, rec, B)
        proj = _conv(self.project, hid)
        fgr_res, pha = proj[:, :3], proj[:, 3:]
        if ratio < 1.0:
            fgr_res, pha = self.refiner(fine, small, fgr_res, pha, hid)
        fgr = (fgr_res + fine).clamp(0.0, 1.0)
        pha = pha.clamp(0.0, 1.0)
        return _ubt(fgr, B), _ubt(pha, B), rec


class RVMPipeline(PipelineBase):
    """Clip-level matting.  ``fork()`` (PipelineBase) shares the weights and owns a private HIP
    stream, so the node / bench can matte one clip on the GPU while another clip's MP4 is encoded
    and hashed on the CPU; every clip's kernels and their order are those of a solo run (bitwise)."""

    def __init__(self, cfg: RVMConfig = None, device="cpu", dtype=None, weight_seed: int = 0, init=True, **_):
        self.cfg = cfg = cfg or RVMConfig()
        self.device = torch.device(device)
        if dtype is None:
            dtype = torch.float16 if self.device.type == "cuda" else torch.float32
        self.dtype = dtype
        with torch.random.fork_rng(devices=[]):
            torch.manual_seed(weight_seed + 7)
            self.net = MattingNetwork(cfg)
        self.net.requires_grad_(False)
        self.net.to(device=self.device, dtype=dtype, memory_format=CL).eval()
        self.timings = {}

    def _reset_graphs(self):
        # eager launches (the recurrent state is per clip): nothing to re-capture; a fork gets its OWN
        # pinned staging buffers (they are written while the fork's previous chunk is in flight)
        self._pin = {}

    def modules(self):
        return {"net": self.net}

    @torch.no_grad()
    def __call__(self, frames: np.ndarray, output_type: str = "green-screen") -> np.ndarray:
        """frames uint8 [T, H, W, 3] -> uint8 [T, H, W, 3] (composite / alpha / foreground)."""
        with self._stream_ctx():
            return self._matte(frames, output_type)

    def _fast_ok(self, ratio) -> bool:
        # every size: ratio < 1 runs the guided filter at full resolution, ratio 1 (inputs <= 512 px)
        # composes the network's own full-resolution output (csrc/rvm.hip rvm_dgf_base ``direct``)
        return (self.device.type == "cuda" and self.dtype == torch.float16 and ratio <= 1.0
                and not ops.reference_ops() and self.net.backbone.features[0].conv.out_channels == 16)

    def _pinned(self, key, nbytes):
        """Reusable page-locked host staging buffers (async H2D / D2H), per pipeline fork."""
        bufs = self.__dict__.setdefault("_pin", {})     # per fork: fork() -> _reset_graphs() -> {}
        b = bufs.get(key)
        if b is None or b.numel() < nbytes:
            b = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
            bufs[key] = b
        return b[:nbytes]

    def _matte_fast(self, frames: np.ndarray, output_type: str, ratio: float, yuv: bool = False):
        """HIP fast path (models/rvm_fast.py): uint8 chunks in through pinned double buffers (async
        H2D), uint8 composites out the same way; chunk i+1's upload and chunk i-1's download overlap
        chunk i's kernels.  Bytes are those of the fast path, bitwise, for any chunk timing."""
        from .rvm_fast import FastMatting
        if getattr(self, "_fast", None) is None:
            self._fast = FastMatting(self.net)
        T, H, W, _ = frames.shape
        n = self.cfg.chunk
        yuv = yuv and _GPU_YUV
        if yuv and _GPU_H264:
            return self._matte_fast_h264(frames, output_type, ratio)
        nout = T * ((H + 15) // 16 * 16) * ((W + 15) // 16 * 16) * 3 // 2 if yuv else T * H * W * 3
        if _PINNED_OUT and nout <= _PINNED_OUT_MAX:
            # the page-locked result array comes from PyTorch's caching host allocator,
            # which rounds up and never returns memory to the OS - bounded per clip; a failed pin
            # (host memory exhausted) falls back to the staged download below (same bytes)
            try:
                res_pin = torch.empty(nout, dtype=torch.uint8, pin_memory=True)
            except RuntimeError:
                res_pin = None
            if res_pin is not None:
                return self._matte_fast_pinned(frames, output_type, ratio, res_pin, yuv)
        res = np.empty((T, H, W, 3), dtype=np.uint8)
        stream = torch.cuda.current_stream(self.device)
        rec = [None] * 4
        pending = []                      # (event, pinned out view, target slice)
        ups = []
        for j, i in enumerate(range(0, T, n)):
            beat()
            t = min(n, T - i)
            nb = t * H * W * 3
            st = self._pinned(("in", j % 2), n * H * W * 3)[:nb]
            if len(ups) >= 2:
                ups[-2].synchronize()     # the staging buffer's previous upload has been consumed
            st.copy_(torch.from_numpy(np.ascontiguousarray(frames[i:i + t]).reshape(-1)))
            dev = st.to(self.device, non_blocking=True).view(t, H, W, 3)
            ev = _event()
            ev.record(stream)
            ups.append(ev)
            out, rec = self._fast(dev, rec, ratio, output_type, GREEN)
            ob = self._pinned(("out", j % 2), n * H * W * 3)[:nb]
            if len(pending) >= 2:         # the staging buffer's previous download must be drained first
                e, v, sl = pending.pop(0)
                e.synchronize()
                _host_copy(res[sl], v)
            ob.copy_(out.view(-1), non_blocking=True)
            e = _event()
            e.record(stream)
            pending.append((e, ob, slice(i, i + t)))
        for e, v, sl in pending:
            e.synchronize()
            _host_copy(res[sl], v)
        return res

    def _matte_fast_pinned(self, frames: np.ndarray, output_type: str, ratio: float, res, yuv: bool = False):
        """As ``_matte_fast``, but every chunk's composite is downloaded straight into one page-locked
        result array (PyTorch's caching host allocator: a freed clip's block is reused), so the
        300 MB host copy out of a staging buffer is gone; the result is that array's numpy view
        (it keeps the block alive until the encode has read it).  Same bytes.
        ``yuv``: each chunk's composite is converted on the GPU to the encoder's macroblock-padded
        4:2:0 planes (``ops.rgb_to_yuv420``) and those are downloaded instead (1.5 instead of 3 bytes
        per pixel, no host colour conversion): returns a ``utils.mp4.Yuv420Clip`` that encodes to the
        RGB path's bytes."""
        from .rvm_fast import FastMatting
        if getattr(self, "_fast", None) is None:
            self._fast = FastMatting(self.net)
        T, H, W, _ = frames.shape
        n = self.cfg.chunk
        fb = H * W * 3
        stream = torch.cuda.current_stream(self.device)
        rec = [None] * 4
        ups = []
        if yuv:
            H16, W16 = (H + 15) // 16 * 16, (W + 15) // 16 * 16
            ly, lc = H16 * W16, H16 * W16 // 4
            planes = (res[:T * ly].view(T, H16, W16), res[T * ly:T * (ly + lc)].view(T, H16 // 2, W16 // 2),
                      res[T * (ly + lc):T * (ly + 2 * lc)].view(T, H16 // 2, W16 // 2))
        for j, i in enumerate(range(0, T, n)):
            beat()
            t = min(n, T - i)
            st = self._pinned(("in", j % 2), n * fb)[:t * fb]
            if len(ups) >= 2:
                ups[-2].synchronize()     # the staging buffer's previous upload has been consumed
            if _NUMPY_IN:                 # one thread (ATen's copy wakes its OpenMP pool)
                st.numpy()[:] = frames[i:i + t].reshape(-1)
            else:
                st.copy_(torch.from_numpy(np.ascontiguousarray(frames[i:i + t]).reshape(-1)))
            dev = st.to(self.device, non_blocking=True).view(t, H, W, 3)
            ev = _event()
            ev.record(stream)
            ups.append(ev)
            out, rec = self._fast(dev, rec, ratio, output_type, GREEN)
            if yuv:
                for dst, src in zip(planes, ops.rgb_to_yuv420(out)):
                    dst[i:i + t].copy_(src, non_blocking=True)
            else:
                res[i * fb:(i + t) * fb].copy_(out.view(-1), non_blocking=True)
        done = _event()
        done.record(stream)
        done.synchronize()
        if yuv:
            from ..utils.mp4 import Yuv420Clip
            return Yuv420Clip(*(pl.numpy() for pl in planes), W, H, keep=res)
        return res.view(T, H, W, 3).numpy()

    def _matte_fast_h264(self, frames: np.ndarray, output_type: str, ratio: float):
        """As ``_matte_fast_pinned`` with ``yuv``, but the 4:2:0 planes stay on the GPU and are encoded
        there (``ops.h264_intra_encode``): returns a ``utils.mp4.H264IntraClip`` (the slices' RBSPs,
        page-locked) whose MP4 is byte-identical to the host encode of the same planes.  A clip the
        GPU encoder flags (output capacity) is downloaded as planes and encoded on the host."""
        from .rvm_fast import FastMatting
        from ..utils.mp4 import INTRA_QP, H264IntraClip, Yuv420Clip
        if getattr(self, "_fast", None) is None:
            self._fast = FastMatting(self.net)
        T, H, W, _ = frames.shape
        n = self.cfg.chunk
        fb = H * W * 3
        H16, W16 = (H + 15) // 16 * 16, (W + 15) // 16 * 16
        dev = self.device
        planes = (torch.empty(T, H16, W16, dtype=torch.uint8, device=dev),
                  torch.empty(T, H16 // 2, W16 // 2, dtype=torch.uint8, device=dev),
                  torch.empty(T, H16 // 2, W16 // 2, dtype=torch.uint8, device=dev))
        stream = torch.cuda.current_stream(dev)
        rec = [None] * 4
        ups = []
        for j, i in enumerate(range(0, T, n)):
            beat()
            t = min(n, T - i)
            st = self._pinned(("in", j % 2), n * fb)[:t * fb]
            if len(ups) >= 2:
                ups[-2].synchronize()     # the staging buffer's previous upload has been consumed
            if _NUMPY_IN:
                st.numpy()[:] = frames[i:i + t].reshape(-1)
            else:
                st.copy_(torch.from_numpy(np.ascontiguousarray(frames[i:i + t]).reshape(-1)))
            x = st.to(dev, non_blocking=True).view(t, H, W, 3)
            ev = _event()
            ev.record(stream)
            ups.append(ev)
            out, rec = self._fast(x, rec, ratio, output_type, GREEN)
            ops.rgb_to_yuv420(out, out=tuple(p[i:i + t] for p in planes))
        enc, meta = ops.h264_intra_encode(*planes, INTRA_QP)
        meta_h = torch.empty(meta.numel(), dtype=torch.int64, pin_memory=True)
        meta_h.copy_(meta, non_blocking=True)
        done = _event()
        done.record(stream)
        done.synchronize()
        m = meta_h.numpy()
        if m[T + 1] != 0:                 # flagged: the host encoder takes the planes (same bytes)
            host = [torch.empty(p.shape, dtype=torch.uint8, pin_memory=True) for p in planes]
            for h, p in zip(host, planes):
                h.copy_(p, non_blocking=True)
            done = _event()
            done.record(stream)
            done.synchronize()
            return Yuv420Clip(*(h.numpy() for h in host), W, H, keep=host)
        total = int(m[T])
        buf = torch.empty(max(total, 1), dtype=torch.uint8, pin_memory=True)
        buf[:total].copy_(enc[:total], non_blocking=True)
        done = _event()
        done.record(stream)
        done.synchronize()
        return H264IntraClip(buf.numpy()[:total], m.copy(), W, H, INTRA_QP, keep=buf)

    @torch.no_grad()
    def matte_for_encode(self, frames: np.ndarray, output_type: str = "green-screen"):
        """As ``__call__``, but on the HIP fast path the result is the encoder's 4:2:0 planes, converted
        on the GPU (``utils.mp4.Yuv420Clip``, the same MP4 bytes); otherwise uint8 RGB frames."""
        with self._stream_ctx():
            return self._matte(frames, output_type, yuv=True)

    def _matte(self, frames: np.ndarray, output_type: str, yuv: bool = False):
        t0 = time.perf_counter()
        T, H, W, _ = frames.shape
        ratio = min(1.0, self.cfg.max_side / max(H, W))
        if self._fast_ok(ratio):
            res = self._matte_fast(frames, output_type, ratio, yuv)
            self.timings = {"matting_s": time.perf_counter() - t0}
            return res
        rec = [None] * 4
        out = []
        green = torch.tensor(GREEN, dtype=self.dtype, device=self.device).view(1, 3, 1, 1)
        for i in range(0, T, self.cfg.chunk):
            beat()
            chunk = torch.from_numpy(np.ascontiguousarray(frames[i:i + self.cfg.chunk])).to(self.device)
            src = (chunk.permute(0, 3, 1, 2).to(self.dtype) / 255.0)[None]     # [1, t, 3, H, W]
            fgr, pha, rec = self.net(src, rec, ratio)
            fgr, pha = fgr[0], pha[0]
            if output_type == "alpha-mask":
                img = pha.expand(-1, 3, -1, -1)
            elif output_type == "foreground-mask":
                img = fgr
            else:                                   # "" and "green-screen"
                img = fgr * pha + green * (1 - pha)
            out.append((img.float() * 255).round().clamp(0, 255).to(torch.uint8).permute(0, 2, 3, 1).cpu())
        res = torch.cat(out).numpy()
        self.timings = {"matting_s": time.perf_counter() - t0}
        return res

    def infer(self, inp: dict):
        """GPU part of a solve (input hydration + matting): host arrays for ``finish``."""
        from ..utils.video_io import load_video
        t0 = time.perf_counter()
        frames, fps = load_video(inp["input_video"])
        out = self.matte_for_encode(frames, inp.get("output_type") or "green-screen")
        tm = dict(self.timings)
        tm["infer_s"] = time.perf_counter() - t0
        return out, fps, tm

    @staticmethod
    def finish(raw) -> "Solution":
        """CPU tail of a solve, no GPU and no pipeline state: H.264 encode + MP4 + CID.  Task slots
        run it while their pipeline mattes the next clip (node/solver.py ``infer_task``)."""
        from ..node.solver import solve_files
        from ..utils.mp4 import encode_mp4
        out, fps, tm = raw
        t1 = time.perf_counter()
        # encode threads at nice 10: the slot's next clip's staging copies keep their CPU
        mp4 = encode_mp4(out, fps, nice=ENCODE_NICE)
        tm = dict(tm, encode_cid_s=time.perf_counter() - t1)
        return solve_files([("out-1.mp4", mp4)], tm)

    def solve(self, inp: dict):
        return self.finish(self.infer(inp))
