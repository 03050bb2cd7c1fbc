"""GPU fast path of the Robust Video Matting network (templates/robust_video_matting.json; BASELINE
config #5): the same MattingNetwork weights as ``models/rvm.py``, run on NHWC fp16 buffers through the
HIP kernels only (VERDICT r2 "RVM hot path on hand-written kernels"):

* frames stay uint8 on the device; ``rvm_resize_u8`` writes the downsampled fp16 source directly, and
  ``rvm_dgf`` reads the uint8 frames again at full resolution for the guided filter + composite, whose
  uint8 output is the only full-resolution tensor;
* the MobileNetV3 stem is a direct conv kernel (K = 27); every other dense conv is the implicit-GEMM
  kernel with the activation (ReLU / hardswish) and the inverted-residual add fused into its epilogue
  and channel counts that are not multiples of 64 read in place (no padded copies);
* decoder inputs are written once by ``rvm_upcat`` (upsample + crop + concat + pad), the pooled source
  pyramid by one ``rvm_pool3`` pass;
* ConvGRU: the UpBlock conv output is updated IN PLACE by ``rvm_gru_out`` (no stack / cat), which also
  assembles the next time step's [x | h] input buffer.

Used for the downsampling case (ratio < 1, every 1080p clip); the PyTorch-op path in ``models/rvm.py``
stays the CPU reference and the small-input path.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..ops import _lib

_ACT = {None: 0, "relu": 1, "hs": 2}
_MODE = {"alpha-mask": 1, "foreground-mask": 2}


def _r8(v):
    return -(-v // 8) * 8


class FastMatting:
    def __init__(self, net, dtype=torch.float16):
        self.net = net
        self.dtype = dtype
        self._w: Dict[int, tuple] = {}
        dev = net.mean.device
        # stem: [co][ky][kx][ci] fp32 + bias + ImageNet normalisation (StemArgs in csrc/rvm.hip)
        stem = net.backbone.features[0].conv
        sw = stem.weight.detach().float().permute(0, 2, 3, 1).reshape(-1)
        sb = stem.bias.detach().float()
        mean = net.mean.detach().float().reshape(3)
        istd = 1.0 / net.std.detach().float().reshape(3)
        blob = torch.cat([sw, sb, mean, istd]).cpu().numpy().astype(np.float32).tobytes()
        assert len(blob) == _lib.rvm_args_size(0), "StemArgs layout"
        self.stem_blob = blob
        # guided filter + projection head (DgfArgs), kept on the device
        rf, pj = net.refiner, net.project
        parts = [pj.weight.reshape(4, 16), pj.bias, rf.c1.conv.weight.reshape(16, 24), rf.c1.conv.bias,
                 rf.c2.conv.weight.reshape(16, 16), rf.c2.conv.bias, rf.c3.weight.reshape(4, 16), rf.c3.bias]
        args = torch.cat([p.detach().float().reshape(-1) for p in parts])
        assert args.numel() * 4 == _lib.rvm_args_size(1), "DgfArgs layout"
        self.dgf_args = args.to(dev).contiguous()

    # ------------------------------------------------------------------ convs
    def _wpad(self, conv: nn.Conv2d):
        ent = self._w.get(id(conv))
        if ent is not None and ent[0] is conv.weight and ent[1] == conv.weight._version:
            return ent[2], ent[3]
        co, ci, k, _ = conv.weight.shape
        cp, cop = -(-ci // 64) * 64, _r8(co)
        w = torch.zeros(cop, k, k, cp, dtype=self.dtype, device=conv.weight.device)
        w[:co, :, :, :ci] = conv.weight.detach().permute(0, 2, 3, 1).to(self.dtype)
        b = torch.zeros(cop, dtype=self.dtype, device=conv.weight.device)
        if conv.bias is not None:
            b[:co] = conv.bias.detach().to(self.dtype)
        ops.derived_ready(w)
        self._w[id(conv)] = (conv.weight, conv.weight._version, w, b)
        return w, b

    def conv(self, x, conv: nn.Conv2d, act=None, residual=None):
        """NHWC conv (1x1 / 3x3, stride 1 / 2) + bias (+ residual) (+ activation) in one launch."""
        w, b = self._wpad(conv)
        k = conv.kernel_size[0]
        if x.shape[-1] % 8:
            x = F.pad(x, (0, _r8(x.shape[-1]) - x.shape[-1]))
        y = _lib.conv_ex(x, w, b, k, conv.stride[0], k // 2, _ACT[act], residual)
        co = conv.weight.shape[0]
        return y if y.shape[-1] == co else y[..., :co].contiguous()

    def convact(self, x, m, residual=None):
        c = m.conv
        if c.groups > 1 and c.groups == c.in_channels == c.out_channels:      # depthwise (HIP pass)
            y = ops.depthwise_conv(x.permute(0, 3, 1, 2), c.weight, c.bias, c.stride[0], c.dilation[0], m.act)
            return y.permute(0, 2, 3, 1)
        return self.conv(x, c, m.act, residual)

    # ------------------------------------------------------------------ encoder
    def _se(self, se, x):
        w = self.conv(self.conv(_lib.rvm_chan_mean(x), se.fc1, "relu"), se.fc2)   # [T, 1, 1, C]
        return _lib.rvm_gate(x, w.contiguous(), 0)                                 # x * hardsigmoid(w), in place

    def _block(self, blk, x):
        h = self.convact(x, blk.expand) if blk.expand is not None else x
        h = self.convact(h, blk.dw)
        if blk.se is not None:
            h = self._se(blk.se, h)
        return self.convact(h, blk.project, residual=x if blk.res else None)

    def encoder(self, small):
        f = self.net.backbone.features
        x = _lib.rvm_stem(small, self.stem_blob)
        x = self._block(f[1], x)
        f1 = x
        for i in range(2, 4):
            x = self._block(f[i], x)
        f2 = x
        for i in range(4, 7):
            x = self._block(f[i], x)
        f3 = x
        for i in range(7, 16):
            x = self._block(f[i], x)
        x = self.convact(x, f[16])
        return f1, f2, f3, x

    # ------------------------------------------------------------------ decoder
    def gru_inplace(self, gru, x, h):
        """ConvGRU over the time axis of x [T,H,W,C] on channels [C/2, C), updated IN PLACE; h [1,H,W,C/2]."""
        T, H, W, C = x.shape
        c = gru.c
        half = C - c
        if h is None:
            h = torch.zeros(1, H, W, c, dtype=x.dtype, device=x.device)
        buf = torch.empty(1, H, W, 2 * c, dtype=x.dtype, device=x.device)
        _lib.rvm_pack(buf, x[0], half, c, h, c)
        wi, bi = self._wpad(gru.ih)
        wh, bh = self._wpad(gru.hh)
        for t in range(T):
            ih = _lib.conv_ex(buf, wi, bi, 3, 1, 1)                     # [1,H,W,2c] (r | z)
            # z <- sigmoid(z part); buf[..., c:] <- sigmoid(r) * h  (the conv_hh input [x | r h])
            z = _lib.convgru_gates1(ih.permute(0, 3, 1, 2), h.permute(0, 3, 1, 2), buf.permute(0, 3, 1, 2),
                                    c).permute(0, 2, 3, 1)
            cc = _lib.conv_ex(buf, wh, bh, 3, 1, 1)                     # [1,H,W,r8(c)]
            nxt = t + 1 < T
            _lib.rvm_gru_out(cc, h, z, x[t], half, buf if nxt else None, x[t + 1] if nxt else None, half)
        return h

    def decoder(self, small, f1, f2, f3, f4, rec):
        dec = self.net.decoder
        s1, s2, s3 = _lib.rvm_pool3(small)
        r4 = self.gru_inplace(dec.decode4.gru, f4, rec[0])
        out = [r4]
        x = f4
        stages = ((dec.decode3, f3, s3, rec[1]), (dec.decode2, f2, s2, rec[2]), (dec.decode1, f1, s1, rec[3]))
        for ub, f, s, r in stages:
            cat = _lib.rvm_upcat(x, f, s, _r8(x.shape[-1] + f.shape[-1] + 3))
            x = self.conv(cat, ub.conv.conv, "relu")
            out.append(self.gru_inplace(ub.gru.gru, x, r))
        cat = _lib.rvm_upcat(x, None, small, _r8(x.shape[-1] + 3))
        hid = self.convact(self.convact(cat, dec.out0), dec.out1)
        return hid, out

    def __call__(self, frames_u8, rec, ratio: float, output_type: str, green):
        """frames uint8 [t,H,W,3] on the device -> composited uint8 [t,H,W,3] on the device, new state."""
        T, H, W, _ = frames_u8.shape
        h, w = int(round(H * ratio)), int(round(W * ratio))
        small = _lib.rvm_resize_u8(frames_u8, h, w)
        f1, f2, f3, f4 = self.encoder(small)
        asp = self.net.aspp
        a1 = self.convact(f4, asp.aspp1)
        g = self.conv(_lib.rvm_chan_mean(f4), asp.aspp2)
        f4 = _lib.rvm_gate(a1.contiguous(), g.contiguous(), 1)                     # a1 * sigmoid(g), in place
        hid, rec = self.decoder(small, f1, f2, f3, f4, rec)
        out = _lib.rvm_dgf(hid.contiguous(), small, self.dgf_args, frames_u8, _MODE.get(output_type, 0), green)
        return out, rec
