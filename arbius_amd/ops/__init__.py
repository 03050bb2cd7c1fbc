"""Fused operators of the inference engine.

Every op here has exactly one GPU implementation: a hand-written gfx950 HIP
kernel in ``csrc/`` (loaded from the in-tree ``libarbius_kernels.so`` through
``_lib``).  Shapes a kernel does not tile natively are zero-padded onto it
(channels, K, N: zeros add nothing to a dot product, so the bytes are those of
an exact-size kernel).  A GPU tensor never falls back to a ROCm library
(hipBLASLt / MIOpen): such a call would pick its reduction order by shape and
break the batch invariance of lock-step groups, so it raises
``LibraryFallback`` instead (``ARBIUS_LIBRARY_FALLBACK=1`` only counts it, in
``LIBRARY_CALLS`` - for experiments).  ``ops/audit.py`` runs every template's
legal operating points on the meta device through this module to prove no
shape reaches that path.  CPU tensors run the PyTorch reference in ``ref.py``
(the no-GPU plumbing config and the numerics oracle for tests).

On a GPU, a missing ``libarbius_kernels.so`` is a hard error (``_lib.lib()``
raises): there is no silent eager fallback.  ``ARBIUS_REFERENCE_OPS=1`` forces
the PyTorch reference on GPU tensors too; it exists only for A/B measurement
(bench.py --reference-ops) and parity tests.
"""
from __future__ import annotations

import collections
import math
import os
import threading
import weakref

import torch
import torch.nn.functional as F

from . import ref
from . import _lib

_FORCE_REF = os.environ.get("ARBIUS_REFERENCE_OPS", "0") == "1"
# GroupNorm-table prologue fused into the conv operand load (1) or applied by a separate
# elementwise kernel in front of the LDS-DMA conv variant (0, default: measured 9098 vs 7925
# tasks/h on SD1.5 512^2 - the register-staged kernel that can take the prologue is slower than
# the LDS-DMA one by more than the extra elementwise pass costs).
# "1": every GN consumer takes the table as an operand prologue; "1x1": only 1x1 convs / linears
# (no tap re-reads of the same activation, so the prologue costs no more VALU than the separate pass)
_NORM_PROLOGUE_MODE = os.environ.get("ARBIUS_NORM_PROLOGUE", "0")
_NORM_PROLOGUE = _NORM_PROLOGUE_MODE == "1"


def _norm_prologue(w) -> bool:
    return _NORM_PROLOGUE or (_NORM_PROLOGUE_MODE == "1x1" and w.shape[1] == 1 and w.shape[2] == 1)

# GPU tensors never reach a library convolution (LibraryFallback above); these flags only matter for
# the ARBIUS_LIBRARY_FALLBACK=1 A/B runs, where MIOpen must at least pick the same solver every call.
torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False


def reference_ops() -> bool:
    """True when every op runs its fp32 PyTorch reference (A/B runs, CPU)."""
    return _FORCE_REF


def set_reference_ops(flag: bool) -> None:
    global _FORCE_REF
    _FORCE_REF = bool(flag)


# ------------------------------------------------------------------ batch-invariant planning
# Consensus needs a task's bytes to be independent of which other tasks share its launches.
# Inside ``plan_batch(unit)`` every conv / GEMM plan (tile config + split-K) is chosen for the
# ``unit``-sample shape even when the tensor holds k*unit samples (lock-step task groups), and
# plain linears run on the implicit-GEMM kernel too (a library GEMM picks its algorithm - and
# so its k-reduction order - by M).  Per-element arithmetic then depends only on the unit
# shape: a group of tasks reproduces every solo task's output bit for bit.  Thread-local, so
# concurrent pipeline forks on other threads keep their own scope.
_TL = threading.local()


class plan_batch:
    def __init__(self, unit: int):
        self.unit = int(unit)

    def __enter__(self):
        self.prev = getattr(_TL, "pb", None)
        _TL.pb = self.unit
        return self

    def __exit__(self, *exc):
        _TL.pb = self.prev


# The canonical batch whose plans every batch-invariant launch uses (a multiple of the unit).
# 2 = a solo task's own plans; 8 = plans tuned for lock-step groups of 4 (bench default),
# which a solo task then also runs (same bits, slightly less fill on its own).
PLAN_CANON = int(os.environ.get("ARBIUS_PLAN_CANON", "8"))


def _canon_batch(batch: int):
    pb = getattr(_TL, "pb", None)
    if not pb or batch % pb:
        return None
    return max(PLAN_CANON, pb) // pb * pb


def _plan_rows(x) -> int:
    """Rows of x [batch, ..., C] at the canonical batch (the actual rows outside ``plan_batch``):
    every size-dependent kernel choice (LayerNorm variant, LN fold) is made on this, so a lock-step
    group makes each of its tasks' solo choices."""
    rows = x.numel() // x.shape[-1]
    canon = _canon_batch(x.shape[0])
    return rows // x.shape[0] * canon if canon else rows


def _hip(t: torch.Tensor) -> bool:
    return (t.is_cuda or (t.device.type == "meta" and _lib.auditing())) and not _FORCE_REF


class LibraryFallback(RuntimeError):
    """A GPU tensor reached a shape no HIP kernel (or padded form of one) serves."""


_ALLOW_LIBRARY = os.environ.get("ARBIUS_LIBRARY_FALLBACK", "0") == "1"
LIBRARY_CALLS = collections.Counter()     # op -> library calls made on GPU tensors (only when allowed)


def _library(op: str, detail: str) -> None:
    """Gate of every library-call branch on GPU tensors (see the module docstring)."""
    if not _ALLOW_LIBRARY:
        raise LibraryFallback(f"{op}: no HIP kernel for {detail}; GPU tensors never take a library fallback")
    LIBRARY_CALLS[op] += 1


# ------------------------------------------------------------------ derived-weight caches
def derived_ready(t) -> None:
    """Call before publishing a derived-weight cache entry (LN fold, GEGLU interleave, padded conv
    weights, ...) computed from ``t``'s device on the calling thread's stream.  Pipeline forks share
    these caches across threads and HIP streams; nothing would order another stream's first consumer
    after the producing kernels, so the entry is published only once they have finished.  A miss
    inside a hipGraph capture is refused: the tensors would be written only when the graph replays
    (every graph warms its ops eagerly before capturing)."""
    if t is None or not t.is_cuda:
        return
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("derived-weight cache miss inside a hipGraph capture (warm the op eagerly first)")
    torch.cuda.current_stream(t.device).synchronize()


# --------------------------------------------------------------------------- GEMM / conv
def _act_ref(y, act):
    if act == "gelu":
        return F.gelu(y)
    if act == "quick_gelu":
        return y * torch.sigmoid(1.702 * y)
    return y


def linear(x, w, b=None, residual=None, act=None):
    """y = act(x @ w^T + b (+ residual)), act None / "gelu" / "quick_gelu" (fused into the GPU epilogue).

    GPU: every linear whose K % 64 == 0 and N % 8 == 0 runs on the implicit-GEMM kernel (bias and
    residual fused into its epilogue, pinned plans - so a task's bytes never depend on which
    library algorithm a GEMM picks).  Library GEMMs (hipBLASLt) only for the other shapes: its
    stream-K kernels spin on other workgroups of their own launch, and two of them replayed
    concurrently on the two task streams of a GPU deadlocked (zeroscope, 2 streams)."""
    if _hip(x) and _gemm_ok(x.shape[-1], w.shape[0]):
        return _lib.gemm(x, w, b, residual, plan_batch=(x.shape[0], _canon_batch(x.shape[0])), act=act)
    if _hip(x):
        if x.dtype != torch.bfloat16:
            _library("linear", f"dtype {x.dtype} x {tuple(x.shape)} w {tuple(w.shape)}")
        else:
            return _padded_linear(x, w, b, residual, act)
    if act is not None:
        return _act_ref(linear(x, w, b, residual), act)
    if residual is not None:
        x2 = x.reshape(-1, x.shape[-1])
        r2 = residual.reshape(-1, w.shape[0])
        y = torch.addmm(r2, x2, w.t())
        if b is not None:
            y = y.add_(b)
        return y.reshape(*x.shape[:-1], w.shape[0])
    return F.linear(x, w, b)


_PAD_LIN = {}


def _padded_linear(x, w, b, residual, act):
    """A bf16 linear whose K (in) % 64 or N (out) % 8 the implicit-GEMM kernel does not tile: zero
    columns of x / w up to K % 64 == 0 (products of zeros add nothing: the exact-K dot product),
    zero rows of w / b up to N % 8 == 0, sliced off the output.  Padded weights are cached per live
    weight (``derived_ready``)."""
    N, K = w.shape
    Kp, Np = -(-K // 64) * 64, -(-N // 8) * 8
    key = (id(w), None if b is None else id(b))
    stamp = (w.data_ptr(), w._version, None if b is None else (b.data_ptr(), b._version))
    ent = _PAD_LIN.get(key)
    if ent is None or ent[0]() is not w or ent[1] != stamp:
        wp = torch.zeros(Np, Kp, dtype=w.dtype, device=w.device)
        wp[:N, :K] = w
        bp = None
        if b is not None:
            bp = torch.zeros(Np, dtype=b.dtype, device=b.device)
            bp[:N] = b
        derived_ready(wp)
        ent = (weakref.ref(w), stamp, wp, bp)
        _PAD_LIN[key] = ent
    wp, bp = ent[2], ent[3]
    xp = F.pad(x, (0, Kp - K)) if Kp != K else x
    if Np != N:
        y = _lib.gemm(xp, wp, bp, None, plan_batch=(x.shape[0], _canon_batch(x.shape[0])))[..., :N]
        if residual is not None:
            y = y + residual
        return _act_ref(y, act).contiguous()
    return _lib.gemm(xp, wp, bp, residual, plan_batch=(x.shape[0], _canon_batch(x.shape[0])), act=act)


_GEGLU_FUSED = os.environ.get("ARBIUS_GEGLU_FUSED", "1") != "0"   # A/B switch (same numerics)
_GEGLU_W = {}   # id(weight) -> (weakref(weight), weakref(bias), interleaved w, interleaved b)


def linear_geglu(x, w, b=None):
    """GEGLU feed-forward projection: value * gelu(gate) of (x @ w^T + b) split in halves.

    GPU: one implicit-GEMM launch with the GEGLU in its epilogue (the [M, 2F] pre-activation
    never reaches HBM; no separate geglu pass).  The projection rows are interleaved once into
    [value 8 | gate 8] blocks so every output tile holds matching value / gate channels."""
    if (_GEGLU_FUSED and _hip(x) and _gemm_ok(x.shape[-1], w.shape[0]) and w.shape[0] % 16 == 0
            and x.dtype == torch.bfloat16):
        ent = _GEGLU_W.get(id(w))
        stamp = (w.data_ptr(), w._version, None if b is None else (b.data_ptr(), b._version))
        if ent is None or ent[0]() is not w or (b is not None and ent[1]() is not b) or ent[4] != stamp:
            wi = _lib.interleave_geglu(w.detach())
            bi = _lib.interleave_geglu(b.detach()) if b is not None else None
            ent = (weakref.ref(w), weakref.ref(b) if b is not None else (lambda: None), wi, bi, stamp)
            derived_ready(wi)
            _GEGLU_W[id(w)] = ent
        return _lib.gemm_geglu(x, ent[2], ent[3], plan_batch=(x.shape[0], _canon_batch(x.shape[0])))
    return geglu(linear(x, w, b))


_LN_FOLD = {}   # (id(ln weight), id(linear weight), geglu) -> folded tensors (weakly keyed, version-stamped)


def ln_fold(gamma, beta, w, b, geglu=False):
    """Fold LayerNorm(gamma, beta) into the following linear (w [N, K], b [N] or None):
    LN(x) w^T + b = rstd (x W'^T - mean wsum) + b' with W' = bf16(w * gamma) (per column k),
    wsum[n] = sum_k W'[n, k] (fp32, of the rounded W' - so the mean term cancels exactly as the
    GEMM sees it) and b' = bf16(b + w beta).  ``geglu``: rows interleaved for the GEGLU epilogue.
    Cached per live (gamma, w) pair; recomputed when either changes."""
    key = (id(gamma), id(w), bool(geglu))
    stamp = (gamma.data_ptr(), gamma._version, beta.data_ptr(), beta._version, w.data_ptr(), w._version,
             None if b is None else (b.data_ptr(), b._version))
    ent = _LN_FOLD.get(key)
    if ent is not None and ent[0]() is gamma and ent[1]() is w and ent[2] == stamp:
        return ent[3]
    with torch.no_grad():
        wf = (w.float() * gamma.float()[None, :]).to(w.dtype)
        wsum = wf.double().sum(dim=1).float()
        bf = w.double() @ beta.double()
        if b is not None:
            bf = bf + b.double()
        bf = bf.to(w.dtype)
        if geglu:
            wf, bf = _lib.interleave_geglu(wf), _lib.interleave_geglu(bf)
            wsum = _lib.interleave_geglu(wsum)
        out = (wf.contiguous(), bf.contiguous(), wsum.contiguous())
    derived_ready(out[0])
    _LN_FOLD[key] = (weakref.ref(gamma), weakref.ref(w), stamp, out)
    return out


# Rows up to which the LayerNorm fold pays: it replaces the LN pass (read + write x) by a row-stats
# pass (read x) but adds ~2 FMAs + the weight-sum loads per output element to the GEMM epilogue.
# Measured per call on MI355X (r3, eager): text encoders / prior / UNet level 2 (<= 2048 rows) win
# (CLIP [2,77,768]: 21 vs 27 us), the 8k-32k-row level-0/1 projections lose (GEGLU [32768, 320 ->
# 2560]: 159 + 13 vs 137 + 17 us) - the epilogue of those short-K GEMMs is already their bottleneck.
LN_FOLD_MAX_ROWS = 2048
# Narrow consumers (N <= LN_FOLD_NARROW_N: the attention Q / QKV projections) fold at any row count when
# ARB_LN_FOLD_NARROW=1: their epilogues are small next to the LN pass they replace (A/B switch).
LN_FOLD_NARROW_N = int(os.environ.get("ARB_LN_FOLD_NARROW_N", "1920"))
_LN_FOLD_NARROW = os.environ.get("ARB_LN_FOLD_NARROW", "0") == "1"


def _ln_fold_ok(x, w, geglu):
    rows_ok = _plan_rows(x) <= LN_FOLD_MAX_ROWS or (_LN_FOLD_NARROW and not geglu and w.shape[0] <= LN_FOLD_NARROW_N)
    return (_hip(x) and x.dtype == torch.bfloat16 and _gemm_ok(x.shape[-1], w.shape[0]) and x.shape[-1] <= 2048
            and rows_ok and (not geglu or w.shape[0] % 16 == 0) and "lnfold" not in _EXP_SKIP)


def ln_linear(x, gamma, beta, eps, w, b=None, residual=None, act=None):
    """act(linear(LayerNorm(x))) - on the GPU the LayerNorm is folded into the GEMM's epilogue (one
    row-stats pass over x, no normalised tensor in HBM), the activation too."""
    if _ln_fold_ok(x, w, False):
        wf, bf, wsum = ln_fold(gamma, beta, w, b)
        rs = _lib.row_stats(x, eps, _plan_rows(x))
        return _lib.gemm_ln(x, wf, bf, wsum, rs, residual, plan_batch=(x.shape[0], _canon_batch(x.shape[0])),
                            act=act)
    return linear(layer_norm(x, gamma, beta, eps), w, b, residual, act=act)


def ln_linear_geglu(x, gamma, beta, eps, w, b=None):
    """linear_geglu(LayerNorm(x)) with the LayerNorm folded in (see ``ln_linear``)."""
    if _GEGLU_FUSED and _ln_fold_ok(x, w, True):
        wf, bf, wsum = ln_fold(gamma, beta, w, b, geglu=True)
        rs = _lib.row_stats(x, eps, _plan_rows(x))
        return _lib.gemm_ln(x, wf, bf, wsum, rs, geglu=True, plan_batch=(x.shape[0], _canon_batch(x.shape[0])))
    return linear_geglu(layer_norm(x, gamma, beta, eps), w, b)


class CatPair:
    """The channel concat [a | b] of two channels-last tensors, NOT materialised: the UNet up-path
    skip connection.  Its consumers (GroupNorm statistics, the GroupNorm table-apply pass and the
    ResBlock shortcut conv) read both parts in place on the GPU, with bytes identical to reading the
    concatenated tensor; anything else calls ``materialize()``."""
    __slots__ = ("a", "b", "shape", "dtype", "device")

    def __init__(self, a, b):
        self.a, self.b = a, b
        self.shape = tuple(a.shape[:-1]) + (a.shape[-1] + b.shape[-1],)
        self.dtype, self.device = a.dtype, a.device

    @property
    def is_cuda(self):
        return self.a.is_cuda

    def dim(self):
        return len(self.shape)

    def materialize(self):
        return torch.cat([self.a, self.b], dim=-1)


def cat_channels(a, b):
    """[a | b] along the channel (last) dim: a lazy ``CatPair`` where the GPU kernels can read it in
    place (bf16, a's channels % 64 == 0), else ``torch.cat``."""
    if (_hip(a) and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.shape[:-1] == b.shape[:-1]
            and a.shape[-1] % 64 == 0 and b.shape[-1] % 8 == 0 and a.is_contiguous() and b.is_contiguous()):
        return CatPair(a, b)
    return torch.cat([a, b], dim=-1)


def materialize(x):
    return x.materialize() if isinstance(x, CatPair) else x


class NormSpec:
    """A GroupNorm(+scale-shift modulation)(+SiLU) of ``x`` to be applied to a consumer's operand.
    Iterating the spec yields ``(table, silu)`` with the affine table computed lazily, so a consumer
    that never needs it (CPU reference paths) never launches the stats kernels.  A fused
    table-and-apply pass that rebuilt each image's table per block measured slower than
    stats + table + table-apply (e.g. 39.8 vs 26.6 us at [8, 4096, 320]: the per-block rebuild
    serialises one partials round trip per group), so the consumer applies the table."""
    __slots__ = ("x", "gamma", "beta", "groups", "eps", "mod", "one_plus", "silu", "_table")

    def __init__(self, x, gamma, beta, groups, eps, mod=None, one_plus=0.0, silu=False):
        self.x, self.gamma, self.beta, self.groups, self.eps = x, gamma, beta, groups, eps
        self.mod, self.one_plus, self.silu, self._table = mod, one_plus, silu, None

    def slice_ok(self):
        """Whether this GroupNorm runs as ONE launch producing the transformed tensor
        (``_lib.group_norm_slice``: small (group, image) slices; chosen by shape only)."""
        x = self.x
        a, b = (x.a, x.b) if isinstance(x, CatPair) else (x, None)
        return (_hip(a) and a.dtype == torch.bfloat16 and "gnstats" not in _EXP_SKIP and "gnapply" not in _EXP_SKIP
                and _lib.group_norm_slice_ok(a, self.groups, b))

    def applied(self):
        """The transformed tensor (GN [+ modulation] [+ SiLU]) in one launch - see ``slice_ok``."""
        x = self.x
        a, b = (x.a, x.b) if isinstance(x, CatPair) else (x, None)
        return _lib.group_norm_slice(a, self.gamma, self.beta, self.groups, self.eps, self.mod, self.one_plus,
                                     self.silu, x2=b)

    def table(self):
        if self._table is None:
            self._table = group_norm_table(self.x, self.gamma, self.beta, self.groups, self.eps, self.mod,
                                           self.one_plus)
        return self._table

    def __iter__(self):
        yield self.table()
        yield self.silu


def _gemm_ok(K, N):
    return K % 64 == 0 and N % 8 == 0


def conv2d(x, w, b=None, stride=1, padding=1, upsample=False, residual=None, temb=None, norm=None):
    """Channels-last conv. x [B,H,W,Cin], w [Cout,kh,kw,Cin]; fused epilogue
    (+bias, +temb[b, n] per-batch bias, +residual); ``norm = (table, silu)`` applies a
    GroupNorm(+SiLU) prologue from ``group_norm_table`` inside the conv's operand load."""
    kern_ok = (w.shape[1] in (1, 3) and w.shape[1] == w.shape[2]) or tuple(w.shape[1:3]) == (3, 1)
    if (isinstance(norm, NormSpec) and kern_ok and not _norm_prologue(w) and w.shape[0] % 8 == 0
            and x.shape[-1] % 64 == 0 and norm.slice_ok()):
        # small slices: statistics, table and transform in one launch instead of three
        x, norm = norm.applied().view(tuple(x.shape)), None
    if isinstance(x, CatPair):
        if (norm is not None and _hip(x.a) and not _norm_prologue(w) and kern_ok and x.shape[-1] % 64 == 0
                and w.shape[0] % 8 == 0 and "gnapply" not in _EXP_SKIP):
            table, nsilu = norm
            x, norm = _lib.norm_table_apply(x.a, table, nsilu, x2=x.b), None     # reads both parts in place
        elif norm is None and _hip(x.a) and kern_ok and x.shape[-1] % 64 == 0 and w.shape[0] % 8 == 0:
            return _lib.conv2d_nhwc(x.a, w, b, padding, upsample, residual, temb, stride, x2=x.b,
                                    plan_b=_canon_batch(x.shape[0]))
        else:
            x = x.materialize()
    if _hip(x) and kern_ok:
        table, nsilu = norm if norm is not None else (None, False)
        if table is not None and not _norm_prologue(w) and x.shape[-1] % 8 == 0:
            if "gnapply" in _EXP_SKIP:
                table, nsilu = None, False
            else:
                x, table, nsilu = _lib.norm_table_apply(x, table, nsilu), None, False
        if x.shape[-1] % 64 == 0 and w.shape[0] % 8 == 0:
            return _lib.conv2d_nhwc(x, w, b, padding, upsample, residual, temb, stride, norm=table,
                                    norm_silu=nsilu, plan_b=_canon_batch(x.shape[0]))
        if table is None or x.shape[-1] % 64 == 0:
            # channel counts the kernel does not tile (3/4-channel conv_in / conv_out / SpatialNorm
            # maps, MobileNet widths 16..960): zero-pad channels onto the MFMA kernel (some wasted
            # FLOPs) instead of a library fallback - MIOpen's deterministic mode picks its naive
            # direct kernel for these shapes (1.1 ms per RVM conv: profiles/rocprof_r1_v11_rvm.md).
            return _padded_conv(x, w, b, padding, upsample, residual, temb, stride, table, nsilu)
    if _hip(x):
        _library("conv2d", f"x {tuple(x.shape)} w {tuple(w.shape)} stride {stride}")
    if norm is not None:
        x = apply_norm_table(x, *norm)
    if x.is_cuda:
        # MIOpen NHWC path (only with ARBIUS_LIBRARY_FALLBACK=1).  A permuted view of a contiguous
        # NHWC tensor is an NCHW tensor in channels_last memory format (no copy).
        xc = x.permute(0, 3, 1, 2)
        if upsample:
            xc = F.interpolate(xc, scale_factor=2.0, mode="nearest")
        pad = (padding, 0) if w.shape[1] != w.shape[2] else padding
        y = F.conv2d(xc, w.permute(0, 3, 1, 2), b, stride=stride, padding=pad)
        y = y.permute(0, 2, 3, 1)
        if not y.is_contiguous():
            y = y.contiguous()
    else:
        y = ref.conv2d_nhwc(x, w, b, stride, padding, upsample)
    if temb is not None:
        y = y + temb[:, None, None, :].to(y.dtype)
    if residual is not None:
        y = y + residual
    return y


_PAD_W = {}


def _padded_weights(w, b):
    """Channel-padded copies of a conv's weight/bias, cached per live weight: the entry holds weak
    references to the owning tensors (a view's base) and is reused only while they are alive and
    unmodified - a freed tensor's address can come back as another weight of another dtype."""
    import weakref

    def owner(t):
        return t if t._base is None else t._base

    key = (w.data_ptr(), w._version, tuple(w.shape), tuple(w.stride()), w.dtype,
           None if b is None else (b.data_ptr(), b._version))
    hit = _PAD_W.get(key)
    if hit is not None and hit[0]() is owner(w) and (b is None or hit[1]() is owner(b)):
        return hit[2], hit[3]
    cout, kh, kw, cin = w.shape
    ci, co = -(-cin // 64) * 64, -(-cout // 8) * 8
    wp = torch.zeros(co, kh, kw, ci, dtype=w.dtype, device=w.device)
    wp[:cout, :, :, :cin] = w
    bp = None
    if b is not None:
        bp = torch.zeros(co, dtype=b.dtype, device=b.device)
        bp[:cout] = b
    derived_ready(wp)
    _PAD_W[key] = (weakref.ref(owner(w)), None if b is None else weakref.ref(owner(b)), wp, bp)
    return wp, bp


def _padded_conv(x, w, b, padding, upsample, residual, temb, stride, table=None, nsilu=False):
    cout, cin = w.shape[0], w.shape[-1]
    wp, bp = _padded_weights(w, b)
    if wp.shape[-1] != cin:
        x = F.pad(x, (0, wp.shape[-1] - cin))
    if wp.shape[0] != cout:
        y = _lib.conv2d_nhwc(x, wp, bp, padding, upsample, None, None, stride, norm=table,
                             norm_silu=nsilu, plan_b=_canon_batch(x.shape[0]))[..., :cout]
        if temb is not None:
            y = y + temb[:, None, None, :].to(y.dtype)
        if residual is not None:
            y = y + residual
        return y.contiguous()
    return _lib.conv2d_nhwc(x, wp, bp, padding, upsample, residual, temb, stride, norm=table, norm_silu=nsilu,
                            plan_b=_canon_batch(x.shape[0]))


_DW_W = {}


def depthwise_conv(x, weight, bias, stride=1, dilation=1, act=None):
    """Depthwise k x k conv (+ bias + ReLU / hardswish), NCHW (channels_last on the GPU).
    GPU fp16: one HIP pass (csrc/depthwise.hip) with the weight transposed once to [k*k, C];
    otherwise the PyTorch reference."""
    C, _, k, _ = weight.shape
    if (_hip(x) and x.dtype == torch.float16 and k in (3, 5) and C % 8 == 0 and stride in (1, 2)
            and x.is_contiguous(memory_format=torch.channels_last)):
        stamp = (weight.data_ptr(), weight._version)
        ent = _DW_W.get(id(weight))
        if ent is None or ent[0]() is not weight or ent[1] != stamp:
            ent = (weakref.ref(weight), stamp, weight.detach().reshape(C, k * k).t().contiguous())
            derived_ready(ent[2])
            _DW_W[id(weight)] = ent
        return _lib.dwconv_f16(x, ent[2], bias, k, stride, dilation, act)
    if _hip(x):
        _library("depthwise_conv", f"x {tuple(x.shape)} {x.dtype} k {k} stride {stride}")
    y = F.conv2d(x, weight, bias, stride=stride, padding=dilation * (k // 2), dilation=dilation, groups=C)
    if act == "relu":
        return F.relu(y)
    if act == "hs":
        return F.hardswish(y)
    return y


# --------------------------------------------------------------------------- normalisation
_EXP_SKIP = os.environ.get("ARBIUS_EXPERIMENT_SKIP", "")   # sensitivity experiments only (wrong outputs)
_EXP_TABLES = {}


def group_norm_table(x, gamma, beta, groups, eps, mod=None, one_plus=0.0):
    """GroupNorm of x as a per-(batch, channel) affine table [B, C, 2] fp32 (scale, shift) for a
    consumer prologue (conv/GEMM); ``mod`` [B, 2C] folds the GLIDE scale-shift modulation
    (out = GN(x) * (mod[:, :C] + one_plus) + mod[:, C:])."""
    if isinstance(x, CatPair):
        if _hip(x.a) and "gnstats" not in _EXP_SKIP:
            return _lib.group_norm_table(x.a, gamma, beta, groups, eps, mod, one_plus, x2=x.b)
        x = x.materialize()
    if _hip(x):
        if "gnstats" in _EXP_SKIP:
            key = (x.shape[0], x.shape[-1])
            if key not in _EXP_TABLES:
                _EXP_TABLES[key] = torch.ones(x.shape[0], x.shape[-1], 2, device=x.device)
            return _EXP_TABLES[key]
        return _lib.group_norm_table(x, gamma, beta, groups, eps, mod, one_plus)
    return ref.group_norm_table(x, gamma, beta, groups, eps, mod, one_plus)


def apply_norm_table(x, table, silu=False):
    """x * scale + shift (+SiLU) per (batch, channel) - the unfused form of a norm prologue."""
    if _hip(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0:
        return _lib.norm_table_apply(x, table, silu)
    B, C = x.shape[0], x.shape[-1]
    shape = (B,) + (1,) * (x.dim() - 2) + (C,)
    y = x.float() * table[..., 0].reshape(shape) + table[..., 1].reshape(shape)
    if silu:
        y = F.silu(y)
    return y.to(x.dtype)
def pool2(x, norm=None):
    """2x2 average pool of x (channels-last [B, H, W, C]) and, with ``norm`` (a ``NormSpec`` /
    ``(table, silu)``), of its GroupNorm(+SiLU) in the same pass: returns (pool(norm(x)), pool(x))
    (the first is None without ``norm``).  The GLIDE down-sampling ResBlock: both branches pool.
    The normalised values round to bf16 before pooling, as the unfused norm-then-pool would."""
    x = materialize(x)
    table, silu = norm if norm is not None else (None, False)
    if _hip(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0 and x.shape[1] % 2 == 0 and x.shape[2] % 2 == 0:
        return _lib.norm_pool2(x, table, silu)

    def pool(t):
        B, H, W, C = t.shape
        v = t.float().view(B, H // 2, 2, W // 2, 2, C)
        return (((v[:, :, 0, :, 0] + v[:, :, 0, :, 1]) + (v[:, :, 1, :, 0] + v[:, :, 1, :, 1])) * 0.25).to(t.dtype)
    return (pool(apply_norm_table(x, table, silu)) if table is not None else None), pool(x)


def upsample2(x):
    """Nearest 2x up-sampling of a channels-last tensor (one HIP pass on the GPU)."""
    x = materialize(x)
    if _hip(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0:
        return _lib.upsample2(x)
    return x.repeat_interleave(2, dim=1).repeat_interleave(2, dim=2)


def group_norm(x, gamma, beta, groups, eps, silu=False):
    if _hip(x):
        return _lib.group_norm_nhwc(x, gamma, beta, groups, eps, silu)
    return ref.group_norm_nhwc(x, gamma, beta, groups, eps, silu)


def spatial_norm(x, yb, gamma, beta, groups, eps, silu=False):
    """MoVQ SpatialNorm: GN(x) * y + b with ``yb`` = [y | b] [B, mh, mw, 2C] at a lower
    (nearest-upsampled) resolution; one fused HIP pass after the GN statistics."""
    if _hip(x):
        return _lib.group_norm_mod_nhwc(x, gamma, beta, groups, eps, silu, yb, 0.0)
    return ref.group_norm_mod_nhwc(x, gamma, beta, groups, eps, silu, yb, 0.0)


def scale_shift_norm(x, ss, gamma, beta, groups, eps, silu=True):
    """GLIDE ResBlock norm: GN(x) * (1 + scale) + shift (+ SiLU), ``ss`` = [scale | shift] [B, 2C]."""
    mod = ss.reshape(ss.shape[0], 1, 1, ss.shape[-1])
    if _hip(x):
        return _lib.group_norm_mod_nhwc(x, gamma, beta, groups, eps, silu, mod, 1.0)
    return ref.group_norm_mod_nhwc(x, gamma, beta, groups, eps, silu, mod, 1.0)


def layer_norm(x, gamma, beta, eps):
    if _hip(x):
        return _lib.layer_norm(x, gamma, beta, eps, _plan_rows(x))
    return ref.layer_norm(x, gamma, beta, eps)


# --------------------------------------------------------------------------- attention
def attention(q, k, v, scale=None, causal=False, kv_prefix=None):
    """q [B,Nq,H,D], k/v [B,Nk,H,D] (last dim contiguous) -> [B,Nq,H,D].
    ``kv_prefix = (kp, vp)``: extra keys/values placed AHEAD of k/v (joint attention over
    context + spatial tokens) read in place by the kernel - no concatenated copy."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    if _hip(q):
        return _lib.flash_attention(q, k, v, scale, causal, kv_prefix)
    if kv_prefix is not None:
        k, v = torch.cat([kv_prefix[0], k], 1), torch.cat([kv_prefix[1], v], 1)
    return ref.attention(q, k, v, scale, causal)


def temporal_attention(q, k, v, scale=None):
    """Frame-axis attention, q/k/v [B, F, P, H, D] strided views of the frame-major
    activation (P = pixels): one MFMA wave per (b, p, h) problem (HIP)."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    if _hip(q):
        B, F_, P, H, D = q.shape
        if F_ <= TEMPORAL_MAX_FRAMES:
            return _lib.temporal_attention(q, k, v, scale)
        # longer clips (damo: num_frames up to 500): the frame axis no longer fits one wave's
        # registers - gather (video, pixel) problems into the flash kernel's [batch, seq, head, d]
        # layout (one copy each way; the UNet3D's common frame counts never take this path)
        def gather(t):
            return t.permute(0, 2, 1, 3, 4).reshape(B * P, F_, H, D).contiguous()
        o = _lib.flash_attention(gather(q), gather(k), gather(v), scale, False)
        return o.view(B, P, F_, H, D).permute(0, 2, 1, 3, 4).contiguous()
    return ref.temporal_attention(q, k, v, scale)


TEMPORAL_MAX_FRAMES = 96     # csrc/temporal_attention.hip keeps <= 96 frames in registers


# --------------------------------------------------------------------------- ConvGRU
def convgru_gates1(ih, h, cat_buf, cx):
    """RVM ConvGRU: [r|z] = sigmoid(ih); z returned, r*h written into cat_buf[:, cx:] (fp16 HIP)."""
    if _hip(ih):
        return _lib.convgru_gates1(ih, h, cat_buf, cx)
    return ref.convgru_gates1(ih, h, cat_buf, cx)


def convgru_gates2(c, h, z):
    """RVM ConvGRU state update h' = (1-z) h + z tanh(c) (fp16 HIP)."""
    if _hip(c):
        return _lib.convgru_gates2(c, h, z)
    return ref.convgru_gates2(c, h, z)


# --------------------------------------------------------------------------- elementwise
def geglu(h):
    if _hip(h):
        return _lib.geglu(h)
    return ref.geglu(h)


def silu(x):
    if _hip(x):
        return _lib.silu(x)
    return ref.silu(x)


# --------------------------------------------------------------------------- sampler
def sampler_step(tasks):
    """Fused CFG + diffusion-sampler update of a lock-step group (models/schedulers.py)."""
    if _hip(tasks[0]["x"]):
        return _lib.sampler_step(tasks)
    return ref.sampler_step(tasks)


def native_loaded() -> bool:
    """True when the HIP kernel library is loaded in this process."""
    return _lib.loaded()


def rgb_to_yuv420(x, out=None):
    """uint8 RGB frames [T, H, W, 3] -> the H.264 encoder's macroblock-padded BT.601 4:2:0 planes
    (y [T, H16, W16], cb, cr [T, H16 / 2, W16 / 2]).  GPU: one HIP pass (``out``: optional device
    destination planes); CPU: the native host conversion (the same integer arithmetic, so the same
    samples)."""
    if _hip(x):
        return _lib.rgb_to_yuv420(x, out)
    if out is not None:
        raise ValueError("rgb_to_yuv420: out= is for GPU planes")
    from .. import native
    return tuple(torch.from_numpy(p) for p in native.rgb_to_yuv420_planes(x.contiguous().numpy()))


def h264_intra_encode(y, cb, cr, qp: int):
    """avc-intra slices of macroblock-padded 4:2:0 planes (csrc/h264_intra.hip): GPU uint8 planes ->
    (out, meta) device tensors, queued on the current stream (layout: native ``h264_nals_from_rbsp``);
    CPU numpy / tensors -> the same functions run on the host (numpy out, meta)."""
    if isinstance(y, torch.Tensor) and _hip(y):
        return _lib.h264_intra_encode(y, cb, cr, qp)
    as_np = [t.numpy() if isinstance(t, torch.Tensor) else t for t in (y, cb, cr)]
    return _lib.h264_intra_host(*as_np, qp)


def image_u8(x, mode: int):
    """Decoded image -> uint8 RGB: mode 0 KL-VAE round(clamp(x / 2 + 0.5, 0, 1) * 255), mode 1 MoVQ
    round(clamp((x + 1) * 127.5, 0, 255)).  GPU bf16: one HIP pass; otherwise the PyTorch chain."""
    if _hip(x) and x.dtype == torch.bfloat16:
        return _lib.image_u8(x, mode)
    x = x.float()
    v = (x / 2 + 0.5).clamp(0, 1) * 255 if mode == 0 else ((x + 1.0) * 127.5).clamp(0, 255)
    return v.round().to(torch.uint8)
