// Implicit-GEMM convolution / GEMM for gfx950 (bf16 in, fp32 accumulate, bf16 out).
//
// Channels-last:  out[m, n] = sum_k A[m, k] * W[n, k]   (+ bias[n] + temb[b(m), n] + residual[m, n])
//   m = (b, ho, wo) output pixel, n = output channel, k = (r, s, cin)
//   A[m, k] = x[b, hi, wi, cin]  gathered on the fly (zero padding, stride 1/2,
//   optional nearest-x2 upsample folded into the index: src = (hi>>1, wi>>1)).
// A 1x1 conv over H=1 is a plain linear layer, so this one kernel family serves
// every UNet / VAE conv AND can serve the transformer linears with fused epilogues.
//
// Mapping (SURVEY.md §2.6a "conv2d 3x3 implicit-GEMM on MFMA"):
//   * swapped product C^T = W X^T on mfma_f32_16x16x32_bf16: each lane ends with 4
//     CONSECUTIVE output channels of one pixel -> 8-byte epilogue stores / residual loads.
//   * 256 threads = 2x2 waves; block tile BN (channels) x BM (pixels) x BK=64.
//   * K tile of 64 always lies inside one (r, s) tap (Cin % 64 == 0), so every A chunk
//     is one 16-byte load of 8 contiguous channels of one input pixel.
//   * LDS rows of 128 B with XOR chunk swizzle (chunk ^ (row & 7)): the ds_read_b128
//     fragment reads are bank-conflict free (checked against the 16-lane groups of
//     MI355X_MICROARCH §LDS).
//   * register-staged double buffer (issue the next tile's global loads before the
//     MFMAs, write LDS after them), ONE barrier per K tile.
//   * XCD-aware bijective block remap: the N-tiles of one pixel tile share an L2.
//   * deterministic split-K for under-filled grids: fp32 slabs + an ordered reduce
//     kernel that applies the epilogue (no atomics -> bitwise reproducible).
#include "common.h"

#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <unordered_map>
#include <vector>

struct ConvArgs {
  const bf16_t* x;      // [B, H, W, Cin]
  const bf16_t* w;      // [N, K]
  const bf16_t* bias;   // [N] or null
  const bf16_t* temb;   // [B, N] (row stride temb_ld) or null (per-batch bias, e.g. ResBlock time embedding)
  const bf16_t* res;    // [M, N] or null
  bf16_t* out;          // [M, N]
  float* ws;            // split-K slabs [S, M, N]
  const float* norm;    // [B, Cin, 2] (scale, shift) GroupNorm prologue or null
  int norm_silu;
  int* counters;        // split-K tile tickets (in-launch reduction) or null
  int B, H, W, Cin;     // input (pre-upsample)
  int Hl, Wl;           // logical input dims (after upsample)
  int Ho, Wo;
  int N, K, M;
  int kw, pad, padw, stride, upsample;
  int ktiles, kt_per_split;
  int tiles_n, tiles_total;
  int nsplit, m_fastest;
  int geglu = 0;        // GEGLU epilogue: W rows interleaved [value 8 | gate 8] per 16; out [M, N/2]
  // LayerNorm folded into this GEMM (x is the RAW LN input, W = W_orig * gamma per column):
  //   out = rstd_m * (acc - mean_m * wsum_n) + bias' (+ ...),  rowstat[m] = (mean, rstd),
  //   wsum[n] = sum_k W[n, k] (fp32, of the bf16 folded weights), bias' = bias + W_orig beta.
  const float2* rowstat = nullptr;
  const float* wsum = nullptr;
  // Channel padding without a padded copy (register-staged kernels): x holds Cx channels per pixel
  // (row stride Cx, Cx % 8 == 0), the K walk runs over Cin = Cx rounded up to 64 per tap, chunks
  // at channel >= Cx read zeros; w is [N, kh, kw, Cin] zero-padded.  Cx == Cin otherwise.
  int Cx = 0;
  int act = 0;          // epilogue activation after bias / temb / residual: 1 ReLU, 2 hardswish
  // Two channel sources (a UNet skip concat read in place): channels [0, C1) from x (row stride
  // C1), [C1, Cin) from x2 (row stride Cin - C1); C1 % 64 == 0, so a K tile never straddles.
  // Register-staged kernel only.
  const bf16_t* x2 = nullptr;
  int C1 = 0;
  int temb_ld = 0;      // temb row stride in elements (a column slice of the batched projection: no copy)
};

// ---- element type: EL = 0 bf16 (the diffusion models), EL = 1 fp16 (robust video matting).
// Storage is raw 16-bit either way; only the MFMA flavour and the f32 <-> 16-bit conversions
// differ, so every tiling / schedule / reduction-order property holds for both.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <int EL>
__device__ __forceinline__ float dec16(uint32_t bits) {
  if constexpr (EL == 0) return __uint_as_float(bits << 16);
  else return (float)__builtin_bit_cast(_Float16, (uint16_t)bits);
}
template <int EL>
__device__ __forceinline__ uint32_t enc16(float v) {
  if constexpr (EL == 0) return (uint32_t)f2bf(v);
  else return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)v);
}
template <int EL>
__device__ __forceinline__ f32x4 mma16(uint4 a, uint4 b, f32x4 c) {
  if constexpr (EL == 0)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                  0, 0, 0);
}
// lo/hi 16-bit halves of a packed pair -> f32
template <int EL>
__device__ __forceinline__ float lo16(uint32_t w) { return dec16<EL>(w & 0xffffu); }
template <int EL>
__device__ __forceinline__ float hi16(uint32_t w) { return dec16<EL>(w >> 16); }
template <int EL>
__device__ __forceinline__ void unpack8e(uint4 v, float (&f)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) { f[2 * i] = lo16<EL>(w[i]); f[2 * i + 1] = hi16<EL>(w[i]); }
}
template <int EL>
__device__ __forceinline__ uint4 pack8e(const float (&f)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = enc16<EL>(f[2 * i]) | (enc16<EL>(f[2 * i + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// 64 zero bytes: the source of every masked 16-byte operand load (zero padding, rows past M,
// channels past N) - loads stay unconditional, so hipcc can count vmcnt instead of draining.
__device__ __attribute__((aligned(16))) uint4 g_conv_zero_page[4];

// 1-D grid of tiles_total * nsplit blocks -> (split, n-tile, m-tile), XCD-aware: consecutive
// logical ids share an XCD (L2).  When the weights outweigh the activations (small-M deep
// levels: a 1280x11520 conv weight is 29 MB) the m-tiles of one weight panel run together
// so the panel is fetched from HBM once per XCD instead of once per m-tile; otherwise the
// n-tiles of one activation panel do.
__device__ __forceinline__ void tile_coords(const ConvArgs& p, int BN, int BM, int& sp, int& n0, int& m0) {
  const int lin = xcd_remap(blockIdx.x, p.tiles_total * p.nsplit);
  const int tiles_m = p.tiles_total / p.tiles_n;
  if (p.m_fastest) {
    const int rest = lin / tiles_m;
    m0 = (lin % tiles_m) * BM;
    n0 = (rest % p.tiles_n) * BN;
    sp = rest / p.tiles_n;
  } else {
    const int rest = lin / p.tiles_n;
    n0 = (lin % p.tiles_n) * BN;
    m0 = (rest % tiles_m) * BM;
    sp = rest / tiles_m;
  }
}


// Epilogue activation (after bias / temb / residual): 1 ReLU, 2 hardswish (RVM, either dtype);
// 3 GELU(erf) and 4 quick-GELU x * sigmoid(1.702 x) (text towers / prior MLPs, bf16): the
// pre-activation is rounded to bf16 first and quick-GELU keeps the bf16 roundings of the unfused
// elementwise chain (h, 1.702 h, sigmoid) - the MLP hidden state never reaches HBM un-activated.
__device__ __forceinline__ float act_f(int act, float v) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return v * fminf(fmaxf(v + 3.f, 0.f), 6.f) * (1.f / 6.f);
  if (act == 3) return gelu_f(bf16_round(v));
  if (act == 4) {
    const float h = bf16_round(v), t = bf16_round(1.702f * h);
    return h * bf16_round(1.f / (1.f + __expf(-t)));
  }
  return v;
}

// LN fold (ConvArgs::rowstat): v[e] <- rstd * (v[e] - mean * wsum[n + e]) for 8 / 4 channels.
__device__ __forceinline__ void ln_fold8(const ConvArgs& p, int m, int n, float (&v)[8]) {
  const float2 rs = p.rowstat[m];
  const float4 w0 = *reinterpret_cast<const float4*>(p.wsum + n), w1 = *reinterpret_cast<const float4*>(p.wsum + n + 4);
  const float ws[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = rs.y * (v[e] - rs.x * ws[e]);
}
__device__ __forceinline__ void ln_fold4(const ConvArgs& p, int m, int n, float& v0, float& v1, float& v2,
                                         float& v3) {
  const float2 rs = p.rowstat[m];
  const float4 w = *reinterpret_cast<const float4*>(p.wsum + n);
  v0 = rs.y * (v0 - rs.x * w.x);
  v1 = rs.y * (v1 - rs.x * w.y);
  v2 = rs.y * (v2 - rs.x * w.z);
  v3 = rs.y * (v3 - rs.x * w.w);
}

// Largest row block whose fp32 staging fits LDSF floats: a multiple of 16 (an MFMA fragment block
// never straddles two row blocks) dividing BM, aligned with the wave rows.  (Halving BM = 192 gave
// 24-row blocks that cut fragments in two: rows 24..31 were staged past the block and never stored.)
template <int BM, int WMR, int OROW, int LDSF>
constexpr int epi_rows() {
  for (int r = BM; r >= 16; r -= 16)
    if (BM % r == 0 && r * OROW <= LDSF && (r % WMR == 0 || WMR % r == 0)) return r;
  return 16;
}

// Non-split epilogue through LDS.  The MFMA layout leaves each lane 4 channels of ONE pixel, so
// direct stores / residual loads touch 16 rows x 32 B per instruction.  Instead the fp32 tile
// is staged in LDS (row = pixel, in row blocks that fit) and re-read as 8-channel chunks along
// the rows: bias / temb / residual loads and the bf16 stores become contiguous 16-B accesses.
// Arithmetic is unchanged (fp32 acc + bias + temb + residual, one rounding), so results are
// bitwise those of the direct epilogue.  Call after the K loop; LDS is reused.
template <int BN, int BM, int WN, int WM, int NT, int LDSF, int EL>
__device__ __forceinline__ void epilogue_lds(const ConvArgs& p, const f32x4 (&acc)[BN / WN / 16][BM / WM / 16],
                                             float* stage, int m0, int n0) {
  constexpr int TN = BN / WN / 16, TM = BM / WM / 16;
  constexpr int OROW = BN + 4;           // floats per staged row (16-B pad: spreads the rows' banks)
  constexpr int PR = epi_rows<BM, BM / WM, OROW, LDSF>();
  static_assert(PR * OROW <= LDSF, "epilogue staging exceeds LDS");
  static_assert(PR % 16 == 0 && BM % PR == 0, "row blocks hold whole MFMA fragment blocks");
  static_assert(PR % (BM / WM) == 0 || (BM / WM) % PR == 0, "row blocks align with wave rows");
  constexpr int CPR = BN / 8;            // 8-channel chunks per row
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WM, wm = wave % WM, g = lane >> 4, l16 = lane & 15;
  const int hw = p.Ho * p.Wo;
#pragma unroll 1
  for (int r0 = 0; r0 < BM; r0 += PR) {
    __syncthreads();                     // K loop / previous block's readers are done with LDS
#pragma unroll
    for (int b = 0; b < TM; ++b) {
      const int rb = wm * (BM / WM) + b * 16;          // wave-uniform 16-row fragment block
      if (rb < r0 || rb >= r0 + PR) continue;
      const int rl = rb - r0 + l16;
#pragma unroll
      for (int a = 0; a < TN; ++a) {
        const int col = wn * (BN / WN) + a * 16 + 4 * g;
        *reinterpret_cast<f32x4*>(&stage[rl * OROW + col]) = acc[a][b];
      }
    }
    __syncthreads();
    if (p.geglu) {
      // value chunk ch, gate chunk ch + 8 -> 8 outputs at column n / 2; both halves rounded to
      // bf16 first (the unfused GEMM -> geglu path's numerics, bitwise)
      constexpr int PPR = BN / 16;
      const int NO = p.N >> 1;
      for (int c = tid; c < PR * PPR; c += NT) {
        const int rl = c / PPR, ch = (c - rl * PPR) * 16;
        const int m = m0 + r0 + rl, n = n0 + ch;
        if (m >= p.M || n >= p.N) continue;
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(&stage[rl * OROW + ch]);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(&stage[rl * OROW + ch + 4]);
        const f32x4 g0 = *reinterpret_cast<const f32x4*>(&stage[rl * OROW + ch + 8]);
        const f32x4 g1 = *reinterpret_cast<const f32x4*>(&stage[rl * OROW + ch + 12]);
        float va[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        float vg[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
        if (p.rowstat) {
          ln_fold8(p, m, n, va);
          ln_fold8(p, m, n + 8, vg);
        }
        if (p.bias) {
          float t[8];
          unpack8e<EL>(ld16(p.bias + n), t);
#pragma unroll
          for (int e = 0; e < 8; ++e) va[e] += t[e];
          unpack8e<EL>(ld16(p.bias + n + 8), t);
#pragma unroll
          for (int e = 0; e < 8; ++e) vg[e] += t[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) va[e] = dec16<EL>(enc16<EL>(va[e])) * gelu_f(dec16<EL>(enc16<EL>(vg[e])));
        st16(p.out + (size_t)m * NO + (n >> 1), pack8e<EL>(va));
      }
      continue;
    }
    // this thread's chunks of the row block: every residual load (the HBM-bound operand) is issued
    // before the first store (the compiler cannot hoist a later chunk's residual load above an
    // earlier chunk's store to out - they may alias), so the block's residual reads overlap instead
    // of running one chunk at a time; bias / temb stay in the loop (L2-hot, and registers: the
    // X-in-registers tiles keep their two blocks per CU).  Same arithmetic and order per element.
    constexpr int ITER = (PR * CPR + NT - 1) / NT;
    uint4 rr[ITER];
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int c = tid + it * NT;
      const int rl = c / CPR, ch = (c - rl * CPR) * 8;
      const int m = m0 + r0 + rl, n = n0 + ch;
      const bool ok = c < PR * CPR && m < p.M && n < p.N;
      rr[it] = (ok && p.res) ? ld16(p.res + (size_t)m * p.N + n) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int c = tid + it * NT;
      const int rl = c / CPR, ch = (c - rl * CPR) * 8;
      const int m = m0 + r0 + rl, n = n0 + ch;
      if (c >= PR * CPR || m >= p.M || n >= p.N) continue;
      const f32x4 s0 = *reinterpret_cast<const f32x4*>(&stage[rl * OROW + ch]);
      const f32x4 s1 = *reinterpret_cast<const f32x4*>(&stage[rl * OROW + ch + 4]);
      float v[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
      float t[8];
      if (p.rowstat) ln_fold8(p, m, n, v);
      if (p.bias) {
        unpack8e<EL>(ld16(p.bias + n), t);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += t[e];
      }
      if (p.temb) {
        unpack8e<EL>(ld16(p.temb + (size_t)(m / hw) * p.temb_ld + n), t);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += t[e];
      }
      if (p.res) {
        unpack8e<EL>(rr[it], t);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += t[e];
      }
      if (p.act) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = act_f(p.act, v[e]);
      }
      st16(p.out + (size_t)m * p.N + n, pack8e<EL>(v));
    }
  }
}

// NORM: the A operand is GroupNorm(+SiLU)(x) computed on the fly from a per-(batch, channel)
// affine table (scale, shift) - the normalised activation is never written to HBM.  Zero
// padding stays zero (the reference pads the NORMALISED tensor), so only in-bounds chunks
// are transformed.
template <int BN, int BM, int WN, int WM, int MINW, bool SPLIT, bool NORM, int EL = 0>
__global__ void __launch_bounds__(256, MINW) conv_igemm_kernel(ConvArgs p) {
  static_assert(EL == 0 || !NORM, "norm prologue: bf16 only");
  constexpr int BK = 64;
  static_assert(WN * WM == 4, "4 waves");
  constexpr int TN = BN / WN / 16, TM = BM / WM / 16;  // 16x16 tiles per wave
  constexpr int WCH = BN * 8 / 256;           // 16-byte chunks per thread (W tile)
  constexpr int XCH = BM * 8 / 256;           // 16-byte chunks per thread (X tile)
  // one LDS array (operand stages, then the epilogue's fp32 staging)
  __shared__ __attribute__((aligned(16))) bf16_t smem_[2 * (BN + BM) * BK];
  bf16_t (*const sW)[BN * BK] = reinterpret_cast<bf16_t (*)[BN * BK]>(smem_);
  bf16_t (*const sX)[BM * BK] = reinterpret_cast<bf16_t (*)[BM * BK]>(smem_ + 2 * BN * BK);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WM, wm = wave % WM;
  const int g = lane >> 4, l16 = lane & 15;

  int split_idx, n0, m0;
  tile_coords(p, BN, BM, split_idx, n0, m0);
  const int kt0 = SPLIT ? split_idx * p.kt_per_split : 0;
  const int kt1 = SPLIT ? min(p.ktiles, kt0 + p.kt_per_split) : p.ktiles;

  // ---- per-thread staging geometry (rows fixed across the K loop)
  const int cc = tid & 7;  // 16-byte chunk within the 128-byte K row
  int xb[XCH], xho[XCH], xwo[XCH];
  bool xok[XCH];
#pragma unroll
  for (int i = 0; i < XCH; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    xok[i] = m < p.M;
    const int mm = xok[i] ? m : 0;
    const int hw = p.Ho * p.Wo;
    xb[i] = mm / hw;
    const int rem = mm - xb[i] * hw;
    xho[i] = (rem / p.Wo) * p.stride - p.pad;
    xwo[i] = (rem % p.Wo) * p.stride - p.padw;
  }

  // Incremental K walk (tap-major, then 64-channel chunks inside the tap): the (r, s) tap, the
  // per-row input offsets and the zero-padding masks change only when the walk crosses into the
  // next tap (every Cin/64 k-tiles), so the per-k-tile address work is two adds per chunk
  // instead of two integer divisions + a 64-bit multiply chain (MFMA:VALU was 1:13-15 on the
  // 64x64 tiles of the UNet's small convs; profiles/pmc_r1_v10_sd15.md).
  int woff[WCH];
#pragma unroll
  for (int i = 0; i < WCH; ++i) {
    const int n = n0 + (tid >> 3) + 32 * i;
    woff[i] = n < p.N ? n * p.K + cc * 8 : -1;
  }
  int wk = kt0 * BK;                                  // K offset of the next tile to load
  int wc = wk % p.Cin, wrs = wk / p.Cin;              // channel chunk, tap index
  int wr = wrs / p.kw, ws = wrs - wr * p.kw;          // tap (r, s)
  int xoff[XCH];                                      // element offset of (b, hi, wi, cc*8) or -1
  auto set_tap = [&]() {
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      int hi = xho[i] + wr, wi = xwo[i] + ws;
      const bool ok = xok[i] && hi >= 0 && hi < p.Hl && wi >= 0 && wi < p.Wl;
      if (p.upsample) { hi >>= 1; wi >>= 1; }
      const int pix = (xb[i] * p.H + hi) * p.W + wi;
      xoff[i] = ok ? (p.x2 ? pix : pix * p.Cx + cc * 8) : -1;    // dual source: the pixel index
    }
  };
  set_tap();
  // activation chunk address of row i at channel offset wc (wave-uniform source select)
  auto xaddr = [&](int i) -> const bf16_t* {
    if (p.x2 == nullptr) return p.x + xoff[i] + wc;
    return wc < p.C1 ? p.x + (size_t)xoff[i] * p.C1 + wc + cc * 8
                     : p.x2 + (size_t)xoff[i] * (p.Cin - p.C1) + (wc - p.C1) + cc * 8;
  };

  // Staging depth: small tiles (MFMA work per k-tile far below a load latency) keep two k-tiles
  // of loads in flight; large tiles keep one (their VGPR budget is spent on accumulators).
  constexpr bool DEEP = BN * BM <= 64 * 128;
  f32x4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if constexpr (DEEP) {
  // Two register sets (A, B) -> two LDS buffers: while the MFMAs consume LDS buffer j, the loads
  // of the NEXT TWO k-tiles are in flight (one set landing, one just issued), and the LDS write
  // waits only for the older set (counted vmcnt: every load is unconditional, masked rows read
  // the zero page).  The old one-set ring exposed a full load latency per k-tile, which on the
  // small UNet tiles is 10-20x the k-tile's MFMA time.
  struct Stage {
    uint4 w[WCH], x[XCH];
    bool xv[XCH];
    int lc;
  };
  Stage A, B;
  // live = false: a dead prefetch past this block's last k-tile - reads the zero page, so the
  // issue stays unconditional (no branch around the loads for hipcc's vmcnt counting to merge)
  const bf16_t* zp = reinterpret_cast<const bf16_t*>(g_conv_zero_page);
  auto load_regs = [&](Stage& S, bool live) {
    S.lc = wc + cc * 8;
#pragma unroll
    for (int i = 0; i < WCH; ++i) S.w[i] = ld16(live && woff[i] >= 0 ? p.w + woff[i] + wk : zp);
    const bool cin_ok = wc + cc * 8 < p.Cx;           // padded channels read zeros
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      S.xv[i] = live && xoff[i] >= 0 && cin_ok;
      S.x[i] = ld16(S.xv[i] ? xaddr(i) : zp);
    }
    wk += BK;
    wc += BK;
    if (wc == p.Cin) {                                // next tap (uniform branch)
      wc = 0;
      if (++ws == p.kw) { ws = 0; ++wr; }
      set_tap();
    }
  };
  auto store_regs = [&](int buf, Stage& S) {
    if constexpr (NORM) {
      // GroupNorm(+SiLU) prologue; zero padding stays zero (only in-bounds chunks transformed)
#pragma unroll
      for (int i = 0; i < XCH; ++i) {
        if (!S.xv[i]) continue;
        const float4* t = reinterpret_cast<const float4*>(p.norm + ((size_t)xb[i] * p.Cin + S.lc) * 2);
        const float4 t0 = t[0], t1 = t[1], t2 = t[2], t3 = t[3];
        const float sc[8] = {t0.x, t0.z, t1.x, t1.z, t2.x, t2.z, t3.x, t3.z};
        const float sh[8] = {t0.y, t0.w, t1.y, t1.w, t2.y, t2.w, t3.y, t3.w};
        float f[8];
        unpack8(S.x[i], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = fmaf(f[e], sc[e], sh[e]);
          f[e] = p.norm_silu ? silu_f(v) : v;
        }
        S.x[i] = pack8(f);
      }
    }
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int row = (tid >> 3) + 32 * i;
      st16(&sW[buf][row * BK + ((cc ^ (row & 7)) << 3)], S.w[i]);
    }
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int row = (tid >> 3) + 32 * i;
      st16(&sX[buf][row * BK + ((cc ^ (row & 7)) << 3)], S.x[i]);
    }
  };

  auto compute = [&](int cur) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      uint4 af[TN], bfr[TM];
#pragma unroll
      for (int a = 0; a < TN; ++a) {
        const int row = wn * (BN / WN) + a * 16 + l16;
        af[a] = ld16(&sW[cur][row * BK + (((kk * 4 + g) ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int b = 0; b < TM; ++b) {
        const int row = wm * (BM / WM) + b * 16 + l16;
        bfr[b] = ld16(&sX[cur][row * BK + (((kk * 4 + g) ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = mma16<EL>(af[a], bfr[b], acc[a][b]);
    }
  };

  // Loads and LDS writes are unconditional (dead ones move zeros into a buffer nobody reads), so
  // every wait in the loop is a counted vmcnt of the older set only.
  const int nk = kt1 - kt0;
  load_regs(A, nk > 0);
  load_regs(B, nk > 1);
  store_regs(0, A);
  __syncthreads();
  for (int i = 0; i < nk; i += 2) {
    // even step: LDS buffer 0 holds tile i; set A (stored) is free, set B holds tile i+1
    load_regs(A, i + 2 < nk);
    compute(0);
    store_regs(1, B);
    __syncthreads();
    if (i + 1 >= nk) break;
    // odd step: LDS buffer 1 holds tile i+1; set B is free, set A holds tile i+2
    load_regs(B, i + 3 < nk);
    compute(1);
    store_regs(0, A);
    __syncthreads();
  }

  } else {
  uint4 rw[WCH], rx[XCH];
  bool xv[XCH];
  int lc0 = 0;
  auto load_tile = [&]() {
    lc0 = wc + cc * 8;
#pragma unroll
    for (int i = 0; i < WCH; ++i)
      rw[i] = woff[i] >= 0 ? ld16(p.w + woff[i] + wk) : make_uint4(0, 0, 0, 0);
    const bool cin_ok = wc + cc * 8 < p.Cx;           // padded channels read zeros
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const bool ok = xoff[i] >= 0 && cin_ok;
      rx[i] = ok ? ld16(xaddr(i)) : make_uint4(0, 0, 0, 0);
      xv[i] = ok;
    }
    wk += BK;
    wc += BK;
    if (wc == p.Cin) {                                // next tap (uniform branch)
      wc = 0;
      if (++ws == p.kw) { ws = 0; ++wr; }
      set_tap();
    }
  };
  auto norm_tile = [&]() {
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      if (!xv[i]) continue;
      const float4* t = reinterpret_cast<const float4*>(p.norm + ((size_t)xb[i] * p.Cin + lc0) * 2);
      const float4 t0 = t[0], t1 = t[1], t2 = t[2], t3 = t[3];
      const float sc[8] = {t0.x, t0.z, t1.x, t1.z, t2.x, t2.z, t3.x, t3.z};
      const float sh[8] = {t0.y, t0.w, t1.y, t1.w, t2.y, t2.w, t3.y, t3.w};
      float f[8];
      unpack8(rx[i], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = fmaf(f[e], sc[e], sh[e]);
        f[e] = p.norm_silu ? silu_f(v) : v;
      }
      rx[i] = pack8(f);
    }
  };
  auto store_tile = [&](int buf) {
    if constexpr (NORM) norm_tile();
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int row = (tid >> 3) + 32 * i;
      st16(&sW[buf][row * BK + ((cc ^ (row & 7)) << 3)], rw[i]);
    }
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int row = (tid >> 3) + 32 * i;
      st16(&sX[buf][row * BK + ((cc ^ (row & 7)) << 3)], rx[i]);
    }
  };


  if (kt0 < kt1) {
    load_tile();
    store_tile(0);
  }
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) load_tile();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      uint4 af[TN], bfr[TM];
#pragma unroll
      for (int a = 0; a < TN; ++a) {
        const int row = wn * (BN / WN) + a * 16 + l16;
        af[a] = ld16(&sW[cur][row * BK + (((kk * 4 + g) ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int b = 0; b < TM; ++b) {
        const int row = wm * (BM / WM) + b * 16 + l16;
        bfr[b] = ld16(&sX[cur][row * BK + (((kk * 4 + g) ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = mma16<EL>(af[a], bfr[b], acc[a][b]);
    }
    if (more) store_tile(cur ^ 1);
    __syncthreads();
  }

  }

  // ---- epilogue: lane holds out[m][n .. n+3]
  const int hw = p.Ho * p.Wo;
  auto emit = [&](int m, int n, float v0, float v1, float v2, float v3) {
    if (p.rowstat) ln_fold4(p, m, n, v0, v1, v2, v3);
    if (p.bias) {
      const uint2 bv = *reinterpret_cast<const uint2*>(p.bias + n);
      v0 += lo16<EL>(bv.x); v1 += hi16<EL>(bv.x);
      v2 += lo16<EL>(bv.y); v3 += hi16<EL>(bv.y);
    }
    if (p.temb) {
      const uint2 tv = *reinterpret_cast<const uint2*>(p.temb + (size_t)(m / hw) * p.temb_ld + n);
      v0 += lo16<EL>(tv.x); v1 += hi16<EL>(tv.x);
      v2 += lo16<EL>(tv.y); v3 += hi16<EL>(tv.y);
    }
    if (p.res) {
      const uint2 rv = *reinterpret_cast<const uint2*>(p.res + (size_t)m * p.N + n);
      v0 += lo16<EL>(rv.x); v1 += hi16<EL>(rv.x);
      v2 += lo16<EL>(rv.y); v3 += hi16<EL>(rv.y);
    }
    if (p.act) { v0 = act_f(p.act, v0); v1 = act_f(p.act, v1); v2 = act_f(p.act, v2); v3 = act_f(p.act, v3); }
    uint2 o;
    o.x = enc16<EL>(v0) | (enc16<EL>(v1) << 16);
    o.y = enc16<EL>(v2) | (enc16<EL>(v3) << 16);
    *reinterpret_cast<uint2*>(p.out + (size_t)m * p.N + n) = o;
  };
  if constexpr (!SPLIT) {
    epilogue_lds<BN, BM, WN, WM, 256, (BN + BM) * BK, EL>(p, acc, reinterpret_cast<float*>(smem_), m0, n0);
    return;
  } else {
    // ---- split-K: fp32 slab, then IN-LAUNCH ordered reduction by the tile's last arriving
    // block (cdna_hip_programming.md "In-launch split-K reduction": agent-scope release before
    // the ticket, acquire in the reducer).  Tickets live in a persistent zero-initialised pool;
    // the reducer re-arms its counter to 0, so no memset node is needed per call.  The
    // reducer sums slabs 0..S-1 in order - the same arithmetic as splitk_reduce_kernel, so
    // results are bitwise identical and independent of which block arrives last.
#pragma unroll
    for (int b = 0; b < TM; ++b) {
      const int m = m0 + wm * (BM / WM) + b * 16 + l16;
      if (m >= p.M) continue;
#pragma unroll
      for (int a = 0; a < TN; ++a) {
        const int n = n0 + wn * (BN / WN) + a * 16 + 4 * g;
        if (n >= p.N) continue;
        *reinterpret_cast<float4*>(p.ws + ((size_t)split_idx * p.M + m) * p.N + n) =
            make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
      }
    }
    if (p.counters == nullptr) return;            // separate reduce kernel (A/B path)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(&sX[0][0]);  // the existing LDS array (no 2nd __shared__)
    const int tile = (m0 / BM) * p.tiles_n + n0 / BN;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int t = __hip_atomic_fetch_add(&p.counters[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = (t == p.nsplit - 1);
    }
    __syncthreads();
    if (!*flag) return;
    if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int b = 0; b < TM; ++b) {
      const int m = m0 + wm * (BM / WM) + b * 16 + l16;
      if (m >= p.M) continue;
#pragma unroll
      for (int a = 0; a < TN; ++a) {
        const int n = n0 + wn * (BN / WN) + a * 16 + 4 * g;
        if (n >= p.N) continue;
        float4 v = *reinterpret_cast<const float4*>(p.ws + (size_t)m * p.N + n);
        for (int sp = 1; sp < p.nsplit; ++sp) {
          const float4 w4 = *reinterpret_cast<const float4*>(p.ws + ((size_t)sp * p.M + m) * p.N + n);
          v.x += w4.x; v.y += w4.y; v.z += w4.z; v.w += w4.w;
        }
        emit(m, n, v.x, v.y, v.z, v.w);
      }
    }
    if (tid == 0) p.counters[tile] = 0;   // re-arm for the next launch on this region
  }
}

// ---------------------------------------------------------------------------------------------
// Multi-stage LDS-DMA variant.  Same tiling / fragment / epilogue as above, but the K-tile
// stream is global_load_lds_dwordx4 (16 B per lane straight into LDS, no VGPR round trip)
// into an NS-deep ring of LDS stages with NS-1 tiles in flight: at ~1 workgroup per CU the
// HBM latency of a tile (~1-2 us) is longer than one tile's MFMA work (~0.3 us), so one-ahead
// register staging leaves the MFMAs starved (cdna_hip_programming.md §5 "Pipelining across
// barriers": counted vmcnt + raw s_barrier, never __syncthreads() while DMA is in flight).
// The XOR swizzle moves to the per-lane SOURCE address (LDS image stays lane-linear, rule 21);
// zero padding / masked rows read a zero page.

// LDS-DMA (16 B per lane, lane-linear at the wave-uniform LDS address) issued as inline asm:
// hipcc's waitcnt pass does not track it, so it adds no conservative vmcnt drains before LDS
// reads.  The kernel owns the RAW ordering: counted wait_vmcnt (builtin) + barrier.
__device__ __forceinline__ void dma16(const void* src, const void* lds) {
  const unsigned a = __builtin_amdgcn_readfirstlane((unsigned)(size_t)lds);
  asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(a) : "memory");
}

// Ring stages as DISTINCT __shared__ objects, each addressed only through a compile-time stage
// index (main loops unrolled by NS).  hipcc's waitcnt pass orders a ds_read after every
// outstanding LDS-DMA unless alias scopes prove them disjoint; scopes exist per LDS variable and
// survive only when a pointer derives from exactly one of them.  With one dynamic array (or a
// runtime stage select) every K step began with s_waitcnt vmcnt(0), draining the whole ring.
template <int S, typename T>
__device__ __forceinline__ T* ring_stage(T* s0, T* s1, T* s2, T* s3) {
  if constexpr (S == 0) return s0;
  else if constexpr (S == 1) return s1;
  else if constexpr (S == 2) return s2;
  else return s3;
}
template <int V>
struct IC {
  static constexpr int value = V;
};

// Counted vmcnt wait as the s_waitcnt BUILTIN (not inline asm): hipcc's waitcnt pass cannot see
// an inline-asm wait, so it still counts the retired stage's DMA as outstanding and drains the
// whole ring (vmcnt(0)) before the next ds_read of that stage.  gfx9 encoding: vmcnt[3:0] in
// bits 3:0, vmcnt[5:4] in bits 15:14; expcnt (6:4) and lgkmcnt (11:8) left at their maxima.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}

// NT = 64 * WN * WM threads: 4 waves (one per SIMD), or 8 waves for the 256-wide tiles (two per
// SIMD: one wave's MFMA cluster runs while the other issues its LDS reads / DMA).
// One 16-byte-per-lane LDS-DMA through a raw buffer resource over [base, base + nbytes): lanes whose
// byte offset is past nbytes get zeros (range check).  A separate device function: hipcc drops a
// kernel's host stub when the target-only resource type appears in the kernel's own (lambda) body.
__device__ __forceinline__ void buf_lds16(const void* base, int nbytes, void* lds, unsigned off) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, nbytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, off, 0, 0, 0);
}

// BUF: LDS-DMA through buffer resources (conv_stag2_kernel BUF): one VALU add per DMA, range-checked
// zero fill for padding taps and rows past N / M instead of the zero-page select.
template <int BN, int BM, int WN, int WM, int NS, bool SPLIT, bool BUF = false>
__global__ void __launch_bounds__(64 * WN * WM, 1) conv_glds_kernel(ConvArgs p) {
  constexpr int EL = 0;   // LDS-DMA variant: bf16 only (fp16 convs use the register-staged kernel)
  constexpr int BK = 64;
  constexpr int NT = 64 * WN * WM;
  constexpr int RPI = NT / 8;        // tile rows covered by one DMA instruction of the workgroup
  static_assert(WN * WM == 4 || WN * WM == 8, "4 or 8 waves");
  static_assert((BN * 8) % NT == 0 && (BM * 8) % NT == 0, "whole DMA rounds per tile");
  constexpr int TN = BN / WN / 16, TM = BM / WM / 16;
  constexpr int WCH = BN * 8 / NT;   // glds per thread per tile (W)
  constexpr int XCH = BM * 8 / NT;   // glds per thread per tile (X)
  constexpr int LPT = WCH + XCH;     // vmcnt units per tile per wave
  constexpr int STAGE = (BN + BM) * BK;  // bf16 elements per stage
  static_assert(NS >= 2 && NS <= 4, "ring depth");
  __shared__ __attribute__((aligned(16))) bf16_t lds0[STAGE];
  __shared__ __attribute__((aligned(16))) bf16_t lds1[STAGE];
  __shared__ __attribute__((aligned(16))) bf16_t lds2[NS > 2 ? STAGE : 8];
  __shared__ __attribute__((aligned(16))) bf16_t lds3[NS > 3 ? STAGE : 8];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WM, wm = wave % WM;
  const int g = lane >> 4, l16 = lane & 15;
  int split_idx, n0, m0;
  tile_coords(p, BN, BM, split_idx, n0, m0);
  const int kt0 = SPLIT ? split_idx * p.kt_per_split : 0;
  const int kt1 = SPLIT ? min(p.ktiles, kt0 + p.kt_per_split) : p.ktiles;
  const int nk = kt1 - kt0;

  // lane-linear LDS image: chunk c = tid + 256 i -> row c/8, position c%8 holds logical
  // chunk (c%8) ^ (row & 7)  (the read side applies the same XOR).
  const int pos = tid & 7;
  int wrow[WCH], wcc[WCH];
#pragma unroll
  for (int i = 0; i < WCH; ++i) {
    wrow[i] = (tid >> 3) + RPI * i;
    wcc[i] = pos ^ (wrow[i] & 7);
  }
  int xb[XCH], xho[XCH], xwo[XCH], xcc[XCH];
  bool xok[XCH];
#pragma unroll
  for (int i = 0; i < XCH; ++i) {
    const int row = (tid >> 3) + RPI * i;
    xcc[i] = pos ^ (row & 7);
    const int m = m0 + row;
    xok[i] = m < p.M;
    const int mm = xok[i] ? m : 0;
    const int hw = p.Ho * p.Wo;
    xb[i] = mm / hw;
    const int rem = mm - xb[i] * hw;
    xho[i] = (rem / p.Wo) * p.stride - p.pad;
    xwo[i] = (rem % p.Wo) * p.stride - p.padw;
  }
  typedef __attribute__((address_space(1))) const void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;

  // incremental K walk, as in conv_igemm_kernel: tap-dependent row offsets recomputed only when
  // the walk enters the next (r, s) tap
  int woff[WCH];
#pragma unroll
  for (int i = 0; i < WCH; ++i) {
    const int n = n0 + wrow[i];
    woff[i] = n < p.N ? n * p.K + wcc[i] * 8 : -1;
  }
  constexpr unsigned kOOB = 0x80000000u;            // BUF: byte offset past every resource (range check)
  unsigned wbo[WCH], xbo[XCH];
#pragma unroll
  for (int i = 0; i < WCH; ++i) wbo[i] = woff[i] >= 0 ? 2u * (unsigned)woff[i] : kOOB;
  int wk = kt0 * BK, wc = wk % p.Cin, wrs = wk / p.Cin;
  int wr = wrs / p.kw, ws = wrs - wr * p.kw;
  int xoff[XCH];
  auto set_tap = [&]() {
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      int hi = xho[i] + wr, wi = xwo[i] + ws;
      const bool ok = xok[i] && hi >= 0 && hi < p.Hl && wi >= 0 && wi < p.Wl;
      if (p.upsample) { hi >>= 1; wi >>= 1; }
      xoff[i] = ok ? ((xb[i] * p.H + hi) * p.W + wi) * p.Cin + xcc[i] * 8 : -1;
      if constexpr (BUF) xbo[i] = ok ? 2u * (unsigned)xoff[i] : kOOB;
    }
  };
  set_tap();
  auto issue = [&](auto stage_c) {
    bf16_t* sW = ring_stage<decltype(stage_c)::value>(lds0, lds1, lds2, lds3);
    bf16_t* sX = sW + BN * BK;
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      // wave-uniform destination: first row of this wave's 8-row slab
      bf16_t* dst = sW + ((wave * 8) + RPI * i) * BK;
      if constexpr (BUF) {
        buf_lds16(p.w, 2 * p.N * p.K, dst, wbo[i] + 2u * (unsigned)wk);
      } else {
        const void* src = woff[i] >= 0 ? (const void*)(p.w + woff[i] + wk) : (const void*)g_conv_zero_page;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)dst, 16, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      bf16_t* dst = sX + ((wave * 8) + RPI * i) * BK;
      if constexpr (BUF) {
        buf_lds16(p.x, 2 * p.B * p.H * p.W * p.Cin, dst, xbo[i] + 2u * (unsigned)wc);
      } else {
        const void* src = xoff[i] >= 0 ? (const void*)(p.x + xoff[i] + wc) : (const void*)g_conv_zero_page;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)dst, 16, 0, 0);
      }
    }
    wk += BK;
    wc += BK;
    if (wc == p.Cin) {
      wc = 0;
      if (++ws == p.kw) { ws = 0; ++wr; }
      set_tap();
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: NS-1 tiles in flight
  if (0 < nk) issue(IC<0>());
  if (NS > 2 && 1 < nk) issue(IC<1>());
  if (NS > 3 && 2 < nk) issue(IC<2>());

  auto step = [&](auto stage_c, int i) __attribute__((always_inline)) {
    constexpr int S = decltype(stage_c)::value;
    // tile i has landed once at most (NS-2) newer tiles are outstanding
    if (i + NS - 2 < nk) wait_vmcnt<(NS - 2) * LPT>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // every wave's DMA for tile i is visible
    if (i + NS - 1 < nk) issue(IC<(S + NS - 1) % NS>());  // that stage was read at i-1
    const bf16_t* sW = ring_stage<S>(lds0, lds1, lds2, lds3);
    const bf16_t* sX = sW + BN * BK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      uint4 af[TN], bfr[TM];
#pragma unroll
      for (int a = 0; a < TN; ++a) {
        const int row = wn * (BN / WN) + a * 16 + l16;
        af[a] = ld16(&sW[row * BK + (((kk * 4 + g) ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int b = 0; b < TM; ++b) {
        const int row = wm * (BM / WM) + b * 16 + l16;
        bfr[b] = ld16(&sX[row * BK + (((kk * 4 + g) ^ (row & 7)) << 3)]);
      }
      if constexpr (NT == 512) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = mma16<EL>(af[a], bfr[b], acc[a][b]);
      if constexpr (NT == 512) __builtin_amdgcn_s_setprio(0);
    }
    // WAR on stage i%NS is covered by the next iteration's barrier: its refill is issued
    // only after every wave has arrived there, i.e. finished this tile's MFMAs (whose
    // operands - these ds_reads - had to complete first).
  };
  // block-uniform guards instead of early exits: with breaks, hipcc gave every exit its own
  // accumulator copy (320x128: 256 VGPRs + scratch spills whose reloads drained the DMA ring)
  for (int i = 0; i < nk; i += NS) {
    step(IC<0>(), i);
    if (i + 1 < nk) step(IC<1>(), i + 1);
    if constexpr (NS > 2) {
      if (i + 2 < nk) step(IC<2 % NS>(), i + 2);
    }
    if constexpr (NS > 3) {
      if (i + 3 < nk) step(IC<3 % NS>(), i + 3);
    }
  }

  if constexpr (!SPLIT) {
    epilogue_lds<BN, BM, WN, WM, NT, STAGE / 2, EL>(p, acc, reinterpret_cast<float*>(lds0), m0, n0);
    return;
  }
  const int hw = p.Ho * p.Wo;
#pragma unroll
  for (int b = 0; b < TM; ++b) {
    const int m = m0 + wm * (BM / WM) + b * 16 + l16;
    if (m >= p.M) continue;
    const int bb = m / hw;
#pragma unroll
    for (int a = 0; a < TN; ++a) {
      const int n = n0 + wn * (BN / WN) + a * 16 + 4 * g;
      if (n >= p.N) continue;
      float v0 = acc[a][b][0], v1 = acc[a][b][1], v2 = acc[a][b][2], v3 = acc[a][b][3];
      if (SPLIT) {
        *reinterpret_cast<float4*>(p.ws + ((size_t)split_idx * p.M + m) * p.N + n) = make_float4(v0, v1, v2, v3);
        continue;
      }
      if (p.rowstat) ln_fold4(p, m, n, v0, v1, v2, v3);
      if (p.bias) {
        const uint2 bv = *reinterpret_cast<const uint2*>(p.bias + n);
        v0 += lo16<EL>(bv.x); v1 += hi16<EL>(bv.x);
        v2 += lo16<EL>(bv.y); v3 += hi16<EL>(bv.y);
      }
      if (p.temb) {
        const uint2 tv = *reinterpret_cast<const uint2*>(p.temb + (size_t)bb * p.temb_ld + n);
        v0 += lo16<EL>(tv.x); v1 += hi16<EL>(tv.x);
        v2 += lo16<EL>(tv.y); v3 += hi16<EL>(tv.y);
      }
      if (p.res) {
        const uint2 rv = *reinterpret_cast<const uint2*>(p.res + (size_t)m * p.N + n);
        v0 += lo16<EL>(rv.x); v1 += hi16<EL>(rv.x);
        v2 += lo16<EL>(rv.y); v3 += hi16<EL>(rv.y);
      }
      uint2 o;
      o.x = enc16<EL>(v0) | (enc16<EL>(v1) << 16);
      o.y = enc16<EL>(v2) | (enc16<EL>(v3) << 16);
      *reinterpret_cast<uint2*>(p.out + (size_t)m * p.N + n) = o;
    }
  }
}

// Staggered two-group variant (cfg 36 + i).  Same LDS-DMA ring, tiling, fragments and epilogue as
// conv_glds_kernel, but the 8 waves form two groups (waves 0-3 and 4-7: one wave of each per SIMD,
// the hardware places waves w and w+4 on one SIMD) that run ONE BARRIER APART
// (cdna_hip_programming.md §5 "The 256^2 8-phase template": staggered wave groups, per-phase
// interleave).  Each K tile is two phases (its two k32 halves); a phase is
//     LOAD:    this k-half's A/B fragments from LDS (+ at odd phases the next-but-one tile's DMA
//              and the counted wait for the next tile), then s_barrier
//     COMPUTE: the k-half's MFMAs at raised priority, then s_barrier
// and group 1 starts with one extra barrier (group 0 ends with one), so every barrier interval
// pairs one group's MFMAs with the other group's LDS reads / DMA issue on each SIMD - in the
// one-barrier-per-K-tile kernel both waves of a SIMD read, then both multiply.
// Ordering (barrier events numbered in group 0's count; group 1 passes event e at its own e-1):
//   RAW: tile j is waited (vmcnt, own DMA) in phase 2j-1 before its first barrier and first read
//        in phase 2j: group 0's wait precedes event 4j-2, group 1's event 4j-1, and the earliest
//        read (group 0, phase 2j) follows event 4j-1.
//   WAR: tile j+2 is issued in phase 2j+1 into the stage of tile j-1, whose last reads (phase
//        2j-1) retire before that phase's MFMAs (lgkmcnt); group 1 finishes those MFMAs at
//        event 4j and group 0 issues only after event 4j+1.  Three stages (NS = 3).
// Per output the MFMA sequence (k-tiles ascending, k-halves ascending) is that of every other
// family, so the results are bitwise those of conv_glds_kernel / conv_igemm_kernel at every split.
// A tile operand of R rows is R/8 DMA wave-instructions (8 rows of 128 B each); wave w issues
// instructions w, w+8, ... - when R/8 is not a multiple of 8 (BN = 160) the surplus ones of a round
// write a 1 KiB dummy buffer nobody reads, so every wave keeps the same vmcnt count per tile.
template <int BN, int BM, int WN, int WM, bool SPLIT, bool BUF = false>
__global__ void __launch_bounds__(512, 1) conv_stag_kernel(ConvArgs p) {
  constexpr int EL = 0, BK = 64, NT = 512, NS = 3;
  static_assert(WN * WM == 8, "8 waves");
  static_assert(BN % 8 == 0 && BM % 8 == 0, "whole DMA wave-instructions per operand");
  constexpr int TN = BN / WN / 16, TM = BM / WM / 16;
  constexpr int WINS = BN / 8, XINS = BM / 8;
  constexpr int WCH = (WINS + 7) / 8, XCH = (XINS + 7) / 8;
  constexpr bool DUMMY = (WINS % 8) != 0 || (XINS % 8) != 0;
  constexpr int LPT = WCH + XCH;
  constexpr int STAGE = (BN + BM) * BK;
  static_assert((size_t)NS * STAGE * 2 + (DUMMY ? 1024 : 0) <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) bf16_t lds0[STAGE];
  __shared__ __attribute__((aligned(16))) bf16_t lds1[STAGE];
  __shared__ __attribute__((aligned(16))) bf16_t lds2[STAGE];
  __shared__ __attribute__((aligned(16))) bf16_t ldsd[DUMMY ? 512 : 8];   // surplus DMA target

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WM, wm = wave % WM;
  const int g = lane >> 4, l16 = lane & 15;
  const bool grp1 = wave >= 4;
  int split_idx, n0, m0;
  tile_coords(p, BN, BM, split_idx, n0, m0);
  const int kt0 = SPLIT ? split_idx * p.kt_per_split : 0;
  const int kt1 = SPLIT ? min(p.ktiles, kt0 + p.kt_per_split) : p.ktiles;
  const int nk = kt1 - kt0;

  const int pos = tid & 7;
  int woff[WCH];
#pragma unroll
  for (int i = 0; i < WCH; ++i) {
    const int j = wave + 8 * i, row = 8 * j + (lane >> 3);
    woff[i] = (j < WINS && n0 + row < p.N) ? (n0 + row) * p.K + ((pos ^ (row & 7)) << 3) : -1;
  }
  constexpr unsigned kOOB = 0x80000000u;            // BUF: byte offset past every resource (range check)
  unsigned wbo[WCH], xbo[XCH];
#pragma unroll
  for (int i = 0; i < WCH; ++i) wbo[i] = woff[i] >= 0 ? 2u * (unsigned)woff[i] : kOOB;
  int xb[XCH], xho[XCH], xwo[XCH], xcc[XCH];
  bool xok[XCH];
  const int hw = p.Ho * p.Wo;
#pragma unroll
  for (int i = 0; i < XCH; ++i) {
    const int j = wave + 8 * i, row = 8 * j + (lane >> 3);
    xcc[i] = pos ^ (row & 7);
    const int m = m0 + row;
    xok[i] = j < XINS && m < p.M;
    const int mm = xok[i] ? m : 0;
    xb[i] = mm / hw;
    const int rem = mm - xb[i] * hw;
    xho[i] = (rem / p.Wo) * p.stride - p.pad;
    xwo[i] = (rem % p.Wo) * p.stride - p.padw;
  }
  typedef __attribute__((address_space(1))) const void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  int wk = kt0 * BK, wc = wk % p.Cin, wrs = wk / p.Cin;
  int wr = wrs / p.kw, ws = wrs - wr * p.kw;
  int xoff[XCH];
  auto set_tap = [&]() {
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      int hi = xho[i] + wr, wi = xwo[i] + ws;
      const bool ok = xok[i] && hi >= 0 && hi < p.Hl && wi >= 0 && wi < p.Wl;
      if (p.upsample) { hi >>= 1; wi >>= 1; }
      xoff[i] = ok ? ((xb[i] * p.H + hi) * p.W + wi) * p.Cin + xcc[i] * 8 : -1;
      if constexpr (BUF) xbo[i] = ok ? 2u * (unsigned)xoff[i] : kOOB;
    }
  };
  set_tap();
  auto issue = [&](auto stage_c) {
    bf16_t* sW = ring_stage<decltype(stage_c)::value>(lds0, lds1, lds2, lds2);
    bf16_t* sX = sW + BN * BK;
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int j = wave + 8 * i;
      bf16_t* dst = (!DUMMY || j < WINS) ? sW + 8 * j * BK : ldsd;
      if constexpr (BUF) {
        buf_lds16(p.w, 2 * p.N * p.K, dst, wbo[i] + 2u * (unsigned)wk);
      } else {
        const void* src = woff[i] >= 0 ? (const void*)(p.w + woff[i] + wk) : (const void*)g_conv_zero_page;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)dst, 16, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int j = wave + 8 * i;
      bf16_t* dst = (!DUMMY || j < XINS) ? sX + 8 * j * BK : ldsd;
      if constexpr (BUF) {
        buf_lds16(p.x, 2 * p.B * p.H * p.W * p.Cin, dst, xbo[i] + 2u * (unsigned)wc);
      } else {
        const void* src = xoff[i] >= 0 ? (const void*)(p.x + xoff[i] + wc) : (const void*)g_conv_zero_page;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)dst, 16, 0, 0);
      }
    }
    wk += BK;
    wc += BK;
    if (wc == p.Cin) {
      wc = 0;
      if (++ws == p.kw) { ws = 0; ++wr; }
      set_tap();
    }
  };
  auto bar = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: tiles 0 and 1 in flight, tile 0 landed for every wave before the first read
  if (0 < nk) issue(IC<0>());
  if (1 < nk) {
    issue(IC<1>());
    wait_vmcnt<LPT>();
  } else {
    wait_vmcnt<0>();
  }
  bar();
  if (grp1) bar();   // group 1 runs one barrier behind group 0

  // one phase: k-half KK of the tile in stage S; at KK = 1 also the DMA of tile i+2 (into stage
  // S+2 mod 3 = the stage of tile i-1) and the wait for tile i+1
  auto phase = [&](auto stage_c, auto kk_c, int i) __attribute__((always_inline)) {
    constexpr int S = decltype(stage_c)::value, KK = decltype(kk_c)::value;
    const bf16_t* sW = ring_stage<S>(lds0, lds1, lds2, lds2);
    const bf16_t* sX = sW + BN * BK;
    uint4 af[TN], bfr[TM];
#pragma unroll
    for (int a = 0; a < TN; ++a) {
      const int row = wn * (BN / WN) + a * 16 + l16;
      af[a] = ld16(&sW[row * BK + (((KK * 4 + g) ^ (row & 7)) << 3)]);
    }
#pragma unroll
    for (int b = 0; b < TM; ++b) {
      const int row = wm * (BM / WM) + b * 16 + l16;
      bfr[b] = ld16(&sX[row * BK + (((KK * 4 + g) ^ (row & 7)) << 3)]);
    }
    if constexpr (KK == 1) {
      if (i + 2 < nk) {
        issue(IC<(S + 2) % NS>());
        wait_vmcnt<LPT>();          // tile i+1 landed (tile i+2 may still be in flight)
      } else {
        wait_vmcnt<0>();
      }
    }
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
      for (int b = 0; b < TM; ++b) acc[a][b] = mma16<EL>(af[a], bfr[b], acc[a][b]);
    __builtin_amdgcn_s_setprio(0);
    bar();
  };
  // unrolled by the ring depth (compile-time stages); a tile past the end is skipped by a
  // block-uniform branch - no early exits, so the accumulators keep one register home
  for (int i = 0; i < nk; i += NS) {
    phase(IC<0>(), IC<0>(), i);
    phase(IC<0>(), IC<1>(), i);
    if (i + 1 < nk) {
      phase(IC<1>(), IC<0>(), i + 1);
      phase(IC<1>(), IC<1>(), i + 1);
    }
    if (i + 2 < nk) {
      phase(IC<2>(), IC<0>(), i + 2);
      phase(IC<2>(), IC<1>(), i + 2);
    }
  }
  if (!grp1) bar();  // equal barrier counts: group 0 makes up group 1's head start

  if constexpr (!SPLIT) {
    epilogue_lds<BN, BM, WN, WM, NT, STAGE / 2, EL>(p, acc, reinterpret_cast<float*>(lds0), m0, n0);
  } else {
#pragma unroll
    for (int b = 0; b < TM; ++b) {
      const int m = m0 + wm * (BM / WM) + b * 16 + l16;
      if (m >= p.M) continue;
#pragma unroll
      for (int a = 0; a < TN; ++a) {
        const int n = n0 + wn * (BN / WN) + a * 16 + 4 * g;
        if (n < p.N)
          *reinterpret_cast<float4*>(p.ws + ((size_t)split_idx * p.M + m) * p.N + n) =
              make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
      }
    }
  }
}

// Half-slot staggered variant (cfg 42 + i): conv_stag_kernel's two wave groups one barrier apart, but
// the LDS-DMA ring is kept in K-HALF slots (32 channels x all rows of both operands per slot): a phase
// reads exactly one slot, the DMA of half u is issued three phases before its first read and waited one
// phase before it, so HS = 5 half slots (2.5 K tiles) carry the same two-phase latency cover as the
// three-stage ring - and a 320 x 128 tile fits in 140 KiB (three full stages would take 168 KiB).
// Slot rows are 64 B (4 x 16-B chunks); the chunk of row r sits at position chunk ^ f(r) with
// f(r) = 2 * ((r >> 3) & 1), which spreads the 16-lane groups of every ds_read_b128 fragment read
// over 16 distinct 16-B slots of the 256-B bank row (checked against the ds_read_b128 lane groups of
// MI355X_MICROARCH.md §LDS).  DMA stays lane-linear: the permutation lives on the source address.
// Ordering, with half u read in phase u (phase = one k-half of one K tile):
//   RAW: half u is waited (vmcnt) in phase u-1 before its first barrier - the conv_stag_kernel
//        argument with half slots for stages.
//   WAR: half u is issued in phase u-3 into the slot of half u-HS, last read in phase u-HS <= u-5:
//        its readers' MFMAs are done by group 1's barrier ending phase u-5 < the event before
//        group 0's load part of phase u-3.
// MFMA order per output (K tiles ascending, k-halves ascending) = every other family: bitwise equal.
__device__ __forceinline__ int half_swz(int r) { return ((r >> 3) & 1) << 1; }


template <int S, typename T>
__device__ __forceinline__ T* half_slot(T* s0, T* s1, T* s2, T* s3, T* s4, T* s5) {
  if constexpr (S == 0) return s0;
  else if constexpr (S == 1) return s1;
  else if constexpr (S == 2) return s2;
  else if constexpr (S == 3) return s3;
  else if constexpr (S == 4) return s4;
  else return s5;
}

// PD = prefetch distance in halves (half P + PD is issued in phase P).  WAR needs HS - PD >= 2 when
// a group's ds_reads may still be in flight at the barrier ending its load part (they retire by the
// next barrier), HS - PD >= 1 when every wave retires them (lgkmcnt(0)) before that barrier - the PD 4
// form on a 5-slot ring, which buys one more phase (two barriers) of DMA lead time.
// BUF: the DMA goes through buffer_load ... lds on two buffer resources (W, X) with 32-bit byte
// offsets - one VALU add per DMA instead of a 64-bit address plus the zero-page select: padding taps
// and rows past N / M carry an offset beyond the resource's size (0x80000000; sizes < 2 GiB), which
// the hardware range check turns into zero-filled LDS (tests/test_kernels_gpu.py probes it).
template <int BN, int BM, int WN, int WM, int HS, bool SPLIT, int PD = 3, bool BUF = false>
__global__ void __launch_bounds__(512, 1) conv_stag2_kernel(ConvArgs p) {
  constexpr int EL = 0, BK = 64, HK = 32, NT = 512;
  static_assert(WN * WM == 8, "8 waves");
  static_assert(HS == 5 || HS == 6, "half-slot ring depth");
  static_assert(PD == 3 || (PD == 4 && HS - PD >= 1), "prefetch distance");
  static_assert(BN % 16 == 0 && BM % 16 == 0, "16-row DMA wave-instructions");
  constexpr int TN = BN / WN / 16, TM = BM / WM / 16;
  constexpr int WINS = BN / 16, XINS = BM / 16;      // DMA wave-instructions per operand and half
  constexpr int WCH = (WINS + 7) / 8, XCH = (XINS + 7) / 8;
  constexpr bool DUMMY = (WINS % 8) != 0 || (XINS % 8) != 0;
  constexpr int LPH = WCH + XCH;                      // vmcnt units per half per wave
  constexpr int SLOT = (BN + BM) * HK;                // bf16 per half slot
  constexpr int U = HS == 5 ? 10 : 6;                 // phases per unrolled round (slot and parity static)
  static_assert((size_t)HS * SLOT * 2 + (DUMMY ? 1024 : 0) <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) bf16_t hs0[SLOT];
  __shared__ __attribute__((aligned(16))) bf16_t hs1[SLOT];
  __shared__ __attribute__((aligned(16))) bf16_t hs2[SLOT];
  __shared__ __attribute__((aligned(16))) bf16_t hs3[SLOT];
  __shared__ __attribute__((aligned(16))) bf16_t hs4[SLOT];
  __shared__ __attribute__((aligned(16))) bf16_t hs5[HS > 5 ? SLOT : 8];
  __shared__ __attribute__((aligned(16))) bf16_t ldsd[DUMMY ? 512 : 8];   // surplus DMA target

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WM, wm = wave % WM;
  const int g = lane >> 4, l16 = lane & 15;
  const bool grp1 = wave >= 4;
  int split_idx, n0, m0;
  tile_coords(p, BN, BM, split_idx, n0, m0);
  const int kt0 = SPLIT ? split_idx * p.kt_per_split : 0;
  const int kt1 = SPLIT ? min(p.ktiles, kt0 + p.kt_per_split) : p.ktiles;
  const int H = 2 * (kt1 - kt0);                      // halves of this block's K range

  // DMA lane geometry: wave-instruction jj = wave + 8 i fills slot rows 16 jj .. 16 jj + 15, lane l
  // writes row 16 jj + l / 4 at chunk position l % 4 (logical chunk = position ^ f(row))
  const int pos = lane & 3;
  int woff[WCH];
#pragma unroll
  for (int i = 0; i < WCH; ++i) {
    const int jj = wave + 8 * i, row = 16 * jj + (lane >> 2);
    woff[i] = (jj < WINS && n0 + row < p.N) ? (n0 + row) * p.K + ((pos ^ half_swz(row)) << 3) : -1;
  }
  constexpr unsigned kOOB = 0x80000000u;            // BUF: byte offset past every resource (range check)
  unsigned wbo[WCH];
#pragma unroll
  for (int i = 0; i < WCH; ++i) wbo[i] = woff[i] >= 0 ? 2u * (unsigned)woff[i] : kOOB;
  int xb[XCH], xho[XCH], xwo[XCH], xcc[XCH];
  bool xok[XCH];
  const int hw = p.Ho * p.Wo;
#pragma unroll
  for (int i = 0; i < XCH; ++i) {
    const int jj = wave + 8 * i, row = 16 * jj + (lane >> 2);
    xcc[i] = pos ^ half_swz(row);
    const int m = m0 + row;
    xok[i] = jj < XINS && m < p.M;
    const int mm = xok[i] ? m : 0;
    xb[i] = mm / hw;
    const int rem = mm - xb[i] * hw;
    xho[i] = (rem / p.Wo) * p.stride - p.pad;
    xwo[i] = (rem % p.Wo) * p.stride - p.padw;
  }
  typedef __attribute__((address_space(1))) const void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  int wk = kt0 * BK, wc = wk % p.Cin, wrs = wk / p.Cin;
  int wr = wrs / p.kw, ws = wrs - wr * p.kw;
  int xoff[XCH];
  unsigned xbo[XCH];
  auto set_tap = [&]() {
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      int hi = xho[i] + wr, wi = xwo[i] + ws;
      const bool ok = xok[i] && hi >= 0 && hi < p.Hl && wi >= 0 && wi < p.Wl;
      if (p.upsample) { hi >>= 1; wi >>= 1; }
      xoff[i] = ok ? ((xb[i] * p.H + hi) * p.W + wi) * p.Cin + xcc[i] * 8 : -1;
      if constexpr (BUF) xbo[i] = ok ? 2u * (unsigned)xoff[i] : kOOB;
    }
  };
  set_tap();
  // DMA of the next half (halves are issued in order; parity PAR = which k-half of the current tile)
  auto issue = [&](auto slot_c, auto par_c) {
    constexpr int S = decltype(slot_c)::value, PAR = decltype(par_c)::value;
    bf16_t* sW = half_slot<S>(hs0, hs1, hs2, hs3, hs4, hs5);
    bf16_t* sX = sW + BN * HK;
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int jj = wave + 8 * i;
      bf16_t* dst = (!DUMMY || jj < WINS) ? sW + 16 * jj * HK : ldsd;
      if constexpr (BUF) {
        buf_lds16(p.w, 2 * p.N * p.K, dst, wbo[i] + 2u * (unsigned)(wk + PAR * HK));
      } else {
        const void* src = woff[i] >= 0 ? (const void*)(p.w + woff[i] + wk + PAR * HK) : (const void*)g_conv_zero_page;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)dst, 16, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int jj = wave + 8 * i;
      bf16_t* dst = (!DUMMY || jj < XINS) ? sX + 16 * jj * HK : ldsd;
      if constexpr (BUF) {
        buf_lds16(p.x, 2 * p.B * p.H * p.W * p.Cin, dst, xbo[i] + 2u * (unsigned)(wc + PAR * HK));
      } else {
        const void* src = xoff[i] >= 0 ? (const void*)(p.x + xoff[i] + wc + PAR * HK) : (const void*)g_conv_zero_page;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)dst, 16, 0, 0);
      }
    }
    if constexpr (PAR == 1) {       // both halves of this K tile issued: next tile
      wk += BK;
      wc += BK;
      if (wc == p.Cin) {
        wc = 0;
        if (++ws == p.kw) { ws = 0; ++wr; }
        set_tap();
      }
    }
  };
  auto bar = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: halves 0..PD-1 in flight (H is even and >= 2), half 0 landed for every wave before any read
  issue(IC<0>(), IC<0>());
  issue(IC<1>(), IC<1>());
  if (2 < H) {
    issue(IC<2>(), IC<0>());
    if constexpr (PD == 4) {
      issue(IC<3>(), IC<1>());     // H even: 2 < H -> half 3 exists
      wait_vmcnt<3 * LPH>();
    } else {
      wait_vmcnt<2 * LPH>();
    }
  } else {
    wait_vmcnt<LPH>();
  }
  bar();
  if (grp1) bar();   // group 1 runs one barrier behind group 0

  // phase P (K = P % U static): reads slot K % HS, issues half P + PD into slot (K + PD) % HS
  auto phase = [&](auto k_c, int P) __attribute__((always_inline)) {
    constexpr int K = decltype(k_c)::value;
    const bf16_t* sW = half_slot<K % HS>(hs0, hs1, hs2, hs3, hs4, hs5);
    const bf16_t* sX = sW + BN * HK;
    uint4 af[TN], bfr[TM];
#pragma unroll
    for (int a = 0; a < TN; ++a) {
      const int row = wn * (BN / WN) + a * 16 + l16;
      af[a] = ld16(&sW[row * HK + ((g ^ half_swz(row)) << 3)]);
    }
#pragma unroll
    for (int b = 0; b < TM; ++b) {
      const int row = wm * (BM / WM) + b * 16 + l16;
      bfr[b] = ld16(&sX[row * HK + ((g ^ half_swz(row)) << 3)]);
    }
    if (P + PD < H) {
      issue(IC<(K + PD) % HS>(), IC<(K + PD) & 1>());
      wait_vmcnt<(PD - 1) * LPH>();   // half P+1 landed (P+2 .. P+PD may be in flight)
    } else if (P + PD - 1 < H) {
      wait_vmcnt<(PD - 2) * LPH>();
    } else if (PD == 4 && P + 2 < H) {
      wait_vmcnt<LPH>();
    } else {
      wait_vmcnt<0>();
    }
    if constexpr (PD == 4) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // slot reads retired (WAR)
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
      for (int b = 0; b < TM; ++b) acc[a][b] = mma16<EL>(af[a], bfr[b], acc[a][b]);
    __builtin_amdgcn_s_setprio(0);
    bar();
  };
  for (int P = 0; P < H; P += U) {   // block-uniform guards, no early exits (see conv_glds_kernel)
    phase(IC<0>(), P);
    phase(IC<1>(), P + 1);           // H is even: a round always has its first two phases
    if (P + 2 < H) phase(IC<2>(), P + 2);
    if (P + 3 < H) phase(IC<3>(), P + 3);
    if (P + 4 < H) phase(IC<4>(), P + 4);
    if (P + 5 < H) phase(IC<5>(), P + 5);
    if constexpr (U > 6) {
      if (P + 6 < H) phase(IC<6>(), P + 6);
      if (P + 7 < H) phase(IC<7>(), P + 7);
      if (P + 8 < H) phase(IC<8>(), P + 8);
      if (P + 9 < H) phase(IC<9>(), P + 9);
    }
  }
  if (!grp1) bar();

  if constexpr (!SPLIT) {
    epilogue_lds<BN, BM, WN, WM, NT, SLOT / 2, EL>(p, acc, reinterpret_cast<float*>(hs0), m0, n0);
  } else {
#pragma unroll
    for (int b = 0; b < TM; ++b) {
      const int m = m0 + wm * (BM / WM) + b * 16 + l16;
      if (m >= p.M) continue;
#pragma unroll
      for (int a = 0; a < TN; ++a) {
        const int n = n0 + wn * (BN / WN) + a * 16 + 4 * g;
        if (n < p.N)
          *reinterpret_cast<float4*>(p.ws + ((size_t)split_idx * p.M + m) * p.N + n) =
              make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
      }
    }
  }
}

// X-in-registers variant (cfg 32 + i), for the big-M SD level-0 convs (M = 32768 pixels at
// lock-step batch 8).  The register-staged 160x128 tile is LDS-bound (profiles/pmc_r2_conv.md:
// per K tile a CU moves 8 waves x (18 ds_read_b128 + 9 ds_write_b128) through LDS against 2 x 640
// MFMA cycles per SIMD; 35 % of wave cycles issue-stalled, 32 % MFMA busy).  Here the activation
// operand never touches LDS: the 16x16x32 MFMA B fragment is "lane = pixel l16, 8 consecutive k at
// chunk g" = 16 contiguous channel bytes of one NHWC pixel, so every lane loads its fragments
// straight from global memory into registers (global_load_dwordx4, NS-1 K tiles ahead).  Only the
// weight tile goes through an NS-deep LDS-DMA ring shared by all WAVES waves, each wave owning
// TMW x 16 pixels x all BN channels.  Per K tile and CU (BN 160, 8 waves, TMW 2): 160 ds_read_b128
// + 24 KB of DMA writes against the same 2 x 640 MFMA cycles per SIMD - about half the LDS
// traffic of the register-staged tile, and no VGPR->LDS store transfers at all.  Split-K writes the
// K range's fp32 slab (summed in slab order by splitk_reduce_kernel).  NS = 2 (tile i+1
// in flight during tile i): a third X register set spills at TMW = 2.  Per output the
// MFMA sequence (k-tiles ascending, two k32 halves each) is that of the other non-split kernels,
// so results are bitwise identical to them at every split.  bf16, no norm prologue / dual source.
template <int BN, int WAVES, int TMW, int NS>
__global__ void __launch_bounds__(64 * WAVES, 1) conv_xreg_kernel(ConvArgs p) {
  constexpr int EL = 0, BK = 64, NT = 64 * WAVES;
  constexpr int BM = WAVES * TMW * 16;
  constexpr int TN = BN / 16;
  constexpr int WINS = BN / 8;                     // W DMA wave-instructions per stage (8 rows each)
  constexpr int WCH = (WINS + WAVES - 1) / WAVES;  // per wave; the remainder target a dummy buffer
  constexpr int LPT = WCH + 2 * TMW;               // vmcnt units per K tile per wave
  constexpr int STAGE = BN * BK;                   // bf16 elements per W stage
  constexpr int OROW = BN + 4;                     // epilogue fp32 staging row (epilogue_lds)
  constexpr int EPI_ROWS = 64;
  constexpr int S0 = STAGE > EPI_ROWS * OROW * 2 ? STAGE : EPI_ROWS * OROW * 2;
  static_assert(BN % 16 == 0 && NS >= 2 && NS <= 3, "tile");
  static_assert((size_t)(S0 + (NS - 1) * STAGE + 512) * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) bf16_t lds0[S0];
  __shared__ __attribute__((aligned(16))) bf16_t lds1[STAGE];
  __shared__ __attribute__((aligned(16))) bf16_t lds2[NS > 2 ? STAGE : 8];
  __shared__ __attribute__((aligned(16))) bf16_t ldsd[512];   // dummy DMA target: zeros, never read

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  int split_idx, n0, m0;
  tile_coords(p, BN, BM, split_idx, n0, m0);
  const bool split = p.nsplit > 1;   // split-K: fp32 slab of this K range, summed by splitk_reduce
  const int kt0 = split ? split_idx * p.kt_per_split : 0;
  const int nk = (split ? min(p.ktiles, kt0 + p.kt_per_split) : p.ktiles) - kt0;
  typedef __attribute__((address_space(1))) const void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  const bf16_t* zp = reinterpret_cast<const bf16_t*>(g_conv_zero_page);

  // W tile: DMA instruction j = wave + WAVES * i fills stage rows 8j .. 8j+7, lane-linear; the
  // source carries the XOR chunk swizzle (row r, position q holds logical chunk q ^ (r & 7)).
  const int pos = lane & 7;
  int woff[WCH];
#pragma unroll
  for (int i = 0; i < WCH; ++i) {
    const int j = wave + WAVES * i;
    const int row = 8 * j + (lane >> 3);
    woff[i] = (j < WINS && n0 + row < p.N) ? (n0 + row) * p.K + ((pos ^ (row & 7)) << 3) : -1;
  }
  // X: this lane's pixel in each of the wave's TMW fragments
  int xb[TMW], xho[TMW], xwo[TMW];
  bool xok[TMW];
  const int hw = p.Ho * p.Wo;
#pragma unroll
  for (int f = 0; f < TMW; ++f) {
    const int m = m0 + (wave * TMW + f) * 16 + l16;
    xok[f] = m < p.M;
    const int mm = xok[f] ? m : 0;
    xb[f] = mm / hw;
    const int rem = mm - xb[f] * hw;
    xho[f] = (rem / p.Wo) * p.stride - p.pad;
    xwo[f] = (rem % p.Wo) * p.stride - p.padw;
  }
  int wk = kt0 * BK, wc = wk % p.Cin, wr = (wk / p.Cin) / p.kw, ws = (wk / p.Cin) % p.kw;
  int xoff[TMW];
  auto set_tap = [&]() {
#pragma unroll
    for (int f = 0; f < TMW; ++f) {
      int hi = xho[f] + wr, wi = xwo[f] + ws;
      const bool ok = xok[f] && hi >= 0 && hi < p.Hl && wi >= 0 && wi < p.Wl;
      if (p.upsample) { hi >>= 1; wi >>= 1; }
      xoff[f] = ok ? ((xb[f] * p.H + hi) * p.W + wi) * p.Cin + g * 8 : -1;
    }
  };
  set_tap();

  uint4 xr[NS][TMW][2];
  auto issue = [&](auto stage_c) {
    constexpr int S = decltype(stage_c)::value;
#pragma unroll
    for (int f = 0; f < TMW; ++f)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) xr[S][f][kk] = ld16(xoff[f] >= 0 ? p.x + xoff[f] + wc + kk * 32 : zp);
    bf16_t* sW = ring_stage<S>(lds0, lds1, lds2, lds2);
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int j = wave + WAVES * i;
      const void* src = woff[i] >= 0 ? (const void*)(p.w + woff[i] + wk) : (const void*)g_conv_zero_page;
      bf16_t* dst = j < WINS ? sW + 8 * j * BK : ldsd;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)dst, 16, 0, 0);
    }
    wk += BK;
    wc += BK;
    if (wc == p.Cin) {
      wc = 0;
      if (++ws == p.kw) { ws = 0; ++wr; }
      set_tap();
    }
  };

  f32x4 acc[TN][TMW];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int f = 0; f < TMW; ++f) acc[a][f] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (0 < nk) issue(IC<0>());
  if (NS > 2 && 1 < nk) issue(IC<1>());
  auto step = [&](auto stage_c, int i) __attribute__((always_inline)) {
    constexpr int S = decltype(stage_c)::value;
    if (i + NS - 2 < nk) wait_vmcnt<(NS - 2) * LPT>();   // tile i (X regs + W DMA) landed
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();                       // every wave's W DMA of tile i is visible
    if (i + NS - 1 < nk) issue(IC<(S + NS - 1) % NS>());  // refill the stage / set read at i-1
    const bf16_t* sW = ring_stage<S>(lds0, lds1, lds2, lds2);
    // both k32 halves of one 16-channel row block back to back on each accumulator: the
    // per-accumulator MFMA order is unchanged (k ascending), and the accumulators stay in place
    // (two separate k-half loops made hipcc ping-pong every accumulator through a second
    // register set and spill at TMW = 2)
    if constexpr (NT == 512) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < TN; ++a) {
      const int row = a * 16 + l16;
      const uint4 a0 = ld16(&sW[row * BK + ((g ^ (row & 7)) << 3)]);
      const uint4 a1 = ld16(&sW[row * BK + (((4 + g) ^ (row & 7)) << 3)]);
#pragma unroll
      for (int f = 0; f < TMW; ++f) {
        const f32x4 t = mma16<EL>(a0, xr[S][f][0], acc[a][f]);
        acc[a][f] = mma16<EL>(a1, xr[S][f][1], t);
      }
    }
    if constexpr (NT == 512) __builtin_amdgcn_s_setprio(0);
  };
  for (int i = 0; i < nk; i += NS) {   // guards, not early exits (see conv_glds_kernel)
    step(IC<0>(), i);
    if (i + 1 < nk) step(IC<1>(), i + 1);
    if constexpr (NS > 2) {
      if (i + 2 < nk) step(IC<2 % NS>(), i + 2);
    }
  }
  if (split) {
#pragma unroll
    for (int f = 0; f < TMW; ++f) {
      const int m = m0 + (wave * TMW + f) * 16 + l16;
      if (m >= p.M) continue;
#pragma unroll
      for (int a = 0; a < TN; ++a) {
        const int n = n0 + a * 16 + 4 * g;
        if (n < p.N)
          *reinterpret_cast<float4*>(p.ws + ((size_t)split_idx * p.M + m) * p.N + n) =
              make_float4(acc[a][f][0], acc[a][f][1], acc[a][f][2], acc[a][f][3]);
      }
    }
    return;
  }
  epilogue_lds<BN, BM, 1, WAVES, NT, EPI_ROWS * OROW, EL>(p, acc, reinterpret_cast<float*>(lds0), m0, n0);
}

// Persistent LDS-DMA variant for short-K GEMMs / 1x1 convs (K = 320..1280 on the UNet: the
// transformer projections, GEGLU proj).  With 5-20 K-tiles per output tile, a one-tile-per-block
// kernel spends most of its life in prologue latency and epilogue; here a grid of ~one block
// per CU walks the flattened (tile, k-tile) sequence of its tiles through ONE NS-deep DMA ring,
// so the next tile's operands are in flight while the current tile's epilogue runs.  The bias
// rides the ring too (one DMA of BN channels with each tile's last k-tile: an ordinary global
// load while LDS-DMA is in flight makes hipcc drain the ring).  Tile order: block b takes
// logical tiles b, b + G, ... through the same bijective XCD remap as the other kernels (G is a
// multiple of 8, so a block's tiles stay on its XCD).  No split-K, no norm prologue; temb /
// residual (rare on short-K shapes) are read directly in the epilogue.
template <int BN, int BM, int WN, int WM, int NS>
__global__ void __launch_bounds__(64 * WN * WM, 1) conv_persist_kernel(ConvArgs p) {
  constexpr int EL = 0;
  constexpr int BK = 64;
  constexpr int NT = 64 * WN * WM;
  constexpr int RPI = NT / 8;
  static_assert((BN * 8) % NT == 0 && (BM * 8) % NT == 0, "whole DMA rounds per tile");
  static_assert(BN % 8 == 0 && BN / 8 <= 64, "bias DMA: one wave, 16 B per lane");
  constexpr int TN = BN / WN / 16, TM = BM / WM / 16;
  constexpr int WCH = BN * 8 / NT, XCH = BM * 8 / NT;
  constexpr int LPT = WCH + XCH;             // vmcnt units per k-tile per wave (bias DMA extra)
  // W and X(+bias slot) of each stage are separate LDS objects: shallow address chains keep every
  // ds_read's alias scope (a scope-less read waits for all LDS-DMA in flight)
  constexpr int XST = BM * BK + BN;
  static_assert(NS >= 2 && NS <= 4, "ring depth");
  __shared__ __attribute__((aligned(16))) bf16_t w0[BN * BK];
  __shared__ __attribute__((aligned(16))) bf16_t w1[BN * BK];
  __shared__ __attribute__((aligned(16))) bf16_t w2[NS > 2 ? BN * BK : 8];
  __shared__ __attribute__((aligned(16))) bf16_t w3[NS > 3 ? BN * BK : 8];
  __shared__ __attribute__((aligned(16))) bf16_t x0[XST];
  __shared__ __attribute__((aligned(16))) bf16_t x1[XST];
  __shared__ __attribute__((aligned(16))) bf16_t x2[NS > 2 ? XST : 8];
  __shared__ __attribute__((aligned(16))) bf16_t x3[NS > 3 ? XST : 8];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WM, wm = wave % WM;
  const int g = lane >> 4, l16 = lane & 15;
  const int nk = p.ktiles, total = p.tiles_total, G = gridDim.x;
  const int mine = (total - (int)blockIdx.x + G - 1) / G;
  const int J = mine * nk;
  const int tiles_m = total / p.tiles_n;
  auto origin = [&](int k, int& n0, int& m0) {
    const int lin = xcd_remap((int)blockIdx.x + k * G, total);
    if (p.m_fastest) {
      m0 = (lin % tiles_m) * BM;
      n0 = (lin / tiles_m) * BN;
    } else {
      n0 = (lin % p.tiles_n) * BN;
      m0 = (lin / p.tiles_n) * BM;
    }
  };

  const int pos = tid & 7;
  int wrow[WCH], wcc[WCH], xcc[XCH];
#pragma unroll
  for (int i = 0; i < WCH; ++i) {
    wrow[i] = (tid >> 3) + RPI * i;
    wcc[i] = pos ^ (wrow[i] & 7);
  }
#pragma unroll
  for (int i = 0; i < XCH; ++i) xcc[i] = pos ^ (((tid >> 3) + RPI * i) & 7);
  typedef __attribute__((address_space(1))) const void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;

  // ---- issue side: geometry of the tile whose k-tiles are being fetched
  int xb[XCH], xho[XCH], xwo[XCH], xoff[XCH], woff[WCH];
  bool xok[XCH];
  int wk = 0, wc = 0, wr = 0, ws = 0, ikt = 0, itile = 0, in0 = 0;
  auto set_tap = [&]() {
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      int hi = xho[i] + wr, wi = xwo[i] + ws;
      const bool ok = xok[i] && hi >= 0 && hi < p.Hl && wi >= 0 && wi < p.Wl;
      if (p.upsample) { hi >>= 1; wi >>= 1; }
      xoff[i] = ok ? ((xb[i] * p.H + hi) * p.W + wi) * p.Cin + xcc[i] * 8 : -1;
    }
  };
  // The issued tile's row geometry is recomputed on EVERY issue (same values within a tile):
  // a branch around it (only at a tile's first k-tile) made hipcc's waitcnt pass drain the ring
  // before every k-tile's ds_reads.
  auto tile_geometry = [&](int k) {
    int n0, m0;
    origin(k, n0, m0);
    in0 = n0;
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int n = n0 + wrow[i];
      woff[i] = n < p.N ? n * p.K + wcc[i] * 8 : -1;
    }
    const int hw = p.Ho * p.Wo;
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int m = m0 + (tid >> 3) + RPI * i;
      xok[i] = m < p.M;
      const int mm = xok[i] ? m : 0;
      xb[i] = mm / hw;
      const int rem = mm - xb[i] * hw;
      xho[i] = (rem / p.Wo) * p.stride - p.pad;
      xwo[i] = (rem % p.Wo) * p.stride - p.padw;
    }
  };
  auto issue = [&](auto stage_c) {
    tile_geometry(itile);
    if (ikt == 0) { wk = 0; wc = 0; wr = 0; ws = 0; }
    set_tap();
    bf16_t* sW = ring_stage<decltype(stage_c)::value>(w0, w1, w2, w3);
    bf16_t* sX = ring_stage<decltype(stage_c)::value>(x0, x1, x2, x3);
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const void* src = woff[i] >= 0 ? (const void*)(p.w + woff[i] + wk) : (const void*)g_conv_zero_page;
      dma16(src, sW + ((wave * 8) + RPI * i) * BK);
    }
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const void* src = xoff[i] >= 0 ? (const void*)(p.x + xoff[i] + wc) : (const void*)g_conv_zero_page;
      dma16(src, sX + ((wave * 8) + RPI * i) * BK);
    }
    if (ikt == nk - 1 && wave == 0) {     // bias of this tile into the stage's bias slot
      const int n = in0 + lane * 8;
      const void* src = (p.bias && n < p.N) ? (const void*)(p.bias + n) : (const void*)g_conv_zero_page;
      // lane l writes slot + 16 l: only the BN/8 lanes of the slot may be active (EXEC mask)
      if (lane < BN / 8) dma16(src, sX + BM * BK);
    }
    wk += BK;
    wc += BK;
    if (wc == p.Cin) {
      wc = 0;
      if (++ws == p.kw) { ws = 0; ++wr; }
      set_tap();
    }
    if (++ikt == nk) { ikt = 0; ++itile; }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (0 < J) issue(IC<0>());
  if (NS > 2 && 1 < J) issue(IC<1>());
  if (NS > 3 && 2 < J) issue(IC<2>());

  int ckt = 0, ctile = 0;
  const int hw = p.Ho * p.Wo;
  auto step = [&](auto stage_c, int j) __attribute__((always_inline)) {
    constexpr int S = decltype(stage_c)::value;
    // stage j has landed once at most (NS-2)*LPT younger VM ops are outstanding (the bias DMA
    // and epilogue stores only make this wait longer, never shorter)
    if (j + NS - 2 < J) wait_vmcnt<(NS - 2) * LPT>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (j + NS - 1 < J) issue(IC<(S + NS - 1) % NS>());
    const bf16_t* sW = ring_stage<S>(w0, w1, w2, w3);
    const bf16_t* sX = ring_stage<S>(x0, x1, x2, x3);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      uint4 af[TN], bfr[TM];
#pragma unroll
      for (int a = 0; a < TN; ++a) {
        const int row = wn * (BN / WN) + a * 16 + l16;
        af[a] = ld16(&sW[row * BK + (((kk * 4 + g) ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int b = 0; b < TM; ++b) {
        const int row = wm * (BM / WM) + b * 16 + l16;
        bfr[b] = ld16(&sX[row * BK + (((kk * 4 + g) ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = mma16<EL>(af[a], bfr[b], acc[a][b]);
    }
    if (++ckt < nk) return;
    // ---- epilogue of the finished tile (the ring keeps fetching the next one meanwhile)
    ckt = 0;
    int n0, m0;
    origin(ctile++, n0, m0);
    const bf16_t* sB = sX + BM * BK;   // this stage's bias slot (issued with this k-tile)
#pragma unroll
    for (int b = 0; b < TM; ++b) {
      const int m = m0 + wm * (BM / WM) + b * 16 + l16;
#pragma unroll
      for (int a = 0; a < TN; ++a) {
        const int nl = wn * (BN / WN) + a * 16 + 4 * g, n = n0 + nl;
        float v0 = acc[a][b][0], v1 = acc[a][b][1], v2 = acc[a][b][2], v3 = acc[a][b][3];
        acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
        if (m >= p.M || n >= p.N) continue;
        if (p.rowstat) ln_fold4(p, m, n, v0, v1, v2, v3);
        const uint2 bv = *reinterpret_cast<const uint2*>(&sB[nl]);
        v0 += lo16<EL>(bv.x); v1 += hi16<EL>(bv.x);
        v2 += lo16<EL>(bv.y); v3 += hi16<EL>(bv.y);
        if (p.temb) {
          const uint2 tv = *reinterpret_cast<const uint2*>(p.temb + (size_t)(m / hw) * p.temb_ld + n);
          v0 += lo16<EL>(tv.x); v1 += hi16<EL>(tv.x);
          v2 += lo16<EL>(tv.y); v3 += hi16<EL>(tv.y);
        }
        if (p.res) {
          const uint2 rv = *reinterpret_cast<const uint2*>(p.res + (size_t)m * p.N + n);
          v0 += lo16<EL>(rv.x); v1 += hi16<EL>(rv.x);
          v2 += lo16<EL>(rv.y); v3 += hi16<EL>(rv.y);
        }
        if (p.act) { v0 = act_f(p.act, v0); v1 = act_f(p.act, v1); v2 = act_f(p.act, v2); v3 = act_f(p.act, v3); }
        uint2 o;
        o.x = enc16<EL>(v0) | (enc16<EL>(v1) << 16);
        o.y = enc16<EL>(v2) | (enc16<EL>(v3) << 16);
        *reinterpret_cast<uint2*>(p.out + (size_t)m * p.N + n) = o;
      }
    }
  };
  for (int j = 0; j < J; j += NS) {   // guards, not early exits (see conv_glds_kernel)
    step(IC<0>(), j);
    if (j + 1 < J) step(IC<1>(), j + 1);
    if constexpr (NS > 2) {
      if (j + 2 < J) step(IC<2 % NS>(), j + 2);
    }
    if constexpr (NS > 3) {
      if (j + 3 < J) step(IC<3 % NS>(), j + 3);
    }
  }
}

// Ordered split-K reduction + epilogue: out[m, n..n+7] from S fp32 slabs.
template <int EL>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(ConvArgs p, int S) {
  if (p.geglu) {   // 16 channels (value 8 | gate 8) -> 8 GEGLU outputs, same rounding as epilogue_lds
    const long tot = (long)p.M * (p.N / 16);
    for (long i = blockIdx.x * 256L + threadIdx.x; i < tot; i += (long)gridDim.x * 256) {
      const int m = (int)(i / (p.N / 16));
      const int n = (int)(i - (long)m * (p.N / 16)) * 16;
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 a = reinterpret_cast<const float4*>(p.ws + (size_t)m * p.N + n)[q];
        v[4 * q] = a.x; v[4 * q + 1] = a.y; v[4 * q + 2] = a.z; v[4 * q + 3] = a.w;
      }
      for (int s = 1; s < S; ++s) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 a = reinterpret_cast<const float4*>(p.ws + ((size_t)s * p.M + m) * p.N + n)[q];
          v[4 * q] += a.x; v[4 * q + 1] += a.y; v[4 * q + 2] += a.z; v[4 * q + 3] += a.w;
        }
      }
      if (p.rowstat) {
        float a[8], b[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) { a[e] = v[e]; b[e] = v[8 + e]; }
        ln_fold8(p, m, n, a);
        ln_fold8(p, m, n + 8, b);
#pragma unroll
        for (int e = 0; e < 8; ++e) { v[e] = a[e]; v[8 + e] = b[e]; }
      }
      if (p.bias) {
        float t[8];
        unpack8e<EL>(ld16(p.bias + n), t);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += t[e];
        unpack8e<EL>(ld16(p.bias + n + 8), t);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[8 + e] += t[e];
      }
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = dec16<EL>(enc16<EL>(v[e])) * gelu_f(dec16<EL>(enc16<EL>(v[8 + e])));
      st16(p.out + (size_t)m * (p.N >> 1) + (n >> 1), pack8e<EL>(o));
    }
    return;
  }
  const long total = (long)p.M * (p.N / 8);
  const int hw = p.Ho * p.Wo;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int m = (int)(i / (p.N / 8));
    const int n = (int)(i - (long)m * (p.N / 8)) * 8;
    float v[8];
    if (S <= 8) {
      // every slab's loads issued before the first add (the per-slab dependent loop exposed one
      // load latency per slab); the adds then run in slab order - bitwise the same sum
      float4 a[8], b[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        if (s < S) {
          const float4* src = reinterpret_cast<const float4*>(p.ws + ((size_t)s * p.M + m) * p.N + n);
          a[s] = src[0];
          b[s] = src[1];
        }
      }
      v[0] = a[0].x; v[1] = a[0].y; v[2] = a[0].z; v[3] = a[0].w;
      v[4] = b[0].x; v[5] = b[0].y; v[6] = b[0].z; v[7] = b[0].w;
#pragma unroll
      for (int s = 1; s < 8; ++s) {
        if (s < S) {
          v[0] += a[s].x; v[1] += a[s].y; v[2] += a[s].z; v[3] += a[s].w;
          v[4] += b[s].x; v[5] += b[s].y; v[6] += b[s].z; v[7] += b[s].w;
        }
      }
    } else {
      {
        const float4* src = reinterpret_cast<const float4*>(p.ws + (size_t)m * p.N + n);
        const float4 a = src[0], b = src[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      }
      for (int s = 1; s < S; ++s) {
        const float4* src = reinterpret_cast<const float4*>(p.ws + ((size_t)s * p.M + m) * p.N + n);
        const float4 a = src[0], b = src[1];
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
      }
    }
    float t[8];
    if (p.rowstat) ln_fold8(p, m, n, v);
    if (p.bias) {
      unpack8e<EL>(ld16(p.bias + n), t);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += t[e];
    }
    if (p.temb) {
      unpack8e<EL>(ld16(p.temb + (size_t)(m / hw) * p.temb_ld + n), t);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += t[e];
    }
    if (p.res) {
      unpack8e<EL>(ld16(p.res + (size_t)m * p.N + n), t);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += t[e];
    }
    if (p.act) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = act_f(p.act, v[e]);
    }
    st16(p.out + (size_t)m * p.N + n, pack8e<EL>(v));
  }
}

// ---------------------------------------------------------------------------------------------
// Tile configurations (BN channels x BM pixels, WN x WM waves) and the plan.  The plan is a
// pure function of the shape (pinned table for the model shapes, cost model otherwise), so
// every GPU runs the same reduction order for the same task (determinism).
struct TileCfg {
  int bn, bm, wn, wm, minw;
};
static const TileCfg kCfgs[] = {
    {128, 128, 2, 2, 2}, {64, 128, 2, 2, 2}, {128, 64, 2, 2, 2}, {64, 64, 2, 2, 2}, {160, 64, 2, 2, 2},
    {160, 128, 2, 2, 1}, {320, 32, 4, 1, 1}, {256, 64, 4, 1, 1}, {128, 256, 2, 2, 1}, {64, 256, 1, 4, 1},
};
static const int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);

struct ConvPlan {
  int cfg, split, kt_per_split;
};

// Pinned choices for shapes measured on MI355X (M, N, K) -> (cfg, split).  Filled by
// scripts/autotune_conv.py; entries not listed fall back to the cost model.
struct PinnedPlan {
  int M, N, K, cfg, split;
};
#include "conv_plans.inc"

// Optional run-time plan table (A/B of autotuned tables without a rebuild): ARB_CONV_PLANS names
// a file in conv_plans.inc format ("{M, N, K, cfg, split},"); its entries take precedence.
static const std::vector<PinnedPlan>& env_plans() {
  static const std::vector<PinnedPlan> plans = [] {
    std::vector<PinnedPlan> v;
    const char* path = std::getenv("ARB_CONV_PLANS");
    if (path == nullptr || path[0] == 0) return v;
    FILE* f = std::fopen(path, "r");
    if (f == nullptr) {
      std::fprintf(stderr, "[arbius] ARB_CONV_PLANS=%s cannot be read: the built-in table is used\n", path);
      return v;
    }
    char line[256];
    while (std::fgets(line, sizeof line, f)) {
      PinnedPlan pp;
      if (std::sscanf(line, " {%d, %d, %d, %d, %d}", &pp.M, &pp.N, &pp.K, &pp.cfg, &pp.split) == 5) v.push_back(pp);
    }
    std::fclose(f);
    return v;
  }();
  return plans;
}

// cfg ids: 0..9 LDS-DMA 4-wave, 10..19 register-staged 4-wave, 20..23 8-wave LDS-DMA 2-stage,
// 24..27 persistent short-K, 28..31 8-wave LDS-DMA 3-stage ring (two K-tiles in flight),
// 32..35 8-wave X-in-registers (weights-only LDS-DMA ring), 36..41 8-wave staggered two-group ring,
// 42..45 the same on K-half slots, 46..47 W-stationary short-K GEMM (conv_sk.inc)
static inline bool is_persist(int cfg) { return cfg >= 24 && cfg < 28; }
// 32..35 X-in-registers 8-wave tiles (weights through an LDS-DMA ring, activations straight to VGPRs)
static inline bool is_xreg(int cfg) { return cfg >= 32 && cfg < 36; }

static ConvPlan conv_plan(int M, int N, int ktiles, int want_cfg, int want_split) {
  const int K = ktiles * 64;
  if (want_cfg >= 0 && (want_cfg < 2 * kNumCfgs || (want_cfg >= 20 && want_cfg < 48))) {
    if (is_persist(want_cfg)) return {want_cfg, 1, ktiles};   // persistent: no split-K
    int split = want_split < 1 ? 1 : want_split;
    if (split > ktiles) split = ktiles;
    const int per = (ktiles + split - 1) / split;
    return {want_cfg, (ktiles + per - 1) / per, per};
  }
  for (const PinnedPlan& pp : env_plans()) {
    if (pp.M == M && pp.N == N && pp.K == K) {
      const int per = (ktiles + pp.split - 1) / pp.split;
      return {pp.cfg, is_persist(pp.cfg) ? 1 : (ktiles + per - 1) / per, is_persist(pp.cfg) ? ktiles : per};
    }
  }
  for (const PinnedPlan& pp : kPinnedPlans) {
    if (pp.M == M && pp.N == N && pp.K == K) {
      const int per = (ktiles + pp.split - 1) / pp.split;
      return {pp.cfg, (ktiles + per - 1) / per, per};
    }
  }
  // cost model: waves of resident workgroups x per-workgroup work / tile efficiency
  double best = 1e30;
  ConvPlan bp = {3, 1, ktiles};
  const int splits[] = {1, 2, 3, 4, 6, 8};
  for (int c = 0; c < kNumCfgs; ++c) {
    const TileCfg& tc = kCfgs[c];
    if (tc.bn > 2 * N && tc.bn > 64) continue;
    const long tiles = (long)((N + tc.bn - 1) / tc.bn) * ((M + tc.bm - 1) / tc.bm);
    const int lds = 2 * (tc.bn + tc.bm) * 128;
    int occ = 163840 / lds;
    if (occ > tc.minw) occ = tc.minw;
    if (occ < 1) occ = 1;
    const double eff = fmin(1.0, (double)tc.bn * tc.bm / (tc.bn + tc.bm) / 64.0);
    for (int si = 0; si < 6; ++si) {
      const int sp = splits[si];
      if (sp > 1 && sp > ktiles / 2) break;
      const int per = (ktiles + sp - 1) / sp;
      const long wgs = tiles * sp;
      const long waves = (wgs + 256L * occ - 1) / (256L * occ);
      // seconds: each resident workgroup slot runs at (45% of 2 PF) * eff / slots
      const double slot_rate = 2.0e15 * 0.45 * eff / (256.0 * occ);
      double t = (double)waves * (2.0 * tc.bn * tc.bm * per * 64.0) / slot_rate;
      if (sp > 1) t += (double)M * N * sp * 8.0 / 4.0e12 + 3.0e-6;  // fp32 slab write+read + reduce launch
      if (t < best) {
        best = t;
        bp = {c, (ktiles + per - 1) / per, per};
      }
    }
  }
  bp.cfg += kNumCfgs;  // register-staged variant: faster than the LDS-DMA ring on every tuned shape
  return bp;
}

// Split-K ticket regions.  A pool of zero-initialised int counters per device, allocated once
// (eagerly, never during stream capture).  Every launch recorded into a hipGraph gets its OWN
// region (graph nodes may replay concurrently on different streams); eager launches share one
// region per stream (same-stream kernels are serialised).  Reducers re-arm counters to 0.
struct CounterPool {
  int* base = nullptr;
  size_t cap = 0, used = 0;
  std::unordered_map<hipStream_t, int*> eager;
};
static std::mutex g_cnt_mu;
static std::unordered_map<int, CounterPool> g_cnt_pools;
static constexpr size_t kCounterPoolInts = size_t(8) << 20;   // 32 MB per device
static constexpr int kEagerRegionInts = 1 << 16;

static int* split_counters(hipStream_t s, int tiles) {
  std::lock_guard<std::mutex> lk(g_cnt_mu);
  int dev = 0;
  hipGetDevice(&dev);
  CounterPool& pool = g_cnt_pools[dev];
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  hipStreamIsCapturing(s, &st);
  const bool capturing = st != hipStreamCaptureStatusNone;
  if (pool.base == nullptr) {
    if (capturing) return nullptr;   // no allocation inside a capture: use the reduce kernel
    if (hipMalloc(&pool.base, kCounterPoolInts * sizeof(int)) != hipSuccess) {
      pool.base = nullptr;
      return nullptr;
    }
    hipMemset(pool.base, 0, kCounterPoolInts * sizeof(int));
    hipDeviceSynchronize();
    pool.cap = kCounterPoolInts;
  }
  if (capturing) {
    if (pool.used + tiles > pool.cap) return nullptr;
    int* r = pool.base + pool.used;
    pool.used += ((size_t)tiles + 63) / 64 * 64;
    return r;
  }
  if (tiles > kEagerRegionInts) return nullptr;
  auto it = pool.eager.find(s);
  if (it != pool.eager.end()) return it->second;
  if (pool.used + kEagerRegionInts > pool.cap) return nullptr;
  int* r = pool.base + pool.used;
  pool.used += kEagerRegionInts;
  pool.eager[s] = r;
  return r;
}

int* arb_tickets(hipStream_t s, int n) { return split_counters(s, n); }

static bool splitk_inlaunch() {
  static const bool on = [] {
    const char* e = std::getenv("ARB_SPLITK_INLAUNCH");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

static size_t slab_bytes(int split, int M, int N) {
  return ((size_t)split * M * N * sizeof(float) + 255) / 256 * 256;
}

// k = 1 / 3: square kernel, padding `pad` on both axes.  k = 31: a 3x1 kernel
// (padding pad x 0) - the (3,1,1) temporal Conv3d of the UNet3D run over the
// frame-major [B, F, H*W, C] activation viewed as an F x HW image.
static void conv_geom(ConvArgs& a, int B, int H, int W, int Cin, int Cout, int k, int pad, int upsample,
                      int stride) {
  const int kh = k == 31 ? 3 : k, kw = k == 31 ? 1 : k, padw = k == 31 ? 0 : pad;
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.Cx = Cin;
  a.Hl = upsample ? 2 * H : H; a.Wl = upsample ? 2 * W : W;
  a.Ho = (a.Hl + 2 * pad - kh) / stride + 1; a.Wo = (a.Wl + 2 * padw - kw) / stride + 1;
  a.N = Cout; a.K = kh * kw * Cin; a.M = B * a.Ho * a.Wo;
  a.kw = kw; a.pad = pad; a.padw = padw; a.stride = stride; a.upsample = upsample;
  a.ktiles = a.K / 64; a.kt_per_split = a.ktiles;
}

ARB_API size_t arb_conv2d_workspace(int B, int H, int W, int Cin, int Cout, int k, int pad, int upsample, int stride,
                                    int cfg, int split) {
  ConvArgs a;
  conv_geom(a, B, H, W, Cin, Cout, k, pad, upsample, stride);
  const ConvPlan pl = conv_plan(a.M, a.N, a.ktiles, cfg, split);
  return pl.split > 1 ? slab_bytes(pl.split, a.M, a.N) : 0;
}

// Buffer-resource LDS-DMA addressing (conv_glds_kernel / conv_stag2_kernel BUF; bitwise equal): default
// on; ARB_DMA_BUF=0 / arb_set_stag2_buf(0) -> the global_load_lds + zero-page form.  Used when W and X
// are below the 2 GiB out-of-range offset and X is one source.
static int g_stag2_buf = -1;
static bool stag2_buf() {
  if (g_stag2_buf < 0) {
    const char* e = std::getenv("ARB_DMA_BUF");
    g_stag2_buf = (e != nullptr && e[0] == '0') ? 0 : 1;
  }
  return g_stag2_buf == 1;
}
ARB_API void arb_set_stag2_buf(int on) { g_stag2_buf = on ? 1 : 0; }
static bool dma_buf_ok(const ConvArgs& p) {
  return stag2_buf() && 2L * p.N * p.K < (1L << 31) && 2L * p.B * p.H * p.W * p.Cin < (1L << 31) &&
         p.x2 == nullptr && (p.Cx == 0 || p.Cx == p.Cin);
}

template <int BN, int BM, int WN, int WM, int NS, bool SPLIT>
static void launch_glds(const ConvArgs& p, dim3 grid, hipStream_t s) {
  static_assert((size_t)NS * (BN + BM) * 64 * sizeof(bf16_t) <= 160 * 1024, "LDS");
  if (dma_buf_ok(p)) conv_glds_kernel<BN, BM, WN, WM, NS, SPLIT, true><<<grid, 64 * WN * WM, 0, s>>>(p);
  else conv_glds_kernel<BN, BM, WN, WM, NS, SPLIT><<<grid, 64 * WN * WM, 0, s>>>(p);   // static LDS ring
}

// Persistent short-K tiles (cfg 24 + i): grid = min(tiles, 256 CUs).
template <int BN, int BM, int WN, int WM, int NS>
static void launch_persist(const ConvArgs& a, hipStream_t s) {
  static_assert((size_t)NS * ((BN + BM) * 64 + BN) * sizeof(bf16_t) <= 160 * 1024, "LDS");   // static ring
  ConvArgs p = a;
  p.tiles_n = (p.N + BN - 1) / BN;
  p.tiles_total = p.tiles_n * ((p.M + BM - 1) / BM);
  p.nsplit = 1;
  p.m_fastest = (long)p.N * p.K > (long)p.M * p.Cin;
  p.norm = nullptr;
  p.counters = nullptr;
  p.kt_per_split = p.ktiles;
  int grid = p.tiles_total < 256 ? p.tiles_total : 256;
  conv_persist_kernel<BN, BM, WN, WM, NS><<<grid, 64 * WN * WM, 0, s>>>(p);
}

// X-in-registers tiles (cfg 32 + i): BN channels x WAVES * TMW * 16 pixels, no split-K.
template <int BN, int WAVES, int TMW, int NS>
static void launch_xreg(const ConvArgs& a, const ConvPlan& pl, hipStream_t s) {
  constexpr int BM = WAVES * TMW * 16;
  ConvArgs p = a;
  p.tiles_n = (p.N + BN - 1) / BN;
  p.tiles_total = p.tiles_n * ((p.M + BM - 1) / BM);
  p.nsplit = pl.split > 1 ? pl.split : 1;
  p.m_fastest = (long)p.N * p.K > (long)p.M * p.Cin;
  p.norm = nullptr;
  p.counters = nullptr;
  p.kt_per_split = p.nsplit > 1 ? pl.kt_per_split : p.ktiles;
  conv_xreg_kernel<BN, WAVES, TMW, NS><<<p.tiles_total * p.nsplit, 64 * WAVES, 0, s>>>(p);
  if (p.nsplit > 1) {
    long blocks = ((long)p.M * (p.N / 8) + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    splitk_reduce_kernel<0><<<(int)blocks, 256, 0, s>>>(p, p.nsplit);
  }
}

// Staggered two-group tiles (cfg 36 + i, i < 6): 8 waves, three-stage LDS-DMA ring.
template <int BN, int BM, int WN, int WM>
static void launch_stag(const ConvArgs& a, const ConvPlan& pl, hipStream_t s) {
  ConvArgs p = a;
  p.tiles_n = (p.N + BN - 1) / BN;
  p.tiles_total = p.tiles_n * ((p.M + BM - 1) / BM);
  p.nsplit = pl.split > 1 ? pl.split : 1;
  p.m_fastest = (long)p.N * p.K > (long)p.M * p.Cin;
  p.norm = nullptr;
  p.counters = nullptr;
  if (pl.split > 1) {
    p.kt_per_split = pl.kt_per_split;
    if (dma_buf_ok(p)) conv_stag_kernel<BN, BM, WN, WM, true, true><<<p.tiles_total * pl.split, 512, 0, s>>>(p);
    else conv_stag_kernel<BN, BM, WN, WM, true><<<p.tiles_total * pl.split, 512, 0, s>>>(p);
    long blocks = ((long)p.M * (p.N / 8) + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    splitk_reduce_kernel<0><<<(int)blocks, 256, 0, s>>>(p, pl.split);
  } else {
    if (dma_buf_ok(p)) conv_stag_kernel<BN, BM, WN, WM, false, true><<<p.tiles_total, 512, 0, s>>>(p);
    else conv_stag_kernel<BN, BM, WN, WM, false><<<p.tiles_total, 512, 0, s>>>(p);
  }
}

// Prefetch distance of the half-slot tiles (bitwise-equal variants: the MFMA sequence is the same):
// 4 (default) = one more phase of DMA lead time; ARB_STAG2_PD=3 or arb_set_stag2_pd(3) -> the r3 form.
// Same-process A/B (profiles/stag2_pd_ab_r4.jsonl): +0..2 % per shape, most on the under-filled
// 24x24 / 16x16-level tiles, never slower beyond noise.
static int g_stag2_pd = -1;
static int stag2_pd() {
  if (g_stag2_pd < 0) {
    const char* e = std::getenv("ARB_STAG2_PD");
    g_stag2_pd = (e != nullptr && e[0] == '3') ? 3 : 4;
  }
  return g_stag2_pd;
}
ARB_API void arb_set_stag2_pd(int pd) { g_stag2_pd = pd == 4 ? 4 : 3; }


// Half-slot staggered tiles (cfg 42 + i): 8 waves, HS-deep ring of K-half slots.
template <int BN, int BM, int WN, int WM, int HS>
static void launch_stag2(const ConvArgs& a, const ConvPlan& pl, hipStream_t s) {
  ConvArgs p = a;
  p.tiles_n = (p.N + BN - 1) / BN;
  p.tiles_total = p.tiles_n * ((p.M + BM - 1) / BM);
  p.nsplit = pl.split > 1 ? pl.split : 1;
  p.m_fastest = (long)p.N * p.K > (long)p.M * p.Cin;
  p.norm = nullptr;
  p.counters = nullptr;
  const bool buf = stag2_pd() == 4 && dma_buf_ok(p);
  if (pl.split > 1) {
    p.kt_per_split = pl.kt_per_split;
    if (buf) conv_stag2_kernel<BN, BM, WN, WM, HS, true, 4, true><<<p.tiles_total * pl.split, 512, 0, s>>>(p);
    else if (stag2_pd() == 4)
      conv_stag2_kernel<BN, BM, WN, WM, HS, true, 4><<<p.tiles_total * pl.split, 512, 0, s>>>(p);
    else conv_stag2_kernel<BN, BM, WN, WM, HS, true><<<p.tiles_total * pl.split, 512, 0, s>>>(p);
    long blocks = ((long)p.M * (p.N / 8) + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    splitk_reduce_kernel<0><<<(int)blocks, 256, 0, s>>>(p, pl.split);
  } else {
    if (buf) conv_stag2_kernel<BN, BM, WN, WM, HS, false, 4, true><<<p.tiles_total, 512, 0, s>>>(p);
    else if (stag2_pd() == 4) conv_stag2_kernel<BN, BM, WN, WM, HS, false, 4><<<p.tiles_total, 512, 0, s>>>(p);
    else conv_stag2_kernel<BN, BM, WN, WM, HS, false><<<p.tiles_total, 512, 0, s>>>(p);
  }
}

// 8-wave LDS-DMA tiles (cfg 20 + i): two full K-tile stages, per-wave 128x64 / 160x64 outputs.
struct BigCfg {
  int bn, bm;
};
static const BigCfg kBigCfgs[] = {{256, 256}, {320, 128}, {256, 128}, {320, 192}};
static_assert(sizeof(kBigCfgs) / sizeof(kBigCfgs[0]) == 4, "conv_plan accepts cfg 20..23");

template <int BN, int BM, int WN, int WM, int NS = 2>
static void launch_big(const ConvArgs& a, const ConvPlan& pl, hipStream_t s) {
  static_assert(NS * (BN + BM) * 64 * 2 <= 160 * 1024, "LDS");
  ConvArgs p = a;
  p.tiles_n = (p.N + BN - 1) / BN;
  p.tiles_total = p.tiles_n * ((p.M + BM - 1) / BM);
  p.nsplit = pl.split > 1 ? pl.split : 1;
  p.m_fastest = (long)p.N * p.K > (long)p.M * p.Cin;
  p.norm = nullptr;
  p.counters = nullptr;
  if (pl.split > 1) {
    p.kt_per_split = pl.kt_per_split;
    launch_glds<BN, BM, WN, WM, NS, true>(p, dim3(p.tiles_total * pl.split), s);
    long work = (long)p.M * (p.N / 8);
    long blocks = (work + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    splitk_reduce_kernel<0><<<(int)blocks, 256, 0, s>>>(p, pl.split);
  } else {
    launch_glds<BN, BM, WN, WM, NS, false>(p, dim3(p.tiles_total), s);
  }
}

template <int BN, int BM, int WN, int WM, int MINW, int EL = 0>
static void launch_conv(const ConvArgs& a, const ConvPlan& pl, bool glds, hipStream_t s) {
  // stages of the LDS-DMA ring: as many as fit 160 KiB, at most 4
  constexpr int STAGE_BYTES = (BN + BM) * 64 * 2;
  constexpr int NS = (4 * STAGE_BYTES <= 160 * 1024) ? 4 : 3;
  ConvArgs p = a;
  p.tiles_n = (p.N + BN - 1) / BN;
  p.tiles_total = p.tiles_n * ((p.M + BM - 1) / BM);
  p.nsplit = pl.split > 1 ? pl.split : 1;
  p.m_fastest = (long)p.N * p.K > (long)p.M * p.Cin;  // weight bytes vs unique activation bytes
  if constexpr (EL != 0) {
    glds = false;        // fp16: register-staged kernel only, no norm prologue
    p.norm = nullptr;
  }
  auto reduce = [&]() {
    long work = (long)p.M * (p.N / 8);
    long blocks = (work + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    splitk_reduce_kernel<EL><<<(int)blocks, 256, 0, s>>>(p, pl.split);
  };
  if (pl.split > 1) {
    p.kt_per_split = pl.kt_per_split;
    dim3 grid(p.tiles_total * pl.split);
    if constexpr (EL == 0) {
      if (glds && !p.norm) {
        p.counters = nullptr;
        launch_glds<BN, BM, WN, WM, NS, true>(p, grid, s);
        reduce();
        return;
      }
    }
    // register-staged kernel.  In-launch reduction is opt-in (ARB_SPLITK_INLAUNCH=1): the
    // agent-scope release/acquire pair writes back / invalidates the XCD's L2 per block, which
    // measured 2-3x slower than the separate ordered reduce on SD1.5 shapes.
    p.counters = (splitk_inlaunch() && !p.geglu) ? split_counters(s, p.tiles_total) : nullptr;
    if constexpr (EL == 0) {
      if (p.norm) conv_igemm_kernel<BN, BM, WN, WM, MINW, true, true><<<grid, 256, 0, s>>>(p);
      else conv_igemm_kernel<BN, BM, WN, WM, MINW, true, false><<<grid, 256, 0, s>>>(p);
    } else {
      conv_igemm_kernel<BN, BM, WN, WM, MINW, true, false, EL><<<grid, 256, 0, s>>>(p);
    }
    if (p.counters == nullptr) reduce();   // separate ordered reduce
  } else {
    dim3 grid(p.tiles_total, 1);
    if constexpr (EL == 0) {
      if (p.norm) conv_igemm_kernel<BN, BM, WN, WM, MINW, false, true><<<grid, 256, 0, s>>>(p);
      else if (glds) launch_glds<BN, BM, WN, WM, NS, false>(p, grid, s);
      else conv_igemm_kernel<BN, BM, WN, WM, MINW, false, false><<<grid, 256, 0, s>>>(p);
    } else {
      conv_igemm_kernel<BN, BM, WN, WM, MINW, false, false, EL><<<grid, 256, 0, s>>>(p);
    }
  }
}

// x [B,H,W,Cin] bf16, w [Cout, k, k, Cin], out [B,Ho,Wo,Cout]; Cin % 64 == 0, Cout % 8 == 0.
// cfg/split = -1: planned; >= 0: forced (autotuning).
// norm: optional [B, Cin, 2] fp32 (scale, shift) GroupNorm table applied to x in the prologue
// (+ SiLU when norm_silu) - see arb_group_norm_table.  Register-staged kernels only.
#include "conv_sk.inc"

template <int EL>
static int conv_run(const void* x, const void* w, const void* bias, const void* temb, const void* res, void* out,
                    void* ws, const void* norm, int B, int H, int W, int Cin, int Cout, int k, int pad, int upsample,
                    int stride, int cfg, int split, int norm_silu, hipStream_t stream, int geglu = 0,
                    const void* x2 = nullptr, int C1 = 0, const void* rowstat = nullptr,
                    const void* wsum = nullptr, int cx = 0, int act = 0, int temb_ld = 0) {
  if (Cin % 64 != 0 || Cout % 8 != 0 || (k != 1 && k != 3 && k != 31) || (stride != 1 && stride != 2)) return -1;
  if (cx == 0) cx = Cin;
  if (cx % 8 != 0 || cx > Cin || Cin - cx >= 64 || act < 0 || act > 4 || (act > 2 && EL != 0)) return -1;
  if (cx != Cin && (norm != nullptr || x2 != nullptr || rowstat != nullptr)) return -1;
  if (x2 != nullptr && (EL != 0 || C1 <= 0 || C1 >= Cin || C1 % 64 != 0 || geglu)) return -1;
  ConvArgs a;
  a.x2 = (const bf16_t*)x2;
  a.C1 = C1;
  a.x = (const bf16_t*)x; a.w = (const bf16_t*)w; a.bias = (const bf16_t*)bias; a.temb = (const bf16_t*)temb;
  a.temb_ld = temb_ld > 0 ? temb_ld : Cout;
  if (temb_ld > 0 && (temb_ld < Cout || temb_ld % 8 != 0)) return -1;
  a.res = (const bf16_t*)res; a.out = (bf16_t*)out; a.ws = (float*)ws;
  a.norm = (const float*)norm; a.norm_silu = norm_silu;
  conv_geom(a, B, H, W, Cin, Cout, k, pad, upsample, stride);
  a.geglu = geglu;
  a.rowstat = (const float2*)rowstat;
  a.wsum = (const float*)wsum;
  a.Cx = cx;
  a.act = act;
  if ((rowstat == nullptr) != (wsum == nullptr) || (rowstat && (norm != nullptr || x2 != nullptr))) return -1;
  ConvPlan pl = conv_plan(a.M, a.N, a.ktiles, cfg, split);
  if (geglu) {
    if (Cout % 16 != 0 || temb != nullptr || res != nullptr || norm != nullptr) return -1;
    if (is_persist(pl.cfg)) pl = {kNumCfgs + 5, 1, a.ktiles};   // persistent kernel has no GEGLU epilogue
  }
  // The 8-wave / persistent families have no GroupNorm prologue: a normed call on a shape pinned to
  // one of them runs the register-staged 128x128 tile at the pinned split (same grid coverage).
  if (norm != nullptr && pl.cfg >= 20) pl = conv_plan(a.M, a.N, a.ktiles, kNumCfgs, is_persist(pl.cfg) ? 1 : pl.split);
  // Dual-source reads exist in the register-staged kernel only: the same tile's register-staged
  // twin (or the 128x128 one for the 8-wave / persistent families) at the same split - the
  // per-output MFMA order and split-K slab order are those of the planned kernel, so the bytes are
  // those of the concatenated-input conv.
  // Padded channels (Cx < Cin) are masked in the register-staged kernels only: same remap.
  if (a.x2 != nullptr || a.Cx != a.Cin) {
    if (pl.cfg >= 20) pl = conv_plan(a.M, a.N, a.ktiles, kNumCfgs, is_persist(pl.cfg) ? 1 : pl.split);
    else if (pl.cfg < kNumCfgs) pl.cfg += kNumCfgs;
  }
  if (pl.split > 1 && ws == nullptr) return -3;
  if (pl.cfg == 46 || pl.cfg == 47) {   // W-stationary short-K GEMM (conv_sk.inc)
    if (EL == 0 && pl.split == 1 && sk_ok(a, pl.cfg)) {
      if (pl.cfg == 46) launch_sk<160, 320>(a, stream);
      else if (a.K == 640) launch_sk<80, 640>(a, stream);
      else launch_sk<80, 320>(a, stream);
      return (int)hipGetLastError();
    }
    pl.cfg = 34;   // outside its shapes: the X-in-registers 160-wide tile at the same split (same bytes)
  }
  if (pl.cfg >= 42) {   // half-slot staggered 8-wave tiles (bf16, no norm prologue / dual source)
    if (EL != 0 || a.norm != nullptr) return -4;
    switch (pl.cfg - 42) {
      case 0: launch_stag2<320, 128, 4, 2, 5>(a, pl, stream); break;
      case 1: launch_stag2<256, 256, 2, 4, 5>(a, pl, stream); break;
      case 2: launch_stag2<256, 192, 4, 2, 5>(a, pl, stream); break;
      default: launch_stag2<192, 192, 2, 4, 5>(a, pl, stream); break;   // cfg 45 (120 KiB ring)
    }
    return (int)hipGetLastError();
  }
  if (pl.cfg >= 36) {   // staggered two-group 8-wave tiles (bf16, no norm prologue / dual source)
    if (EL != 0 || a.norm != nullptr) return -4;
    switch (pl.cfg - 36) {
      case 0: launch_stag<256, 128, 4, 2>(a, pl, stream); break;
      case 1: launch_stag<128, 256, 2, 4>(a, pl, stream); break;
      case 2: launch_stag<192, 192, 2, 4>(a, pl, stream); break;
      case 3: launch_stag<320, 64, 4, 2>(a, pl, stream); break;
      case 4: launch_stag<160, 256, 2, 4>(a, pl, stream); break;
      default: launch_stag<160, 128, 2, 4>(a, pl, stream); break;
    }
    return (int)hipGetLastError();
  }
  if (is_xreg(pl.cfg)) {   // X-in-registers 8-wave tiles (bf16, no norm prologue / dual source)
    if (EL != 0 || a.norm != nullptr) return -4;
    switch (pl.cfg - 32) {
      case 0: launch_xreg<160, 8, 2, 2>(a, pl, stream); break;
      case 1: launch_xreg<128, 8, 2, 2>(a, pl, stream); break;
      case 2: launch_xreg<160, 8, 1, 2>(a, pl, stream); break;
      default: launch_xreg<256, 8, 1, 2>(a, pl, stream); break;
    }
    return (int)hipGetLastError();
  }
  if (pl.cfg >= 28) {   // 8-wave 3-stage LDS-DMA ring (bf16, no norm prologue)
    if (EL != 0 || a.norm != nullptr) return -4;
    switch (pl.cfg - 28) {
      case 0: launch_big<128, 256, 2, 4, 3>(a, pl, stream); break;
      case 1: launch_big<256, 128, 4, 2, 3>(a, pl, stream); break;
      case 2: launch_big<192, 192, 2, 4, 3>(a, pl, stream); break;
      default: launch_big<320, 64, 4, 2, 3>(a, pl, stream); break;
    }
    return (int)hipGetLastError();
  }
  if (pl.cfg >= 24) {   // persistent short-K tiles (bf16, no norm prologue, no split)
    if (EL != 0 || a.norm != nullptr) return -4;
    switch (pl.cfg - 24) {
      case 0: launch_persist<128, 128, 2, 2, 4>(a, stream); break;
      case 1: launch_persist<256, 128, 4, 2, 3>(a, stream); break;
      case 2: launch_persist<160, 128, 2, 2, 4>(a, stream); break;
      default: launch_persist<128, 64, 2, 2, 4>(a, stream); break;
    }
    return (int)hipGetLastError();
  }
  if (pl.cfg >= 20) {   // 8-wave LDS-DMA tiles (bf16, no norm prologue)
    if (EL != 0 || a.norm != nullptr) return -4;
    switch (pl.cfg - 20) {
      case 0: launch_big<256, 256, 2, 4>(a, pl, stream); break;
      case 1: launch_big<320, 128, 4, 2>(a, pl, stream); break;
      case 2: launch_big<256, 128, 4, 2>(a, pl, stream); break;
      default: launch_big<320, 192, 2, 4>(a, pl, stream); break;
    }
    return (int)hipGetLastError();
  }
  const bool glds = pl.cfg < kNumCfgs;  // cfg >= kNumCfgs: register-staged variant (A/B)
  switch (pl.cfg % kNumCfgs) {
    case 0: launch_conv<128, 128, 2, 2, 2, EL>(a, pl, glds, stream); break;
    case 1: launch_conv<64, 128, 2, 2, 2, EL>(a, pl, glds, stream); break;
    case 2: launch_conv<128, 64, 2, 2, 2, EL>(a, pl, glds, stream); break;
    case 3: launch_conv<64, 64, 2, 2, 2, EL>(a, pl, glds, stream); break;
    case 4: launch_conv<160, 64, 2, 2, 2, EL>(a, pl, glds, stream); break;
    case 5: launch_conv<160, 128, 2, 2, 1, EL>(a, pl, glds, stream); break;
    case 6: launch_conv<320, 32, 4, 1, 1, EL>(a, pl, glds, stream); break;
    case 7: launch_conv<256, 64, 4, 1, 1, EL>(a, pl, glds, stream); break;
    case 8: launch_conv<128, 256, 2, 2, 1, EL>(a, pl, glds, stream); break;
    default: launch_conv<64, 256, 1, 4, 1, EL>(a, pl, glds, stream); break;
  }
  return (int)hipGetLastError();
}

ARB_API int arb_conv2d_nhwc(const void* x, const void* w, const void* bias, const void* temb, const void* res,
                            void* out, void* ws, const void* norm, int B, int H, int W, int Cin, int Cout, int k,
                            int pad, int upsample, int stride, int cfg, int split, int norm_silu,
                            hipStream_t stream) {
  return conv_run<0>(x, w, bias, temb, res, out, ws, norm, B, H, W, Cin, Cout, k, pad, upsample, stride, cfg, split,
                     norm_silu, stream);
}

// As arb_conv2d_nhwc with the time embedding read at row stride temb_ld (a column slice of the batched
// [B, sum(Cout)] ResBlock projection, no contiguous copy); temb_ld % 8 == 0 (16-byte rows).
ARB_API int arb_conv2d_nhwc_tld(const void* x, const void* w, const void* bias, const void* temb, int temb_ld,
                                const void* res, void* out, void* ws, const void* norm, int B, int H, int W, int Cin,
                                int Cout, int k, int pad, int upsample, int stride, int cfg, int split, int norm_silu,
                                hipStream_t stream) {
  return conv_run<0>(x, w, bias, temb, res, out, ws, norm, B, H, W, Cin, Cout, k, pad, upsample, stride, cfg, split,
                     norm_silu, stream, 0, nullptr, 0, nullptr, nullptr, 0, 0, temb_ld);
}

// Conv over the channel concat [x | x2] without materialising it (UNet up-path skip connections):
// x [B,H,W,C1], x2 [B,H,W,Cin-C1]; otherwise as arb_conv2d_nhwc (no norm prologue).
ARB_API int arb_conv2d_nhwc_cat(const void* x, const void* x2, int C1, const void* w, const void* bias,
                                const void* temb, const void* res, void* out, void* ws, int B, int H, int W, int Cin,
                                int Cout, int k, int pad, int upsample, int stride, int cfg, int split,
                                hipStream_t stream) {
  return conv_run<0>(x, w, bias, temb, res, out, ws, nullptr, B, H, W, Cin, Cout, k, pad, upsample, stride, cfg, split,
                     0, stream, 0, x2, C1);
}

// fp16 twin (robust video matting): same plans and tiles on mfma_f32_16x16x32_f16, no norm prologue.
ARB_API int arb_conv2d_nhwc_f16(const void* x, const void* w, const void* bias, const void* temb, const void* res,
                                void* out, void* ws, int B, int H, int W, int Cin, int Cout, int k, int pad,
                                int upsample, int stride, int cfg, int split, hipStream_t stream) {
  return conv_run<1>(x, w, bias, temb, res, out, ws, nullptr, B, H, W, Cin, Cout, k, pad, upsample, stride, cfg,
                     split, 0, stream);
}

// Tile family for the ACTUAL shape at a plan's split-K (solo tasks run the canonical batch-8 split;
// at a fixed split every family reduces each output in the same order, so the family is a free,
// bitwise-neutral choice - scripts/tune_family.py pins the fastest per shape).  Unknown: keep cfg.
// ratio = canonical batch / actual batch (4: a solo task under the batch-8 plans; 1: a lock-step
// group of 4 on its own plans, tuned with the second task stream running concurrently).
struct FamilyPlan {
  int M, N, K, split, ratio, cfg;
};
#include "conv_family.inc"

// Optional run-time family table (A/B of a re-tuned table without a rebuild): ARB_CONV_FAMILY names a
// file in conv_family.inc format ("{M, N, K, split, ratio, cfg},"); its entries take precedence.
static const std::vector<FamilyPlan>& env_families() {
  static const std::vector<FamilyPlan> fams = [] {
    std::vector<FamilyPlan> v;
    const char* path = std::getenv("ARB_CONV_FAMILY");
    if (path == nullptr || path[0] == 0) return v;
    FILE* f = std::fopen(path, "r");
    if (f == nullptr) {
      std::fprintf(stderr, "[arbius] ARB_CONV_FAMILY=%s cannot be read: the built-in table is used\n", path);
      return v;
    }
    char line[256];
    while (std::fgets(line, sizeof line, f)) {
      FamilyPlan fp;
      if (std::sscanf(line, " {%d, %d, %d, %d, %d, %d}", &fp.M, &fp.N, &fp.K, &fp.split, &fp.ratio, &fp.cfg) == 6)
        v.push_back(fp);
    }
    std::fclose(f);
    return v;
  }();
  return fams;
}

ARB_API int arb_conv_family(int M, int N, int K, int split, int ratio, int cfg) {
  if (std::getenv("ARB_NO_FAMILY") != nullptr) return cfg;
  for (const FamilyPlan& fp : env_families())
    if (fp.M == M && fp.N == N && fp.K == K && fp.split == split && fp.ratio == ratio) return fp.cfg;
  for (const FamilyPlan& fp : kFamilyPlans)
    if (fp.M == M && fp.N == N && fp.K == K && fp.split == split && fp.ratio == ratio) return fp.cfg;
  return cfg;
}

ARB_API int arb_conv2d_plan(int B, int H, int W, int Cin, int Cout, int k, int pad, int upsample, int stride,
                            int* cfg_split) {
  ConvArgs a;
  conv_geom(a, B, H, W, Cin, Cout, k, pad, upsample, stride);
  const ConvPlan pl = conv_plan(a.M, a.N, a.ktiles, -1, -1);
  cfg_split[0] = pl.cfg;
  cfg_split[1] = pl.split;
  return 0;
}

// GEGLU projection: out[M, N/2] = value * gelu(gate) of x W^T + b, with W / b rows interleaved in
// blocks of 16 as [value 8 | gate 8] (see ops.linear_geglu); N % 16 == 0, K % 64 == 0.
ARB_API int arb_gemm_geglu(const void* x, const void* w, const void* bias, void* out, void* ws, int M, int N, int K,
                           int cfg, int split, hipStream_t stream) {
  return conv_run<0>(x, w, bias, nullptr, nullptr, out, ws, nullptr, 1, 1, M, K, N, 1, 0, 0, 1, cfg, split, 0, stream,
                     1);
}

// Plain GEMM with fused epilogue: out[M,N] = x[M,K] W[N,K]^T (+bias +residual); K % 64 == 0.
ARB_API int arb_gemm_bias_res(const void* x, const void* w, const void* bias, const void* res, void* out, void* ws,
                              int M, int N, int K, int cfg, int split, hipStream_t stream) {
  return arb_conv2d_nhwc(x, w, bias, nullptr, res, out, ws, nullptr, 1, 1, M, K, N, 1, 0, 0, 1, cfg, split, 0, stream);
}

// As arb_gemm_bias_res with an epilogue activation (act_f: 3 GELU, 4 quick-GELU; bf16).
ARB_API int arb_gemm_act(const void* x, const void* w, const void* bias, const void* res, void* out, void* ws, int M,
                         int N, int K, int cfg, int split, int act, hipStream_t stream) {
  return conv_run<0>(x, w, bias, nullptr, res, out, ws, nullptr, 1, 1, M, K, N, 1, 0, 0, 1, cfg, split, 0, stream, 0,
                     nullptr, 0, nullptr, nullptr, 0, act);
}

// GEMM with a LayerNorm folded in (see ConvArgs::rowstat): x is the LN's INPUT [M, K], w the
// gamma-scaled weights, bias the beta-folded bias, rowstat[m] = (mean, rstd) of x's row m
// (arb_row_stats), wsum[n] = sum_k w[n, k] in fp32.  geglu: w / bias / wsum interleaved as for
// arb_gemm_geglu, out [M, N/2].  The normalised activation never exists in memory.
ARB_API int arb_gemm_ln(const void* x, const void* w, const void* bias, const void* res, void* out, void* ws,
                        const void* rowstat, const void* wsum, int M, int N, int K, int cfg, int split, int geglu,
                        int act, hipStream_t stream) {
  if (rowstat == nullptr || wsum == nullptr || (geglu && (res != nullptr || act != 0))) return -1;
  return conv_run<0>(x, w, bias, nullptr, res, out, ws, nullptr, 1, 1, M, K, N, 1, 0, 0, 1, cfg, split, 0, stream,
                     geglu, nullptr, 0, rowstat, wsum, 0, act);
}

// General entry: x has Cx channels per pixel (Cx % 8 == 0; the K walk pads to Cin = Cx rounded up to
// 64 and reads zeros for the padded channels - no padded copy of x), w is [Cout, k, k, Cin]
// zero-padded; act 0/1/2 = none / ReLU / hardswish in the epilogue; f16 selects the fp16 twin.
ARB_API int arb_conv2d_ex(const void* x, const void* w, const void* bias, const void* temb, const void* res, void* out,
                          void* ws, int B, int H, int W, int Cx, int Cout, int k, int pad, int upsample, int stride,
                          int cfg, int split, int act, int f16, hipStream_t stream) {
  const int Cin = (Cx + 63) / 64 * 64;
  if (f16)
    return conv_run<1>(x, w, bias, temb, res, out, ws, nullptr, B, H, W, Cin, Cout, k, pad, upsample, stride, cfg,
                       split, 0, stream, 0, nullptr, 0, nullptr, nullptr, Cx, act);
  return conv_run<0>(x, w, bias, temb, res, out, ws, nullptr, B, H, W, Cin, Cout, k, pad, upsample, stride, cfg, split,
                     0, stream, 0, nullptr, 0, nullptr, nullptr, Cx, act);
}
