// LayerNorm over token rows [M, C] bf16 (transformer blocks, CLIP).
#include "common.h"

#include <cstdlib>

// LayerNorm: one wave per R consecutive rows, rows held in registers (exact two-pass mean/var per
// row), 4 waves per block.  All R rows' loads are issued before any reduction (R x the bytes in
// flight per wave - the kernel is HBM-latency bound at C = 320..1280), gamma / beta loaded once.
// Per-row arithmetic is identical for every R (same order), so results do not depend on R.
// STATS = true: write only the row's (mean, rstd) to rs[row] (a LayerNorm folded into the consuming
// GEMM's epilogue, conv.hip "LN fold") - same arithmetic, one read of x and no write of it.
template <int NVMAX, int R, bool STATS = false>
__global__ void __launch_bounds__(256) layer_norm_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         const bf16_t* __restrict__ gamma,
                                                         const bf16_t* __restrict__ beta, int M, int C, float eps,
                                                         float2* __restrict__ rs = nullptr) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= M) return;
  const int NV = C >> 3;
  float v[R][NVMAX][8];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const bool rok = row0 + r < M;
    const bf16_t* xr = x + (size_t)(row0 + r) * C;
#pragma unroll
    for (int i = 0; i < NVMAX; ++i) {
      const int vi = lane + 64 * i;
      if (rok && vi < NV) {
        unpack8(ld16(xr + vi * 8), v[r][i]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[r][i][e] = 0.f;
      }
    }
  }
  float g[NVMAX][8], bb[NVMAX][8];
#pragma unroll
  for (int i = 0; i < NVMAX; ++i) {
    const int vi = lane + 64 * i;
    if (!STATS && vi < NV) {
      unpack8(ld16(gamma + vi * 8), g[i]);
      unpack8(ld16(beta + vi * 8), bb[i]);
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (row0 + r >= M) break;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NVMAX; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[r][i][e];
    const float mean = wave_sum(s) / (float)C;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NVMAX; ++i) {
      const int vi = lane + 64 * i;
      if (vi < NV) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = v[r][i][e] - mean;
          ss += d * d;
        }
      }
    }
    const float rstd = rsqrtf(wave_sum(ss) / (float)C + eps);
    if constexpr (STATS) {
      if (lane == 0) rs[row0 + r] = make_float2(mean, rstd);
      continue;
    }
#pragma unroll
    for (int i = 0; i < NVMAX; ++i) {
      const int vi = lane + 64 * i;
      if (vi < NV) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (v[r][i][e] - mean) * rstd * g[i][e] + bb[i][e];
        st16(y + (size_t)(row0 + r) * C + vi * 8, pack8(o));
      }
    }
  }
}

// Packed-row LayerNorm: LPR lanes per row (a power of two dividing 64), each lane VPL contiguous
// 8-channel vectors (C = 8 * LPR * VPL), so every lane of the wave is busy (the one-row-per-wave
// kernel leaves 24 of 64 lanes idle at C = 320 / 640 / 1280) and 64 / LPR rows' loads are in
// flight per wave.  Two exact passes over registers, fixed xor-butterfly row reductions.
template <int LPR, int VPL, bool STATS = false>
__global__ void __launch_bounds__(256) layer_norm_packed_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                                const bf16_t* __restrict__ gamma,
                                                                const bf16_t* __restrict__ beta, int M, int C,
                                                                float eps, float2* __restrict__ rs = nullptr) {
  constexpr int RPW = 64 / LPR;                    // rows per wave
  const int lane = threadIdx.x & 63, sub = lane % LPR;
  const int row = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const bool ok = row < M;
  const bf16_t* xr = x + (size_t)(ok ? row : 0) * C + sub * VPL * 8;
  float v[VPL][8];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    if (ok) {
      unpack8(ld16(xr + i * 8), v[i]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[i][e];
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / (float)C;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[i][e] - mean;
      ss += d * d;
    }
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1) ss += __shfl_xor(ss, o, 64);
  const float rstd = rsqrtf(ss / (float)C + eps);
  if (!ok) return;
  if constexpr (STATS) {
    if (sub == 0) rs[row] = make_float2(mean, rstd);
    return;
  }
  bf16_t* yr = y + (size_t)row * C + sub * VPL * 8;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    float g[8], bb[8], o[8];
    unpack8(ld16(gamma + sub * VPL * 8 + i * 8), g);
    unpack8(ld16(beta + sub * VPL * 8 + i * 8), bb);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * rstd * g[e] + bb[e];
    st16(yr + i * 8, pack8(o));
  }
}

// (LPR, VPL) for C: the largest power-of-two lanes-per-row with at most 8 vectors per lane
static bool ln_packed_geom(int C, int& lpr, int& vpl) {
  if (C % 8 != 0) return false;
  const int NV = C / 8;
  for (int l = 64; l >= 4; l >>= 1)
    if (NV % l == 0 && NV / l <= 8) {
      lpr = l;
      vpl = NV / l;
      return true;
    }
  return false;
}

// plan_rows: the row count the kernel choice is made for - the CANONICAL batch's rows under
// batch-invariant planning (ops.plan_batch), never the launch's own M: the packed and wave-per-row
// kernels reduce a row in different orders, so a choice by M would make a lock-step group's bytes
// differ from its solo tasks'.
template <bool STATS>
static bool ln_packed_launch(const void* x, void* y, const void* gamma, const void* beta, void* rs, int M, int C,
                             float eps, long plan_rows, hipStream_t stream) {
  static const bool on = [] {
    const char* e = std::getenv("ARB_LN_PACKED");
    return e == nullptr || e[0] != '0';
  }();
  // Measured (graph replay, profiles/norm_kernels_ab_r3.jsonl): faster only for short inputs
  // (154 x 768 text-tower rows: 2.9 vs 4.1 us); at the UNet token counts the wave-per-row kernel
  // wins (32768 x 320: 13.2 vs 13.7 us, 8192 x 640: 6.6 vs 8.0 us).
  int lpr = 0, vpl = 0;
  if (!on || plan_rows * C > (1L << 18) || !ln_packed_geom(C, lpr, vpl)) return false;
  const int rows_per_block = 4 * (64 / lpr);
  const dim3 grid((M + rows_per_block - 1) / rows_per_block);
#define LNP(L, V)                                                                                   \
  if (lpr == L && vpl == V) {                                                                       \
    layer_norm_packed_kernel<L, V, STATS><<<grid, 256, 0, stream>>>(                                \
        (const bf16_t*)x, (bf16_t*)y, (const bf16_t*)gamma, (const bf16_t*)beta, M, C, eps, (float2*)rs); \
    return true;                                                                                    \
  }
  // C = 320 / 640 / 1280 (UNet), 768 (CLIP), 384 / 1024 / 2048 / 2560 and the small widths
  LNP(8, 5) LNP(16, 5) LNP(32, 5) LNP(32, 3) LNP(64, 1) LNP(64, 2) LNP(64, 3) LNP(64, 4) LNP(64, 5)
  LNP(16, 3) LNP(32, 1) LNP(16, 1)
#undef LNP
  return false;
}

ARB_API int arb_layer_norm(const void* x, void* y, const void* gamma, const void* beta, int M, int C, float eps,
                           long plan_rows, hipStream_t stream) {
  if (C % 8 != 0) return -1;
  if (ln_packed_launch<false>(x, y, gamma, beta, nullptr, M, C, eps, plan_rows, stream)) return (int)hipGetLastError();
  const int NV = C / 8;
#define LN_LAUNCH(NVM, R)                                                                                   \
  layer_norm_kernel<NVM, R><<<dim3((M + 4 * R - 1) / (4 * R)), 256, 0, stream>>>(                                \
      (const bf16_t*)x, (bf16_t*)y, (const bf16_t*)gamma, (const bf16_t*)beta, M, C, eps)
  static const bool one_row = [] {   // A/B switch: ARB_LN_ROWS=1 -> one row per wave
    const char* e = std::getenv("ARB_LN_ROWS");
    return e != nullptr && e[0] == '1';
  }();
  if (NV <= 64) {
    if (one_row) LN_LAUNCH(1, 1); else LN_LAUNCH(1, 4);
  } else if (NV <= 128) {
    if (one_row) LN_LAUNCH(2, 1); else LN_LAUNCH(2, 2);
  }
  else if (NV <= 256)
    LN_LAUNCH(4, 1);
  else
    return -1;
#undef LN_LAUNCH
  return (int)hipGetLastError();
}

// Per-row (mean, rstd) of x [M, C] - the statistics of a LayerNorm folded into the next GEMM.
ARB_API int arb_row_stats(const void* x, void* rs, int M, int C, float eps, long plan_rows, hipStream_t stream) {
  if (C % 8 != 0) return -1;
  if (ln_packed_launch<true>(x, nullptr, nullptr, nullptr, rs, M, C, eps, plan_rows, stream))
    return (int)hipGetLastError();
  const int NV = C / 8;
#define RS_LAUNCH(NVM, R)                                                                                   \
  layer_norm_kernel<NVM, R, true><<<dim3((M + 4 * R - 1) / (4 * R)), 256, 0, stream>>>(                          \
      (const bf16_t*)x, nullptr, nullptr, nullptr, M, C, eps, (float2*)rs)
  if (NV <= 64) RS_LAUNCH(1, 4);
  else if (NV <= 128) RS_LAUNCH(2, 2);
  else if (NV <= 256) RS_LAUNCH(4, 1);
  else return -1;
#undef RS_LAUNCH
  return (int)hipGetLastError();
}
