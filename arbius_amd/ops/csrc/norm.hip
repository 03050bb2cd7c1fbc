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

ARB_API int arb_layer_norm(const void* x, void* y, const void* gamma, const void* beta, int M, int C, float eps,
                           hipStream_t stream) {
  if (C % 8 != 0) return -1;
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
ARB_API int arb_row_stats(const void* x, void* rs, int M, int C, float eps, hipStream_t stream) {
  if (C % 8 != 0) return -1;
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
