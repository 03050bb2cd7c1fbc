// LayerNorm over token rows [M, C] bf16 (transformer blocks, CLIP).
#include "common.h"

// LayerNorm: one wave per row, row held in registers (exact two-pass mean/var), 4 rows/block.
template <int NVMAX>
__global__ void __launch_bounds__(256) layer_norm_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         const bf16_t* __restrict__ gamma,
                                                         const bf16_t* __restrict__ beta, int M, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int NV = C >> 3;
  const bf16_t* xr = x + (size_t)row * C;
  float v[NVMAX][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NVMAX; ++i) {
    const int vi = lane + 64 * i;
    if (vi < NV) {
      unpack8(ld16(xr + vi * 8), v[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[i][e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)C;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NVMAX; ++i) {
    const int vi = lane + 64 * i;
    if (vi < NV) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[i][e] - mean;
        ss += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / (float)C + eps);
#pragma unroll
  for (int i = 0; i < NVMAX; ++i) {
    const int vi = lane + 64 * i;
    if (vi < NV) {
      float g[8], bb[8], o[8];
      unpack8(ld16(gamma + vi * 8), g);
      unpack8(ld16(beta + vi * 8), bb);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * rstd * g[e] + bb[e];
      st16(y + (size_t)row * C + vi * 8, pack8(o));
    }
  }
}

ARB_API int arb_layer_norm(const void* x, void* y, const void* gamma, const void* beta, int M, int C, float eps,
                           hipStream_t stream) {
  if (C % 8 != 0) return -1;
  const int NV = C / 8;
  dim3 grid((M + 3) / 4);
  if (NV <= 64)
    layer_norm_kernel<1><<<grid, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (const bf16_t*)gamma,
                                                   (const bf16_t*)beta, M, C, eps);
  else if (NV <= 128)
    layer_norm_kernel<2><<<grid, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (const bf16_t*)gamma,
                                                   (const bf16_t*)beta, M, C, eps);
  else if (NV <= 256)
    layer_norm_kernel<4><<<grid, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (const bf16_t*)gamma,
                                                   (const bf16_t*)beta, M, C, eps);
  else
    return -1;
  return (int)hipGetLastError();
}
