// Depthwise k x k convolution, fp16 channels-last, + bias + activation in one pass: the
// MobileNetV3-Large encoder of Robust Video Matting (3x3 / 5x5 taps, stride
// 1 / 2, dilation 1 / 2 in the last stage).  MIOpen's deterministic mode serves these shapes with
// its naive direct kernel (profiles/rocprof_r1_v11_rvm_miopen_naive.md), so they get their own.
//
// Thread = one output pixel x 8 consecutive channels (16-B vector loads and stores: adjacent
// threads cover adjacent channel vectors, so every tap's load is a coalesced row segment; the
// k*k overlapping taps of neighbouring pixels hit L1/L2).  Weights are pre-transposed to
// [k*k, C] so the per-tap weight vector is one 16-B load.  fp32 accumulation in fixed tap order
// (r-major, then s), bias after the sum, activation on the fp32 value, one rounding to fp16:
// deterministic, and identical for any batch / chunk split of the frames.
#include "common.h"

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void unpack_h8(uint4 v, float (&f)[8]) {
  const h8 h = __builtin_bit_cast(h8, v);
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = (float)h[e];
}

__device__ __forceinline__ uint4 pack_h8(const float (&f)[8]) {
  h8 h;
#pragma unroll
  for (int e = 0; e < 8; ++e) h[e] = (_Float16)f[e];
  return __builtin_bit_cast(uint4, h);
}

// act: 0 none, 1 ReLU, 2 hardswish (x * relu6(x + 3) / 6)
template <int K>
__global__ void __launch_bounds__(256) dwconv_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ wt,
                                                     const uint16_t* __restrict__ bias, uint16_t* __restrict__ y,
                                                     int B, int H, int W, int C, int Ho, int Wo, int stride, int dil,
                                                     int act) {
  const int NV = C >> 3;
  const long total = (long)B * Ho * Wo * NV;
  const int pad = dil * (K / 2);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int cv = (int)(i % NV);
    long p = i / NV;
    const int wo = (int)(p % Wo);
    p /= Wo;
    const int ho = (int)(p % Ho);
    const int b = (int)(p / Ho);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    const int h0 = ho * stride - pad, w0 = wo * stride - pad;
#pragma unroll
    for (int r = 0; r < K; ++r) {
      const int hi = h0 + r * dil;
      if (hi < 0 || hi >= H) continue;
      const uint16_t* xr = x + (((size_t)b * H + hi) * W) * C + cv * 8;
#pragma unroll
      for (int s = 0; s < K; ++s) {
        const int wi = w0 + s * dil;
        if (wi < 0 || wi >= W) continue;
        float xv[8], wv[8];
        unpack_h8(ld16(xr + (size_t)wi * C), xv);
        unpack_h8(ld16(wt + (size_t)(r * K + s) * C + cv * 8), wv);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(xv[e], wv[e], acc[e]);
      }
    }
    float bv[8];
    if (bias != nullptr) {
      unpack_h8(ld16(bias + cv * 8), bv);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) bv[e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = acc[e] + bv[e];
      if (act == 1) v = fmaxf(v, 0.f);
      else if (act == 2) v = v * fminf(fmaxf(v + 3.f, 0.f), 6.f) * (1.f / 6.f);
      acc[e] = v;
    }
    st16(y + (((size_t)b * Ho + ho) * Wo + wo) * C + cv * 8, pack_h8(acc));
  }
}

// x [B, H, W, C] fp16, wt [k*k, C] fp16, bias [C] fp16 or null -> y [B, Ho, Wo, C];
// padding = dil * (k / 2) (same-size for stride 1).  C % 8 == 0, k in {3, 5}.
ARB_API int arb_dwconv_f16(const void* x, const void* wt, const void* bias, void* y, int B, int H, int W, int C,
                           int k, int stride, int dil, int act, hipStream_t stream) {
  if (C % 8 != 0 || (k != 3 && k != 5) || (stride != 1 && stride != 2) || dil < 1 || act < 0 || act > 2) return -1;
  const int pad = dil * (k / 2);
  const int Ho = (H + 2 * pad - dil * (k - 1) - 1) / stride + 1;
  const int Wo = (W + 2 * pad - dil * (k - 1) - 1) / stride + 1;
  const long total = (long)B * Ho * Wo * (C / 8);
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  if (k == 3)
    dwconv_kernel<3><<<(int)blocks, 256, 0, stream>>>((const uint16_t*)x, (const uint16_t*)wt,
                                                      (const uint16_t*)bias, (uint16_t*)y, B, H, W, C, Ho, Wo, stride,
                                                      dil, act);
  else
    dwconv_kernel<5><<<(int)blocks, 256, 0, stream>>>((const uint16_t*)x, (const uint16_t*)wt,
                                                      (const uint16_t*)bias, (uint16_t*)y, B, H, W, C, Ho, Wo, stride,
                                                      dil, act);
  return (int)hipGetLastError();
}
