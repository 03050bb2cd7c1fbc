// ConvGRU gate kernels of the Robust Video Matting recurrent decoder
// (templates/robust_video_matting.json; SURVEY.md §2.6(d): "recurrent ConvGRU as
// CDNA4 HIP, fp16").  The two 3x3 convolutions of the cell are library convs
// (MIOpen, channels-last fp16); everything between and after them is fused here:
//
//   gates1:  [r | z] = sigmoid(conv_ih(cat(x, h)))
//            z  -> zbuf              r*h -> cat buffer columns [cx, cx+C)
//            (the x columns of the same buffer are written by the caller once, so
//             the second conv reads cat(x, r*h) without a concat copy)
//   gates2:  h' = (1 - z) * h + z * tanh(conv_hh(cat(x, r*h)))
//
// Layout: channels-last rows of P pixels; fp16 storage, fp32 math; 8 channels per
// thread (16-byte vectors).  Pure elementwise -> bitwise deterministic.
#include "common.h"

typedef _Float16 h16;
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + fast_exp(-x)); }
__device__ __forceinline__ float tanh_f(float x) {
  const float e = fast_exp(-2.f * fabsf(x));
  const float t = (1.f - e) * __builtin_amdgcn_rcpf(1.f + e);
  return copysignf(t, x);
}

// ih [P, 2C] (r | z), h [P, C]  ->  z [P, C], cat[p * cat_stride + cx + c] = r * h
__global__ void __launch_bounds__(256) gru_gates1_kernel(const h16* __restrict__ ih, const h16* __restrict__ h,
                                                         h16* __restrict__ z, h16* __restrict__ cat, long P, int C,
                                                         int cat_stride, int cx) {
  const int nv = C >> 3;
  const long total = P * nv;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / nv;
    const int c = (int)(i - p * nv) * 8;
    const h16x8 rr = *reinterpret_cast<const h16x8*>(ih + p * 2 * C + c);
    const h16x8 zz = *reinterpret_cast<const h16x8*>(ih + p * 2 * C + C + c);
    const h16x8 hh = *reinterpret_cast<const h16x8*>(h + p * C + c);
    h16x8 zo, rh;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      zo[e] = (h16)sigm((float)zz[e]);
      rh[e] = (h16)(sigm((float)rr[e]) * (float)hh[e]);
    }
    *reinterpret_cast<h16x8*>(z + p * C + c) = zo;
    *reinterpret_cast<h16x8*>(cat + p * cat_stride + cx + c) = rh;
  }
}

// c [P, C] (conv_hh output), h [P, C], z [P, C] -> hout [P, C]
__global__ void __launch_bounds__(256) gru_gates2_kernel(const h16* __restrict__ cc, const h16* __restrict__ h,
                                                         const h16* __restrict__ z, h16* __restrict__ hout, long P,
                                                         int C) {
  const long total = P * (C >> 3);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const h16x8 cv = *reinterpret_cast<const h16x8*>(cc + i * 8);
    const h16x8 hv = *reinterpret_cast<const h16x8*>(h + i * 8);
    const h16x8 zv = *reinterpret_cast<const h16x8*>(z + i * 8);
    h16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float zf = (float)zv[e];
      o[e] = (h16)((1.f - zf) * (float)hv[e] + zf * tanh_f((float)cv[e]));
    }
    *reinterpret_cast<h16x8*>(hout + i * 8) = o;
  }
}

// Scalar variants for channel counts that are not a multiple of 8 (RVM decode2: 20).
__global__ void __launch_bounds__(256) gru_gates1_scalar(const h16* __restrict__ ih, const h16* __restrict__ h,
                                                         h16* __restrict__ z, h16* __restrict__ cat, long P, int C,
                                                         int cat_stride, int cx) {
  const long total = P * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / C;
    const int c = (int)(i - p * C);
    z[i] = (h16)sigm((float)ih[p * 2 * C + C + c]);
    cat[p * cat_stride + cx + c] = (h16)(sigm((float)ih[p * 2 * C + c]) * (float)h[i]);
  }
}

__global__ void __launch_bounds__(256) gru_gates2_scalar(const h16* __restrict__ cc, const h16* __restrict__ h,
                                                         const h16* __restrict__ z, h16* __restrict__ hout,
                                                         long total) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const float zf = (float)z[i];
    hout[i] = (h16)((1.f - zf) * (float)h[i] + zf * tanh_f((float)cc[i]));
  }
}

static int grid_for(long work) {
  long b = (work + 255) / 256;
  return (int)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

// mode 1: a = ih [P,2C], b = h, c = z (out), d = cat buffer (out, row stride cat_stride, column offset cx)
// mode 2: a = conv_hh out [P,C], b = h, c = z, d = h' (out)
ARB_API int arb_convgru_gates(int mode, const void* a, const void* b, void* c, void* d, long P, int C, int cat_stride,
                              int cx, hipStream_t stream) {
  const bool vec = C % 8 == 0 && cat_stride % 8 == 0 && cx % 8 == 0;
  if (mode == 1) {
    if (vec)
      gru_gates1_kernel<<<grid_for(P * (C / 8)), 256, 0, stream>>>((const h16*)a, (const h16*)b, (h16*)c, (h16*)d,
                                                                    P, C, cat_stride, cx);
    else
      gru_gates1_scalar<<<grid_for(P * C), 256, 0, stream>>>((const h16*)a, (const h16*)b, (h16*)c, (h16*)d, P, C,
                                                              cat_stride, cx);
  } else if (mode == 2) {
    if (C % 8 == 0)
      gru_gates2_kernel<<<grid_for(P * (C / 8)), 256, 0, stream>>>((const h16*)a, (const h16*)b, (const h16*)c,
                                                                    (h16*)d, P, C);
    else
      gru_gates2_scalar<<<grid_for(P * C), 256, 0, stream>>>((const h16*)a, (const h16*)b, (const h16*)c, (h16*)d,
                                                              P * C);
  } else {
    return -2;
  }
  return (int)hipGetLastError();
}
