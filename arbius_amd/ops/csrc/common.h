// Shared helpers for the gfx950 (CDNA4, MI355X) kernels of arbius_amd.
// Wave64 everywhere; bf16 storage, fp32 math; 16-byte vector global access.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ARB_API extern "C" __attribute__((visibility("default")))

typedef uint16_t bf16_t;  // raw bf16 bits
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// max of non-NaN floats as ONE instruction each: hipcc lowers fmaxf on MFMA results with a
// canonicalising v_max_f32 x, x per operand first (IEEE maxnum quieting), doubling the VALU of a
// softmax row max (MI355X_MICROARCH.md).  Inputs here are finite or -inf, so max is exact and
// order-free: bitwise the fmaxf result.
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float vmax2(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Lane pairs (l, l ^ 16) and (l, l ^ 32) combined with the gfx950 lane-swap VALU ops instead of
// __shfl_xor, which hipcc lowers to ds_bpermute_b32 (an LDS round trip in the softmax's critical
// chain).  permlane{16,32}_swap(x, x) returns {x with its odd 16-lane rows (upper 32 lanes) replaced by
// the even rows (lower half), x with its even rows (lower half) replaced by the odd rows (upper half)}:
// in every lane one element is x[l] and the other x[l ^ 16] (x[l ^ 32]).  max / + of the pair are
// exact and commutative, so the results are bitwise those of the shuffle forms.
__device__ __forceinline__ float max_xor16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax2(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float max_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax2(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_xor16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float sum_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// n zero-initialised int tickets for one launch on stream s (conv.hip's per-device pool): a region
// of its own per graph-captured launch, one shared region per stream for eager launches (same-
// stream kernels are serialised).  The launch's last arriving block re-arms its ticket to 0.
// nullptr: no pool (e.g. the first use is inside a capture) - the caller takes its two-kernel path.
int* arb_tickets(hipStream_t s, int n);

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// round-to-nearest-even f32 -> bf16 (NaN kept NaN via the cast path the compiler emits)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

// 16-byte accesses as ONE <4 x i32> IR load/store: a HIP uint4 struct copy is lowered as two
// <2 x i32> halves, and the second half's extra GEP can fall outside the LDS lowering's alias-
// scope walk - the merged ds_read_b128 then carries no scope and hipcc drains every LDS-DMA
// before it (s_waitcnt vmcnt(0)).
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16(const void* p) {
  const u32x4_t v = *reinterpret_cast<const u32x4_t*>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16(void* p, uint4 v) {
  *reinterpret_cast<u32x4_t*>(p) = (u32x4_t){v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ void unpack8(uint4 v, float (&f)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// round-to-nearest-even to bf16 and back (an intermediate the unfused op would store as bf16)
__device__ __forceinline__ float bf16_round(float v) { return __uint_as_float((uint32_t)f2bf(v) << 16); }

// raw v_exp_f32 / v_rcp_f32 (no denormal range fix-up sequences; results are bf16-rounded anyway)
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ float silu_f(float x) { return x * __builtin_amdgcn_rcpf(1.f + fast_exp(-x)); }
// GELU(erf) = x * Phi(x) with erfc from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7 on erf) on the
// raw rcp / exp2: ~16 VALU instead of ocml erff's ~40 - the GEGLU epilogue evaluates one per output of
// the feed-forward GEMMs.  Phi(x) = 1 - c/2 (x >= 0) or c/2 (x < 0) with c = erfc(|x| / sqrt 2), so the
// negative tail has no 1 + erf cancellation.
__device__ __forceinline__ float gelu_f(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  float q = fmaf(t, 1.061405429f, -1.453152027f);
  q = fmaf(t, q, 1.421413741f);
  q = fmaf(t, q, -0.284496736f);
  q = fmaf(t, q, 0.254829592f);
  const float c = q * t * __builtin_amdgcn_exp2f(z * z * -1.4426950408889634f);
  return x >= 0.f ? fmaf(-0.5f * c, x, x) : 0.5f * c * x;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5 / T1):
// consecutive logical tiles land on the same XCD (shared L2).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}
