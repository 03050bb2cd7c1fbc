// GroupNorm (+SiLU) over channels-last activations [B, HW, C] bf16.
//
// The normalisation of every ResBlock / Transformer2D input of the SD1.5 UNet
// and VAE.  Three short, wide kernels (each fills the chip;
// hipGraph replay keeps the launch gaps at ~1 us):
//   1. gn_stats    grid (chunks, B): each block walks ~64 KB of rows in slabs; per slab every
//      thread keeps RPT rows x 8 channels in registers (next slab's loads in flight), computes
//      EXACT per-channel (n, mean, M2) by two passes over registers and Chan-combines the slabs;
//      the block then combines them once
//      per group with the exact parallel-variance algebra
//      (N = sum n, mu = sum n*mean / N, M2 = sum [M2_c + n_c (mean_c - mu)^2]).
//   2. gn_finalize grid (G, B): one group per block, 256 threads combine the
//      chunk stats (Chan) and a fixed-shape LDS tree -> mean, rstd.
//   3. gn_apply    grid (blocks, B): normalise + gamma/beta (+SiLU), 16 B stores.
// No atomics, fixed reduction order everywhere -> bitwise deterministic, and the
// same partition for a given shape on every GPU.
#include "common.h"

#include <cstdlib>

#define GN_RPT 4  // rows per thread in the stats / apply kernels

struct Stat {
  float n, mean, m2, pad;
};

__device__ __forceinline__ Stat chan_combine(Stat a, Stat b) {
  if (b.n == 0.f) return a;
  if (a.n == 0.f) return b;
  const float n = a.n + b.n;
  const float d = b.mean - a.mean;
  const float f = b.n / n;
  Stat r;
  r.n = n;
  r.mean = a.mean + d * f;
  r.m2 = a.m2 + b.m2 + d * d * a.n * f;
  r.pad = 0.f;
  return r;
}

#define GN_TAIL_GPB 4
#define GN_TAIL_MAXG 32
struct GnTail {
  int* tickets;            // [B], zero on entry; null = partials only (separate table kernel)
  float2* table;
  const bf16_t* gamma;
  const bf16_t* beta;
  const bf16_t* mod;
  float one_plus, eps;
};

__device__ void gn_tail(const Stat* __restrict__ part, const GnTail& tl, int b, int chunks, int C, int G);

// Stats partition, a function of (HW, C) only - so the reduction order never depends on the
// batch (lock-step groups stay bitwise equal to solo tasks).  Large images (>= 1M elements per
// image): slabs of 8 rows per thread (16 x 16-B loads in flight with the next slab's), up to
// ~64 KB of rows per block and at least 16 blocks per image.  Small images: one 4-row slab per
// block (as many blocks as possible: these calls are latency-bound).
__host__ __device__ inline int gn_srpt(int HW, int C) { return (long)HW * C >= (1L << 20) ? 8 : 4; }
// One slab per block: the stats pass is bandwidth / latency bound, so it wants as many blocks in
// flight as possible (SD level 0 at batch 8: 688 blocks of ~30 KB instead of 344 of ~61 KB); the
// finalize / table combine of the extra partials costs far less than the idle CUs did.
__host__ __device__ inline int gn_iters(int HW, int C) { return 1; }

// Thread geometry: NV = C/8 channel vectors.  NV < 256: k = 256/NV row lanes, thread
// (v = t % NV, rl = t / NV).  NV >= 256: one row lane, thread owns vectors t, t+256 (VPT).
template <int VPT, int GN_SRPT, bool TAIL = false>
__global__ void __launch_bounds__(256) gn_stats_kernel(const bf16_t* __restrict__ x, Stat* __restrict__ part,
                                                       int HW, int C, int G, const bf16_t* __restrict__ x2, int C1,
                                                       GnTail tl) {
  const int chunk = blockIdx.x, b = blockIdx.y, chunks = gridDim.x;
  const int NV = C >> 3;
  const int k = NV >= 256 ? 1 : 256 / NV;
  const int t = threadIdx.x;
  const int v = NV >= 256 ? t : t % NV, rl = NV >= 256 ? 0 : t / NV;
  const int r0 = chunk * k * GN_SRPT * gn_iters(HW, C);
  __shared__ float sh_n[256];
  __shared__ float sh_mean[256 * 8 * VPT];
  __shared__ float sh_m2[256 * 8 * VPT];

  // Per channel vector: source tensor, row stride and channel offset.  x2 != null: the channels
  // [C1, C) live in x2 (a skip concat read in place; C1 % 8 == 0, so a vector never straddles).
  const bf16_t* sbase[VPT];
  int sstride[VPT], scoff[VPT];
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int ch = (v + 256 * j) * 8;
    const bool second = x2 != nullptr && ch >= C1;
    const int cs = x2 == nullptr ? C : (second ? C - C1 : C1);
    sbase[j] = (second ? x2 : x) + (size_t)b * HW * cs;
    sstride[j] = cs;
    scoff[j] = second ? ch - C1 : ch;
  }
  // The block walks ITER slabs of k*GN_SRPT rows (ITER from (HW, C) only: batch-invariant).  Per
  // slab each thread takes the EXACT (mean, M2) of its GN_SRPT rows per channel (two passes over
  // registers) and Chan-combines it into a running per-channel Stat; the next slab's loads are in
  // flight meanwhile.  The per-group LDS combine below then runs once per block, not per slab.
  const int iters = gn_iters(HW, C);
  Stat acc[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[j][e] = Stat{0.f, 0.f, 0.f, 0.f};
  uint4 raw[2][VPT][GN_SRPT];
  auto load = [&](uint4 (&dst)[VPT][GN_SRPT], int it) {
#pragma unroll
    for (int i = 0; i < GN_SRPT; ++i) {
      const int r = r0 + it * k * GN_SRPT + rl + i * k;
      const bool ok = rl < k && it < iters && r < HW;
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int vv = v + 256 * j;
        dst[j][i] = (ok && vv < NV) ? ld16(sbase[j] + (size_t)r * sstride[j] + scoff[j]) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  float nt = 0.f;
  auto process = [&](const uint4 (&src)[VPT][GN_SRPT], int it) {
    float n = 0.f;
#pragma unroll
    for (int i = 0; i < GN_SRPT; ++i) {
      const int r = r0 + it * k * GN_SRPT + rl + i * k;
      n += (rl < k && it < iters && r < HW) ? 1.f : 0.f;
    }
    if (n == 0.f) return;
    nt += n;
    const float inv_n = 1.f / n;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      float f[GN_SRPT][8];
#pragma unroll
      for (int i = 0; i < GN_SRPT; ++i) unpack8(src[j][i], f[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < GN_SRPT; ++i) s += f[i][e];
        const float mean = s * inv_n;
        float m2 = 0.f;
#pragma unroll
        for (int i = 0; i < GN_SRPT; ++i) {
          const int r = r0 + it * k * GN_SRPT + rl + i * k;
          const float d = f[i][e] - mean;
          m2 += (rl < k && r < HW) ? d * d : 0.f;
        }
        acc[j][e] = chan_combine(acc[j][e], Stat{n, mean, m2, 0.f});
      }
    }
  };
  // two register sets: slab it+1 is loading while slab it is reduced
  load(raw[0], 0);
  for (int it = 0; it < iters; it += 2) {
    load(raw[1], it + 1);
    process(raw[0], it);
    if (it + 1 >= iters) break;
    load(raw[0], it + 2);
    process(raw[1], it + 1);
  }
  sh_n[t] = nt;
#pragma unroll
  for (int j = 0; j < VPT; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sh_mean[(t * VPT + j) * 8 + e] = acc[j][e].mean;
      sh_m2[(t * VPT + j) * 8 + e] = acc[j][e].m2;
    }
  __syncthreads();
  // Per-group combine, parallel: L = 256/G lanes per group (consecutive lanes of one wave),
  // each takes every L-th (channel, row-lane) item; the L partials are merged by a fixed
  // xor-shuffle butterfly -> deterministic.
  const int Cg = C / G;
  int L = 1;  // largest power of two with G * L <= 256, at most one wave
  while (L < 64 && 2 * L * G <= 256) L *= 2;
  const int g = t / L, sl = t % L;
  const int items = Cg * k;
  float N = 0.f, sum = 0.f;
  if (g < G) {
    for (int it = sl; it < items; it += L) {
      const int c = g * Cg + it / k, j = it % k;
      const int vv = c >> 3, e = c & 7;
      const int tt = NV >= 256 ? (vv & 255) : j * NV + vv;
      const int o = (tt * VPT + (NV >= 256 ? (vv >> 8) : 0)) * 8 + e;
      N += sh_n[tt];
      sum += sh_n[tt] * sh_mean[o];
    }
  }
  for (int o = 1; o < L; o <<= 1) {
    N += __shfl_xor(N, o, 64);
    sum += __shfl_xor(sum, o, 64);
  }
  const float mu = N > 0.f ? sum / N : 0.f;
  float m2 = 0.f;
  if (g < G) {
    for (int it = sl; it < items; it += L) {
      const int c = g * Cg + it / k, j = it % k;
      const int vv = c >> 3, e = c & 7;
      const int tt = NV >= 256 ? (vv & 255) : j * NV + vv;
      const int o = (tt * VPT + (NV >= 256 ? (vv >> 8) : 0)) * 8 + e;
      const float d = sh_mean[o] - mu;
      m2 += sh_m2[o] + sh_n[tt] * d * d;
    }
  }
  for (int o = 1; o < L; o <<= 1) m2 += __shfl_xor(m2, o, 64);
  if (g < G && sl == 0) {
    Stat st = {N, mu, m2, 0.f};
    part[((size_t)b * chunks + chunk) * G + g] = st;
  }
  if constexpr (TAIL) gn_tail(part, tl, b, chunks, C, G);
}

__global__ void __launch_bounds__(256) gn_finalize_kernel(const Stat* __restrict__ part, float2* __restrict__ stats,
                                                          int chunks, int G, float eps) {
  const int g = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  __shared__ Stat sh[256];
  Stat acc = {0.f, 0.f, 0.f, 0.f};
  for (int c = t; c < chunks; c += 256) acc = chan_combine(acc, part[((size_t)b * chunks + c) * G + g]);
  sh[t] = acc;
  __syncthreads();
#pragma unroll
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) sh[t] = chan_combine(sh[t], sh[t + s]);
    __syncthreads();
  }
  if (t == 0) {
    const Stat r = sh[0];
    stats[b * G + g] = make_float2(r.mean, rsqrtf(r.m2 / fmaxf(r.n, 1.f) + eps));
  }
}

// MOD: per-pixel modulation after the affine GN, read from a [B, mh, mw, 2C] map
// at (nearest-)lower resolution:  out = gn * (y + one_plus) + b   (y = channels
// [0,C), b = [C,2C)).  SpatialNorm of the MoVQ decoder (mh x mw = latent grid,
// computed once per layer at latent resolution) and the scale-shift norm of the
// GLIDE ResBlock (mh = mw = 1, one_plus = 1) both run as this one pass.
template <int VPT, bool MOD>
__global__ void __launch_bounds__(256) gn_apply_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                       const float2* __restrict__ stats,
                                                       const bf16_t* __restrict__ gamma,
                                                       const bf16_t* __restrict__ beta, int HW, int C, int G,
                                                       int silu, const bf16_t* __restrict__ mod, int W, int H,
                                                       int mh, int mw, float one_plus) {
  const int blk = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  __shared__ float2 sh_st[256];
  if (t < G) sh_st[t] = stats[b * G + t];
  __syncthreads();
  const int NV = C >> 3;
  const int k = NV >= 256 ? 1 : 256 / NV;
  const int v = NV >= 256 ? t : t % NV, rl = NV >= 256 ? 0 : t / NV;
  if (rl >= k) return;
  const int Cg = C / G;
  const int r0 = blk * k * GN_RPT;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int vv = v + 256 * j;
    if (vv >= NV) continue;
    float sc[8], sf[8];
    {
      float gm[8], bt[8];
      unpack8(ld16(gamma + vv * 8), gm);
      unpack8(ld16(beta + vv * 8), bt);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float2 st = sh_st[(vv * 8 + e) / Cg];
        sc[e] = st.y * gm[e];
        sf[e] = bt[e] - st.x * sc[e];
      }
    }
    const size_t off = ((size_t)b * HW) * C + vv * 8;
    uint4 raw[GN_RPT];
#pragma unroll
    for (int i = 0; i < GN_RPT; ++i) {
      const int r = r0 + rl + i * k;
      raw[i] = r < HW ? ld16(x + off + (size_t)r * C) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < GN_RPT; ++i) {
      const int r = r0 + rl + i * k;
      if (r >= HW) continue;
      float f[8];
      unpack8(raw[i], f);
      if constexpr (MOD) {
        const int my = (r / W) * mh / H, mx = (r % W) * mw / W;
        const bf16_t* mp = mod + (((size_t)b * mh + my) * mw + mx) * (2 * C) + vv * 8;
        float my8[8], mb8[8];
        unpack8(ld16(mp), my8);
        unpack8(ld16(mp + C), mb8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float o = (f[e] * sc[e] + sf[e]) * (my8[e] + one_plus) + mb8[e];
          f[e] = silu ? silu_f(o) : o;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float o = f[e] * sc[e] + sf[e];
          f[e] = silu ? silu_f(o) : o;
        }
      }
      st16(y + off + (size_t)r * C, pack8(f));
    }
  }
}

static int gn_chunks(int HW, int C) {
  const int NV = C / 8;
  const int k = NV >= 256 ? 1 : 256 / NV;
  const int rows = k * GN_RPT;
  return (HW + rows - 1) / rows;
}

// stats blocks per image: gn_iters slabs of k * gn_srpt rows each
static int gn_stat_chunks(int HW, int C) {
  const int NV = C / 8;
  const int k = NV >= 256 ? 1 : 256 / NV;
  const int rows = k * gn_srpt(HW, C) * gn_iters(HW, C);
  return (HW + rows - 1) / rows;
}

static void launch_gn_stats(const void* x, Stat* part, int B, int HW, int C, int G, hipStream_t stream,
                            const void* x2 = nullptr, int C1 = 0, GnTail tl = GnTail{}) {
  dim3 grid(gn_stat_chunks(HW, C), B);
  const bool wide = C / 8 > 256, big = gn_srpt(HW, C) == 8;
  const bf16_t* xb = (const bf16_t*)x;
  const bf16_t* xb2 = (const bf16_t*)x2;
  const bool tail = tl.tickets != nullptr;
  if (wide) {
    if (big) gn_stats_kernel<2, 8><<<grid, 256, 0, stream>>>(xb, part, HW, C, G, xb2, C1, tl);
    else if (tail) gn_stats_kernel<2, 4, true><<<grid, 256, 0, stream>>>(xb, part, HW, C, G, xb2, C1, tl);
    else gn_stats_kernel<2, 4><<<grid, 256, 0, stream>>>(xb, part, HW, C, G, xb2, C1, tl);
  } else {
    if (big && tail) gn_stats_kernel<1, 8, true><<<grid, 256, 0, stream>>>(xb, part, HW, C, G, xb2, C1, tl);
    else if (big) gn_stats_kernel<1, 8><<<grid, 256, 0, stream>>>(xb, part, HW, C, G, xb2, C1, tl);
    else if (tail) gn_stats_kernel<1, 4, true><<<grid, 256, 0, stream>>>(xb, part, HW, C, G, xb2, C1, tl);
    else gn_stats_kernel<1, 4><<<grid, 256, 0, stream>>>(xb, part, HW, C, G, xb2, C1, tl);
  }
}

ARB_API size_t arb_group_norm_workspace(int B, int HW, int C, int G) {
  // partial stats + final (mean, rstd); 256-byte aligned split
  const size_t part = (size_t)B * gn_stat_chunks(HW, C) * G * sizeof(Stat);
  return ((part + 255) / 256) * 256 + (size_t)B * G * sizeof(float2);
}

// One block per (group, batch) for small groups of rows (HW * Cg <= GN_GROUP_MAX elements, the
// UNet levels): the block reads its group's Cg channels of every row (Cg/2 dword loads per row),
// takes each row's exact (mean, M2) over its Cg values, Chan-combines rows per thread and then
// across the block in a fixed LDS tree, and writes the group's affine table (or mean / rstd)
// directly: one launch instead of stats + table, and no partials round trip.  The choice
// depends on (HW, C, G) only - never on the batch - so lock-step groups stay bitwise equal to
// solo runs.
#define GN_GROUP_MAX 65536
#define GN_GROUP_THREADS 1024
template <int CWMAX, int U>
__global__ void __launch_bounds__(GN_GROUP_THREADS) gn_group_kernel(
    const bf16_t* __restrict__ x, float2* __restrict__ table, float2* __restrict__ stats,
    const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta, const bf16_t* __restrict__ mod,
    float one_plus, int HW, int C, int G, float eps, const bf16_t* __restrict__ x2, int C1) {
  const int g = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int Cg = C / G, Cw = Cg >> 1;                 // Cg even (C % 8 == 0, checked by the host)
  // channels [0, C1) from x (row stride C1), [C1, C) from x2 (a skip concat read in place; C1 even, so
  // a dword never straddles); C1 == C without x2
  const int g0 = g * Cg;
  const uint32_t* base1 = reinterpret_cast<const uint32_t*>(x + (size_t)b * HW * C1);
  const uint32_t* base2 = x2 ? reinterpret_cast<const uint32_t*>(x2 + (size_t)b * HW * (C - C1)) : nullptr;
  const int rowd1 = C1 >> 1, rowd2 = (C - C1) >> 1;   // row strides in dwords
  Stat acc = {0.f, 0.f, 0.f, 0.f};
  for (int r0 = 0; r0 < HW; r0 += U * GN_GROUP_THREADS) {
    uint32_t w[U][CWMAX];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = r0 + u * GN_GROUP_THREADS + t;
#pragma unroll
      for (int j = 0; j < CWMAX; ++j)
        if (j < Cw) {
          const int c = g0 + 2 * j;
          w[u][j] = r >= HW ? 0u
                    : c < C1 ? base1[(size_t)r * rowd1 + (c >> 1)] : base2[(size_t)r * rowd2 + ((c - C1) >> 1)];
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = r0 + u * GN_GROUP_THREADS + t;
      if (r >= HW) continue;
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < CWMAX; ++j)
        if (j < Cw) s += __uint_as_float(w[u][j] << 16) + __uint_as_float(w[u][j] & 0xffff0000u);
      const float mean = s / (float)Cg;
      float m2 = 0.f;
#pragma unroll
      for (int j = 0; j < CWMAX; ++j)
        if (j < Cw) {
          const float d0 = __uint_as_float(w[u][j] << 16) - mean, d1 = __uint_as_float(w[u][j] & 0xffff0000u) - mean;
          m2 += d0 * d0 + d1 * d1;
        }
      acc = chan_combine(acc, Stat{(float)Cg, mean, m2, 0.f});
    }
  }
  __shared__ Stat sh[GN_GROUP_THREADS];
  sh[t] = acc;
  __syncthreads();
#pragma unroll
  for (int st = GN_GROUP_THREADS / 2; st > 0; st >>= 1) {
    if (t < st) sh[t] = chan_combine(sh[t], sh[t + st]);
    __syncthreads();
  }
  const Stat r = sh[0];
  const float mean = r.mean, rstd = rsqrtf(r.m2 / fmaxf(r.n, 1.f) + eps);
  if (stats != nullptr) {
    if (t == 0) stats[b * G + g] = make_float2(mean, rstd);
    return;
  }
  for (int i = t; i < Cg; i += GN_GROUP_THREADS) {
    const int c = g * Cg + i;
    float sc = rstd * bf2f(gamma[c]);
    float sf = bf2f(beta[c]) - mean * sc;
    if (mod) {
      const float m = bf2f(mod[(size_t)b * 2 * C + c]) + one_plus, a = bf2f(mod[(size_t)b * 2 * C + C + c]);
      sc *= m;
      sf = fmaf(sf, m, a);
    }
    table[(size_t)b * C + c] = make_float2(sc, sf);
  }
}

// One block per (group, image) building the table directly: opt-in (ARB_GN_GROUP=1: HW <= 256 only,
// 2: every eligible shape).  Measured slower than stats + table at every SD1.5 level (r3: 36 vs 14 us
// at [8, 16, 16, 1280], 30 vs 12 us at [8, 8, 8, 1280]; r2: 2.5 % end to end used everywhere) - the
// 1024-thread blocks walk whole groups with most lanes idle.  Batch-invariant either way; reads a
// skip concat in place like the slab path.
static bool gn_group_path(int HW, int C, int G) {
  static const int mode = [] {
    const char* e = std::getenv("ARB_GN_GROUP");
    return e ? std::atoi(e) : 0;
  }();
  const int Cg = C / G;
  if (mode == 0 || Cg % 2 != 0 || Cg > 64 || (long)HW * Cg > GN_GROUP_MAX) return false;
  return mode == 2 || HW <= 256;
}

// table != null: affine table; else stats (mean, rstd)
static void launch_gn_group(const void* x, float2* table, float2* stats, const void* gamma, const void* beta,
                            const void* mod, float one_plus, int B, int HW, int C, int G, float eps,
                            hipStream_t stream, const void* x2 = nullptr, int C1 = 0) {
  if (x2 == nullptr) C1 = C;
  const int Cw = C / G / 2;
  dim3 grid(G, B);
#define GN_GROUP_LAUNCH(CW, U)                                                                                   \
  gn_group_kernel<CW, U><<<grid, GN_GROUP_THREADS, 0, stream>>>((const bf16_t*)x, table, stats, (const bf16_t*)gamma, \
                                                                (const bf16_t*)beta, (const bf16_t*)mod, one_plus, HW, \
                                                                C, G, eps, (const bf16_t*)x2, C1)
  if (Cw <= 8) GN_GROUP_LAUNCH(8, 4);
  else if (Cw <= 20) GN_GROUP_LAUNCH(20, 2);
  else GN_GROUP_LAUNCH(32, 1);
#undef GN_GROUP_LAUNCH
}

static int gn_run(const void* x, void* y, const void* gamma, const void* beta, void* workspace, int B, int HW,
                  int C, int G, float eps, int silu, const void* mod, int H, int W, int mh, int mw, float one_plus,
                  hipStream_t stream) {
  if (C % 8 != 0 || C / 8 > 512 || C % G != 0 || G > 256) return -1;
  const int chunks = gn_chunks(HW, C), schunks = gn_stat_chunks(HW, C);
  Stat* part = (Stat*)workspace;
  const size_t part_bytes = ((size_t)B * schunks * G * sizeof(Stat) + 255) / 256 * 256;
  float2* stats = (float2*)((char*)workspace + part_bytes);
  dim3 g1(chunks, B);
  const bool wide = C / 8 > 256;
  if (gn_group_path(HW, C, G)) {
    launch_gn_group(x, nullptr, stats, nullptr, nullptr, nullptr, 0.f, B, HW, C, G, eps, stream);
  } else {
    launch_gn_stats(x, part, B, HW, C, G, stream);
    gn_finalize_kernel<<<dim3(G, B), 256, 0, stream>>>(part, stats, schunks, G, eps);
  }
#define GN_APPLY(VPT, MOD)                                                                                    \
  gn_apply_kernel<VPT, MOD><<<g1, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, stats, (const bf16_t*)gamma, \
                                                    (const bf16_t*)beta, HW, C, G, silu, (const bf16_t*)mod, W, H, \
                                                    mh, mw, one_plus)
  if (mod) {
    if (wide) GN_APPLY(2, true); else GN_APPLY(1, true);
  } else {
    if (wide) GN_APPLY(2, false); else GN_APPLY(1, false);
  }
#undef GN_APPLY
  return (int)hipGetLastError();
}

ARB_API int arb_group_norm_nhwc(const void* x, void* y, const void* gamma, const void* beta, void* workspace, int B,
                                int HW, int C, int G, float eps, int silu, hipStream_t stream) {
  return gn_run(x, y, gamma, beta, workspace, B, HW, C, G, eps, silu, nullptr, 1, HW, 1, 1, 0.f, stream);
}

// x [B, H, W, C]; mod [B, mh, mw, 2C] with H % mh == 0 and W % mw == 0.
ARB_API int arb_group_norm_mod_nhwc(const void* x, void* y, const void* gamma, const void* beta, void* workspace,
                                    const void* mod, int B, int H, int W, int C, int G, float eps, int silu, int mh,
                                    int mw, float one_plus, hipStream_t stream) {
  if (mh <= 0 || mw <= 0 || H % mh != 0 || W % mw != 0) return -1;
  return gn_run(x, y, gamma, beta, workspace, B, H * W, C, G, eps, silu, mod, H, W, mh, mw, one_plus, stream);
}

// ---------------------------------------------------------------------------------------------
// GroupNorm as an affine TABLE for a consumer's prologue (conv / GEMM A-operand transform):
//   table[b, c] = (scale, shift),  GN(x)[b, p, c] = x * scale + shift
// with an optional per-(b, c) modulation folded in (GLIDE scale-shift norm):
//   out = GN(x) * (mod[b, c] + one_plus) + mod[b, C + c]  ->  scale *= m, shift = shift * m + t
// Grid (G, B): the exact Chan combine of gn_finalize, then Cg threads write the group's channels.
__global__ void __launch_bounds__(256) gn_table_kernel(const Stat* __restrict__ part, float2* __restrict__ table,
                                                       const bf16_t* __restrict__ gamma,
                                                       const bf16_t* __restrict__ beta,
                                                       const bf16_t* __restrict__ mod, float one_plus, int chunks,
                                                       int C, int G, float eps) {
  const int g = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  __shared__ Stat sh[256];
  Stat acc = {0.f, 0.f, 0.f, 0.f};
  for (int c = t; c < chunks; c += 256) acc = chan_combine(acc, part[((size_t)b * chunks + c) * G + g]);
  sh[t] = acc;
  __syncthreads();
#pragma unroll
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) sh[t] = chan_combine(sh[t], sh[t + s]);
    __syncthreads();
  }
  const Stat r = sh[0];
  const float mean = r.mean, rstd = rsqrtf(r.m2 / fmaxf(r.n, 1.f) + eps);
  const int Cg = C / G;
  for (int i = t; i < Cg; i += 256) {
    const int c = g * Cg + i;
    float sc = rstd * bf2f(gamma[c]);
    float sf = bf2f(beta[c]) - mean * sc;
    if (mod) {
      const float m = bf2f(mod[(size_t)b * 2 * C + c]) + one_plus, a = bf2f(mod[(size_t)b * 2 * C + C + c]);
      sc *= m;
      sf = fmaf(sf, m, a);
    }
    table[(size_t)b * C + c] = make_float2(sc, sf);
  }
}

// gn_table as ONE WAVE per (group, image): the same combine tree as the 256-thread LDS version, bit for
// bit - lane l holds tree leaves l, l+64, l+128, l+192 (leaf t = the sequential Chan combine of chunks
// t, t+256, ...); levels 128 and 64 combine in-lane, levels 32..1 through __shfl_down (node t takes node
// t+s) - with no LDS round trips and no block barriers (the 256-thread version was launch/latency bound:
// 6 us per call, 2 % of the SD1.5 bench's kernel time).
// Tree leaves of lane l for group g of image b: leaf q = the sequential Chan combine of chunks l + 64q,
// l + 64q + 256, ...
__device__ __forceinline__ void gn_table_leaves(const Stat* __restrict__ part, int b, int chunks, int G, int g, int l,
                                                Stat (&leaf)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    Stat acc = {0.f, 0.f, 0.f, 0.f};
    for (int c = l + 64 * q; c < chunks; c += 256) acc = chan_combine(acc, part[((size_t)b * chunks + c) * G + g]);
    leaf[q] = acc;
  }
}

// The rest of the one-wave table: combine tree over the 4 x 64 leaves, then the group's Cg table entries.
__device__ __forceinline__ void gn_table_tree(Stat (&leaf)[4], float2* __restrict__ table,
                                              const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta,
                                              const bf16_t* __restrict__ mod, float one_plus, int C, int G, float eps,
                                              int g, int b, int l) {
  // level 128: t <- (t, t + 128) for t < 128  (t = l: leaf 0 with leaf 2; t = l + 64: leaf 1 with leaf 3)
  Stat n0 = chan_combine(leaf[0], leaf[2]);
  const Stat n1 = chan_combine(leaf[1], leaf[3]);
  // level 64: t <- (t, t + 64) for t < 64
  n0 = chan_combine(n0, n1);
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    Stat o;
    o.n = __shfl_down(n0.n, s, 64);
    o.mean = __shfl_down(n0.mean, s, 64);
    o.m2 = __shfl_down(n0.m2, s, 64);
    o.pad = 0.f;
    n0 = chan_combine(n0, o);
  }
  const float mean = __shfl(n0.mean, 0, 64), m2 = __shfl(n0.m2, 0, 64), n = __shfl(n0.n, 0, 64);
  const float rstd = rsqrtf(m2 / fmaxf(n, 1.f) + eps);
  const int Cg = C / G;
  for (int i = l; i < Cg; i += 64) {
    const int c = g * Cg + i;
    float sc = rstd * bf2f(gamma[c]);
    float sf = bf2f(beta[c]) - mean * sc;
    if (mod) {
      const float m = bf2f(mod[(size_t)b * 2 * C + c]) + one_plus, a = bf2f(mod[(size_t)b * 2 * C + C + c]);
      sc *= m;
      sf = fmaf(sf, m, a);
    }
    table[(size_t)b * C + c] = make_float2(sc, sf);
  }
}

__global__ void __launch_bounds__(64) gn_table_wave_kernel(const Stat* __restrict__ part, float2* __restrict__ table,
                                                           const bf16_t* __restrict__ gamma,
                                                           const bf16_t* __restrict__ beta,
                                                           const bf16_t* __restrict__ mod, float one_plus,
                                                           int chunks, int C, int G, float eps) {
  const int g = blockIdx.x, b = blockIdx.y, l = threadIdx.x;
  Stat leaf[4];
  gn_table_leaves(part, b, chunks, G, g, l, leaf);
  gn_table_tree(leaf, table, gamma, beta, mod, one_plus, C, G, eps, g, b, l);
}

// Statistics + table in ONE launch, bitwise equal to gn_stats + gn_table_wave: the stats blocks of
// image b take a ticket after their partials are stored (agent-scope release before it); the block
// that draws the last one (acquire) runs gn_table_wave's arithmetic for every group of the image,
// wave w taking groups w, w + 4, ... with the leaf loads of GPB groups in flight together, then
// re-arms the ticket.  Saves the table launch and its cross-XCD partials round trip (K2 solo: ~96
// GroupNorms per UNet step).  G <= GN_TAIL_MAXG (4 waves x 2 batches of GPB).  Not on the wide
// big-image variant (C > 2048 at >= 1M elements per image): there the tail's registers spill.
__device__ void gn_tail(const Stat* __restrict__ part, const GnTail& tl, int b, int chunks, int C,
                                        int G) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this block's partials are stored
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const int t = __hip_atomic_fetch_add(&tl.tickets[b], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == chunks - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __syncthreads();
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int i0 = 0; i0 < GN_TAIL_MAXG / 4; i0 += GN_TAIL_GPB) {
    Stat leaf[GN_TAIL_GPB][4];
    if (chunks <= 256) {   // one partial per leaf at most: every load of the batch in flight at once
      Stat raw[GN_TAIL_GPB][4];
#pragma unroll
      for (int i = 0; i < GN_TAIL_GPB; ++i) {
        const int g = w + 4 * (i0 + i);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = l + 64 * q;
          raw[i][q] = (g < G && c < chunks) ? part[((size_t)b * chunks + c) * G + g] : Stat{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int i = 0; i < GN_TAIL_GPB; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) leaf[i][q] = chan_combine(Stat{0.f, 0.f, 0.f, 0.f}, raw[i][q]);
    } else {
#pragma unroll
      for (int i = 0; i < GN_TAIL_GPB; ++i) {
        const int g = w + 4 * (i0 + i);
        if (g < G) gn_table_leaves(part, b, chunks, G, g, l, leaf[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < GN_TAIL_GPB; ++i) {
      const int g = w + 4 * (i0 + i);
      if (g < G) gn_table_tree(leaf[i], tl.table, tl.gamma, tl.beta, tl.mod, tl.one_plus, C, G, tl.eps, g, b, l);
    }
  }
  if (threadIdx.x == 0) tl.tickets[b] = 0;   // re-arm for the next launch on this region
}

// A/B switch (bitwise-equal variants): ARB_GN_TABLE_LDS=1 or arb_set_gn_table_lds(1) -> the 256-thread
// LDS-tree table kernel instead of the one-wave one (tests/test_kernels_gpu.py compares the two).
static int g_gn_table_lds = -1;
static bool gn_table_lds() {
  if (g_gn_table_lds < 0) {
    const char* e = std::getenv("ARB_GN_TABLE_LDS");
    g_gn_table_lds = (e != nullptr && e[0] == '1') ? 1 : 0;
  }
  return g_gn_table_lds == 1;
}
ARB_API void arb_set_gn_table_lds(int on) { g_gn_table_lds = on ? 1 : 0; }

static int gn_table_run(const void* x, const void* x2, int C1, const void* gamma, const void* beta, const void* mod,
                        float one_plus, void* workspace, void* table, int B, int HW, int C, int G, float eps,
                        hipStream_t stream);

// Opt-in (ARB_GN_TAIL=1 or arb_set_gn_tail(1)); bitwise equal to the two launches either way.
// Measured slower everywhere (round 5, same box: SD 4x4 31.0k -> 28.1k tasks/h, K2 solo 1.09 ->
// 1.26 s): every stats block's agent-scope release before its ticket is an L2 write-back on
// MI355X, which costs far more than the table launch it saves (profiles/k2_plan_r5.md).
static int g_gn_tail = -1;
static bool gn_tail_on() {
  if (g_gn_tail < 0) {
    const char* e = std::getenv("ARB_GN_TAIL");
    g_gn_tail = (e != nullptr && e[0] == '1') ? 1 : 0;
  }
  return g_gn_tail == 1;
}
ARB_API void arb_set_gn_tail(int on) { g_gn_tail = on ? 1 : 0; }

// ---------------------------------------------------------------------------------------------
// Small images (HW * C <= GN_FUSED_MAX, the deep UNet levels): statistics AND table in ONE launch.
// Grid (G / GB, B): a block owns GB consecutive groups (CB = GB * Cg channels, a multiple of 8) of
// one image and walks every row of them - thread (v, rl) takes channel vector v of the slice and
// rows rl, rl + k, ... (k = 256 / (CB / 8) row lanes), 4 rows' 16-byte loads in flight, exact
// per-channel (n, mean, M2) per 4-row batch Chan-combined; then a fixed LDS / xor-butterfly combine
// per group and the (scale, shift) table of the slice.  Two launches (stats partials + table) and
// the partials round trip become one; the partition depends on (HW, C, G) only, never on the batch.
#define GN_FUSED_MAX (1 << 20)
__host__ __device__ inline int gn_fused_gb(int C, int G) {
  const int Cg = C / G;
  for (int gb = 1; gb <= G && gb <= 8; ++gb)
    if (G % gb == 0 && (gb * Cg) % 8 == 0 && (gb * Cg) / 8 <= 128) return gb;
  return 0;
}

__global__ void __launch_bounds__(256) gn_fused_table_kernel(
    const bf16_t* __restrict__ x, float2* __restrict__ table, const bf16_t* __restrict__ gamma,
    const bf16_t* __restrict__ beta, const bf16_t* __restrict__ mod, float one_plus, int HW, int C, int G, int GB,
    float eps, const bf16_t* __restrict__ x2, int C1) {
  const int gs = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int Cg = C / G, CB = GB * Cg, NVB = CB >> 3;
  const int k = 256 / NVB;
  const int v = t % NVB, rl = t / NVB;
  const int c0 = gs * CB, ch = c0 + 8 * v;
  const bool active = rl < k;
  __shared__ float sh_n[256];
  __shared__ float sh_mean[256 * 8];
  __shared__ float sh_m2[256 * 8];
  __shared__ float2 sh_g[8];
  const bool second = x2 != nullptr && ch >= C1;
  const int cs = x2 == nullptr ? C : (second ? C - C1 : C1);
  const bf16_t* base = (second ? x2 : x) + (size_t)b * HW * cs + (second ? ch - C1 : ch);
  Stat acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = Stat{0.f, 0.f, 0.f, 0.f};
  float nt = 0.f;
  if (active) {
    for (int r0 = rl; r0 < HW; r0 += 4 * k) {
      uint4 raw[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = r0 + i * k;
        raw[i] = r < HW ? ld16(base + (size_t)r * cs) : make_uint4(0, 0, 0, 0);
      }
      float n = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) n += (r0 + i * k < HW) ? 1.f : 0.f;
      nt += n;
      const float inv_n = 1.f / n;
      float f[4][8];
#pragma unroll
      for (int i = 0; i < 4; ++i) unpack8(raw[i], f[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float sm = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) sm += f[i][e];
        const float mean = sm * inv_n;
        float m2 = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float d = f[i][e] - mean;
          m2 += (r0 + i * k < HW) ? d * d : 0.f;
        }
        acc[e] = chan_combine(acc[e], Stat{n, mean, m2, 0.f});
      }
    }
  }
  sh_n[t] = nt;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sh_mean[t * 8 + e] = acc[e].mean;
    sh_m2[t * 8 + e] = acc[e].m2;
  }
  __syncthreads();
  // per group of the slice: L lanes (one wave at most) take every L-th (channel, row lane) item
  int L = 1;
  while (L < 64 && 2 * L * GB <= 256) L *= 2;
  const int g = t / L, sl = t % L;
  const int items = Cg * k;
  float N = 0.f, sum = 0.f;
  if (g < GB) {
    for (int it = sl; it < items; it += L) {
      const int c = g * Cg + it / k, j = it % k;           // channel within the slice, row lane
      const int tt = j * NVB + (c >> 3), o = tt * 8 + (c & 7);
      N += sh_n[tt];
      sum += sh_n[tt] * sh_mean[o];
    }
  }
  for (int o = 1; o < L; o <<= 1) {
    N += __shfl_xor(N, o, 64);
    sum += __shfl_xor(sum, o, 64);
  }
  const float mu = N > 0.f ? sum / N : 0.f;
  float m2 = 0.f;
  if (g < GB) {
    for (int it = sl; it < items; it += L) {
      const int c = g * Cg + it / k, j = it % k;
      const int tt = j * NVB + (c >> 3), o = tt * 8 + (c & 7);
      const float d = sh_mean[o] - mu;
      m2 += sh_m2[o] + sh_n[tt] * d * d;
    }
  }
  for (int o = 1; o < L; o <<= 1) m2 += __shfl_xor(m2, o, 64);
  if (g < GB && sl == 0) sh_g[g] = make_float2(mu, rsqrtf(m2 / fmaxf(N, 1.f) + eps));
  __syncthreads();
  for (int i = t; i < CB; i += 256) {
    const int c = c0 + i;
    const float2 st = sh_g[i / Cg];
    float sc = st.y * bf2f(gamma[c]);
    float sf = bf2f(beta[c]) - st.x * sc;
    if (mod) {
      const float m = bf2f(mod[(size_t)b * 2 * C + c]) + one_plus, a = bf2f(mod[(size_t)b * 2 * C + C + c]);
      sc *= m;
      sf = fmaf(sf, m, a);
    }
    table[(size_t)b * C + c] = make_float2(sc, sf);
  }
}

// Opt-in (ARB_GN_FUSED=1): measured slower than stats + table on the SD1.5 batch-8 shapes under
// graph replay (10.6 vs 7.8 us at [8, 8, 8, 1280], 11.9 vs 8.7 at [8, 16, 16, 1280], 15.1 vs 11.0
// at [8, 32, 32, 640]: profiles/norm_kernels_ab_r3.jsonl) - 256 small blocks spend their time in
// the per-group (channel x row-lane) LDS combine, while the two-kernel path spreads it.
static bool gn_fused_path(int HW, int C, int G) {
  static const bool on = [] {
    const char* e = std::getenv("ARB_GN_FUSED");
    return e != nullptr && e[0] == '1';
  }();
  return on && (long)HW * C <= GN_FUSED_MAX && gn_fused_gb(C, G) > 0;
}

ARB_API int arb_group_norm_table(const void* x, const void* gamma, const void* beta, const void* mod, float one_plus,
                                 void* workspace, void* table, int B, int HW, int C, int G, float eps,
                                 hipStream_t stream) {
  return gn_table_run(x, nullptr, 0, gamma, beta, mod, one_plus, workspace, table, B, HW, C, G, eps, stream);
}

// GroupNorm table over the channel concat [x | x2] (x: C1 channels, x2: C - C1) without materialising it.
ARB_API int arb_group_norm_table_cat(const void* x, const void* x2, int C1, const void* gamma, const void* beta,
                                     const void* mod, float one_plus, void* workspace, void* table, int B, int HW,
                                     int C, int G, float eps, hipStream_t stream) {
  if (x2 == nullptr || C1 <= 0 || C1 >= C || C1 % 8 != 0) return -1;
  return gn_table_run(x, x2, C1, gamma, beta, mod, one_plus, workspace, table, B, HW, C, G, eps, stream);
}

static int gn_table_run(const void* x, const void* x2, int C1, const void* gamma, const void* beta, const void* mod,
                        float one_plus, void* workspace, void* table, int B, int HW, int C, int G, float eps,
                        hipStream_t stream) {
  if (C % 8 != 0 || C / 8 > 512 || C % G != 0 || G > 256) return -1;
  if (gn_group_path(HW, C, G)) {   // same path (and bits) with or without the concat read in place
    launch_gn_group(x, (float2*)table, nullptr, gamma, beta, mod, one_plus, B, HW, C, G, eps, stream, x2, C1);
    return (int)hipGetLastError();
  }
  if (gn_fused_path(HW, C, G)) {   // small images: stats + table in one launch (concat read in place)
    const int gb = gn_fused_gb(C, G);
    gn_fused_table_kernel<<<dim3(G / gb, B), 256, 0, stream>>>(
        (const bf16_t*)x, (float2*)table, (const bf16_t*)gamma, (const bf16_t*)beta, (const bf16_t*)mod, one_plus,
        HW, C, G, gb, eps, (const bf16_t*)x2, x2 ? C1 : C);
    return (int)hipGetLastError();
  }
  const int chunks = gn_stat_chunks(HW, C);
  Stat* part = (Stat*)workspace;
  if (gn_tail_on() && !gn_table_lds() && G <= GN_TAIL_MAXG && (gn_srpt(HW, C) == 4 || C / 8 <= 256)) {
    int* tickets = arb_tickets(stream, B);
    if (tickets != nullptr) {   // statistics + table in one launch (bitwise equal)
      launch_gn_stats(x, part, B, HW, C, G, stream, x2, C1,
                      GnTail{tickets, (float2*)table, (const bf16_t*)gamma, (const bf16_t*)beta, (const bf16_t*)mod,
                             one_plus, eps});
      return (int)hipGetLastError();
    }
  }
  launch_gn_stats(x, part, B, HW, C, G, stream, x2, C1);
  if (gn_table_lds())
    gn_table_kernel<<<dim3(G, B), 256, 0, stream>>>(part, (float2*)table, (const bf16_t*)gamma, (const bf16_t*)beta,
                                                    (const bf16_t*)mod, one_plus, chunks, C, G, eps);
  else
    gn_table_wave_kernel<<<dim3(G, B), 64, 0, stream>>>(part, (float2*)table, (const bf16_t*)gamma,
                                                        (const bf16_t*)beta, (const bf16_t*)mod, one_plus, chunks, C,
                                                        G, eps);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// GroupNorm (+scale-shift modulation)(+SiLU) of SMALL (group, image) slices in ONE launch: statistics,
// affine table and the transformed output (what stats + table + norm_table_apply produce in three
// ~5 us launches).  Grid (G, B), one block per slice of HW rows x Cg channels (HW * Cg <= GN_SLICE_MAX,
// Cg even and <= 64).  Thread (p, rl) owns channel pair p (one dword of every row) of rows
// rl, rl + R, ... (R = 256 / (Cg / 2) row lanes), kept in registers; the mean and then the sum of
// squared deviations are exact two-pass fp32 sums, each thread's in row order, combined by a fixed
// xor butterfly per wave and the 4 wave partials in wave order (LDS).  Table: sc = rstd * gamma
// (* (mod + one_plus)), sf = beta - mean * sc (then fma(sf, m, mod_shift)) - the formula of the table
// kernels; apply: silu?(fma(x, sc, sf)) - the formula of norm_table_apply.  The choice depends on
// (HW, C, G) only, so lock-step groups stay bitwise equal to solo tasks.  x2 != null: channels
// [C1, C) come from x2 (the skip concat read in place); the output is the full C-channel tensor.
#define GN_SLICE_MAX 24576
#define GN_SLICE_MAXD 56          // rows per thread: ceil(GN_SLICE_MAX / 2 / 225) (R * P >= 225)

__device__ __forceinline__ float gn_block_sum(float v, float* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  return ((sh[0] + sh[1]) + sh[2]) + sh[3];
}

__global__ void __launch_bounds__(256) gn_slice_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ x2,
                                                       int C1, bf16_t* __restrict__ y,
                                                       const bf16_t* __restrict__ gamma,
                                                       const bf16_t* __restrict__ beta,
                                                       const bf16_t* __restrict__ mod, float one_plus, int HW,
                                                       int C, int G, float eps, int silu) {
  const int g = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int Cg = C / G, P = Cg >> 1, R = 256 / P;
  const int p = t % P, rl = t / P;
  const bool act = rl < R;
  const int c = g * Cg + 2 * p;
  const bool second = x2 != nullptr && c >= C1;
  const int cs = x2 == nullptr ? C : (second ? C - C1 : C1);
  const uint32_t* src = reinterpret_cast<const uint32_t*>((second ? x2 : x) + (size_t)b * HW * cs +
                                                          (second ? c - C1 : c));
  const int rs = cs >> 1;                         // row stride in dwords
  __shared__ float sh[4];
  __shared__ float2 tab[64];
  uint32_t w[GN_SLICE_MAXD];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < GN_SLICE_MAXD; ++i) {
    const int r = rl + i * R;
    w[i] = (act && r < HW) ? src[(size_t)r * rs] : 0u;
  }
#pragma unroll
  for (int i = 0; i < GN_SLICE_MAXD; ++i)
    s += __uint_as_float(w[i] << 16) + __uint_as_float(w[i] & 0xffff0000u);
  const float n = (float)HW * (float)Cg;
  const float mean = gn_block_sum(s, sh) / n;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < GN_SLICE_MAXD; ++i) {
    const int r = rl + i * R;
    if (act && r < HW) {
      const float d0 = __uint_as_float(w[i] << 16) - mean, d1 = __uint_as_float(w[i] & 0xffff0000u) - mean;
      q += d0 * d0 + d1 * d1;
    }
  }
  const float rstd = rsqrtf(gn_block_sum(q, sh) / n + eps);
  if (t < Cg) {
    const int cc = g * Cg + t;
    float sc = rstd * bf2f(gamma[cc]);
    float sf = bf2f(beta[cc]) - mean * sc;
    if (mod) {
      const float m = bf2f(mod[(size_t)b * 2 * C + cc]) + one_plus, a = bf2f(mod[(size_t)b * 2 * C + C + cc]);
      sc *= m;
      sf = fmaf(sf, m, a);
    }
    tab[t] = make_float2(sc, sf);
  }
  __syncthreads();
  if (!act) return;
  const float2 t0 = tab[2 * p], t1 = tab[2 * p + 1];
  uint32_t* dst = reinterpret_cast<uint32_t*>(y + (size_t)b * HW * C + c);
#pragma unroll
  for (int i = 0; i < GN_SLICE_MAXD; ++i) {
    const int r = rl + i * R;
    if (r < HW) {
      float o0 = fmaf(__uint_as_float(w[i] << 16), t0.x, t0.y);
      float o1 = fmaf(__uint_as_float(w[i] & 0xffff0000u), t1.x, t1.y);
      if (silu) { o0 = silu_f(o0); o1 = silu_f(o1); }
      dst[(size_t)r * (C >> 1)] = (uint32_t)f2bf(o0) | ((uint32_t)f2bf(o1) << 16);
    }
  }
}

static bool gn_slice_shape_ok(int HW, int C, int G) {
  if (C % 8 != 0 || G <= 0 || C % G != 0) return false;
  const int Cg = C / G;
  return Cg % 2 == 0 && Cg <= 64 && (long)HW * Cg <= GN_SLICE_MAX;
}

// Off switch (A/B): ARB_GN_SLICE=0 -> the caller takes stats + table + table-apply.
ARB_API int arb_group_norm_slice_ok(int HW, int C, int G) {
  static const bool on = [] {
    const char* e = std::getenv("ARB_GN_SLICE");
    return e == nullptr || e[0] != '0';
  }();
  return on && gn_slice_shape_ok(HW, C, G) ? 1 : 0;
}

ARB_API int arb_group_norm_slice(const void* x, const void* x2, int C1, void* y, const void* gamma, const void* beta,
                                 const void* mod, float one_plus, int B, int HW, int C, int G, float eps, int silu,
                                 hipStream_t stream) {
  if (!gn_slice_shape_ok(HW, C, G)) return -1;
  if (x2 == nullptr) C1 = C;
  else if (C1 <= 0 || C1 >= C || C1 % 8 != 0) return -1;
  gn_slice_kernel<<<dim3(G, B), 256, 0, stream>>>((const bf16_t*)x, (const bf16_t*)x2, C1, (bf16_t*)y,
                                                  (const bf16_t*)gamma, (const bf16_t*)beta, (const bf16_t*)mod,
                                                  one_plus, HW, C, G, eps, silu);
  return (int)hipGetLastError();
}
