// GroupNorm (+SiLU) over channels-last activations and LayerNorm over token rows.
//
// GroupNorm is the normalisation of every ResBlock / Transformer2D input of the
// SD1.5 UNet and VAE.  Activations are [B, HW, C] bf16.
// Deterministic two-phase reduction (no atomics, fixed combine order, so the
// same task gives the same bytes on every GPU - SURVEY.md §7.3.1):
//   1. gn_partial : grid (chunks, B).  Each block reduces `rows` rows of one
//      batch into per-group (n, mean, M2) with a per-channel shift (first row)
//      and Chan's parallel combine -> robust to |mean| >> std.
//   2. gn_apply   : grid (chunks, B).  Every block re-combines the partials of
//      its batch in a fixed order (256 threads, G groups x 256/G slices), then
//      normalises its rows with gamma/beta (+SiLU) and 16-byte stores.
#include "common.h"

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

#define GN_MAX_CHUNKS 64

// Phase 1. x: [B, HW, C]; part: [B, chunks, G].  Thread t owns channel vectors {v, v+256,..}
// (VPT of them) and row lane rl.  Per channel it accumulates sums of (x - shift) with
// shift = its first row (robust to |mean| >> std); the per-group combine over channels
// and row lanes is exact algebra on those sums (no divisions in the loop).
template <int VPT>
__global__ void __launch_bounds__(256) gn_stats_kernel(const bf16_t* __restrict__ x, Stat* __restrict__ part,
                                                       int HW, int C, int G, int rows_per_chunk) {
  const int chunk = blockIdx.x, b = blockIdx.y, chunks = gridDim.x;
  const int NV = C >> 3;
  const int k = NV >= 256 ? 1 : 256 / NV;
  const int t = threadIdx.x;
  const int v = NV >= 256 ? t : t % NV, rl = NV >= 256 ? 0 : t / NV;
  const int r_begin = chunk * rows_per_chunk;
  const int r_end = min(HW, r_begin + rows_per_chunk);
  __shared__ float sh_n[256];
  __shared__ float sh_shift[256 * 8 * VPT];
  __shared__ float sh_s[256 * 8 * VPT];
  __shared__ float sh_q[256 * 8 * VPT];
  __shared__ float sh_mu[256];

  float shift[VPT][8], s[VPT][8], q[VPT][8];
  float n = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) { s[j][i] = 0.f; q[j][i] = 0.f; shift[j][i] = 0.f; }
  if (rl < k) {
    const bf16_t* base = x + ((size_t)b * HW) * C;
    int r = r_begin + rl;
    if (r < r_end) {
#pragma unroll
      for (int j = 0; j < VPT; ++j)
        if (v + 256 * j < NV) unpack8(ld16(base + (size_t)r * C + (v + 256 * j) * 8), shift[j]);
    }
    for (; r < r_end; r += k) {
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        if (v + 256 * j < NV) {
          float f[8];
          unpack8(ld16(base + (size_t)r * C + (v + 256 * j) * 8), f);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float d = f[i] - shift[j][i];
            s[j][i] += d;
            q[j][i] = fmaf(d, d, q[j][i]);
          }
        }
      }
      n += 1.f;
    }
  }
  sh_n[t] = n;
#pragma unroll
  for (int j = 0; j < VPT; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int o = (t * VPT + j) * 8 + i;
      sh_shift[o] = shift[j][i];
      sh_s[o] = s[j][i];
      sh_q[o] = q[j][i];
    }
  __syncthreads();
  const int Cg = C / G;
  if (t < G) {
    float N = 0.f, sum = 0.f;
    for (int c = t * Cg; c < (t + 1) * Cg; ++c) {
      const int vv = c >> 3, e = c & 7;
      for (int j = 0; j < k; ++j) {
        const int tt = NV >= 256 ? (vv & 255) : j * NV + vv;
        const int o = (tt * VPT + (NV >= 256 ? (vv >> 8) : 0)) * 8 + e;
        const float nn = sh_n[tt];
        N += nn;
        sum += nn * sh_shift[o] + sh_s[o];
      }
    }
    const float mu = N > 0.f ? sum / N : 0.f;
    float m2 = 0.f;
    for (int c = t * Cg; c < (t + 1) * Cg; ++c) {
      const int vv = c >> 3, e = c & 7;
      for (int j = 0; j < k; ++j) {
        const int tt = NV >= 256 ? (vv & 255) : j * NV + vv;
        const int o = (tt * VPT + (NV >= 256 ? (vv >> 8) : 0)) * 8 + e;
        const float dsh = sh_shift[o] - mu;
        m2 += sh_q[o] + 2.f * dsh * sh_s[o] + sh_n[tt] * dsh * dsh;
      }
    }
    Stat st = {N, mu, fmaxf(m2, 0.f), 0.f};
    part[((size_t)b * chunks + chunk) * G + t] = st;
  }
}

// Phase 2: every block combines its batch's <= 64 chunk stats (loads issued back to back,
// fixed combine order -> identical in every block), then normalises `rows` rows.
__global__ void __launch_bounds__(256) gn_apply_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                       const Stat* __restrict__ part, const bf16_t* __restrict__ gamma,
                                                       const bf16_t* __restrict__ beta, int HW, int C, int G,
                                                       int chunks, int rows, float eps, int silu) {
  const int blk = blockIdx.x, b = blockIdx.y;
  const int t = threadIdx.x;
  __shared__ Stat sh[256];
  __shared__ float sh_mean[256], sh_rstd[256];
  const int S = (G <= 64 && 256 % G == 0) ? 256 / G : 1;
  {
    Stat acc = {0.f, 0.f, 0.f, 0.f};
    const int g = t % G, sl = t / G;
    if (sl < S) {
      Stat loc[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = sl + i * S;
        loc[i] = c < chunks ? part[((size_t)b * chunks + c) * G + g] : Stat{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) acc = chan_combine(acc, loc[i]);
      for (int c = sl + 16 * S; c < chunks; c += S) acc = chan_combine(acc, part[((size_t)b * chunks + c) * G + g]);
    }
    sh[t] = acc;
  }
  __syncthreads();
  if (t < G) {
    Stat acc = sh[t];
    for (int sl = 1; sl < S; ++sl) acc = chan_combine(acc, sh[sl * G + t]);
    sh_mean[t] = acc.mean;
    sh_rstd[t] = rsqrtf(acc.m2 / fmaxf(acc.n, 1.f) + eps);
  }
  __syncthreads();

  const int NV = C >> 3;
  const int k = NV >= 256 ? 1 : 256 / NV;
  const int v = NV >= 256 ? t : t % NV, rl = NV >= 256 ? 0 : t / NV;
  if (rl >= k) return;
  const int Cg = C / G;
  const int r_begin = blk * rows;
  const int r_end = min(HW, r_begin + rows);
  for (int vv = v; vv < NV; vv += 256) {
    float sc[8], sf[8];
    {
      float gm[8], bt[8];
      unpack8(ld16(gamma + vv * 8), gm);
      unpack8(ld16(beta + vv * 8), bt);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int g = (vv * 8 + i) / Cg;
        sc[i] = sh_rstd[g] * gm[i];
        sf[i] = bt[i] - sh_mean[g] * sc[i];
      }
    }
    const size_t off = ((size_t)b * HW) * C + vv * 8;
    for (int r = r_begin + rl; r < r_end; r += k) {
      float f[8];
      unpack8(ld16(x + off + (size_t)r * C), f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float o = f[i] * sc[i] + sf[i];
        f[i] = silu ? silu_f(o) : o;
      }
      st16(y + off + (size_t)r * C, pack8(f));
    }
    if (NV < 256) break;
  }
}

struct GnPlan {
  int chunks, rows, apply_blocks, apply_rows;
};

static GnPlan gn_plan(int B, int HW, int C) {
  const int NV = C / 8;
  const int k = NV >= 256 ? 1 : 256 / NV;
  GnPlan p;
  int target = 512 / (B > 0 ? B : 1);
  if (target > GN_MAX_CHUNKS) target = GN_MAX_CHUNKS;
  if (target < 1) target = 1;
  p.rows = (HW + target - 1) / target;
  if (p.rows < k) p.rows = k;
  p.chunks = (HW + p.rows - 1) / p.rows;
  // apply: ~2-4 rows per row lane, >= ~512 blocks where the tensor allows
  p.apply_rows = 4 * k;
  long want = 1024 / (B > 0 ? B : 1);
  long r = (HW + want - 1) / want;
  if (r > p.apply_rows) p.apply_rows = (int)r;
  p.apply_blocks = (HW + p.apply_rows - 1) / p.apply_rows;
  return p;
}

ARB_API size_t arb_group_norm_workspace(int B, int HW, int C, int G) {
  const GnPlan p = gn_plan(B, HW, C);
  return (size_t)B * p.chunks * G * sizeof(Stat);
}

ARB_API int arb_group_norm_nhwc(const void* x, void* y, const void* gamma, const void* beta, void* workspace, int B,
                                int HW, int C, int G, float eps, int silu, hipStream_t stream) {
  if (C % 8 != 0 || C / 8 > 512 || C % G != 0 || G > 256) return -1;
  const GnPlan p = gn_plan(B, HW, C);
  dim3 g1(p.chunks, B);
  if (C / 8 > 256)
    gn_stats_kernel<2><<<g1, 256, 0, stream>>>((const bf16_t*)x, (Stat*)workspace, HW, C, G, p.rows);
  else
    gn_stats_kernel<1><<<g1, 256, 0, stream>>>((const bf16_t*)x, (Stat*)workspace, HW, C, G, p.rows);
  dim3 g2(p.apply_blocks, B);
  gn_apply_kernel<<<g2, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (const Stat*)workspace, (const bf16_t*)gamma,
                                          (const bf16_t*)beta, HW, C, G, p.chunks, p.apply_rows, eps, silu);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
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
