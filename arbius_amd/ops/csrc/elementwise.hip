// Vectorised (16-byte per lane) elementwise kernels: GEGLU gate, SiLU, add.
// Memory-bound; grid capped at ~2048 blocks with a grid-stride loop
// (cdna_hip_programming.md Guideline 11/13).
#include "common.h"

#include <cstdlib>

// h: [M, 2F] (value | gate) -> out [M, F] = value * gelu(gate)
__global__ void __launch_bounds__(256) geglu_kernel(const bf16_t* __restrict__ h, bf16_t* __restrict__ out,
                                                    long M, int F) {
  const int FV = F >> 3;
  const long total = M * FV;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long row = i / FV;
    const int col = (int)(i - row * FV) * 8;
    float a[8], g[8];
    unpack8(ld16(h + row * 2 * F + col), a);
    unpack8(ld16(h + row * 2 * F + F + col), g);
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = a[e] * gelu_f(g[e]);
    st16(out + row * F + col, pack8(a));
  }
}

__global__ void __launch_bounds__(256) silu_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long n8) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float f[8];
    unpack8(ld16(x + i * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = silu_f(f[e]);
    st16(y + i * 8, pack8(f));
  }
}


// Unfused form of a GroupNorm-table prologue: y[b, p, c] = x * table[b, c].x + table[b, c].y
// (+SiLU).  Used in front of the LDS-DMA conv variant, which stages operands straight into
// LDS and so cannot transform them on the way in.
// x2 != null: channels [C1, C) are read from x2 (the concat [x | x2] is written, never read, whole).
__global__ void __launch_bounds__(256) norm_table_apply_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                               const float2* __restrict__ table, long HW, int C,
                                                               long total8, int silu, const bf16_t* __restrict__ x2,
                                                               int C1) {
  const int CV = C >> 3;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total8; i += (long)gridDim.x * 256) {
    const long pix = i / CV;
    const int c = (int)(i - pix * CV) * 8;
    const long b = pix / HW;
    const float2* t = table + b * C + c;
    float f[8];
    const bf16_t* src = x2 == nullptr ? x + i * 8
                                      : (c < C1 ? x + pix * C1 + c : x2 + pix * (C - C1) + (c - C1));
    unpack8(ld16(src), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float2 ss = t[e];
      const float o = fmaf(f[e], ss.x, ss.y);
      f[e] = silu ? silu_f(o) : o;
    }
    st16(y + i * 8, pack8(f));
  }
}

// The same transform in a 2-D geometry (grid: row slabs x images): thread (v, rl) owns channel
// vector v (8 channels) for RP rows of the slab, keeps its 8 (scale, shift) pairs in registers and
// issues all RP 16-byte loads before the first store - no 64-bit index division, table read once
// per thread instead of per element.  Bitwise identical to norm_table_apply_kernel.
template <int VPT, int RP>
__global__ void __launch_bounds__(256) norm_table_apply2_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                                const float2* __restrict__ table, int HW, int C,
                                                                int silu, const bf16_t* __restrict__ x2, int C1) {
  const int b = blockIdx.y, t = threadIdx.x;
  const int CV = C >> 3;
  const int k = CV >= 256 ? 1 : 256 / CV;
  const int v0 = CV >= 256 ? t : t % CV, rl = CV >= 256 ? 0 : t / CV;
  if (rl >= k) return;
  const int r0 = blockIdx.x * k * RP + rl;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int v = v0 + 256 * j;
    if (v >= CV) break;
    const int c = 8 * v;
    float sc[8], sh[8];
    const float4* tp = reinterpret_cast<const float4*>(table + (size_t)b * C + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float4 q = tp[e];
      sc[2 * e] = q.x; sh[2 * e] = q.y; sc[2 * e + 1] = q.z; sh[2 * e + 1] = q.w;
    }
    const bf16_t* src;
    int sstride;
    if (x2 == nullptr) { src = x + (size_t)b * HW * C + c; sstride = C; }
    else if (c < C1) { src = x + (size_t)b * HW * C1 + c; sstride = C1; }
    else { src = x2 + (size_t)b * HW * (C - C1) + (c - C1); sstride = C - C1; }
    bf16_t* dst = y + (size_t)b * HW * C + c;
    uint4 raw[RP];
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      const int r = r0 + i * k;
      raw[i] = r < HW ? ld16(src + (size_t)r * sstride) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      const int r = r0 + i * k;
      if (r >= HW) break;
      float f[8];
      unpack8(raw[i], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float o = fmaf(f[e], sc[e], sh[e]);
        f[e] = silu ? silu_f(o) : o;
      }
      st16(dst + (size_t)r * C, pack8(f));
    }
  }
}

static int launch_apply2(const void* x, const void* x2, int C1, void* y, const void* table, int B, long HW, int C,
                         int silu, hipStream_t stream) {
  if (HW > (1L << 30)) return -1;
  const int CV = C / 8;
  const int k = CV >= 256 ? 1 : 256 / CV;
  constexpr int RP = 8;
  dim3 grid((unsigned)((HW + (long)k * RP - 1) / ((long)k * RP)), B);
  if (CV > 512) return -1;
  if (CV > 256)
    norm_table_apply2_kernel<2, RP><<<grid, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (const float2*)table,
                                                              (int)HW, C, silu, (const bf16_t*)x2, C1);
  else
    norm_table_apply2_kernel<1, RP><<<grid, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (const float2*)table,
                                                              (int)HW, C, silu, (const bf16_t*)x2, C1);
  return (int)hipGetLastError();
}

static bool apply2_on() {
  static const bool on = [] {
    const char* e = std::getenv("ARB_GN_APPLY2");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

// Row softmax of a score matrix: P = softmax(scale * S) per row over the first nv columns (the rest
// of the row, key padding up to the GEMM tile, is written 0), S / P [R, N] bf16 (N % 8 == 0), fp32
// math, one wave per row (three sweeps of the row: max, sum of exp, write; the row stays in L1/L2).
// The middle launch of the large-head attention (d = 512 single-head VAE / MoVQ mid-block
// attention): S = Q K^T and O = P V run on the implicit-GEMM kernel.  Fixed reduction order.
__global__ void __launch_bounds__(256) softmax_rows_kernel(const bf16_t* __restrict__ s, bf16_t* __restrict__ p,
                                                           int R, int N, int nv, float scale) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= R) return;
  const bf16_t* sr = s + (size_t)row * N;
  bf16_t* pr = p + (size_t)row * N;
  float m = -INFINITY;
  for (int c = lane * 8; c < N; c += 512) {
    float f[8];
    unpack8(ld16(sr + c), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) m = c + e < nv ? fmaxf(m, f[e] * scale) : m;
  }
  m = wave_max(m);
  float sum = 0.f;
  for (int c = lane * 8; c < N; c += 512) {
    float f[8];
    unpack8(ld16(sr + c), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) sum += c + e < nv ? __expf(f[e] * scale - m) : 0.f;
  }
  const float inv = 1.f / wave_sum(sum);
  for (int c = lane * 8; c < N; c += 512) {
    float f[8];
    unpack8(ld16(sr + c), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = c + e < nv ? __expf(f[e] * scale - m) * inv : 0.f;
    st16(pr + c, pack8(f));
  }
}

ARB_API int arb_softmax_rows(const void* s, void* p, int R, int N, int nv, float scale, hipStream_t stream) {
  if (N % 8 != 0 || R <= 0 || nv <= 0 || nv > N) return -1;
  softmax_rows_kernel<<<(R + 3) / 4, 256, 0, stream>>>((const bf16_t*)s, (bf16_t*)p, R, N, nv, scale);
  return (int)hipGetLastError();
}

static int grid_for(long work) {
  long g = (work + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

ARB_API int arb_geglu(const void* h, void* out, long M, int F, hipStream_t stream) {
  if (F % 8 != 0) return -1;
  geglu_kernel<<<grid_for(M * (F / 8)), 256, 0, stream>>>((const bf16_t*)h, (bf16_t*)out, M, F);
  return (int)hipGetLastError();
}

ARB_API int arb_silu(const void* x, void* y, long n, hipStream_t stream) {
  if (n % 8 != 0) return -1;
  silu_kernel<<<grid_for(n / 8), 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, n / 8);
  return (int)hipGetLastError();
}

ARB_API int arb_norm_table_apply(const void* x, void* y, const void* table, int B, long HW, int C, int silu,
                                 hipStream_t stream) {
  if (C % 8 != 0) return -1;
  // 2-D kernel for large tensors only (graph replay: 9.4 vs 10.6 us at [8, 64, 64, 320], 15.4 vs 17.6 at
  // [8, 64, 64, 640], 21.3 vs 24.9 at [1, 512, 512, 128]; slower below ~8M elements: 3.7 vs 2.6 us at
  // [8, 8, 8, 1280] - profiles/norm_kernels_ab_r3.jsonl)
  if (apply2_on() && C / 8 <= 512 && (long)B * HW * C >= (8L << 20))
    return launch_apply2(x, nullptr, 0, y, table, B, HW, C, silu, stream);
  const long total8 = (long)B * HW * (C / 8);
  norm_table_apply_kernel<<<grid_for(total8), 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (const float2*)table,
                                                                HW, C, total8, silu, nullptr, 0);
  return (int)hipGetLastError();
}

ARB_API int arb_norm_table_apply_cat(const void* x, const void* x2, int C1, void* y, const void* table, int B, long HW,
                                     int C, int silu, hipStream_t stream) {
  if (C % 8 != 0 || C1 <= 0 || C1 >= C || C1 % 8 != 0 || x2 == nullptr) return -1;
  if (apply2_on() && C / 8 <= 512 && (long)B * HW * C >= (8L << 20))
    return launch_apply2(x, x2, C1, y, table, B, HW, C, silu, stream);
  const long total8 = (long)B * HW * (C / 8);
  norm_table_apply_kernel<<<grid_for(total8), 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (const float2*)table,
                                                                HW, C, total8, silu, (const bf16_t*)x2, C1);
  return (int)hipGetLastError();
}

// 2x2 average pool (GLIDE down-sampling ResBlock, guided-diffusion AvgPool2d) of x and, with a
// GroupNorm table, of its normalised form in the same pass: yx = pool(x), yn = pool(bf16(act(x *
// scale + shift))).  The normalised values are rounded to bf16 before pooling (the unfused
// norm-then-pool arithmetic); sums in fixed order (p00 + p01) + (p10 + p11), times 0.25 (exact).
// x [B, H, W, C] (H, W even), yn / yx [B, H/2, W/2, C]; either output may be null.
__global__ void __launch_bounds__(256) norm_pool2_kernel(const bf16_t* __restrict__ x, const float2* __restrict__ table,
                                                         int silu, bf16_t* __restrict__ yn, bf16_t* __restrict__ yx,
                                                         int Ho, int Wo, int C, long total8) {
  const int CV = C >> 3;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total8; i += (long)gridDim.x * 256) {
    const long pix = i / CV;                     // output pixel (b, oy, ox)
    const int c = (int)(i - pix * CV) * 8;
    const long b = pix / ((long)Ho * Wo);
    const int rem = (int)(pix - b * Ho * Wo), oy = rem / Wo, ox = rem - oy * Wo;
    const long W = 2L * Wo;
    const bf16_t* p0 = x + ((b * 2 * Ho + 2 * oy) * W + 2 * ox) * C + c;
    float f[4][8];
    unpack8(ld16(p0), f[0]);
    unpack8(ld16(p0 + C), f[1]);
    unpack8(ld16(p0 + W * C), f[2]);
    unpack8(ld16(p0 + W * C + C), f[3]);
    if (yx != nullptr) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = ((f[0][e] + f[1][e]) + (f[2][e] + f[3][e])) * 0.25f;
      st16(yx + i * 8, pack8(o));
    }
    if (yn != nullptr) {
      const float2* t = table + b * C + c;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float2 ss = t[e];
        float q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = fmaf(f[j][e], ss.x, ss.y);
          q[j] = bf16_round(silu ? silu_f(v) : v);
        }
        o[e] = ((q[0] + q[1]) + (q[2] + q[3])) * 0.25f;
      }
      st16(yn + i * 8, pack8(o));
    }
  }
}

ARB_API int arb_norm_pool2(const void* x, const void* table, int silu, void* yn, void* yx, int B, int H, int W, int C,
                           hipStream_t stream) {
  if (C % 8 != 0 || H % 2 != 0 || W % 2 != 0 || B <= 0 || (yn != nullptr && table == nullptr)) return -1;
  const long total8 = (long)B * (H / 2) * (W / 2) * (C / 8);
  norm_pool2_kernel<<<grid_for(total8), 256, 0, stream>>>((const bf16_t*)x, (const float2*)table, silu, (bf16_t*)yn,
                                                          (bf16_t*)yx, H / 2, W / 2, C, total8);
  return (int)hipGetLastError();
}

// Nearest 2x up-sampling of a channels-last tensor (GLIDE up-sampling ResBlock skip path):
// y [B, 2H, 2W, C] from x [B, H, W, C]; one read of x, 16-byte stores.
__global__ void __launch_bounds__(256) upsample2_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int H,
                                                        int W, int C, long total8) {
  const int CV = C >> 3;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total8; i += (long)gridDim.x * 256) {
    const long pix = i / CV;                     // input pixel (b, iy, ix)
    const int c = (int)(i - pix * CV) * 8;
    const long b = pix / ((long)H * W);
    const int rem = (int)(pix - b * H * W), iy = rem / W, ix = rem - iy * W;
    const uint4 v = ld16(x + i * 8);
    const long W2 = 2L * W;
    bf16_t* q = y + ((b * 2 * H + 2 * iy) * W2 + 2 * ix) * C + c;
    st16(q, v);
    st16(q + C, v);
    st16(q + W2 * C, v);
    st16(q + W2 * C + C, v);
  }
}

ARB_API int arb_upsample2(const void* x, void* y, int B, int H, int W, int C, hipStream_t stream) {
  if (C % 8 != 0 || B <= 0) return -1;
  const long total8 = (long)B * H * W * (C / 8);
  upsample2_kernel<<<grid_for(total8), 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, H, W, C, total8);
  return (int)hipGetLastError();
}

// Decoded image -> uint8 RGB in one pass (the tail of every VAE / MoVQ decode; was 5-6 ATen launches):
// mode 0 (SD KL-VAE): round(clamp(x / 2 + 0.5, 0, 1) * 255); mode 1 (MoVQ): round(clamp((x + 1) * 127.5, 0, 255)).
// fp32 arithmetic in the order of the PyTorch expressions (x / 2 exact, so a contracted fma rounds the
// same), round half to even - bitwise the ATen chain for finite inputs.
__global__ void __launch_bounds__(256) image_u8_kernel(const bf16_t* __restrict__ x, uint8_t* __restrict__ y, long n,
                                                       int mode) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float f = bf2f(x[i]);
    float v;
    if (mode == 0) {
      v = fminf(fmaxf(f * 0.5f + 0.5f, 0.f), 1.f) * 255.f;
    } else {
      const float s = f + 1.f;
      v = fminf(fmaxf(s * 127.5f, 0.f), 255.f);
    }
    y[i] = (uint8_t)rintf(v);
  }
}

ARB_API int arb_image_u8(const void* x, void* y, long n, int mode, hipStream_t stream) {
  if (n <= 0 || mode < 0 || mode > 1) return -1;
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  image_u8_kernel<<<dim3((unsigned)blocks), 256, 0, stream>>>((const bf16_t*)x, (uint8_t*)y, n, mode);
  return (int)hipGetLastError();
}

// uint8 RGB frames [T, H, W, 3] -> BT.601 limited-range 4:2:0 planes padded to whole macroblocks:
// Y [T, H16, W16], Cb / Cr [T, H16 / 2, W16 / 2] - the H.264 encoder's input, so the video tail
// downloads 1.5 bytes per pixel instead of 3 and the host skips the colour conversion.  Integer
// arithmetic identical to native/src/native.cpp rgb_to_420 (samples clipped to [1, 254]; rows and
// columns past the picture replicate the last one; chroma = the 2x2 sum's matrix, >> 10 with
// rounding), so the encoded bytes are the same.  One thread per chroma sample: its 2x2 luma samples
// and Cb, Cr.
__global__ void rgb_to_yuv420_kernel(const uint8_t* __restrict__ rgb, uint8_t* __restrict__ yp,
                                     uint8_t* __restrict__ cbp, uint8_t* __restrict__ crp, int T, int H, int W,
                                     int H16, int W16) {
  const int Wc = W16 / 2, Hc = H16 / 2;
  const long total = (long)T * Hc * Wc;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int x = (int)(i % Wc);
    const long rest = i / Wc;
    const int r = (int)(rest % Hc), t = (int)(rest / Hc);
    const uint8_t* f = rgb + (size_t)t * H * W * 3;
    int sr = 0, sg = 0, sb = 0;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      const int yy = 2 * r + dy;
      const uint8_t* row = f + (size_t)min(yy, H - 1) * W * 3;
      uint8_t* yo = yp + ((size_t)t * H16 + yy) * W16;
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int xx = 2 * x + dx;
        const uint8_t* p = row + 3 * min(xx, W - 1);
        const int R = p[0], G = p[1], B = p[2];
        yo[xx] = (uint8_t)min(max(((66 * R + 129 * G + 25 * B + 128) >> 8) + 16, 1), 254);
        sr += R; sg += G; sb += B;
      }
    }
    const size_t co = ((size_t)t * Hc + r) * Wc + x;
    cbp[co] = (uint8_t)min(max(((-38 * sr - 74 * sg + 112 * sb + 512) >> 10) + 128, 1), 254);
    crp[co] = (uint8_t)min(max(((112 * sr - 94 * sg - 18 * sb + 512) >> 10) + 128, 1), 254);
  }
}

ARB_API int arb_rgb_to_yuv420(const void* rgb, void* y, void* cb, void* cr, int T, int H, int W, hipStream_t stream) {
  if (T <= 0 || H <= 0 || W <= 0) return -1;
  const int H16 = (H + 15) / 16 * 16, W16 = (W + 15) / 16 * 16;
  const long total = (long)T * (H16 / 2) * (W16 / 2);
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  rgb_to_yuv420_kernel<<<dim3((unsigned)blocks), 256, 0, stream>>>((const uint8_t*)rgb, (uint8_t*)y, (uint8_t*)cb,
                                                                   (uint8_t*)cr, T, H, W, H16, W16);
  return (int)hipGetLastError();
}
