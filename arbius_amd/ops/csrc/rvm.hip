// Robust Video Matting: the non-GEMM stages as fused fp16/fp32 HIP passes (templates/
// robust_video_matting.json; VERDICT r2 "RVM hot path on hand-written kernels").
//
//   rvm_resize_u8   uint8 frames [T,H,W,3] -> bilinear (align_corners=False, output size given) /255
//                   -> fp16 [T,h,w,3]: the downsampled source; the full-res fp16 clip never exists
//   rvm_stem        3x3 stride-2 conv (3 -> 16) on the ImageNet-normalised source + bias + hardswish
//                   (a direct VALU conv: K = 27 is too short for an MFMA tile)
//   rvm_pool3       the decoder's 2x2 ceil-mode average-pool pyramid s1, s2, s3 in one pass
//   rvm_upcat       bilinear x2 upsample (+ crop) of the coarser decoder state, concatenated with the
//                   encoder skip and the pooled source, zero-padded to a multiple of 8 channels: the
//                   input of the UpBlock conv, written once (no interpolate / cat / pad copies)
//   rvm_pack        [a | b | 0] channel packing (ConvGRU input buffer)
//   rvm_gru_out     h' = (1 - z) h + z tanh(c), written to the state, IN PLACE into the GRU half of the
//                   UpBlock output (time t), and into the next step's [x_{t+1} | h'] input buffer
//   rvm_dgf_base    the projection head (16 -> fgr residual 3 + alpha 1) and the guided filter's
//                   low-res inputs [x | y] (fp32)
//   rvm_dgf_ab      3x3 box means / covariance / variance + the 3 1x1 convs (24 -> 16 -> 16 -> 4) -> A, b
//   rvm_dgf_out     full resolution: bilinear A, b; out = A [src, mean(src)] + b; fgr / alpha clamp;
//                   green-screen / alpha / foreground composite -> uint8 [T,H,W,3]
//   rvm_chan_mean   per-(t, channel) spatial mean (squeeze-excite / LR-ASPP pooling), fixed-order tree
//   rvm_gate        x *= hardsigmoid(w) / sigmoid(w) per (t, channel), in place
// Every pass is elementwise or a fixed-order local reduction: bitwise deterministic.
#include "common.h"

#include <cstring>

typedef _Float16 h16;

__device__ __forceinline__ float hsw(float v) { return v * fminf(fmaxf(v + 3.f, 0.f), 6.f) * (1.f / 6.f); }

// PyTorch area_pixel_compute_source_index (linear, align_corners=False): max(0, (dst+0.5)*scale-0.5)
__device__ __forceinline__ void lin_src(int dst, float scale, int in, int& i0, int& i1, float& l1) {
  float s = (dst + 0.5f) * scale - 0.5f;
  s = s < 0.f ? 0.f : s;
  i0 = (int)s;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = s - (float)i0;
}

__global__ void __launch_bounds__(256) rvm_resize_u8(const uint8_t* __restrict__ src, h16* __restrict__ dst, int T,
                                                     int H, int W, int h, int w, float sh, float sw) {
  const long total = (long)T * h * w;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int x = (int)(i % w), y = (int)((i / w) % h), t = (int)(i / ((long)w * h));
    int y0, y1, x0, x1;
    float ly, lx;
    lin_src(y, sh, H, y0, y1, ly);
    lin_src(x, sw, W, x0, x1, lx);
    const uint8_t* f = src + (size_t)t * H * W * 3;
    const uint8_t* p00 = f + ((size_t)y0 * W + x0) * 3;
    const uint8_t* p01 = f + ((size_t)y0 * W + x1) * 3;
    const uint8_t* p10 = f + ((size_t)y1 * W + x0) * 3;
    const uint8_t* p11 = f + ((size_t)y1 * W + x1) * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = (1.f - ly) * ((1.f - lx) * p00[c] + lx * p01[c]) + ly * ((1.f - lx) * p10[c] + lx * p11[c]);
      dst[i * 3 + c] = (h16)(v * (1.f / 255.f));
    }
  }
}

struct StemArgs {
  float w[16 * 27];   // [co][ky][kx][ci]
  float b[16];
  float mean[3], istd[3];
};

__global__ void __launch_bounds__(256) rvm_stem(const h16* __restrict__ x, h16* __restrict__ out, const StemArgs a,
                                                int T, int h, int w, int ho, int wo) {
  const long total = (long)T * ho * wo;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int ox = (int)(i % wo), oy = (int)((i / wo) % ho), t = (int)(i / ((long)wo * ho));
    float in[27];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int yy = 2 * oy - 1 + ky, xx = 2 * ox - 1 + kx;
        const bool ok = yy >= 0 && yy < h && xx >= 0 && xx < w;
        const h16* p = x + (((size_t)t * h + (ok ? yy : 0)) * w + (ok ? xx : 0)) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) in[(ky * 3 + kx) * 3 + c] = ok ? ((float)p[c] - a.mean[c]) * a.istd[c] : 0.f;
      }
    h16 o[16];
#pragma unroll
    for (int co = 0; co < 16; ++co) {
      float acc = a.b[co];
#pragma unroll
      for (int k = 0; k < 27; ++k) acc = fmaf(a.w[co * 27 + k], in[k], acc);
      o[co] = (h16)hsw(acc);
    }
    uint4* d = reinterpret_cast<uint4*>(out + i * 16);
    d[0] = *reinterpret_cast<const uint4*>(&o[0]);
    d[1] = *reinterpret_cast<const uint4*>(&o[8]);
  }
}

// ceil-mode 2x2 average pooling, three levels: thread per level-3 pixel (its 8x8 level-0 block).
// Each level rounds to fp16 before the next (F.avg_pool2d on fp16 tensors, level by level).
__global__ void __launch_bounds__(256) rvm_pool3(const h16* __restrict__ s0, h16* __restrict__ s1, h16* __restrict__ s2,
                                                 h16* __restrict__ s3, int T, int h0, int w0) {
  const int h1 = (h0 + 1) / 2, w1 = (w0 + 1) / 2, h2 = (h1 + 1) / 2, w2 = (w1 + 1) / 2;
  const int h3 = (h2 + 1) / 2, w3 = (w2 + 1) / 2;
  const long total = (long)T * h3 * w3;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int X3 = (int)(i % w3), Y3 = (int)((i / w3) % h3), t = (int)(i / ((long)w3 * h3));
    float l2[2][2][3];
    int n2y = 0, n2x = 0;
    for (int dy2 = 0; dy2 < 2; ++dy2) {
      const int Y2 = 2 * Y3 + dy2;
      if (Y2 >= h2) break;
      n2y = dy2 + 1;
      for (int dx2 = 0; dx2 < 2; ++dx2) {
        const int X2 = 2 * X3 + dx2;
        if (X2 >= w2) break;
        if (dy2 == 0) n2x = dx2 + 1;
        float l1[2][2][3];
        int n1y = 0, n1x = 0;
        for (int dy1 = 0; dy1 < 2; ++dy1) {
          const int Y1 = 2 * Y2 + dy1;
          if (Y1 >= h1) break;
          n1y = dy1 + 1;
          for (int dx1 = 0; dx1 < 2; ++dx1) {
            const int X1 = 2 * X2 + dx1;
            if (X1 >= w1) break;
            if (dy1 == 0) n1x = dx1 + 1;
            float acc[3] = {0.f, 0.f, 0.f};
            int n0 = 0;
            for (int dy0 = 0; dy0 < 2; ++dy0) {
              const int Y0 = 2 * Y1 + dy0;
              if (Y0 >= h0) break;
              for (int dx0 = 0; dx0 < 2; ++dx0) {
                const int X0 = 2 * X1 + dx0;
                if (X0 >= w0) break;
                const h16* p = s0 + (((size_t)t * h0 + Y0) * w0 + X0) * 3;
#pragma unroll
                for (int c = 0; c < 3; ++c) acc[c] += (float)p[c];
                ++n0;
              }
            }
            h16* q = s1 + (((size_t)t * h1 + Y1) * w1 + X1) * 3;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              q[c] = (h16)(acc[c] / (float)n0);
              l1[dy1][dx1][c] = (float)q[c];
            }
          }
        }
        float acc[3] = {0.f, 0.f, 0.f};
        for (int dy1 = 0; dy1 < n1y; ++dy1)
          for (int dx1 = 0; dx1 < n1x; ++dx1)
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c] += l1[dy1][dx1][c];
        h16* q = s2 + (((size_t)t * h2 + Y2) * w2 + X2) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          q[c] = (h16)(acc[c] / (float)(n1y * n1x));
          l2[dy2][dx2][c] = (float)q[c];
        }
      }
    }
    float acc[3] = {0.f, 0.f, 0.f};
    for (int dy2 = 0; dy2 < n2y; ++dy2)
      for (int dx2 = 0; dx2 < n2x; ++dx2)
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] += l2[dy2][dx2][c];
    h16* q = s3 + (((size_t)t * h3 + Y3) * w3 + X3) * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) q[c] = (h16)(acc[c] / (float)(n2y * n2x));
  }
}

// dst [T,H,W,Cd] = [up2x(x)[:H,:W] (cx) | f (cf) | s (cs) | 0]; x [T,hx,wx,cx]; f may be null (cf = 0)
__global__ void __launch_bounds__(256) rvm_upcat(const h16* __restrict__ x, int hx, int wx, int cx,
                                                 const h16* __restrict__ f, int cf, const h16* __restrict__ s, int cs,
                                                 h16* __restrict__ dst, int T, int H, int W, int Cd) {
  const long total = (long)T * H * W * Cd;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % Cd);
    const long p = i / Cd;
    const int xx = (int)(p % W), yy = (int)((p / W) % H), t = (int)(p / ((long)W * H));
    float v = 0.f;
    if (c < cx) {
      int y0, y1, x0, x1;
      float ly, lx;
      lin_src(yy, 0.5f, hx, y0, y1, ly);
      lin_src(xx, 0.5f, wx, x0, x1, lx);
      const h16* b = x + (size_t)t * hx * wx * cx + c;
      const float v00 = (float)b[((size_t)y0 * wx + x0) * cx], v01 = (float)b[((size_t)y0 * wx + x1) * cx];
      const float v10 = (float)b[((size_t)y1 * wx + x0) * cx], v11 = (float)b[((size_t)y1 * wx + x1) * cx];
      v = (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
      dst[i] = (h16)v;
      continue;
    }
    if (c < cx + cf) {
      dst[i] = f[p * cf + (c - cx)];
      continue;
    }
    if (c < cx + cf + cs) {
      dst[i] = s[p * cs + (c - cx - cf)];
      continue;
    }
    dst[i] = (h16)0.f;
  }
}

// buf[p, 0:CA) = a[p * as + aoff + c]; buf[p, CA:CA+CB) = b ? b[p * CB + c] : 0; row stride bs
__global__ void __launch_bounds__(256) rvm_pack(h16* __restrict__ buf, int bs, const h16* __restrict__ a, long as,
                                                int aoff, int CA, const h16* __restrict__ b, int CB, long P) {
  const int C = CA + CB;
  const long total = P * C;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long p = i / C;
    buf[p * bs + c] = c < CA ? a[p * as + aoff + c] : (b ? b[p * CB + (c - CA)] : (h16)0.f);
  }
}

__device__ __forceinline__ float tanh_g(float x) {
  const float e = __expf(-2.f * fabsf(x));
  const float t = (1.f - e) / (1.f + e);
  return copysignf(t, x);
}

__global__ void __launch_bounds__(256) rvm_gru_out(const h16* __restrict__ cc, int ccs, h16* __restrict__ h,
                                                   const h16* __restrict__ z, h16* __restrict__ out, long os, int oc,
                                                   h16* __restrict__ buf, int bs, const h16* __restrict__ nx, long ns,
                                                   int noff, long P, int C) {
  const long total = P * C;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long p = i / C;
    const float zf = (float)z[i];
    const h16 hn = (h16)((1.f - zf) * (float)h[i] + zf * tanh_g((float)cc[p * ccs + c]));
    h[i] = hn;
    out[p * os + oc + c] = hn;
    if (buf) {
      buf[p * bs + C + c] = hn;
      buf[p * bs + c] = nx[p * ns + noff + c];
    }
  }
}

struct DgfArgs {
  float wp[4 * 16], bp[4];          // projection head [4][16]
  float w1[16 * 24], b1[16];        // [out][in]: in = cov(4) | var(4) | hid(16)
  float w2[16 * 16], b2[16];
  float w3[4 * 16], b3[4];
};

// per low-res pixel: y = proj(hid) (fgr residual 3 | alpha 1), x = [small, mean(small)] -> xy [P, 8] fp32.
// direct (no downsampling, ratio 1: the network ran at full resolution, no guided filter): write the
// affine map A = 0, b = y straight to xy, so rvm_dgf_out composes fgr = src + residual, alpha = y[3].
__global__ void __launch_bounds__(256) rvm_dgf_base(const h16* __restrict__ hid, const h16* __restrict__ small,
                                                    const DgfArgs* __restrict__ a, float* __restrict__ xy, long P,
                                                    int direct) {
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < P; p += (long)gridDim.x * 256) {
    float hv[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) hv[k] = (float)hid[p * 16 + k];
    float o[8];
    const float s0 = (float)small[p * 3], s1 = (float)small[p * 3 + 1], s2 = (float)small[p * 3 + 2];
    o[0] = s0; o[1] = s1; o[2] = s2; o[3] = (s0 + s1 + s2) * (1.f / 3.f);
    if (direct) o[0] = o[1] = o[2] = o[3] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float acc = a->bp[j];
#pragma unroll
      for (int k = 0; k < 16; ++k) acc = fmaf(a->wp[j * 16 + k], hv[k], acc);
      o[4 + j] = acc;
    }
    float4* d = reinterpret_cast<float4*>(xy + p * 8);
    d[0] = make_float4(o[0], o[1], o[2], o[3]);
    d[1] = make_float4(o[4], o[5], o[6], o[7]);
  }
}

// 3x3 box means (zero padding, /9 - count_include_pad) -> cov, var -> 1x1 convs -> A, b (= mean_y - A mean_x)
__global__ void __launch_bounds__(256) rvm_dgf_ab(const float* __restrict__ xy, const h16* __restrict__ hid,
                                                  const DgfArgs* __restrict__ a, float* __restrict__ ab, int T, int h,
                                                  int w) {
  const long total = (long)T * h * w;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int x = (int)(i % w), y = (int)((i / w) % h), t = (int)(i / ((long)w * h));
    float mx[4] = {0.f, 0.f, 0.f, 0.f}, my[4] = {0.f, 0.f, 0.f, 0.f}, mxy[4] = {0.f, 0.f, 0.f, 0.f};
    float mxx[4] = {0.f, 0.f, 0.f, 0.f};
    for (int dy = -1; dy <= 1; ++dy) {
      const int yy = y + dy;
      if (yy < 0 || yy >= h) continue;
      for (int dx = -1; dx <= 1; ++dx) {
        const int xx = x + dx;
        if (xx < 0 || xx >= w) continue;
        const float* q = xy + (((size_t)t * h + yy) * w + xx) * 8;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          mx[c] += q[c];
          my[c] += q[4 + c];
          mxy[c] += q[c] * q[4 + c];
          mxx[c] += q[c] * q[c];
        }
      }
    }
    float feat[24];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      mx[c] *= (1.f / 9.f);
      my[c] *= (1.f / 9.f);
      feat[c] = mxy[c] * (1.f / 9.f) - mx[c] * my[c];
      feat[4 + c] = mxx[c] * (1.f / 9.f) - mx[c] * mx[c];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) feat[8 + k] = (float)hid[i * 16 + k];
    float h1[16], h2[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      float acc = a->b1[j];
#pragma unroll
      for (int k = 0; k < 24; ++k) acc = fmaf(a->w1[j * 24 + k], feat[k], acc);
      h1[j] = fmaxf(acc, 0.f);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      float acc = a->b2[j];
#pragma unroll
      for (int k = 0; k < 16; ++k) acc = fmaf(a->w2[j * 16 + k], h1[k], acc);
      h2[j] = fmaxf(acc, 0.f);
    }
    float o[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float acc = a->b3[j];
#pragma unroll
      for (int k = 0; k < 16; ++k) acc = fmaf(a->w3[j * 16 + k], h2[k], acc);
      o[j] = acc;
      o[4 + j] = my[j] - acc * mx[j];
    }
    float4* d = reinterpret_cast<float4*>(ab + i * 8);
    d[0] = make_float4(o[0], o[1], o[2], o[3]);
    d[1] = make_float4(o[4], o[5], o[6], o[7]);
  }
}

// full resolution: A, b bilinear (size given: scale = low / full); mode 0 green-screen, 1 alpha-mask,
// 2 foreground-mask -> uint8 [T,H,W,3]
__global__ void __launch_bounds__(256) rvm_dgf_out(const uint8_t* __restrict__ src, const float* __restrict__ ab,
                                                   uint8_t* __restrict__ dst, int T, int H, int W, int h, int w,
                                                   float sh, float sw, int mode, float g0, float g1, float g2) {
  const long total = (long)T * H * W;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int x = (int)(i % W), y = (int)((i / W) % H), t = (int)(i / ((long)W * H));
    int y0, y1, x0, x1;
    float ly, lx;
    lin_src(y, sh, h, y0, y1, ly);
    lin_src(x, sw, w, x0, x1, lx);
    const float* b = ab + (size_t)t * h * w * 8;
    const float* q00 = b + ((size_t)y0 * w + x0) * 8;
    const float* q01 = b + ((size_t)y0 * w + x1) * 8;
    const float* q10 = b + ((size_t)y1 * w + x0) * 8;
    const float* q11 = b + ((size_t)y1 * w + x1) * 8;
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c)
      v[c] = (1.f - ly) * ((1.f - lx) * q00[c] + lx * q01[c]) + ly * ((1.f - lx) * q10[c] + lx * q11[c]);
    const uint8_t* sp = src + i * 3;
    const float f0 = sp[0] * (1.f / 255.f), f1 = sp[1] * (1.f / 255.f), f2 = sp[2] * (1.f / 255.f);
    const float fm = (f0 + f1 + f2) * (1.f / 3.f);
    const float fg[3] = {fminf(fmaxf(v[0] * f0 + v[4] + f0, 0.f), 1.f), fminf(fmaxf(v[1] * f1 + v[5] + f1, 0.f), 1.f),
                         fminf(fmaxf(v[2] * f2 + v[6] + f2, 0.f), 1.f)};
    const float pha = fminf(fmaxf(v[3] * fm + v[7], 0.f), 1.f);
    const float gr[3] = {g0, g1, g2};
    uint8_t* d = dst + i * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float o = mode == 1 ? pha : mode == 2 ? fg[c] : fg[c] * pha + gr[c] * (1.f - pha);
      d[c] = (uint8_t)fminf(fmaxf(rintf(o * 255.f), 0.f), 255.f);
    }
  }
}

// Per-(t, channel) spatial mean (squeeze-excite / LR-ASPP global pool): x fp16 [T, P, C] -> fp16
// [T, C], fp32 accumulation.  Block (t, 64-channel slab): thread (vector v of 8 channels, row lane
// rl) sums rows rl, rl + k, ...; the k row-lane partials are added in a fixed LDS tree order.
__global__ void __launch_bounds__(256) rvm_chan_mean(const h16* __restrict__ x, h16* __restrict__ out, long P, int C) {
  const int t = blockIdx.y, tid = threadIdx.x;
  const int v = tid & 7, rl = tid >> 3;                 // 8 vectors (64 channels) x 32 row lanes
  const int c = blockIdx.x * 64 + 8 * v;
  __shared__ float sh[32][65];
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    const h16* base = x + (size_t)t * P * C + c;
    for (long r = rl; r < P; r += 32) {
      const uint4 raw = *reinterpret_cast<const uint4*>(base + (size_t)r * C);
      const h16* hv = reinterpret_cast<const h16*>(&raw);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += (float)hv[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) sh[rl][8 * v + e] = acc[e];
  __syncthreads();
  for (int st = 16; st > 0; st >>= 1) {
    if (rl < st) {
#pragma unroll
      for (int e = 0; e < 8; ++e) sh[rl][8 * v + e] += sh[rl + st][8 * v + e];
    }
    __syncthreads();
  }
  if (rl == 0 && c < C) {
#pragma unroll
    for (int e = 0; e < 8; ++e) out[(size_t)t * C + c + e] = (h16)(sh[0][8 * v + e] / (float)P);
  }
}

// x[t, p, c] *= gate(w[t, c]) in place: mode 0 hardsigmoid (squeeze-excite), 1 sigmoid (LR-ASPP)
__global__ void __launch_bounds__(256) rvm_gate(h16* __restrict__ x, const h16* __restrict__ w, long P, int C,
                                                int mode, long total8) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total8; i += (long)gridDim.x * 256) {
    const long e0 = i * 8;
    const long row = e0 / C;
    const int c = (int)(e0 - row * C);
    const long t = row / P;
    uint4 raw = *reinterpret_cast<const uint4*>(x + e0);
    const uint4 wr = *reinterpret_cast<const uint4*>(w + t * C + c);
    h16* hv = reinterpret_cast<h16*>(&raw);
    const h16* gv = reinterpret_cast<const h16*>(&wr);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float g = (float)gv[e];
      const float a = mode == 0 ? fminf(fmaxf(g * (1.f / 6.f) + 0.5f, 0.f), 1.f) : 1.f / (1.f + __expf(-g));
      hv[e] = (h16)((float)hv[e] * (float)(h16)a);
    }
    *reinterpret_cast<uint4*>(x + e0) = raw;
  }
}

static int rgrid(long work) {
  long b = (work + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

ARB_API int arb_rvm_resize_u8(const void* src, void* dst, int T, int H, int W, int h, int w, hipStream_t s) {
  if (T < 1 || h < 1 || w < 1 || h > H || w > W) return -1;
  rvm_resize_u8<<<rgrid((long)T * h * w), 256, 0, s>>>((const uint8_t*)src, (h16*)dst, T, H, W, h, w,
                                                        (float)H / (float)h, (float)W / (float)w);
  return (int)hipGetLastError();
}

ARB_API int arb_rvm_stem(const void* x, void* out, const void* args, int T, int h, int w, hipStream_t s) {
  const int ho = (h + 1) / 2, wo = (w + 1) / 2;
  StemArgs a;
  memcpy(&a, args, sizeof(StemArgs));
  rvm_stem<<<rgrid((long)T * ho * wo), 256, 0, s>>>((const h16*)x, (h16*)out, a, T, h, w, ho, wo);
  return (int)hipGetLastError();
}

ARB_API int arb_rvm_pool3(const void* s0, void* s1, void* s2, void* s3, int T, int h0, int w0, hipStream_t s) {
  const int h3 = (((h0 + 1) / 2 + 1) / 2 + 1) / 2, w3 = (((w0 + 1) / 2 + 1) / 2 + 1) / 2;
  rvm_pool3<<<rgrid((long)T * h3 * w3), 256, 0, s>>>((const h16*)s0, (h16*)s1, (h16*)s2, (h16*)s3, T, h0, w0);
  return (int)hipGetLastError();
}

ARB_API int arb_rvm_upcat(const void* x, int hx, int wx, int cx, const void* f, int cf, const void* sp, int cs,
                          void* dst,
                          int T, int H, int W, int Cd, hipStream_t s) {
  if (cx + cf + cs > Cd || 2 * hx < H || 2 * wx < W) return -1;
  rvm_upcat<<<rgrid((long)T * H * W * Cd), 256, 0, s>>>((const h16*)x, hx, wx, cx, (const h16*)f, cf, (const h16*)sp,
                                                         cs, (h16*)dst, T, H, W, Cd);
  return (int)hipGetLastError();
}

ARB_API int arb_rvm_pack(void* buf, int bs, const void* a, long as, int aoff, int CA, const void* b, int CB, long P,
                         hipStream_t s) {
  if (CA + CB > bs) return -1;
  rvm_pack<<<rgrid(P * (CA + CB)), 256, 0, s>>>((h16*)buf, bs, (const h16*)a, as, aoff, CA, (const h16*)b, CB, P);
  return (int)hipGetLastError();
}

ARB_API int arb_rvm_gru_out(const void* cc, int ccs, void* h, const void* z, void* out, long os, int oc, void* buf,
                            int bs, const void* nx, long ns, int noff, long P, int C, hipStream_t s) {
  if ((buf != nullptr && (nx == nullptr || bs < 2 * C)) || ccs < C) return -1;
  rvm_gru_out<<<rgrid(P * C), 256, 0, s>>>((const h16*)cc, ccs, (h16*)h, (const h16*)z, (h16*)out, os, oc, (h16*)buf,
                                            bs, (const h16*)nx, ns, noff, P, C);
  return (int)hipGetLastError();
}

ARB_API int arb_rvm_dgf(const void* hid, const void* small, const void* dgf_args_dev, void* xy, void* ab,
                        const void* src, void* dst, int T, int H, int W, int h, int w, int mode, float g0, float g1,
                        float g2, hipStream_t s) {
  const long P = (long)T * h * w;
  const int direct = h == H && w == W;      // full-resolution network (inputs <= 512 px): no guided filter
  rvm_dgf_base<<<rgrid(P), 256, 0, s>>>((const h16*)hid, (const h16*)small, (const DgfArgs*)dgf_args_dev, (float*)xy,
                                         P, direct);
  if (!direct)
    rvm_dgf_ab<<<rgrid(P), 256, 0, s>>>((const float*)xy, (const h16*)hid, (const DgfArgs*)dgf_args_dev, (float*)ab,
                                         T, h, w);
  rvm_dgf_out<<<rgrid((long)T * H * W), 256, 0, s>>>((const uint8_t*)src, (const float*)(direct ? xy : ab),
                                                      (uint8_t*)dst, T, H, W, h, w, (float)h / (float)H,
                                                      (float)w / (float)W, mode, g0, g1, g2);
  return (int)hipGetLastError();
}

ARB_API int arb_rvm_chan_mean(const void* x, void* out, int T, long P, int C, hipStream_t s) {
  if (T < 1 || P < 1 || C % 8 != 0) return -1;
  rvm_chan_mean<<<dim3((C + 63) / 64, T), 256, 0, s>>>((const h16*)x, (h16*)out, P, C);
  return (int)hipGetLastError();
}

ARB_API int arb_rvm_gate(void* x, const void* w, int T, long P, int C, int mode, hipStream_t s) {
  if (T < 1 || P < 1 || C % 8 != 0 || mode < 0 || mode > 1) return -1;
  const long total8 = (long)T * P * C / 8;
  rvm_gate<<<rgrid(total8), 256, 0, s>>>((h16*)x, (const h16*)w, P, C, mode, total8);
  return (int)hipGetLastError();
}

ARB_API size_t arb_rvm_args_sizes(int which) { return which == 0 ? sizeof(StemArgs) : sizeof(DgfArgs); }
