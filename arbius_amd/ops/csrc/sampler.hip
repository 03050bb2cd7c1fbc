// Fused classifier-free-guidance + diffusion sampler step (SURVEY.md §2.6(a) "CFG combine +
// scheduler step ... fused elementwise", §7.1 kernel list).
//
// ONE launch per denoising step per lock-step group: for every task k of the group and every
// latent pixel (4 channels), in fp32 with a fixed operation order:
//
//   e    = u + g * (c - u)                         (CFG; u / c = the UNet's uncond / cond rows)
//   E    = he0*e + he1*H1 + he2*H2 + he3*H3        (multistep history: PNDM / k-LMS)
//   x0   = clamp(px*X + pe*E, +-clamp)             (eps- or x0-prediction; clamp optional)
//   out  = ox*Xsrc + oe*E + ox0*x0 + od*(x0 - P) + std*noise
//          std = a scalar, or exp(0.5*(f*logb + (1-f)*plv)) with f = (v+1)/2 (learned variance v,
//          the cond row's extra channels: Kandinsky 2 p_sample)
//   stores: Hs = e, P = x0, CUR = X, X = out, xin_next[2 rows] = bf16(out * in_scale)
//
// DDIM / Euler / Euler-a / DPM-Solver++(2M) / PNDM / k-LMS / p_sample are all this one form with
// host-computed coefficients (models/schedulers.py ``StepPlan``), so every sampler runs the same
// audited arithmetic; the next step's UNet input (scale_model_input, bf16 cast, CFG duplication)
// is written here too, so no elementwise PyTorch kernel runs inside the denoise loop.
// Pure elementwise, no reductions, no atomics -> bitwise reproducible.
#include "common.h"

#include <cstring>

constexpr int MAXT = 8;   // tasks per launch (lock-step groups are <= 8)

struct SampTask {
  const bf16_t* u;       // uncond UNet output, [n_pix, cout]
  const bf16_t* c;       // cond UNet output
  float* x;              // fp32 state [n_pix, 4]  (read, then overwritten by out)
  const float* xsrc;     // Xsrc (== x, or PNDM's stored sample)
  float* p;              // previous x0 (DPM++2M), read and/or written
  float* cur;            // PNDM current sample store (or null)
  float* hs;             // history slot written with e (or null)
  const float* h1;       // history reads (null when the coefficient is 0)
  const float* h2;
  const float* h3;
  const float* noise;    // [n_pix, 4] or null
  bf16_t* xin0;          // next UNet input rows (or null)
  bf16_t* xin1;
  float g, he0, he1, he2, he3, px, pe, clampv, ox, oe, ox0, od, stdv, logb, plv, in_scale;
  int flags;             // bit0 store_x0, bit1 store_cur, bit2 learned_std, bit3 clamp, bit4 read_p
};

struct SampArgs {
  SampTask t[MAXT];
  int ntask, n_pix, cout;
};

__global__ void __launch_bounds__(256) sampler_step_kernel(const SampArgs a) {
  const int k = blockIdx.y;
  const SampTask& T = a.t[k];
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= a.n_pix) return;
  float u[4], c[4], v[4];
  if (a.cout == 8) {
    float fu[8], fc[8];
    unpack8(ld16(T.u + (size_t)pix * 8), fu);
    unpack8(ld16(T.c + (size_t)pix * 8), fc);
#pragma unroll
    for (int j = 0; j < 4; ++j) { u[j] = fu[j]; c[j] = fc[j]; v[j] = fc[4 + j]; }
  } else {
    const uint2 ru = *reinterpret_cast<const uint2*>(T.u + (size_t)pix * 4);
    const uint2 rc = *reinterpret_cast<const uint2*>(T.c + (size_t)pix * 4);
    u[0] = __uint_as_float(ru.x << 16); u[1] = __uint_as_float(ru.x & 0xffff0000u);
    u[2] = __uint_as_float(ru.y << 16); u[3] = __uint_as_float(ru.y & 0xffff0000u);
    c[0] = __uint_as_float(rc.x << 16); c[1] = __uint_as_float(rc.x & 0xffff0000u);
    c[2] = __uint_as_float(rc.y << 16); c[3] = __uint_as_float(rc.y & 0xffff0000u);
    v[0] = v[1] = v[2] = v[3] = 0.f;
  }
  const size_t o = (size_t)pix * 4;
  const float4 X = *reinterpret_cast<const float4*>(T.x + o);
  const float4 XS = *reinterpret_cast<const float4*>(T.xsrc + o);
  float4 H1 = make_float4(0.f, 0.f, 0.f, 0.f), H2 = H1, H3 = H1, P = H1, N = H1;
  if (T.h1) H1 = *reinterpret_cast<const float4*>(T.h1 + o);
  if (T.h2) H2 = *reinterpret_cast<const float4*>(T.h2 + o);
  if (T.h3) H3 = *reinterpret_cast<const float4*>(T.h3 + o);
  if (T.flags & 16) P = *reinterpret_cast<const float4*>(T.p + o);
  if (T.noise) N = *reinterpret_cast<const float4*>(T.noise + o);
  const float xs[4] = {X.x, X.y, X.z, X.w}, xsrc[4] = {XS.x, XS.y, XS.z, XS.w};
  const float h1[4] = {H1.x, H1.y, H1.z, H1.w}, h2[4] = {H2.x, H2.y, H2.z, H2.w};
  const float h3[4] = {H3.x, H3.y, H3.z, H3.w}, pp[4] = {P.x, P.y, P.z, P.w}, nn[4] = {N.x, N.y, N.z, N.w};
  float e[4], x0[4], out[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    e[j] = u[j] + T.g * (c[j] - u[j]);
    const float E = T.he0 * e[j] + T.he1 * h1[j] + T.he2 * h2[j] + T.he3 * h3[j];
    float z = T.px * xs[j] + T.pe * E;
    if (T.flags & 8) z = fminf(fmaxf(z, -T.clampv), T.clampv);
    x0[j] = z;
    float s = T.stdv;
    if (T.flags & 4) {
      const float f = (v[j] + 1.0f) * 0.5f;
      s = expf(0.5f * (f * T.logb + (1.0f - f) * T.plv));
    }
    out[j] = T.ox * xsrc[j] + T.oe * E + T.ox0 * z + T.od * (z - pp[j]) + s * nn[j];
  }
  if (T.hs) *reinterpret_cast<float4*>(T.hs + o) = make_float4(e[0], e[1], e[2], e[3]);
  if (T.flags & 1) *reinterpret_cast<float4*>(T.p + o) = make_float4(x0[0], x0[1], x0[2], x0[3]);
  if (T.flags & 2) *reinterpret_cast<float4*>(T.cur + o) = X;
  *reinterpret_cast<float4*>(T.x + o) = make_float4(out[0], out[1], out[2], out[3]);
  if (T.xin0) {
    uint2 b;
    b.x = (uint32_t)f2bf(out[0] * T.in_scale) | ((uint32_t)f2bf(out[1] * T.in_scale) << 16);
    b.y = (uint32_t)f2bf(out[2] * T.in_scale) | ((uint32_t)f2bf(out[3] * T.in_scale) << 16);
    *reinterpret_cast<uint2*>(T.xin0 + o) = b;
    if (T.xin1) *reinterpret_cast<uint2*>(T.xin1 + o) = b;
  }
}

// host layout of one task (pointers as uint64, then floats, then flags) - mirrors SampTask
static_assert(sizeof(SampTask) == 13 * 8 + 16 * 4 + 8, "SampTask layout");

ARB_API int arb_sampler_step(const void* tasks, int ntask, int n_pix, int cout, hipStream_t stream) {
  if (ntask < 1 || ntask > MAXT || n_pix < 1 || (cout != 4 && cout != 8)) return -1;
  SampArgs a;
  memcpy(a.t, tasks, sizeof(SampTask) * ntask);
  for (int k = 0; k < ntask; ++k) {
    const SampTask& t = a.t[k];
    if (!t.u || !t.c || !t.x || !t.xsrc) return -2;
    if ((t.flags & (1 | 16)) && !t.p) return -3;
    if ((t.flags & 2) && !t.cur) return -4;
    if ((reinterpret_cast<uintptr_t>(t.x) | reinterpret_cast<uintptr_t>(t.xsrc)) & 15) return -5;
    if (cout == 8 && ((reinterpret_cast<uintptr_t>(t.u) | reinterpret_cast<uintptr_t>(t.c)) & 15)) return -5;
    if (cout == 4 && ((reinterpret_cast<uintptr_t>(t.u) | reinterpret_cast<uintptr_t>(t.c)) & 7)) return -5;
  }
  a.ntask = ntask;
  a.n_pix = n_pix;
  a.cout = cout;
  dim3 grid((n_pix + 255) / 256, ntask);
  sampler_step_kernel<<<grid, 256, 0, stream>>>(a);
  return (int)hipGetLastError();
}
