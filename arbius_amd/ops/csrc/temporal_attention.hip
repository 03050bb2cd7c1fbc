// Temporal self-attention over the frames axis (UNet3D of zeroscopev2xl / damo,
// SURVEY.md §2.6(c), §5.7): a SHORT sequence (F = 1..96 frames) for a HUGE batch
// (every latent pixel x head x CFG branch: 2 x 2880 x 5 = 28800 problems at the
// 576x320x24f level-0 blocks).  The generic flash kernel tiles 64+ queries per
// wave and would idle >60% of every MFMA here, so this kernel gives each wave
// ONE (video, pixel, head) problem and keeps the whole frame axis in registers:
//
//   S^T = K Q^T  on mfma_f32_16x16x32_bf16 (K rows / Q rows are 16-byte loads
//                straight from the activation - no LDS, no transposes)
//   softmax over keys: in-lane over the 4 C rows x key tiles, then xor 16/32
//   O^T = V^T P^T: P^T is consumed from the S^T accumulators in place through
//                a permuted key order (slot 8g+j <-> key tile/row held by lane
//                group g); V^T comes from the wave's V rows staged in LDS by
//                16-byte loads and read back with the CDNA4 transposing read
//                ds_read_b64_tr_b16 (the flash kernel's PV fragment path, row
//                stride 16*(odd) elements: conflict free) - round 5 gathered it
//                with 2-byte loads, 32 per lane (MFMA:VALU 1:45, pmc_r4_zeroscope).
//
// Activations stay in the UNet's frame-major channels-last layout
// [B*F, H, W, C] (fused QKV adds a 3x): element (b, f, p, h, d) is at
// b*sb + f*sf + p*sp + h*sh + d, so no permute/copy exists on either side.
// Deterministic: fixed reduction order, no atomics.
#include "common.h"

struct TAArgs {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  bf16_t* o;
  long q_sb, q_sf, q_sp, q_sh;
  long k_sb, k_sf, k_sp, k_sh;
  long v_sb, v_sf, v_sp, v_sh;
  long o_sb, o_sf, o_sp, o_sh;
  int B, F, P, H;
  long items;
  float scale_log2;
};

template <int KT32, int DD>
__global__ void __launch_bounds__(256) temporal_attn_kernel(TAArgs a) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long item = (long)blockIdx.x * 4 + wave;
  if (item >= a.items) return;
  const int h = (int)(item % a.H);
  const long t = item / a.H;
  const int p = (int)(t % a.P);
  const int b = (int)(t / a.P);
  const bf16_t* qb = a.q + b * a.q_sb + p * a.q_sp + h * a.q_sh;
  const bf16_t* kb = a.k + b * a.k_sb + p * a.k_sp + h * a.k_sh;
  const bf16_t* vb = a.v + b * a.v_sb + p * a.v_sp + h * a.v_sh;
  bf16_t* ob = a.o + b * a.o_sb + p * a.o_sp + h * a.o_sh;
  const int F = a.F;
  const int r16 = lane & 15, g = lane >> 4;
  constexpr int KS = DD / 32;     // contraction steps of S
  constexpr int NKT = 2 * KT32;   // 16-key tiles
  constexpr int DT = DD / 16;     // 16-row d tiles of O^T
  const bf16x8 zero8 = __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));

  // K as the A operand of S^T: lane holds K[kt*16 + r16][ks*32 + 8g .. +7]
  bf16x8 kf[NKT][KS];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    const int key = kt * 16 + r16;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      kf[kt][ks] = key < F ? __builtin_bit_cast(bf16x8, ld16(kb + key * a.k_sf + ks * 32 + 8 * g)) : zero8;
  }
  // V^T as the A operand of O^T, permuted key slots: slot 8g+j <-> key
  //   j < 4: tile 2s, row 4g+j      j >= 4: tile 2s+1, row 4g+j-4
  // V rows [0, 32*KT32) of this wave's problem -> LDS (keys >= F zero), 16-byte chunks
  constexpr int VROWT = 16 * (DT | 1);
  constexpr int CPR = DD / 8;
  __shared__ __attribute__((aligned(16))) bf16_t sV[4][32 * KT32 * VROWT];
  bf16_t* myV = sV[wave];
#pragma unroll
  for (int c = lane; c < 32 * KT32 * CPR; c += 64) {
    const int row = c / CPR, col = (c % CPR) * 8;
    st16(&myV[row * VROWT + col], row < F ? ld16(vb + row * a.v_sf + col) : make_uint4(0, 0, 0, 0));
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's rows are in LDS (reads are wave-local)
  __builtin_amdgcn_wave_barrier();
  bf16x8 vf[KT32][DT];
  const int qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
  for (int s = 0; s < KT32; ++s) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const bf16_t* a0 = &myV[(32 * s + 4 * g + qq) * VROWT + 16 * dt + 4 * pp];
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0 + 16 * VROWT));
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      const s16x8 vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      vf[s][dt] = __builtin_bit_cast(bf16x8, vv);
    }
  }

  // two query tiles per pass (F = 24: both of them): their QK -> max -> exp -> PV chains are independent,
  // so the scheduler interleaves them; per query tile the arithmetic (and the order of the row sum) is
  // unchanged.  A second tile past F (odd tile counts) computes masked garbage and stores nothing.
  const int QT = (F + 15) >> 4;
  for (int qt0 = 0; qt0 < QT; qt0 += 2) {
    int qrow[2];
    f32x4 sc[2][NKT];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      qrow[u] = (qt0 + u) * 16 + r16;
      bf16x8 qf[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        qf[ks] = qrow[u] < F ? __builtin_bit_cast(bf16x8, ld16(qb + qrow[u] * a.q_sf + ks * 32 + 8 * g)) : zero8;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        sc[u][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          sc[u][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][ks], qf[ks], sc[u][kt], 0, 0, 0);
      }
    }
    // sc[u][kt][r] = S^T[key = kt*16 + 4g + r][query = (qt0 + u)*16 + r16]
    float mx[2], sum[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      mx[u] = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt * 16 + 4 * g + r;
          const float v = key < F ? sc[u][kt][r] * a.scale_log2 : -INFINITY;
          sc[u][kt][r] = v;
        }
        mx[u] = vmax3(mx[u], vmax2(sc[u][kt][0], sc[u][kt][1]), vmax2(sc[u][kt][2], sc[u][kt][3]));
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) mx[u] = max_xor16(mx[u]);
#pragma unroll
    for (int u = 0; u < 2; ++u) mx[u] = max_xor32(mx[u]);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      sum[u] = 0.f;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(sc[u][kt][r] - mx[u]);
          sc[u][kt][r] = e;
          sum[u] += e;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) sum[u] = sum_xor16(sum[u]);
#pragma unroll
    for (int u = 0; u < 2; ++u) sum[u] = sum_xor32(sum[u]);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      f32x4 oc[DT];
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) oc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KT32; ++s) {
        u16x8 pu;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pu[j] = f2bf(sc[u][2 * s][j]);
          pu[4 + j] = f2bf(sc[u][2 * s + 1][j]);
        }
        const bf16x8 pb = __builtin_bit_cast(bf16x8, pu);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
          oc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[s][dt], pb, oc[dt], 0, 0, 0);
      }
      // oc[dt][r] = O^T[d = dt*16 + 4g + r][query = qrow]
      if (qrow[u] < F) {
        const float inv = 1.f / sum[u];
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const uint32_t w0 = (uint32_t)f2bf(oc[dt][0] * inv) | ((uint32_t)f2bf(oc[dt][1] * inv) << 16);
          const uint32_t w1 = (uint32_t)f2bf(oc[dt][2] * inv) | ((uint32_t)f2bf(oc[dt][3] * inv) << 16);
          *reinterpret_cast<uint2*>(ob + qrow[u] * a.o_sf + dt * 16 + 4 * g) = make_uint2(w0, w1);
        }
      }
    }
  }
}

// strides: 16 longs (q, k, v, o) x (sb, sf, sp, sh) in elements.  F <= 96, D in {32, 64, 128}.
ARB_API int arb_temporal_attention(const void* q, const void* k, const void* v, void* o, const long* st, int B, int F,
                                   int P, int H, int D, float scale, hipStream_t stream) {
  if (F < 1 || F > 96 || (D != 32 && D != 64 && D != 128)) return -1;
  TAArgs a;
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.o = (bf16_t*)o;
  a.q_sb = st[0]; a.q_sf = st[1]; a.q_sp = st[2]; a.q_sh = st[3];
  a.k_sb = st[4]; a.k_sf = st[5]; a.k_sp = st[6]; a.k_sh = st[7];
  a.v_sb = st[8]; a.v_sf = st[9]; a.v_sp = st[10]; a.v_sh = st[11];
  a.o_sb = st[12]; a.o_sf = st[13]; a.o_sp = st[14]; a.o_sh = st[15];
  a.B = B; a.F = F; a.P = P; a.H = H;
  a.items = (long)B * P * H;
  a.scale_log2 = scale * 1.4426950408889634f;
  const long blocks = (a.items + 3) / 4;
  if (blocks > 0x7fffffffL) return -2;
  const int kt32 = (F + 31) / 32;
#define TA_CASE(KT, DDV) \
  if (kt32 == KT && D == DDV) {                                                  \
    temporal_attn_kernel<KT, DDV><<<(unsigned)blocks, 256, 0, stream>>>(a);      \
    return (int)hipGetLastError();                                                \
  }
  TA_CASE(1, 64) TA_CASE(2, 64) TA_CASE(3, 64)
  TA_CASE(1, 32) TA_CASE(2, 32) TA_CASE(3, 32)
  TA_CASE(1, 128) TA_CASE(2, 128) TA_CASE(3, 128)
#undef TA_CASE
  return -3;
}
