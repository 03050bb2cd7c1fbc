// Blockwise single-head attention at head dim 512 for gfx950: the SD / zeroscope KL-VAE and the
// Kandinsky MoVQ mid-block self-attention (seq 4096 at 512^2, 9216 at
// the MoVQ's 96^2 latent, 16384 at 1024^2; batch = frames for the video VAE).  O(N) memory: the
// score matrix never exists - online softmax in fp32 over 32-key tiles streamed through LDS.
//
//   * one workgroup = 4 waves x 16 queries; every wave keeps its 16 queries' Q fragments (prescaled
//     by scale * log2 e, 64 VGPRs) and O^T accumulators (16 x 512 fp32, 128 VGPRs) in registers for
//     the whole key range - the 512-wide head is split over the O^T d-tiles of each wave, not over
//     waves, so no partial-score reduction across waves is needed.
//   * swapped products as in attention.hip: S^T = K Q^T (each lane owns one query column), P^T
//     straight from the S^T accumulators into the B operand of O^T = V^T P^T, V^T fragments by the
//     transposing LDS read ds_read_b64_tr_b16.  mfma_f32_16x16x32_bf16 throughout.
//   * K / V tiles (32 keys x 1 KiB) arrive by LDS-DMA (global_load_lds_dwordx4, one wave-instruction
//     per 1 KiB row, so rows can be padded): K rows at a 1040-B pitch (ds_read_b128 fragments: at most
//     one 2-way bank collision per 16-lane group, and every k-step's read is the lane's base address
//     plus an immediate - no per-fragment address registers), V rows at 1056 B (conflict-free
//     transposing reads).  Two stages (131 KiB of LDS),
//     the next tile's DMA in flight under the current tile's MFMAs.
//   * the key axis is split over S workgroups when (batch x query blocks) alone cannot fill the chip
//     (S from the launch geometry only, at most 8): each writes an fp32 partial O^T and its (max, sum);
//     attn512_combine_kernel merges the S partials in split order.  S = 1 normalises in place.
//   * no atomics, fixed reduction order -> bitwise deterministic.
#include "common.h"

#define A5_D 512
#define A5_KT 32                  // keys per tile
#define A5_QB 64                  // queries per workgroup (4 waves x 16)
#define A5_KROW (A5_D + 8)        // K row pitch in LDS (elements): 1040 B
#define A5_VROW (A5_D + 16)       // V row pitch in LDS (elements): 1056 B

struct A5Args {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  bf16_t* o;
  long q_sb, q_sn, q_sh;
  long k_sb, k_sn, k_sh;
  long v_sb, v_sn, v_sh;
  long o_sb, o_sn, o_sh;
  int B, H, Nq, Nk;
  float scale_log2;
  int nsplit, kper;               // key splits and keys per split (multiple of A5_KT)
  float* wo;                      // [S, B*H, Nq, 512] fp32 partial O (nsplit > 1)
  float2* wml;                    // [S, B*H, Nq] (running max in log2 units, row sum)
};

__device__ __attribute__((aligned(16))) uint4 g_a5_zero[4];

template <int S_ONE>
__global__ void __launch_bounds__(256, 1) attn512_kernel(A5Args a) {
  constexpr int KS = A5_D / 32;                 // QK k-steps
  constexpr int DT = A5_D / 16;                 // O^T d-tiles
  constexpr int STAGE = A5_KT * A5_KROW + A5_KT * A5_VROW;
  __shared__ __attribute__((aligned(16))) bf16_t sS0[STAGE];
  __shared__ __attribute__((aligned(16))) bf16_t sS1[STAGE];

  const int nqb = (a.Nq + A5_QB - 1) / A5_QB;
  const int total = nqb * a.H * a.B * a.nsplit;
  const int lin = xcd_remap(blockIdx.x, total);
  const int split = lin % a.nsplit;             // the splits of one query block share an XCD
  const int rest = lin / a.nsplit;
  const int qb = rest % nqb;
  const int bh = rest / nqb;
  const int h = bh % a.H, b = bh / a.H;

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lq = lane & 15, g = lane >> 4;
  const bf16_t* qbase = a.q + b * a.q_sb + h * a.q_sh;
  const bf16_t* kbase = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vbase = a.v + b * a.v_sb + h * a.v_sh;
  const int k0 = split * a.kper;
  const int k1 = min(a.Nk, k0 + a.kper);

  // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[q][32 s + 8 g .. +7] * scale * log2 e
  const int qi = qb * A5_QB + wave * 16 + lq;
  bf16x8 qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    uint4 raw = make_uint4(0, 0, 0, 0);
    if (qi < a.Nq) raw = ld16(qbase + (long)qi * a.q_sn + 32 * s + 8 * g);
    float f[8];
    unpack8(raw, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] *= a.scale_log2;
    qf[s] = __builtin_bit_cast(bf16x8, pack8(f));
  }

  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  typedef __attribute__((address_space(1))) const void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  // DMA of one tile: rows r = wave + 4 i (i < 8) of K and of V, one 1 KiB wave-instruction each
  auto issue = [&](int kv, bf16_t* dst) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < A5_KT / 4; ++i) {
      const int r = wave + 4 * i;
      const bool ok = kv + r < k1;
      const void* src = ok ? (const void*)(kbase + (long)(kv + r) * a.k_sn + (lane << 3)) : (const void*)g_a5_zero;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + r * A5_KROW), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < A5_KT / 4; ++i) {
      const int r = wave + 4 * i;
      const bool ok = kv + r < k1;
      const void* src = ok ? (const void*)(vbase + (long)(kv + r) * a.v_sn + (lane << 3)) : (const void*)g_a5_zero;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + A5_KT * A5_KROW + r * A5_VROW), 16, 0, 0);
    }
  };

  // ---- one 32-key tile, software-pipelined by hand (one wave per SIMD: nothing else hides an LDS
  // round trip).  LDS fragment reads go in batches of 8 MFMAs' worth, each batch issued before the
  // MFMAs of the previous one (sched_group_barrier pins the order; hipcc's counted lgkmcnt then
  // waits only for the batch being consumed):
  //   QK:  K0 | K1 . mma K0 | K2 . mma K1 | K3 . mma K2 | V0 . mma K3 | softmax | V1 . mma V0 | ...
  // with K batches b = (key tile t, k-steps 8 h .. 8 h + 7) and V batches = 8 O^T d-tiles each.
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const int qq = (lane & 15) >> 2, pp = lane & 3;
  auto compute = [&](int kv0, const bf16_t* cK, const bf16_t* cV) __attribute__((always_inline)) {
    const float mi = m_run != -INFINITY ? -m_run : 0.f;
    f32x4 st[2];
    st[0] = (f32x4){mi, mi, mi, mi};
    st[1] = st[0];
    const bf16_t* kb0 = &cK[lq * A5_KROW + 8 * g];      // + 16 rows per key tile, + 32 per k-step
    const bf16_t* vb = &cV[(4 * g + qq) * A5_VROW + 4 * pp];
    bf16x8 ka[8], kb[8];
    auto kread = [&](bf16x8 (&kf)[8], int b) __attribute__((always_inline)) {
#pragma unroll
      for (int s = 0; s < 8; ++s)
        kf[s] = __builtin_bit_cast(bf16x8, ld16(kb0 + (b >> 1) * 16 * A5_KROW + 32 * (8 * (b & 1) + s)));
    };
    auto kmma = [&](const bf16x8 (&kf)[8], int b) __attribute__((always_inline)) {
#pragma unroll
      for (int s = 0; s < 8; ++s)
        st[b >> 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[s], qf[8 * (b & 1) + s], st[b >> 1], 0, 0, 0);
    };
    s16x4 va[16], vc[16];                                   // one V batch: lo / hi halves of 8 d-tiles
    auto vread = [&](s16x4 (&vf)[16], int d0) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        vf[2 * j] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, vb + 16 * (d0 + j)));
        vf[2 * j + 1] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, vb + 16 * (d0 + j) + 16 * A5_VROW));
      }
    };
    auto vmma = [&](const s16x4 (&vf)[16], int d0, const bf16x8& pf) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const s16x4 lo = vf[2 * j], hi = vf[2 * j + 1];
        s16x8 vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[d0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pf, o[d0 + j], 0, 0, 0);
      }
    };
#define A5_GRP(nread, nmma)                                 \
  __builtin_amdgcn_sched_group_barrier(0x100, nread, 0);    \
  __builtin_amdgcn_sched_group_barrier(0x008, nmma, 0);
    kread(ka, 0);
    kread(kb, 1);
    kmma(ka, 0);
    A5_GRP(16, 8)
    kread(ka, 2);
    kmma(kb, 1);
    A5_GRP(8, 8)
    kread(kb, 3);
    kmma(ka, 2);
    A5_GRP(8, 8)
    vread(va, 0);
    kmma(kb, 3);
    A5_GRP(16, 8)
    if (kv0 + A5_KT > k1) {                     // keys past this split's range / past Nk
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kv0 + 16 * t + 4 * g + r >= k1) st[t][r] = -INFINITY;
    }
    float mloc = vmax3(st[0][0], st[0][1], st[0][2]);       // single-instruction maxes (common.h)
    mloc = vmax3(mloc, st[0][3], st[1][0]);
    mloc = vmax3(mloc, st[1][1], st[1][2]);
    mloc = vmax2(mloc, st[1][3]);
    mloc = max_xor16(mloc);
    mloc = max_xor32(mloc);
    // lazy rescale (attention.hip T13): the running max moves only when it grew by > 8 (log2 units)
    const float m_old = m_run;
    const float m_cand = (m_old == -INFINITY ? 0.f : m_old) + mloc;
    const bool need = m_cand > m_old + 8.f;
    float alpha = 1.f;
    if (need) {
      alpha = (m_old == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m_old - m_cand);
      m_run = m_cand;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) st[t][r] -= mloc;
    }
    float lsum = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[t][r] = __builtin_amdgcn_exp2f(st[t][r]);
        lsum += st[t][r];
      }
    l_run = l_run * alpha + lsum;
    if (__any(need)) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
    }
    // P^T fragment (k order: 8 g + j <-> key 4 g + j, 8 g + 4 + j <-> 16 + 4 g + j, as the V^T reads)
    bf16x8 pf;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pf[j] = (__bf16)st[0][j];
      pf[j + 4] = (__bf16)st[1][j];
    }
    vread(vc, 8);
    vmma(va, 0, pf);
    A5_GRP(16, 8)
    vread(va, 16);
    vmma(vc, 8, pf);
    A5_GRP(16, 8)
    vread(vc, 24);
    vmma(va, 16, pf);
    A5_GRP(16, 8)
    vmma(vc, 24, pf);
#undef A5_GRP
  };

  // two stages with static roles (loop unrolled by 2); a stage is refilled only after the barrier
  // that retired its last reads
  if (k0 < k1) issue(k0, sS0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kv0 = k0; kv0 < k1; kv0 += 2 * A5_KT) {
    const int kv1 = kv0 + A5_KT;
    if (kv1 < k1) issue(kv1, sS1);
    compute(kv0, sS0, sS0 + A5_KT * A5_KROW);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kv1 >= k1) break;
    if (kv1 + A5_KT < k1) issue(kv1 + A5_KT, sS0);
    compute(kv1, sS1, sS1 + A5_KT * A5_KROW);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  float l = l_run;
  l = sum_xor16(l);
  l = sum_xor32(l);
  if (qi >= a.Nq) return;
  if constexpr (S_ONE) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16_t* orow = a.o + b * a.o_sb + h * a.o_sh + (long)qi * a.o_sn;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      uint2 w;
      w.x = (uint32_t)f2bf(o[dt][0] * inv) | ((uint32_t)f2bf(o[dt][1] * inv) << 16);
      w.y = (uint32_t)f2bf(o[dt][2] * inv) | ((uint32_t)f2bf(o[dt][3] * inv) << 16);
      *reinterpret_cast<uint2*>(orow + 16 * dt + 4 * g) = w;
    }
  } else {
    const long row = ((long)split * a.B * a.H + bh) * a.Nq + qi;
    float* wrow = a.wo + row * A5_D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) *reinterpret_cast<f32x4*>(wrow + 16 * dt + 4 * g) = o[dt];
    if (g == 0) a.wml[row] = make_float2(m_run, l);
  }
}

// out[q, d..d+7] = sum_s 2^(m_s - M) O_s / sum_s 2^(m_s - M) l_s, splits summed in order
__global__ void __launch_bounds__(256) attn512_combine_kernel(A5Args a) {
  const long rows = (long)a.B * a.H * a.Nq;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * (A5_D / 8)) return;
  const long r = i / (A5_D / 8);
  const int d = (int)(i - r * (A5_D / 8)) * 8;
  const int qi = (int)(r % a.Nq);
  const int bh = (int)(r / a.Nq);
  const int h = bh % a.H, b = bh / a.H;
  float M = -INFINITY;
  for (int s = 0; s < a.nsplit; ++s) M = fmaxf(M, a.wml[(long)s * rows + r].x);
  float L = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < a.nsplit; ++s) {
    const float2 ml = a.wml[(long)s * rows + r];
    const float w = ml.x == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(ml.x - M);
    L += w * ml.y;
    const float4* src = reinterpret_cast<const float4*>(a.wo + ((long)s * rows + r) * A5_D + d);
    const float4 x0 = src[0], x1 = src[1];
    acc[0] += w * x0.x; acc[1] += w * x0.y; acc[2] += w * x0.z; acc[3] += w * x0.w;
    acc[4] += w * x1.x; acc[5] += w * x1.y; acc[6] += w * x1.z; acc[7] += w * x1.w;
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] *= inv;
  st16(a.o + b * a.o_sb + h * a.o_sh + (long)qi * a.o_sn + d, pack8(acc));
}

// Key splits of one call, from the launch geometry only (equal calls split equally): only when the
// query blocks alone leave CUs idle (< 256 workgroups; one workgroup per CU), then the split count
// 1..8 (>= 512 keys each) whose workgroups fill the last round of 256 best, a larger split only for a
// clearly fuller chip (4096 tokens: 4 splits, 256 workgroups; 9216: 5 splits, 720 of 768 slots).
static int a5_splits(int B, int H, int Nq, int Nk) {
  const long blocks = (long)B * H * ((Nq + A5_QB - 1) / A5_QB);
  if (blocks >= 256) return 1;
  auto fill = [&](int s) { const long n = blocks * s; return (double)n / (256.0 * ((n + 255) / 256)); };
  int best = 1;
  for (int s = 2; s <= 8 && Nk >= s * 512; ++s)
    if (fill(s) > fill(best) + 0.05) best = s;
  return best;
}

// workspace bytes for arb_attention512 (0 when the call does not split)
ARB_API long arb_attention512_workspace(int B, int H, int Nq, int Nk) {
  const int s = a5_splits(B, H, Nq, Nk);
  if (s == 1) return 0;
  const long rows = (long)B * H * Nq;
  return (long)s * rows * (A5_D * 4 + 8);
}

// q/k/v/o [B, N, H, 512] with element strides {sb, sn, sh} x 4 (q, k, v, o); last dim contiguous.
ARB_API int arb_attention512(const void* q, const void* k, const void* v, void* o, const long* strides, int B, int H,
                             int Nq, int Nk, float scale, void* ws, hipStream_t stream) {
  if (Nq <= 0 || Nk <= 0) return -1;
  A5Args a;
  a.q = (const bf16_t*)q;
  a.k = (const bf16_t*)k;
  a.v = (const bf16_t*)v;
  a.o = (bf16_t*)o;
  a.q_sb = strides[0]; a.q_sn = strides[1]; a.q_sh = strides[2];
  a.k_sb = strides[3]; a.k_sn = strides[4]; a.k_sh = strides[5];
  a.v_sb = strides[6]; a.v_sn = strides[7]; a.v_sh = strides[8];
  a.o_sb = strides[9]; a.o_sn = strides[10]; a.o_sh = strides[11];
  a.B = B; a.H = H; a.Nq = Nq; a.Nk = Nk;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.nsplit = a5_splits(B, H, Nq, Nk);
  a.kper = ((Nk + a.nsplit - 1) / a.nsplit + A5_KT - 1) / A5_KT * A5_KT;
  a.nsplit = (Nk + a.kper - 1) / a.kper;        // no empty split
  const long rows = (long)B * H * Nq;
  a.wo = nullptr;
  a.wml = nullptr;
  if (a.nsplit > 1) {
    if (ws == nullptr) return -3;
    a.wo = (float*)ws;
    a.wml = (float2*)((char*)ws + (long)a.nsplit * rows * A5_D * 4);
  }
  const long blocks = (long)B * H * ((Nq + A5_QB - 1) / A5_QB) * a.nsplit;
  if (blocks > 0x7fffffffL) return -4;
  if (a.nsplit == 1) {
    attn512_kernel<1><<<dim3((unsigned)blocks), 256, 0, stream>>>(a);
  } else {
    attn512_kernel<0><<<dim3((unsigned)blocks), 256, 0, stream>>>(a);
    const long n = rows * (A5_D / 8);
    attn512_combine_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, stream>>>(a);
  }
  return (int)hipGetLastError();
}
