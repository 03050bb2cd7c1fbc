// Flash attention forward for gfx950 (bf16 in/out, fp32 softmax + accumulate).
//
// Serves every attention of the engine: UNet self-attention (seq 4096/1024/256/64,
// head dims 40/80/160), cross-attention against 77 text tokens, CLIP causal
// self-attention (d 64), Kandinsky joint attention and the UNet3D temporal
// attention (seq = frames).  SURVEY.md §2.6 (a)-(c), §5.7.
//
// Structure (one workgroup = 4 waves, QT x 16 query rows per wave):
//   * swapped product S^T = K Q^T on mfma_f32_16x16x32_bf16, so each lane owns
//     ONE query column (q = lane&15) and 4 keys per 16-key tile: softmax row
//     statistics need only two cross-lane steps (xor 16/32) and the O^T
//     accumulator rows are lane-aligned with them.
//   * P^T goes straight from the S^T accumulators into the B operand of
//     O^T = V^T P^T with a permuted k order (no LDS round-trip for P).
//   * V^T fragments come from the row-major V tile through the CDNA4 transposing
//     read ds_read_b64_tr_b16; row stride 16*(odd) elements -> conflict free (T10).
//   * ROW SUMS ON THE MATRIX CORE: when D % 16 != 0 (d=40: the 4096-token SD
//     self-attention, VALU-bound) the zero-padded V column D is set to 1.0, so
//     O^T row D accumulates sum_k P[q,k] with the same rescaling as O - the
//     per-score add of the softmax denominator disappears from the VALU.
//   * scores stay raw; the scale is folded into the exp2 fma (max commutes).
//   * K/V: register-staged prefetch of tile j+1 while tile j is consumed, LDS
//     double buffer -> one barrier per 64-key tile (T14).
//   * head dim padded to 32 (QK^T k-dim) / 16 (PV n-dim) with zero fill; key
//     padding masked with -inf only on partial tiles; V padding rows zero.
//   * 1-D XCD-aware block remap: the q-blocks of one (batch, head) share an L2.
//   * no atomics, fixed reduction order -> bitwise deterministic.
#include "common.h"

#include <cstdlib>

#define KV_BLK 64

struct AttnArgs {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  bf16_t* o;
  long q_sb, q_sn, q_sh;
  long k_sb, k_sn, k_sh;
  long v_sb, v_sn, v_sh;
  long o_sb, o_sn, o_sh;
  int B, H, Nq, Nk, D;
  float scale_log2;
  int causal;
  // optional K/V PREFIX segment (keys [0, Np) read from kp/vp, keys [Np, Nk) from k/v at
  // j - Np): the Kandinsky joint attention's text+image context tokens ahead of the spatial
  // tokens, without materialising cat(ctx_kv, kv) every layer and step.
  const bf16_t* kp;
  const bf16_t* vp;
  long kp_sb, kp_sn, vp_sb, vp_sn;
  int Np;
};

// 16-byte sources of the LDS-DMA staging: zero padding, and V's ones column (row-sum trick)
__device__ __attribute__((aligned(16))) uint4 g_attn_zero[1];
__device__ __attribute__((aligned(16))) uint4 g_attn_ones[1] = {{0x3F80u, 0u, 0u, 0u}};

// GLDS: K/V tiles arrive by LDS-DMA (global_load_lds, 16 B per lane straight into LDS, no VGPR
// staging, no ds_write): K rows are 8 chunks (128 B, KSTEPS == 2 only) with the chunk XOR-swizzled
// by (row & 7) on the SOURCE address (lane-linear LDS image, rule 21) and on the QK read; V rows
// are VROW/8 chunks, already lane-linear; padding chunks read a zero page, V's row-sum column a
// ones page.  One LDS array for everything (hipcc's vmcnt trap with two __shared__ objects).
template <int KSTEPS, int DT, int QT, bool ONES, bool GLDS = false, bool PP = false, bool PS = true, bool ILP = true,
          bool PFX = false>
__global__ void __launch_bounds__(256, 2) flash_attn_fwd_kernel(AttnArgs a) {
  static_assert(!GLDS || KSTEPS == 2, "LDS-DMA staging: 8-chunk K rows only");
  constexpr int KROW = GLDS ? KSTEPS * 32 : KSTEPS * 32 + 8;   // K tile row (elements)
  constexpr int VROW = 16 * (DT | 1);      // V tile row: 16*(odd) -> tr-read conflict free
  constexpr int QBLK = 4 * QT * 16;        // queries per workgroup
  constexpr int KCH = KV_BLK * KSTEPS * 4;
  constexpr int VCH = KV_BLK * DT * 2;
  constexpr int KPT = (KCH + 255) / 256, VPT = (VCH + 255) / 256;
  // one array per pipeline stage: K rows then V rows.  Two distinct __shared__ objects give the
  // LDS accesses disjoint alias scopes, so (GLDS, loop unrolled by 2 with static stage roles)
  // hipcc need not drain the DMA into one stage before the ds_reads of the other.
  constexpr int STAGE = KV_BLK * (KROW + VROW);
  __shared__ __attribute__((aligned(16))) bf16_t sS0[STAGE];
  __shared__ __attribute__((aligned(16))) bf16_t sS1[STAGE];

  const int nqb = (a.Nq + QBLK - 1) / QBLK;
  const int total = nqb * a.H * a.B;
  const int lin = xcd_remap(blockIdx.x, total);
  const int qb = lin % nqb;
  const int h = (lin / nqb) % a.H;
  const int b = lin / (nqb * a.H);

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int lq = lane & 15, g = lane >> 4, g4 = 4 * g;
  const int D = a.D;
  // lane-pair reductions: the gfx950 lane swaps (VALU) where the registers allow; at 4 query tiles of a
  // 48/64-wide head (and the 129..160-wide heads) they push the kernel past 256 VGPRs (up to 45 spills),
  // so those keep the LDS permute
  constexpr bool SWAPS = !(QT >= 4 && (DT >= 4 || !ONES)) && KSTEPS < 5;
  auto mx16 = [](float x) __attribute__((always_inline)) {
    return SWAPS ? max_xor16(x) : vmax2(x, __shfl_xor(x, 16, 64));
  };
  auto mx32 = [](float x) __attribute__((always_inline)) {
    return SWAPS ? max_xor32(x) : vmax2(x, __shfl_xor(x, 32, 64));
  };
  // ONES: D % 16 != 0 -> the spare zero-padded V column D carries the row sum

  const bf16_t* qbase = a.q + b * a.q_sb + h * a.q_sh;
  const bf16_t* kbase = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vbase = a.v + b * a.v_sb + h * a.v_sh;
  const bf16_t* kpbase = a.Np ? a.kp + b * a.kp_sb + h * a.k_sh : nullptr;
  const bf16_t* vpbase = a.Np ? a.vp + b * a.vp_sb + h * a.v_sh : nullptr;
  auto krow = [&](int j) { return j < a.Np ? kpbase + (long)j * a.kp_sn : kbase + (long)(j - a.Np) * a.k_sn; };
  auto vrow = [&](int j) { return j < a.Np ? vpbase + (long)j * a.vp_sn : vbase + (long)(j - a.Np) * a.v_sn; };

  // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[q][32s + 8g .. +7]
  bf16x8 qf[QT][KSTEPS];
  int qidx[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    qidx[qt] = qb * QBLK + (wave * QT + qt) * 16 + lq;
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      const int d = 32 * s + 8 * g;
      uint4 raw = make_uint4(0, 0, 0, 0);
      if (qidx[qt] < a.Nq && d < D) raw = ld16(qbase + (long)qidx[qt] * a.q_sn + d);
      if constexpr (PS) {   // Q * scale * log2(e), rounded to bf16 once
        float f[8];
        unpack8(raw, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] *= a.scale_log2;
        raw = pack8(f);
      }
      qf[qt][s] = __builtin_bit_cast(bf16x8, raw);
    }
  }

  f32x4 o[QT][DT];
  float m_run[QT], l_run[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    m_run[qt] = -INFINITY;
    l_run[qt] = 0.f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[qt][dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  int kv_end = a.Nk;
  if (a.causal) {
    const int qmax = min(a.Nq, (qb + 1) * QBLK) - 1;
    kv_end = min(a.Nk, qmax + 1);
  }

  uint4 rk[KPT], rv[VPT];
  const uint32_t one_bits = 0x3F80u;  // bf16 1.0
  // Per-thread staging geometry is fixed across key tiles: row / column of each 16-byte chunk,
  // its in-range flag, and the row pointer (main K/V segment).  Full tiles of the main segment
  // then cost one uniform offset add per chunk; partial / prefix-straddling tiles take the
  // general path (bounds + prefix select per row).
  int kr[KPT], kc[KPT], vr[VPT], vc[VPT];
  bool kok[KPT], vok[VPT], vone[VPT];
  const bf16_t* kp0[KPT];
  const bf16_t* vp0[VPT];
#pragma unroll
  for (int i = 0; i < KPT; ++i) {
    const int c = tid + 256 * i;
    kr[i] = c / (KSTEPS * 4);
    kc[i] = (c % (KSTEPS * 4)) * 8;
    kok[i] = c < KCH && kc[i] < D;
    kp0[i] = kbase + (long)kr[i] * a.k_sn + kc[i];
  }
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = tid + 256 * i;
    vr[i] = c / (DT * 2);
    vc[i] = (c % (DT * 2)) * 8;
    vok[i] = c < VCH && vc[i] < D;
    // column D is the first element of the first all-padding 8-chunk when D % 16 == 8
    vone[i] = ONES && c < VCH && vc[i] == (D & ~7);
    vp0[i] = vbase + (long)vr[i] * a.v_sn + vc[i];
  }
  auto load_kv = [&](int kv) {
    if (kv >= a.Np && kv + KV_BLK <= a.Nk) {          // full tile of the main segment (uniform)
      const long ko = (long)(kv - a.Np) * a.k_sn, vo = (long)(kv - a.Np) * a.v_sn;
#pragma unroll
      for (int i = 0; i < KPT; ++i) rk[i] = kok[i] ? ld16(kp0[i] + ko) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        uint4 val = vok[i] ? ld16(vp0[i] + vo) : make_uint4(0, 0, 0, 0);
        if (vone[i]) val.x = (val.x & 0xffff0000u) | one_bits;
        rv[i] = val;
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < KPT; ++i)
      rk[i] = (kok[i] && kv + kr[i] < a.Nk) ? ld16(krow(kv + kr[i]) + kc[i]) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      uint4 val = (vok[i] && kv + vr[i] < a.Nk) ? ld16(vrow(kv + vr[i]) + vc[i]) : make_uint4(0, 0, 0, 0);
      if (vone[i]) val.x = (val.x & 0xffff0000u) | one_bits;
      rv[i] = val;
    }
  };
  auto store_kv = [&](int buf) {
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int c = tid + 256 * i;
      if (c < KCH) st16(&(buf ? sS1 : sS0)[(c / (KSTEPS * 4)) * KROW + (c % (KSTEPS * 4)) * 8], rk[i]);
    }
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = tid + 256 * i;
      if (c < VCH) st16(&(buf ? sS1 : sS0)[KV_BLK * KROW + (c / (DT * 2)) * VROW + (c % (DT * 2)) * 8], rv[i]);
    }
  };
  // ---- LDS-DMA staging geometry (GLDS): per wave-instruction block b (64 chunks), lane l
  constexpr int KBLK = KV_BLK * KSTEPS * 4 / 64;        // K blocks per tile (8)
  constexpr int VCPR = VROW / 8;                         // V chunks per LDS row
  constexpr int VBLK = KV_BLK * VCPR / 64;               // V blocks per tile
  constexpr int KBW = (KBLK + 3) / 4, VBW = (VBLK + 3) / 4;   // blocks per wave
  typedef __attribute__((address_space(1))) const void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  const bf16_t* gk[KBW];
  const bf16_t* gv[VBW];
  int gkr[KBW], gvr[VBW];
  int gkm[KBW], gvm[VBW];           // 0: zero page, 1: data, 2: ones page (V row-sum column)
  int gvb[VBW];
  if constexpr (GLDS) {
    static_assert(KBLK % 4 == 0, "K blocks split evenly over the 4 waves");
#pragma unroll
    for (int i = 0; i < KBW; ++i) {
      const int blk = wave + 4 * i;
      const int row = blk * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ (row & 7);               // logical chunk at this position
      gkr[i] = row;
      gkm[i] = (blk < KBLK && lc * 8 < D) ? 1 : 0;
      gk[i] = kbase + (long)row * a.k_sn + lc * 8;
    }
#pragma unroll
    for (int i = 0; i < VBW; ++i) {
      // a wave short of V blocks re-issues its first one (same bytes to the same LDS slot), so
      // every DMA is unconditional and the wait counts stay static
      const int blk = (wave + 4 * i < VBLK) ? wave + 4 * i : wave;
      gvb[i] = blk;
      const int q = blk * 64 + lane;
      const int row = q / VCPR, col = (q % VCPR) * 8;
      gvr[i] = row;
      gvm[i] = col < D ? 1 : (ONES && col == (D & ~7)) ? 2 : 0;
      gv[i] = vbase + (long)row * a.v_sn + col;
    }
  }
  // per-lane DMA sources resolved once (data row / zero page / ones page): a tile then costs one uniform
  // offset per chunk, and the range check runs only on a partial tile (the same bytes as resolving
  // them per tile, without the divergent page selection on every tile)
  const char* kb0[KBW];
  const char* vb0[VBW];
  if constexpr (GLDS) {
#pragma unroll
    for (int i = 0; i < KBW; ++i) kb0[i] = gkm[i] ? (const char*)gk[i] : (const char*)g_attn_zero;
#pragma unroll
    for (int i = 0; i < VBW; ++i)
      vb0[i] = gvm[i] == 1 ? (const char*)gv[i] : gvm[i] == 2 ? (const char*)g_attn_ones : (const char*)g_attn_zero;
  }
  auto issue_kv = [&](int kv, bf16_t* dst) __attribute__((always_inline)) {
    if (PFX && kv < a.Np) {
      // a tile holding PREFIX keys (Kandinsky joint attention: the first one or two tiles): every row
      // picks its segment - prefix row j from kp/vp, main row j - Np from k/v
#pragma unroll
      for (int i = 0; i < KBW; ++i) {
        const int j = kv + gkr[i], col = ((lane & 7) ^ (gkr[i] & 7)) * 8;
        const void* src = !gkm[i] || j >= a.Nk ? (const void*)g_attn_zero
                          : j < a.Np ? (const void*)(kpbase + (long)j * a.kp_sn + col)
                                     : (const void*)(kbase + (long)(j - a.Np) * a.k_sn + col);
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + (wave + 4 * i) * 512), 16, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < VBW; ++i) {
        const int j = kv + gvr[i], col = ((gvb[i] * 64 + lane) % VCPR) * 8;
        const void* src = gvm[i] == 2 ? (const void*)g_attn_ones
                          : gvm[i] != 1 || j >= a.Nk ? (const void*)g_attn_zero
                          : j < a.Np ? (const void*)(vpbase + (long)j * a.vp_sn + col)
                                     : (const void*)(vbase + (long)(j - a.Np) * a.v_sn + col);
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + KV_BLK * KROW + gvb[i] * 512), 16, 0, 0);
      }
      return;
    }
    // main-segment tile: the row offset is uniform (PFX: the kernel serves a prefix launch; the others
    // never see one and keep the prefix-free addressing and register budget)
    const int np = PFX ? a.Np : 0;
    const long ko = (long)(kv - np) * a.k_sn * 2, vo = (long)(kv - np) * a.v_sn * 2;   // bytes
    const bool full = kv + KV_BLK <= a.Nk;
#pragma unroll
    for (int i = 0; i < KBW; ++i) {
      const char* src = kb0[i] + (gkm[i] ? ko : 0);
      if (!full && kv + gkr[i] >= a.Nk) src = (const char*)g_attn_zero;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + (wave + 4 * i) * 512), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < VBW; ++i) {
      const char* src = vb0[i] + (gvm[i] == 1 ? vo : 0);
      if (!full && gvm[i] == 1 && kv + gvr[i] >= a.Nk) src = (const char*)g_attn_zero;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + KV_BLK * KROW + gvb[i] * 512), 16, 0, 0);
    }
  };

  // ---- S^T tiles of one 64-key tile: 4 key tiles x QT query tiles
  auto qk = [&](const bf16_t* cK, f32x4 (&st)[QT][4]) __attribute__((always_inline)) {
    float mi[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) mi[qt] = (PS && m_run[qt] != -INFINITY) ? -m_run[qt] : 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) st[qt][t] = (f32x4){mi[qt], mi[qt], mi[qt], mi[qt]};
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        const int krw = 16 * t + lq;
        const int kch = GLDS ? ((4 * s + g) ^ (krw & 7)) : (4 * s + g);
        const bf16x8 kf = __builtin_bit_cast(bf16x8, ld16(&cK[krw * KROW + kch * 8]));
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
          st[qt][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qt][s], st[qt][t], 0, 0, 0);
      }
    }
  };

  // ---- online softmax of one query tile (per query column = lane&15): P^T fragments, and the
  // running max / sum update; returns whether O needs the rescale by alpha (any lane)
  auto softmax = [&](int kv0, int qt, f32x4 (&st)[QT][4], bf16x8 (&pf)[QT][2],
                     float& alpha) __attribute__((always_inline)) {
    const bool full = !a.causal && kv0 + KV_BLK <= a.Nk;
    if (!full) {
      // key kv0 + 16t + 4g + r: compare the lane-invariant 4g against per-(t, r) uniform bounds, so
      // no per-element key index is built (hipcc hoisted those 16 v_or above the branch, onto
      // every full tile)
      const int lim = a.Nk - kv0;                                   // keys >= lim are padding
      const int qrel = a.causal ? qidx[qt] - kv0 : 0x7fffffff;       // keys > qrel are causal-masked
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool masked = g4 >= lim - (16 * t + r) || g4 > qrel - (16 * t + r);
          st[qt][t][r] = masked ? -INFINITY : st[qt][t][r];
        }
    }
    // row max: v_max3 chain (values are finite or -inf: same bits as the fmaxf tree)
    float mloc = vmax3(st[qt][0][0], st[qt][0][1], st[qt][0][2]);
    mloc = vmax3(mloc, st[qt][0][3], st[qt][1][0]);
    mloc = vmax3(mloc, st[qt][1][1], st[qt][1][2]);
    mloc = vmax3(mloc, st[qt][1][3], st[qt][2][0]);
    mloc = vmax3(mloc, st[qt][2][1], st[qt][2][2]);
    mloc = vmax3(mloc, st[qt][2][3], st[qt][3][0]);
    mloc = vmax3(mloc, st[qt][3][1], st[qt][3][2]);
    mloc = vmax2(mloc, st[qt][3][3]);
    mloc = mx16(mloc);
    mloc = mx32(mloc);
    // lazy rescale (T13): keep the running max unless it grew by > 8 (log2 units), so
    // p <= 2^8; the O/l rescale then runs only on the (rare) tiles where some lane needs it.
    if constexpr (PS) {
      // st = S' - m_use already (log2 units; m_use = 0 before the first finite max)
      const float m_old = m_run[qt];
      const float m_cand = (m_old == -INFINITY ? 0.f : m_old) + mloc;
      const bool need = m_cand > m_old + 8.f;
      alpha = 1.f;
      if (need) {
        alpha = (m_old == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m_old - m_cand);
        m_run[qt] = m_cand;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) st[qt][t][r] -= mloc;
      }
      float lsum = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          st[qt][t][r] = __builtin_amdgcn_exp2f(st[qt][t][r]);
          if (!ONES) lsum += st[qt][t][r];
        }
      if (!ONES) l_run[qt] = l_run[qt] * alpha + lsum;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 p;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          p[j] = (__bf16)st[qt][2 * ks][j];
          p[j + 4] = (__bf16)st[qt][2 * ks + 1][j];
        }
        pf[qt][ks] = p;
      }
      return __any(need);
    }
    const float m_cand = mloc * a.scale_log2;
    const bool need = m_cand > m_run[qt] + 8.f;
    alpha = 1.f;
    if (need) {
      alpha = (m_run[qt] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m_run[qt] - m_cand);
      m_run[qt] = m_cand;
    }
    const float m_use = (m_run[qt] == -INFINITY) ? 0.f : m_run[qt];
    if (ONES) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          st[qt][t][r] = __builtin_amdgcn_exp2f(fmaf(st[qt][t][r], a.scale_log2, -m_use));
    } else {
      float lsum = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __builtin_amdgcn_exp2f(fmaf(st[qt][t][r], a.scale_log2, -m_use));
          st[qt][t][r] = p;
          lsum += p;
        }
      l_run[qt] = l_run[qt] * alpha + lsum;
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 p;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        p[j] = (__bf16)st[qt][2 * ks][j];
        p[j + 4] = (__bf16)st[qt][2 * ks + 1][j];
      }
      pf[qt][ks] = p;
    }
    return __any(need);
  };

  // ---- O^T += V^T P^T  (A = V^T via transposing LDS reads)
  auto pv = [&](const bf16_t* cV, const bf16x8 (&pf)[QT][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int qq = (lane & 15) >> 2, pp = lane & 3;
        const bf16_t* a0 = &cV[(32 * ks + 4 * g + qq) * VROW + 16 * dt + 4 * pp];
        const bf16_t* a1 = a0 + 16 * VROW;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a1));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        s16x8 vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const bf16x8 vf = __builtin_bit_cast(bf16x8, vv);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
          o[qt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qt][ks], o[qt][dt], 0, 0, 0);
      }
    }
  };
  auto rescale = [&](int qt, float alpha) __attribute__((always_inline)) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[qt][dt] *= alpha;
  };

  // ---- ILP form of the prescaled (PS) online softmax, all query tiles of one key tile at once: bitwise
  // `softmax` + `rescale` per query tile, written so the query tiles' dependency chains interleave.  The
  // row max is a max3 tree (max is exact and order-free); every step runs over all query tiles before
  // the next; the lazy rescale is a wave-uniform branch per query tile with per-lane selects inside (a
  // lane that needs none subtracts 0: x - 0 == x bit for bit) - `softmax`'s divergent per-tile branches
  // cut the schedule into one serial chain per query tile (max -> lane swaps -> decision -> exp -> cvt).
  auto softmax_all = [&](int kv0, f32x4 (&st)[QT][4], bf16x8 (&pf)[QT][2]) __attribute__((always_inline)) {
    const bool full = !a.causal && kv0 + KV_BLK <= a.Nk;
    if (!full) {
      const int lim = a.Nk - kv0;
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        const int qrel = a.causal ? qidx[qt] - kv0 : 0x7fffffff;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool masked = g4 >= lim - (16 * t + r) || g4 > qrel - (16 * t + r);
            st[qt][t][r] = masked ? -INFINITY : st[qt][t][r];
          }
      }
    }
    float mloc[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      const f32x4* x = st[qt];
      const float a0 = vmax3(x[0][0], x[0][1], x[0][2]), a1 = vmax3(x[0][3], x[1][0], x[1][1]);
      const float a2 = vmax3(x[1][2], x[1][3], x[2][0]), a3 = vmax3(x[2][1], x[2][2], x[2][3]);
      const float a4 = vmax3(x[3][0], x[3][1], x[3][2]);
      mloc[qt] = vmax2(vmax3(a0, a1, a2), vmax3(a3, a4, x[3][3]));
    }
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) mloc[qt] = mx16(mloc[qt]);
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) mloc[qt] = mx32(mloc[qt]);
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      const float m_old = m_run[qt];
      const float m_cand = (m_old == -INFINITY ? 0.f : m_old) + mloc[qt];
      const bool need = m_cand > m_old + 8.f;
      float alpha = 1.f;
      const bool any = __any(need);
      if (any) {                                   // wave-uniform, rare (lazy rescale)
        const float al = (m_old == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m_old - m_cand);
        alpha = need ? al : 1.f;
        m_run[qt] = need ? m_cand : m_old;
        const float sub = need ? mloc[qt] : 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) st[qt][t][r] -= sub;
      }
      float lsum = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          st[qt][t][r] = __builtin_amdgcn_exp2f(st[qt][t][r]);
          if (!ONES) lsum += st[qt][t][r];
        }
      if (!ONES) l_run[qt] = l_run[qt] * alpha + lsum;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 p;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          p[j] = (__bf16)st[qt][2 * ks][j];
          p[j + 4] = (__bf16)st[qt][2 * ks + 1][j];
        }
        pf[qt][ks] = p;
      }
      if (any) rescale(qt, alpha);
    }
  };

  auto compute = [&](int kv0, const bf16_t* cK, const bf16_t* cV) __attribute__((always_inline)) {
    f32x4 st[QT][4];
    bf16x8 pf[QT][2];
    qk(cK, st);
    if constexpr (PS && ILP) {
      softmax_all(kv0, st, pf);
    } else {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        float alpha;
        if (softmax(kv0, qt, st, pf, alpha)) rescale(qt, alpha);
      }
    }
    pv(cV, pf);
  };

  if constexpr (GLDS && PP) {
    // Software-pipelined K / V rings (bitwise the same arithmetic on O as the plain loop: O sees
    // *alpha_j then +PV_j in the same order): iteration j runs QK(j) on K(j) while the MFMAs of
    // PV(j-1) on V(j-1) (from the previous iteration's P) keep the matrix core busy through the
    // softmax VALU of tile j.  V lags K by one tile: K(j+1) and V(j) are in flight during
    // iteration j, in the stage whose previous occupant was last read in iteration j-1 (K) / j-2
    // (V) - both retired by the barrier that opens iteration j.
    auto issue_k = [&](int kv, bf16_t* dst) __attribute__((always_inline)) {
      const long ko = (long)kv * a.k_sn;
#pragma unroll
      for (int i = 0; i < KBW; ++i) {
        const void* src = (gkm[i] && kv + gkr[i] < a.Nk) ? (const void*)(gk[i] + ko) : (const void*)g_attn_zero;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + (wave + 4 * i) * 512), 16, 0, 0);
      }
    };
    auto issue_v = [&](int kv, bf16_t* dst) __attribute__((always_inline)) {
      const long vo = (long)kv * a.v_sn;
#pragma unroll
      for (int i = 0; i < VBW; ++i) {
        const void* src = gvm[i] == 2 ? (const void*)g_attn_ones
                          : (gvm[i] == 1 && kv + gvr[i] < a.Nk) ? (const void*)(gv[i] + vo) : (const void*)g_attn_zero;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + KV_BLK * KROW + gvb[i] * 512), 16, 0, 0);
      }
    };
    bf16x8 pprev[QT][2];
    // one pipelined iteration on tile kv0 (stage roles static: CUR holds K(kv0), OTH holds V(kv0 - 64))
    auto step = [&](int kv0, bf16_t* cur, bf16_t* oth, bool first) __attribute__((always_inline)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (kv0 + KV_BLK < kv_end) issue_k(kv0 + KV_BLK, oth);
      issue_v(kv0, cur);
      f32x4 st[QT][4];
      bf16x8 pf[QT][2];
      qk(cur, st);
      if (!first) pv(oth + KV_BLK * KROW, pprev);
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        float alpha;
        if (softmax(kv0, qt, st, pf, alpha)) rescale(qt, alpha);
      }
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        pprev[qt][0] = pf[qt][0];
        pprev[qt][1] = pf[qt][1];
      }
    };
    if (kv_end > 0) {
      issue_k(0, sS0);
      int kv0 = 0;
      step(0, sS0, sS1, true);
      for (kv0 = KV_BLK; kv0 + KV_BLK < kv_end; kv0 += 2 * KV_BLK) {
        step(kv0, sS1, sS0, false);
        step(kv0 + KV_BLK, sS0, sS1, false);
      }
      // tail: at most one more K tile, then the last tile's PV (its V went to the stage of its K)
      bf16_t* vlast = sS0;
      if (kv0 < kv_end) {
        step(kv0, sS1, sS0, false);
        vlast = sS1;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      pv(vlast + KV_BLK * KROW, pprev);
    }
  } else if constexpr (GLDS) {
    // stage roles are static (loop unrolled by 2): DMA into one stage while the other is read;
    // a stage is refilled only after the barrier that retired its last reads
    if (kv_end > 0) issue_kv(0, sS0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kv0 = 0; kv0 < kv_end; kv0 += 2 * KV_BLK) {
      const int kv1 = kv0 + KV_BLK;
      if (kv1 < kv_end) issue_kv(kv1, sS1);
      compute(kv0, sS0, sS0 + KV_BLK * KROW);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (kv1 >= kv_end) break;
      if (kv1 + KV_BLK < kv_end) issue_kv(kv1 + KV_BLK, sS0);
      compute(kv1, sS1, sS1 + KV_BLK * KROW);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    if (kv_end > 0) {
      load_kv(0);
      store_kv(0);
    }
    __syncthreads();
    int buf = 0;
    for (int kv0 = 0; kv0 < kv_end; kv0 += KV_BLK, buf ^= 1) {
      const bool more = kv0 + KV_BLK < kv_end;
      if (more) load_kv(kv0 + KV_BLK);
      const bf16_t* cS = buf ? sS1 : sS0;
      compute(kv0, cS, cS + KV_BLK * KROW);
      // the prefetched tile goes to the other buffer (last read one iteration ago, fenced by
      // the previous barrier); this barrier publishes it and retires reads of `buf`.
      if (more) store_kv(buf ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue: denominator (MFMA ones-column or lane sums), normalise, store O[q][d]
  bf16_t* obase = a.o + b * a.o_sb + h * a.o_sh;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    float l;
    if (ONES) {
      // O^T row D lives in d-tile D/16, lane group (D%16)/4, register (D%4) = 0 (D % 8 == 0)
      const int dtl = D >> 4;
      float cand = 0.f;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        if (dt == dtl) cand = o[qt][dt][0];
      l = __shfl(cand, ((D & 15) >> 2) * 16 + lq, 64);
    } else {
      l = l_run[qt];
      l = SWAPS ? sum_xor16(l) : l + __shfl_xor(l, 16, 64);
      l = SWAPS ? sum_xor32(l) : l + __shfl_xor(l, 32, 64);
    }
    const float inv = l > 0.f ? 1.f / l : 0.f;
    if (qidx[qt] < a.Nq) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int d = 16 * dt + 4 * g;
        if (d < D) {
          uint2 w;
          w.x = (uint32_t)f2bf(o[qt][dt][0] * inv) | ((uint32_t)f2bf(o[qt][dt][1] * inv) << 16);
          w.y = (uint32_t)f2bf(o[qt][dt][2] * inv) | ((uint32_t)f2bf(o[qt][dt][3] * inv) << 16);
          *reinterpret_cast<uint2*>(obase + (long)qidx[qt] * a.o_sn + d) = w;
        }
      }
    }
  }
}

static int g_attn_glds = -1;
static bool attn_glds_enabled() {
  if (g_attn_glds < 0) {
    const char* e = std::getenv("ARB_ATTN_GLDS");
    g_attn_glds = (e == nullptr || e[0] != '0') ? 1 : 0;
  }
  return g_attn_glds == 1;
}
// register-staged K/V (0) vs LDS-DMA (1, default): bitwise-equal paths (test hook / A/B)
ARB_API void arb_set_attn_glds(int on) { g_attn_glds = on ? 1 : 0; }

// A/B switch (bitwise-equal paths): ARB_ATTN_PP=1 runs the software-pipelined K / V ring (PV of
// tile j-1 overlapped with QK and softmax of tile j) on the LDS-DMA kernels
static int g_attn_pp = -1;
static bool attn_pp_enabled() {
  if (g_attn_pp < 0) {
    const char* e = std::getenv("ARB_ATTN_PP");
    g_attn_pp = (e != nullptr && e[0] == '1') ? 1 : 0;
  }
  return g_attn_pp == 1;
}
ARB_API void arb_set_attn_pp(int on) { g_attn_pp = on ? 1 : 0; }
// PS (prescaled-Q softmax, default): Q is scaled by scale * log2(e) once (bf16) and every S^T MFMA
// chain starts from -m_run, so the accumulators leave the matrix core as exp2 arguments - one VALU
// op less per score (the fma of the raw-score form).  ARB_ATTN_PRESCALE=0 / arb_set_attn_prescale(0):
// the raw-score form (different bytes: Q rounds to bf16 after the scale).
static int g_attn_prescale = -1;
static bool attn_prescale_enabled() {
  if (g_attn_prescale < 0) {
    const char* e = std::getenv("ARB_ATTN_PRESCALE");
    g_attn_prescale = (e != nullptr && e[0] == '0') ? 0 : 1;
  }
  return g_attn_prescale == 1;
}
ARB_API void arb_set_attn_prescale(int on) { g_attn_prescale = on ? 1 : 0; }

// ARB_ATTN_ILP=0 / arb_set_attn_ilp(0): the per-query-tile softmax instead of softmax_all (bitwise equal:
// the A/B of the ILP form, and its bitwise test)
static int g_attn_ilp = -1;
static bool attn_ilp_enabled() {
  if (g_attn_ilp < 0) {
    const char* e = std::getenv("ARB_ATTN_ILP");
    g_attn_ilp = (e != nullptr && e[0] == '0') ? 0 : 1;
  }
  return g_attn_ilp == 1;
}
ARB_API void arb_set_attn_ilp(int on) { g_attn_ilp = on ? 1 : 0; }

template <int KSTEPS, int DT, int QT, bool PS>
static void launch_fa_ps(const AttnArgs& a, hipStream_t s) {
  constexpr int QBLK = 4 * QT * 16;
  const int nqb = (a.Nq + QBLK - 1) / QBLK;
  dim3 grid(nqb * a.H * a.B);
  if constexpr (KSTEPS == 2) {
    if (attn_glds_enabled()) {     // LDS-DMA staging (a K/V prefix segment included)
      // pipelined variants that fit the 256-VGPR budget of two waves per SIMD without spilling
      // (the 4-q-tile d = 48 / 64 ones carry two S tile sets + P(j-1) past it); no prefix
      if constexpr (PS && (QT <= 2 || DT == 3)) {
        if (a.Np == 0 && attn_pp_enabled() && (QT <= 2 || (a.D & 15))) {
          if (a.D & 15) flash_attn_fwd_kernel<KSTEPS, DT, QT, true, true, true, PS><<<grid, 256, 0, s>>>(a);
          else if constexpr (QT <= 2)
            flash_attn_fwd_kernel<KSTEPS, DT, QT, false, true, true, PS><<<grid, 256, 0, s>>>(a);
          return;
        }
      }
      if constexpr (QT <= 2) {   // K/V prefix segment (joint attention; never a 4-q-tile launch)
        if (a.Np > 0) {
          if (a.D & 15)
            flash_attn_fwd_kernel<KSTEPS, DT, QT, true, true, false, PS, true, true><<<grid, 256, 0, s>>>(a);
          else
            flash_attn_fwd_kernel<KSTEPS, DT, QT, false, true, false, PS, true, true><<<grid, 256, 0, s>>>(a);
          return;
        }
      }
      if (PS && !attn_ilp_enabled()) {
        if (a.D & 15) flash_attn_fwd_kernel<KSTEPS, DT, QT, true, true, false, PS, false><<<grid, 256, 0, s>>>(a);
        else flash_attn_fwd_kernel<KSTEPS, DT, QT, false, true, false, PS, false><<<grid, 256, 0, s>>>(a);
        return;
      }
      if (a.D & 15) flash_attn_fwd_kernel<KSTEPS, DT, QT, true, true, false, PS><<<grid, 256, 0, s>>>(a);
      else flash_attn_fwd_kernel<KSTEPS, DT, QT, false, true, false, PS><<<grid, 256, 0, s>>>(a);
      return;
    }
  }
  if (a.D & 15) flash_attn_fwd_kernel<KSTEPS, DT, QT, true, false, false, PS><<<grid, 256, 0, s>>>(a);
  else flash_attn_fwd_kernel<KSTEPS, DT, QT, false, false, false, PS><<<grid, 256, 0, s>>>(a);
}

template <int KSTEPS, int DT, int QT>
static void launch_fa(const AttnArgs& a, hipStream_t s) {
  if (attn_prescale_enabled()) launch_fa_ps<KSTEPS, DT, QT, true>(a, s);
  else launch_fa_ps<KSTEPS, DT, QT, false>(a, s);
}

// kp/vp (may be null): prefix K/V segment of Np keys with strides pstrides = {kp_sb, kp_sn, vp_sb, vp_sn}
// (head stride shared with k/v); Nk counts prefix + main keys.
ARB_API int arb_flash_attention(const void* q, const void* k, const void* v, void* o, const long* strides, int B,
                                int H, int Nq, int Nk, int D, float scale, int causal, const void* kp,
                                const void* vp, const long* pstrides, int Np, hipStream_t stream) {
  if (D % 8 != 0 || D > 160 || (Np > 0 && (kp == nullptr || vp == nullptr || causal))) return -1;
  AttnArgs a;
  a.kp = (const bf16_t*)kp;
  a.vp = (const bf16_t*)vp;
  a.Np = Np;
  a.kp_sb = Np ? pstrides[0] : 0; a.kp_sn = Np ? pstrides[1] : 0;
  a.vp_sb = Np ? pstrides[2] : 0; a.vp_sn = Np ? pstrides[3] : 0;
  a.q = (const bf16_t*)q;
  a.k = (const bf16_t*)k;
  a.v = (const bf16_t*)v;
  a.o = (bf16_t*)o;
  a.q_sb = strides[0]; a.q_sn = strides[1]; a.q_sh = strides[2];
  a.k_sb = strides[3]; a.k_sn = strides[4]; a.k_sh = strides[5];
  a.v_sb = strides[6]; a.v_sn = strides[7]; a.v_sh = strides[8];
  a.o_sb = strides[9]; a.o_sn = strides[10]; a.o_sh = strides[11];
  a.B = B; a.H = H; a.Nq = Nq; a.Nk = Nk; a.D = D;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.causal = causal;
  const int ks = (D + 31) / 32, dt = (D + 15) / 16;
  // Small query counts: 1 q-tile per wave keeps more workgroups in flight.  Large ones (>= 1024
  // workgroups even at 4 q-tiles per wave, e.g. the batched SD level-0 self-attention): 4 q-tiles
  // per wave halve the K/V fragment LDS reads per query (LDS bandwidth is the shared limit).
  const long rows = (long)B * H * Nq;
  const bool small = rows < 256L * 128;
  static const int qt_env = [] {
    const char* e = std::getenv("ARB_ATTN_QT");
    return e ? std::atoi(e) : 0;
  }();
  const bool wide = Np == 0 && (qt_env == 4 || (qt_env == 0 && rows >= 256L * 1024));
#define FA_CASE(KS, DTT)                                  \
  if (ks == KS && dt == DTT) {                            \
    if (small) launch_fa<KS, DTT, 1>(a, stream);          \
    else launch_fa<KS, DTT, 2>(a, stream);                \
    return (int)hipGetLastError();                        \
  }
#define FA_CASE4(KS, DTT)                                 \
  if (ks == KS && dt == DTT) {                            \
    if (small) launch_fa<KS, DTT, 1>(a, stream);          \
    else if (wide) launch_fa<KS, DTT, 4>(a, stream);      \
    else launch_fa<KS, DTT, 2>(a, stream);                \
    return (int)hipGetLastError();                        \
  }
  FA_CASE(1, 1) FA_CASE(1, 2)
  FA_CASE4(2, 3) FA_CASE4(2, 4)
  FA_CASE(3, 5) FA_CASE(3, 6)
  FA_CASE(4, 7) FA_CASE(4, 8)
  FA_CASE(5, 9) FA_CASE(5, 10)
#undef FA_CASE
#undef FA_CASE4
  return -2;
}
