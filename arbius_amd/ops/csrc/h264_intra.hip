// H.264 avc-intra encoder on the GPU: the same bytes as native/src/h264.cpp encode_idr (one IDR
// slice per picture, Intra_16x16 + chroma modes by SAD, dead-zone quantisation at a fixed QP,
// CAVLC, deblocking off), so a video task's MP4 (robust_video_matting out-1.mp4,
// /root/reference/templates/robust_video_matting.json:1-31) no longer costs ~17 ms of host CPU per
// 1080p frame.  The host keeps only emulation prevention and the MP4 mux.
//
// Work split (one launch each, all on the caller's stream):
//   analyse  one workgroup per picture walks the macroblock anti-diagonals (mx + my = d): an
//            Intra_16x16 macroblock reads only its left / top / top-left neighbours' reconstruction,
//            so every macroblock of a diagonal is independent.  One lane per macroblock runs the
//            encoder's decisions (mode SADs, forward transform, quantisation, reconstruction);
//            levels, modes and TotalCoeff go to a workspace.
//   count    one lane per macroblock (all pictures at once): its CAVLC bits.
//   scan     one workgroup per picture: exclusive prefix of the macroblock bit counts after the
//            slice header -> each macroblock's bit offset and the picture's RBSP length.
//   frames   one wave: byte offset of every picture in the output (4-byte aligned), capacity check,
//            the slice header bits and the rbsp stop bit.
//   zero     clears the used output bytes;  write: one lane per macroblock writes its CAVLC bits at
//            its offset (whole 32-bit words with plain stores, the two boundary words with atomicOr:
//            the result is an OR of disjoint bit ranges, so it does not depend on lane order).
//
// The per-macroblock code is __host__ __device__: arb_h264_intra_host runs the identical functions
// on the CPU in raster order (tests/test_h264_gpu_algo.py compares its NALs with the native
// encoder on a machine without a GPU); the GPU path is checked against the native encoder by
// tests/test_h264_gpu.py.  Integer arithmetic only: nothing here depends on evaluation order.
#include "common.h"

#include <algorithm>
#include <cstring>
#include <vector>

#define HD __host__ __device__

namespace h264g {

// ---- tables (ITU-T H.264 9.2, 8.5; the values native/src/h264.cpp encodes with)
constexpr uint8_t kCoeffTokenLen[4][68] = {
    {1, 0, 0, 0, 6, 2, 0, 0, 8, 6, 3, 0, 9, 8, 7, 5, 10, 9, 8, 6, 11, 10, 9, 7, 13, 11, 10, 8,
     13, 13, 11, 9, 13, 13, 13, 10, 14, 14, 13, 11, 14, 14, 14, 13, 15, 15, 14, 14, 15, 15, 15, 14,
     16, 15, 15, 15, 16, 16, 16, 15, 16, 16, 16, 16, 16, 16, 16, 16},
    {2, 0, 0, 0, 6, 2, 0, 0, 6, 5, 3, 0, 7, 6, 6, 4, 8, 6, 6, 4, 8, 7, 7, 5, 9, 8, 8, 6,
     11, 9, 9, 6, 11, 11, 11, 7, 12, 11, 11, 9, 12, 12, 12, 11, 12, 12, 12, 11, 13, 13, 13, 12,
     13, 13, 13, 13, 13, 14, 13, 13, 14, 14, 14, 13, 14, 14, 14, 14},
    {4, 0, 0, 0, 6, 4, 0, 0, 6, 5, 4, 0, 6, 5, 5, 4, 7, 5, 5, 4, 7, 5, 5, 4, 7, 6, 6, 4,
     7, 6, 6, 4, 8, 7, 7, 5, 8, 8, 7, 6, 9, 8, 8, 7, 9, 9, 8, 8, 9, 9, 9, 8,
     10, 9, 9, 9, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10},
    {6, 0, 0, 0, 6, 6, 0, 0, 6, 6, 6, 0, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6,
     6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6,
     6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6},
};
constexpr uint8_t kCoeffTokenBits[4][68] = {
    {1, 0, 0, 0, 5, 1, 0, 0, 7, 4, 1, 0, 7, 6, 5, 3, 7, 6, 5, 3, 7, 6, 5, 4, 15, 6, 5, 4,
     11, 14, 5, 4, 8, 10, 13, 4, 15, 14, 9, 4, 11, 10, 13, 12, 15, 14, 9, 12, 11, 10, 13, 8,
     15, 1, 9, 12, 11, 14, 13, 8, 7, 10, 9, 12, 4, 6, 5, 8},
    {3, 0, 0, 0, 11, 2, 0, 0, 7, 7, 3, 0, 7, 10, 9, 5, 7, 6, 5, 4, 4, 6, 5, 6, 7, 6, 5, 8,
     15, 6, 5, 4, 11, 14, 13, 4, 15, 10, 9, 4, 11, 14, 13, 12, 8, 10, 9, 8, 15, 14, 13, 12,
     11, 10, 9, 12, 7, 11, 6, 8, 9, 8, 10, 1, 7, 6, 5, 4},
    {15, 0, 0, 0, 15, 14, 0, 0, 11, 15, 13, 0, 8, 12, 14, 12, 15, 10, 11, 11, 11, 8, 9, 10, 9, 14, 13, 9,
     8, 10, 9, 8, 15, 14, 13, 13, 11, 14, 10, 12, 15, 10, 13, 12, 11, 14, 9, 12, 8, 10, 13, 8,
     13, 7, 9, 12, 9, 12, 11, 10, 5, 8, 7, 6, 1, 4, 3, 2},
    {3, 0, 0, 0, 0, 1, 0, 0, 4, 5, 6, 0, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23,
     24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47,
     48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63},
};
constexpr uint8_t kChromaDcTokenLen[20] = {2, 0, 0, 0, 6, 1, 0, 0, 6, 6, 3, 0, 6, 7, 7, 6, 6, 8, 8, 7};
constexpr uint8_t kChromaDcTokenBits[20] = {1, 0, 0, 0, 7, 1, 0, 0, 4, 6, 1, 0, 3, 3, 2, 5, 2, 3, 2, 0};
constexpr uint8_t kTotalZerosLen[15][16] = {
    {1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9}, {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6},
    {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6},       {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5},
    {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5},             {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6},
    {6, 5, 3, 3, 3, 2, 3, 4, 3, 6},                   {6, 4, 5, 3, 2, 2, 3, 3, 6},
    {6, 6, 4, 2, 2, 3, 2, 5},                         {5, 5, 3, 2, 2, 2, 4},
    {4, 4, 3, 3, 1, 3},                               {4, 4, 2, 1, 3},
    {3, 3, 1, 2},                                     {2, 2, 1},
    {1, 1},
};
constexpr uint8_t kTotalZerosBits[15][16] = {
    {1, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 1}, {7, 6, 5, 4, 3, 5, 4, 3, 2, 3, 2, 3, 2, 1, 0},
    {5, 7, 6, 5, 4, 3, 4, 3, 2, 3, 2, 1, 1, 0},       {3, 7, 5, 4, 6, 5, 4, 3, 3, 2, 2, 1, 0},
    {5, 4, 3, 7, 6, 5, 4, 3, 2, 1, 1, 0},             {1, 1, 7, 6, 5, 4, 3, 2, 1, 1, 0},
    {1, 1, 5, 4, 3, 3, 2, 1, 1, 0},                   {1, 1, 1, 3, 3, 2, 2, 1, 0},
    {1, 0, 1, 3, 2, 1, 1, 1},                         {1, 0, 1, 3, 2, 1, 1},
    {0, 1, 1, 2, 1, 3},                               {0, 1, 1, 1, 1},
    {0, 1, 1, 1},                                     {0, 1, 1},
    {0, 1},
};
constexpr uint8_t kChromaDcTotalZerosLen[3][4] = {{1, 2, 3, 3}, {1, 2, 2, 0}, {1, 1, 0, 0}};
constexpr uint8_t kChromaDcTotalZerosBits[3][4] = {{1, 1, 1, 0}, {1, 1, 0, 0}, {1, 0, 0, 0}};
constexpr uint8_t kRunLen[7][15] = {
    {1, 1}, {1, 2, 2}, {2, 2, 2, 2}, {2, 2, 2, 3, 3}, {2, 2, 3, 3, 3, 3}, {2, 3, 3, 3, 3, 3, 3},
    {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11},
};
constexpr uint8_t kRunBits[7][15] = {
    {1, 0}, {1, 1, 0}, {3, 2, 1, 0}, {3, 2, 1, 1, 0}, {3, 2, 3, 2, 1, 0}, {3, 0, 1, 3, 2, 5, 4},
    {7, 6, 5, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1},
};
constexpr uint8_t kZigzag[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
constexpr uint8_t kBlkX[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
constexpr uint8_t kBlkY[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};
constexpr int kV[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
constexpr int kMF[6][3] = {{13107, 5243, 8066}, {11916, 4660, 7490}, {10082, 4194, 6554},
                           {9362, 3647, 5825},  {8192, 3355, 5243}, {7282, 2893, 4559}};
constexpr uint8_t kChromaQp[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
                                   18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33,
                                   34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};

constexpr int kLevels = 384;   // per macroblock: luma DC 16 | luma AC 16 x 15 | chroma DC 2 x 4 | chroma AC 2 x 4 x 15
constexpr int kLvAc = 16, kLvCdc = 256, kLvCac = 264;

HD inline int pos_class(int r) {
  const int i = r >> 2, j = r & 3;
  return ((i & 1) == 0 && (j & 1) == 0) ? 0 : ((i & 1) && (j & 1)) ? 1 : 2;
}
HD inline int clip255(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }
// clip255(v >> 5) as clamp-then-shift (the same integer for every v).  The shift-then-clamp form,
// packed 4 samples per dword, is selected into gfx950 v_ashr_pk_u8_i32 by hipcc (ROCm 7.2) at -O1
// and above, and that sequence produced wrong plane-prediction samples on the device (one sample of
// a chroma block in tests/test_h264_gpu.py's smooth case; -O0, which emits none, matched the native
// encoder): scripts/h264_debug.py, gpurun_out/r6h264dbg.
HD inline int plane_px(int v) { return (v < 0 ? 0 : v > 8191 ? 8191 : v) >> 5; }
HD inline int sat16(int v) { return v < -32768 ? -32768 : v > 32767 ? 32767 : v; }
HD inline int quant(int w, int mf, int f, int qbits) {
  const int a = w < 0 ? -w : w;
  int z = (a * mf + f) >> qbits;
  z = z < 2047 ? z : 2047;
  return w < 0 ? -z : z;
}
HD inline int clz32(uint32_t x) { return __builtin_clz(x); }
HD inline uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

HD inline void fwd4x4(const int* x, int* out) {
  int t[16];
  for (int i = 0; i < 4; ++i) {
    const int* r = x + 4 * i;
    const int s03 = r[0] + r[3], d03 = r[0] - r[3], s12 = r[1] + r[2], d12 = r[1] - r[2];
    t[4 * i + 0] = s03 + s12;
    t[4 * i + 1] = 2 * d03 + d12;
    t[4 * i + 2] = s03 - s12;
    t[4 * i + 3] = d03 - 2 * d12;
  }
  for (int j = 0; j < 4; ++j) {
    const int s03 = t[j] + t[12 + j], d03 = t[j] - t[12 + j], s12 = t[4 + j] + t[8 + j], d12 = t[4 + j] - t[8 + j];
    out[j] = s03 + s12;
    out[4 + j] = 2 * d03 + d12;
    out[8 + j] = s03 - s12;
    out[12 + j] = d03 - 2 * d12;
  }
}

HD inline void inv4x4(const int* d, int* r) {
  int f[16];
  for (int i = 0; i < 4; ++i) {
    const int* x = d + 4 * i;
    const int e0 = x[0] + x[2], e1 = x[0] - x[2], e2 = (x[1] >> 1) - x[3], e3 = x[1] + (x[3] >> 1);
    f[4 * i + 0] = e0 + e3;
    f[4 * i + 1] = e1 + e2;
    f[4 * i + 2] = e1 - e2;
    f[4 * i + 3] = e0 - e3;
  }
  for (int j = 0; j < 4; ++j) {
    const int g0 = f[j] + f[8 + j], g1 = f[j] - f[8 + j];
    const int g2 = (f[4 + j] >> 1) - f[12 + j], g3 = f[4 + j] + (f[12 + j] >> 1);
    r[j] = (g0 + g3 + 32) >> 6;
    r[4 + j] = (g1 + g2 + 32) >> 6;
    r[8 + j] = (g1 - g2 + 32) >> 6;
    r[12 + j] = (g0 - g3 + 32) >> 6;
  }
}

HD inline void hadamard4(const int* c, int* f) {
  int t[16];
  for (int i = 0; i < 4; ++i) {
    const int* x = c + 4 * i;
    t[4 * i + 0] = x[0] + x[1] + x[2] + x[3];
    t[4 * i + 1] = x[0] + x[1] - x[2] - x[3];
    t[4 * i + 2] = x[0] - x[1] - x[2] + x[3];
    t[4 * i + 3] = x[0] - x[1] + x[2] - x[3];
  }
  for (int j = 0; j < 4; ++j) {
    f[j] = t[j] + t[4 + j] + t[8 + j] + t[12 + j];
    f[4 + j] = t[j] + t[4 + j] - t[8 + j] - t[12 + j];
    f[8 + j] = t[j] - t[4 + j] - t[8 + j] + t[12 + j];
    f[12 + j] = t[j] - t[4 + j] + t[8 + j] - t[12 + j];
  }
}

// AC dequantisation of one QP: (c * mul[class] + add) >> sh (native AcDequant, per position class)
struct Dq {
  int mul[3], add, sh;
  HD explicit Dq(int qp) {
    const int q6 = qp / 6;
    for (int k = 0; k < 3; ++k) mul[k] = qp >= 24 ? 16 * kV[qp % 6][k] * (1 << (q6 - 4)) : 16 * kV[qp % 6][k];
    add = qp >= 24 ? 0 : 1 << (3 - q6);
    sh = qp >= 24 ? 0 : 4 - q6;
  }
  HD int operator()(int c, int r) const { return (c * mul[pos_class(r)] + add) >> sh; }
};

// One picture's planes and the encoder state the kernels share (device or host pointers).
struct Pic {
  const uint8_t* sy;
  const uint8_t* sc[2];
  uint8_t* ry;             // reconstruction (what a decoder outputs; neighbours predict from it)
  uint8_t* rc[2];
  uint8_t* tcy;            // TotalCoeff per 4x4 luma block [4 mbh][4 mbw] (CAVLC nC)
  uint8_t* tcc[2];         // per 4x4 chroma block [2 mbh][2 mbw]
  int16_t* lv;             // levels, kLevels per macroblock
  uint32_t* info;          // per macroblock: mode | cmode << 2 | cbp_chroma << 4 | cbp_luma != 0 << 6
  uint32_t* bits;          // per macroblock: CAVLC bits (analyse), then bit offset in the RBSP (scan)
  int W, mbw, mbh, qp;
};

HD inline uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }   // 4-byte aligned
// Per-lane work arrays (source and prediction samples, 4 per dword): on the GPU in LDS,
// lane-interleaved (element j of lane t at j * stride + t: the unrolled code touches one j on every
// lane at once -> consecutive banks), which keeps the analyse kernel's live registers small; on the
// host a local array (stride 1).
struct WBuf {
  uint32_t* p;
  int stride;
  HD uint32_t& operator[](int j) const { return p[j * stride]; }
  HD WBuf at(int off) const { return WBuf{p + off * stride, stride}; }
};
constexpr int kWork = 192;   // dwords per lane: luma src 64 | luma pred 64 | Cb, Cr src 16 + 16 | Cb, Cr pred 16 + 16
HD inline int byte_of(const WBuf& s, int i) { return int((s[i >> 2] >> (8 * (i & 3))) & 255u); }

// Intra_16x16 prediction sample (8.3.3): mode 0 V, 1 H, 2 DC, 3 plane
struct Pred16 {
  int top[16], left[16], dc, a, b, c;
  HD int at(int mode, int x, int y) const {
    if (mode == 0) return top[x];
    if (mode == 1) return left[y];
    if (mode == 2) return dc;
    return plane_px(a + b * (x - 7) + c * (y - 7) + 16);
  }
};
// Intra chroma 8x8 prediction sample (8.3.4): mode 0 DC (per 4x4 quadrant), 1 H, 2 V, 3 plane
struct PredC {
  int top[8], left[8], dcq[4], a, b, c;
  HD int at(int mode, int x, int y) const {
    if (mode == 0) return dcq[(y >> 2) * 2 + (x >> 2)];
    if (mode == 1) return left[y];
    if (mode == 2) return top[x];
    return plane_px(a + b * (x - 3) + c * (y - 3) + 16);
  }
};

// the chosen prediction packed 4 samples per dword (one divergent section per macroblock instead of
// a mode branch per sample), and the SAD of a source block against one mode
template <int M>
HD inline void fill16(const Pred16& P, const WBuf& pr) {
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) v |= uint32_t(P.at(M, (4 * i + k) & 15, (4 * i + k) >> 4)) << (8 * k);
    pr[i] = v;
  }
}
template <int M>
HD inline int sad16(const WBuf& s, const Pred16& P) {
  int sad = 0;
#pragma unroll
  for (int i = 0; i < 256; ++i) {
    const int d = byte_of(s, i) - P.at(M, i & 15, i >> 4);
    sad += d < 0 ? -d : d;
  }
  return sad;
}
template <int M>
HD inline void fillc(const PredC& Q, const WBuf& pr) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) v |= uint32_t(Q.at(M, (4 * i + k) & 7, (4 * i + k) >> 3)) << (8 * k);
    pr[i] = v;
  }
}
template <int M>
HD inline int sadc(const WBuf& s, const PredC& Q) {
  int sad = 0;
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const int d = byte_of(s, i) - Q.at(M, i & 7, i >> 3);
    sad += d < 0 ? -d : d;
  }
  return sad;
}

// ---- the per-macroblock decisions, levels and reconstruction (native encode_mb)
HD inline void analyse_mb(const Pic& p, int mx, int my, const WBuf& wk, uint32_t* dbg = nullptr) {
  const int W = p.W, Wc = W / 2, mb = my * p.mbw + mx;
  const bool L = mx > 0, T = my > 0, TL = L && T;
  const int x0 = 16 * mx, y0 = 16 * my;
  int16_t* lv = p.lv + (size_t)mb * kLevels;

  // ---- luma: neighbours and the 4 candidate predictions
  Pred16 P;
  int tl = 0;
  for (int i = 0; i < 16; ++i) {
    P.top[i] = T ? p.ry[(size_t)(y0 - 1) * W + x0 + i] : 0;
    P.left[i] = L ? p.ry[(size_t)(y0 + i) * W + x0 - 1] : 0;
  }
  if (TL) tl = p.ry[(size_t)(y0 - 1) * W + x0 - 1];
  {
    int st = 0, sl = 0;
    for (int i = 0; i < 16; ++i) {
      st += P.top[i];
      sl += P.left[i];
    }
    P.dc = (L && T) ? (st + sl + 16) >> 5 : L ? (sl + 8) >> 4 : T ? (st + 8) >> 4 : 128;
    int H = 0, V = 0;
    for (int i = 0; i < 8; ++i) {
      const int t0 = P.top[8 + i], t1 = 6 - i < 0 ? tl : P.top[6 - i];
      const int l0 = P.left[8 + i], l1 = 6 - i < 0 ? tl : P.left[6 - i];
      H += (i + 1) * (t0 - t1);
      V += (i + 1) * (l0 - l1);
    }
    P.a = 16 * (P.left[15] + P.top[15]);
    P.b = (5 * H + 32) >> 6;
    P.c = (5 * V + 32) >> 6;
  }
  const WBuf s = wk;   // source macroblock, 16 rows x 16 bytes
  for (int y = 0; y < 16; ++y)
    for (int k = 0; k < 4; ++k) s[4 * y + k] = ld32(p.sy + (size_t)(y0 + y) * W + x0 + 4 * k);
  // candidates in mode order, ties to the lowest mode
  int mode = 2, best = 1 << 30;
  if (T) {
    best = sad16<0>(s, P);
    mode = 0;
  }
  if (L) {
    const int v = sad16<1>(s, P);
    if (v < best) { best = v; mode = 1; }
  }
  {
    const int v = sad16<2>(s, P);
    if (v < best) { best = v; mode = 2; }
  }
  if (TL) {
    const int v = sad16<3>(s, P);
    if (v < best) { best = v; mode = 3; }
  }
  const WBuf pr = wk.at(64);
  if (mode == 0) fill16<0>(P, pr);
  else if (mode == 1) fill16<1>(P, pr);
  else if (mode == 2) fill16<2>(P, pr);
  else fill16<3>(P, pr);

  // ---- luma levels: AC per block now, the DC after the Hadamard of all 16 block DCs
  const int qp = p.qp, qp6 = qp % 6, qbits = 15 + qp / 6, fq = (1 << qbits) / 3;
  int dcm[16];
  int any_ac = 0;
#pragma unroll
  for (int blk = 0; blk < 16; ++blk) {
    const int bx = kBlkX[blk], by = kBlkY[blk];
    int res[16], w4[16];
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int i = 16 * (4 * by + y) + 4 * bx + x;
        res[4 * y + x] = byte_of(s, i) - byte_of(pr, i);
      }
    fwd4x4(res, w4);
    dcm[4 * by + bx] = w4[0];
    int tc = 0;
#pragma unroll
    for (int k = 0; k < 15; ++k) {
      const int r = kZigzag[k + 1];
      const int q = quant(w4[r], kMF[qp6][pos_class(r)], fq, qbits);
      lv[kLvAc + 15 * blk + k] = (int16_t)q;
      tc += q != 0;
    }
    p.tcy[(size_t)(4 * my + by) * 4 * p.mbw + 4 * mx + bx] = (uint8_t)tc;
    any_ac |= tc;
  }
  int hd[16], dc[16];
  hadamard4(dcm, hd);
  for (int k = 0; k < 16; ++k) {
    dc[k] = quant(hd[kZigzag[k]] / 2, kMF[qp6][0], 2 * fq, qbits + 1);
    lv[k] = (int16_t)dc[k];
  }

  // ---- luma reconstruction (native recon_luma16)
  {
    int c[16], fdc[16];
    for (int k = 0; k < 16; ++k) c[kZigzag[k]] = dc[k];
    hadamard4(c, fdc);
    const int ls = 16 * kV[qp6][0];
    const Dq dq(qp);
#pragma unroll
    for (int blk = 0; blk < 16; ++blk) {
      const int bx = kBlkX[blk], by = kBlkY[blk];
      const int fv = fdc[4 * by + bx];
      int d[16];
      for (int k = 0; k < 16; ++k) d[k] = 0;
      d[0] = qp >= 36 ? fv * ls * (1 << (qp / 6 - 6)) : (fv * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
      int any = 0;
      for (int k = 0; k < 15; ++k) {
        const int r = kZigzag[k + 1];
        const int q = lv[kLvAc + 15 * blk + k];
        d[r] = dq(q, r);
        any |= q;
      }
      int r16[16];
      if (any) {
        inv4x4(d, r16);
      } else {
        const int v = (d[0] + 32) >> 6;
        for (int k = 0; k < 16; ++k) r16[k] = v;
      }
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const int yy = 4 * by + y;
        uint32_t v = 0;
#pragma unroll
        for (int x = 0; x < 4; ++x)
          v |= uint32_t(clip255(byte_of(pr, 16 * yy + 4 * bx + x) + sat16(r16[4 * y + x]))) << (8 * x);
        *reinterpret_cast<uint32_t*>(p.ry + (size_t)(y0 + yy) * W + x0 + 4 * bx) = v;
      }
    }
  }

  // ---- chroma: one mode for both components by the summed SAD
  const int qpc = kChromaQp[qp], qc6 = qpc % 6, qcbits = 15 + qpc / 6, fqc = (1 << qcbits) / 3;
  const int cx0 = 8 * mx, cy0 = 8 * my;
  PredC C[2];
  const WBuf sc[2] = {wk.at(128), wk.at(144)};
  #pragma unroll
  for (int c = 0; c < 2; ++c) {
    PredC& Q = C[c];
    const uint8_t* r = p.rc[c];
    int ctl = 0;
    for (int i = 0; i < 8; ++i) {
      Q.top[i] = T ? r[(size_t)(cy0 - 1) * Wc + cx0 + i] : 0;
      Q.left[i] = L ? r[(size_t)(cy0 + i) * Wc + cx0 - 1] : 0;
    }
    if (TL) ctl = r[(size_t)(cy0 - 1) * Wc + cx0 - 1];
    for (int q = 0; q < 4; ++q) {
      const int bx = q & 1, by = q >> 1;
      int st = 0, sl = 0;
      for (int i = 0; i < 4; ++i) {
        st += Q.top[4 * bx + i];
        sl += Q.left[4 * by + i];
      }
      int v = 128;
      if (bx == by) {
        if (T && L) v = (st + sl + 4) >> 3;
        else if (L) v = (sl + 2) >> 2;
        else if (T) v = (st + 2) >> 2;
      } else if (bx == 1) {
        if (T) v = (st + 2) >> 2;
        else if (L) v = (sl + 2) >> 2;
      } else {
        if (L) v = (sl + 2) >> 2;
        else if (T) v = (st + 2) >> 2;
      }
      Q.dcq[q] = v;
    }
    int H = 0, V = 0;
    for (int i = 0; i < 4; ++i) {
      const int t1 = 2 - i < 0 ? ctl : Q.top[2 - i], l1 = 2 - i < 0 ? ctl : Q.left[2 - i];
      H += (i + 1) * (Q.top[4 + i] - t1);
      V += (i + 1) * (Q.left[4 + i] - l1);
    }
    Q.a = 16 * (Q.left[7] + Q.top[7]);
    Q.b = (34 * H + 32) >> 6;
    Q.c = (34 * V + 32) >> 6;
    for (int y = 0; y < 8; ++y)
      for (int k = 0; k < 2; ++k) sc[c][2 * y + k] = ld32(p.sc[c] + (size_t)(cy0 + y) * Wc + cx0 + 4 * k);
  }
  int cmode = 0, cbest = sadc<0>(sc[0], C[0]) + sadc<0>(sc[1], C[1]);
  if (L) {
    const int v = sadc<1>(sc[0], C[0]) + sadc<1>(sc[1], C[1]);
    if (v < cbest) { cbest = v; cmode = 1; }
  }
  if (T) {
    const int v = sadc<2>(sc[0], C[0]) + sadc<2>(sc[1], C[1]);
    if (v < cbest) { cbest = v; cmode = 2; }
  }
  if (TL) {
    const int v = sadc<3>(sc[0], C[0]) + sadc<3>(sc[1], C[1]);
    if (v < cbest) { cbest = v; cmode = 3; }
  }
  const WBuf pc[2] = {wk.at(160), wk.at(176)};
  #pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (cmode == 0) fillc<0>(C[c], pc[c]);
    else if (cmode == 1) fillc<1>(C[c], pc[c]);
    else if (cmode == 2) fillc<2>(C[c], pc[c]);
    else fillc<3>(C[c], pc[c]);
  }
  if (dbg) {   // diagnostics (arb_h264_debug): chroma predictor state of one macroblock
    int o = 0;
    dbg[o++] = uint32_t(cmode);
    dbg[o++] = uint32_t(sadc<0>(sc[0], C[0]) + sadc<0>(sc[1], C[1]));
    dbg[o++] = uint32_t(sadc<3>(sc[0], C[0]) + sadc<3>(sc[1], C[1]));
    for (int c = 0; c < 2; ++c) {
      dbg[o++] = uint32_t(C[c].a);
      dbg[o++] = uint32_t(C[c].b);
      dbg[o++] = uint32_t(C[c].c);
      for (int i = 0; i < 4; ++i) dbg[o++] = uint32_t(C[c].dcq[i]);
      for (int i = 0; i < 8; ++i) dbg[o++] = uint32_t(C[c].top[i]);
      for (int i = 0; i < 8; ++i) dbg[o++] = uint32_t(C[c].left[i]);
      for (int i = 0; i < 16; ++i) dbg[o++] = sc[c][i];
      for (int i = 0; i < 16; ++i) dbg[o++] = pc[c][i];
    }
  }
  int c_any_ac = 0, c_any_dc = 0;
  int cdc[2][4];
  #pragma unroll
  for (int c = 0; c < 2; ++c) {
    int d4[4];
    for (int blk = 0; blk < 4; ++blk) {
      const int bx = blk & 1, by = blk >> 1;
      int res[16], w4[16];
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          const int i = 8 * (4 * by + y) + 4 * bx + x;
          res[4 * y + x] = byte_of(sc[c], i) - byte_of(pc[c], i);
        }
      fwd4x4(res, w4);
      d4[blk] = w4[0];
      int tc = 0;
      for (int k = 0; k < 15; ++k) {
        const int r = kZigzag[k + 1];
        const int q = quant(w4[r], kMF[qc6][pos_class(r)], fqc, qcbits);
        lv[kLvCac + 60 * c + 15 * blk + k] = (int16_t)q;
        tc += q != 0;
      }
      p.tcc[c][(size_t)(2 * my + by) * 2 * p.mbw + 2 * mx + bx] = (uint8_t)tc;
      c_any_ac |= tc;
    }
    const int h[4] = {d4[0] + d4[1] + d4[2] + d4[3], d4[0] - d4[1] + d4[2] - d4[3], d4[0] + d4[1] - d4[2] - d4[3],
                      d4[0] - d4[1] - d4[2] + d4[3]};
    for (int k = 0; k < 4; ++k) {
      cdc[c][k] = quant(h[k], kMF[qc6][0], 2 * fqc, qcbits + 1);
      lv[kLvCdc + 4 * c + k] = (int16_t)cdc[c][k];
      c_any_dc |= cdc[c][k];
    }
  }
  const int cbp_chroma = c_any_ac ? 2 : c_any_dc ? 1 : 0;
  p.info[mb] = uint32_t(mode) | uint32_t(cmode) << 2 | uint32_t(cbp_chroma) << 4 | uint32_t(any_ac != 0) << 6;

  // ---- chroma reconstruction (native recon_chroma)
  {
    const int ls = 16 * kV[qc6][0];
    const Dq dq(qpc);
    #pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int* q4 = cdc[c];
      const int fv4[4] = {q4[0] + q4[1] + q4[2] + q4[3], q4[0] - q4[1] + q4[2] - q4[3], q4[0] + q4[1] - q4[2] - q4[3],
                          q4[0] - q4[1] - q4[2] + q4[3]};
      for (int blk = 0; blk < 4; ++blk) {
        const int bx = blk & 1, by = blk >> 1;
        int d[16];
        for (int k = 0; k < 16; ++k) d[k] = 0;
        d[0] = (fv4[blk] * ls * (1 << (qpc / 6))) >> 5;
        int any = 0;
        for (int k = 0; k < 15; ++k) {
          const int r = kZigzag[k + 1];
          const int q = lv[kLvCac + 60 * c + 15 * blk + k];
          d[r] = dq(q, r);
          any |= q;
        }
        int r16[16];
        if (any) {
          inv4x4(d, r16);
        } else {
          const int v = (d[0] + 32) >> 6;
          for (int k = 0; k < 16; ++k) r16[k] = v;
        }
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int yy = 4 * by + y;
          uint32_t v = 0;
#pragma unroll
          for (int x = 0; x < 4; ++x)
            v |= uint32_t(clip255(byte_of(pc[c], 8 * yy + 4 * bx + x) + sat16(r16[4 * y + x]))) << (8 * x);
          *reinterpret_cast<uint32_t*>(p.rc[c] + (size_t)(cy0 + yy) * Wc + cx0 + 4 * bx) = v;
        }
      }
    }
  }
}

// ---- CAVLC (native write_block) into a bit sink: Count (lengths only) or Put (the bits)
struct Count {
  uint32_t n = 0;
  int err = 0;
  HD void put(uint32_t, int len) { n += (uint32_t)len; }
};

HD inline void or_word(uint32_t* w, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicOr(w, v);
#else
  *w |= v;
#endif
}

// MSB-first bits from an absolute bit position of a big-endian word buffer.  Words wholly inside
// this writer's range are stored; its first and last words may hold a neighbour's bits (OR).
struct Put {
  uint32_t* out;
  size_t w;
  uint64_t acc = 0;
  int n;
  bool first = true;
  int err = 0;
  HD Put(uint32_t* o, uint64_t bitpos) : out(o), w((size_t)(bitpos >> 5)), n((int)(bitpos & 31)) {}
  HD void put(uint32_t v, int len) {
    if (len == 0) return;
    acc = (acc << len) | (len == 32 ? v : (v & ((1u << len) - 1)));
    n += len;
    if (n >= 32) {
      n -= 32;
      const uint32_t word = bswap32(uint32_t(acc >> n));
      if (first) or_word(out + w, word);
      else out[w] = word;
      first = false;
      ++w;
    }
  }
  HD void finish() {
    if (n > 0) or_word(out + w, bswap32(uint32_t(acc << (32 - n))));
  }
};

template <class S>
HD inline void ue(S& s, uint32_t v) {
  const uint32_t x = v + 1;
  const int len = 32 - clz32(x);
  s.put(0, len - 1);
  s.put(x, len);
}

template <class S>
HD inline void write_block(S& s, const int16_t* coef, int max_num, int nC) {
  int levels[16], runs[16], tc = 0;
  uint32_t nzm = 0;
  for (int i = 0; i < max_num; ++i) nzm |= uint32_t(coef[i] != 0) << i;
  const int last = nzm ? 31 - clz32(nzm) : -1;
  for (uint32_t m = nzm; m;) {
    const int i = 31 - clz32(m);
    m &= ~(1u << i);
    levels[tc] = coef[i];
    runs[tc++] = m ? i - 1 - (31 - clz32(m)) : i;
  }
  const int total_zeros = last + 1 - tc;
  int t1 = 0;
  while (t1 < tc && t1 < 3 && (levels[t1] == 1 || levels[t1] == -1)) ++t1;
  if (nC == -1) {
    s.put(kChromaDcTokenBits[tc * 4 + t1], kChromaDcTokenLen[tc * 4 + t1]);
  } else {
    const int t = nC < 2 ? 0 : nC < 4 ? 1 : nC < 8 ? 2 : 3;
    s.put(kCoeffTokenBits[t][tc * 4 + t1], kCoeffTokenLen[t][tc * 4 + t1]);
  }
  if (tc == 0) return;
  uint32_t signs = 0;
  for (int k = 0; k < t1; ++k) signs = (signs << 1) | uint32_t(levels[k] < 0);
  s.put(signs, t1);
  int sl = (tc > 10 && t1 < 3) ? 1 : 0;
  for (int k = t1; k < tc; ++k) {
    const int lv = levels[k];
    int code = lv > 0 ? 2 * lv - 2 : -2 * lv - 1;
    if (k == t1 && t1 < 3) code -= 2;
    if (sl == 0) {
      if (code < 14) {
        s.put(1, code + 1);
      } else if (code < 30) {
        s.put(16 | uint32_t(code - 14), 19);
      } else {
        if (code - 30 >= 4096) s.err = 1;
        s.put(4096 | uint32_t(code - 30), 28);
      }
    } else {
      if (code < (15 << sl)) {
        s.put((1u << sl) | uint32_t(code & ((1 << sl) - 1)), (code >> sl) + 1 + sl);
      } else {
        if (code - (15 << sl) >= 4096) s.err = 1;
        s.put(4096 | uint32_t(code - (15 << sl)), 28);
      }
    }
    if (sl == 0) sl = 1;
    if ((lv < 0 ? -lv : lv) > (3 << (sl - 1)) && sl < 6) ++sl;
  }
  if (tc < max_num) {
    if (nC == -1) s.put(kChromaDcTotalZerosBits[tc - 1][total_zeros], kChromaDcTotalZerosLen[tc - 1][total_zeros]);
    else s.put(kTotalZerosBits[tc - 1][total_zeros], kTotalZerosLen[tc - 1][total_zeros]);
  }
  int zl = total_zeros;
  for (int k = 0; k < tc - 1 && zl > 0; ++k) {
    const int t = (zl < 7 ? zl : 7) - 1;
    s.put(kRunBits[t][runs[k]], kRunLen[t][runs[k]]);
    zl -= runs[k];
  }
}

// nC (9.2.1) of the 4x4 block (bx, by) of a plane with `per` blocks per macroblock side; one slice,
// so a neighbour is available iff it is inside the picture
HD inline int nc(const uint8_t* tcs, int mbw, int bx, int by, int per) {
  const int stride = per * mbw;
  const bool a = bx > 0, b = by > 0;
  const int na = a ? tcs[(size_t)by * stride + bx - 1] : 0, nb = b ? tcs[(size_t)(by - 1) * stride + bx] : 0;
  if (a && b) return (na + nb + 1) >> 1;
  return a ? na : b ? nb : 0;
}

template <class S>
HD inline void mb_syntax(S& s, const Pic& p, int mx, int my) {
  const int mb = my * p.mbw + mx;
  const uint32_t inf = p.info[mb];
  const int mode = inf & 3, cmode = (inf >> 2) & 3, cbpc = (inf >> 4) & 3, cbpl = (inf >> 6) & 1;
  const int16_t* lv = p.lv + (size_t)mb * kLevels;
  ue(s, uint32_t(1 + mode + 4 * cbpc + (cbpl ? 12 : 0)));
  ue(s, uint32_t(cmode));
  s.put(1, 1);   // mb_qp_delta = se(0)
  write_block(s, lv, 16, nc(p.tcy, p.mbw, 4 * mx, 4 * my, 4));
  if (cbpl)
    for (int blk = 0; blk < 16; ++blk)
      write_block(s, lv + kLvAc + 15 * blk, 15, nc(p.tcy, p.mbw, 4 * mx + kBlkX[blk], 4 * my + kBlkY[blk], 4));
  if (cbpc)
    for (int c = 0; c < 2; ++c) write_block(s, lv + kLvCdc + 4 * c, 4, -1);
  if (cbpc == 2)
    for (int c = 0; c < 2; ++c)
      for (int blk = 0; blk < 4; ++blk)
        write_block(s, lv + kLvCac + 60 * c + 15 * blk, 15,
                    nc(p.tcc[c], p.mbw, 2 * mx + (blk & 1), 2 * my + (blk >> 1), 2));
}

// IDR slice header of native encode_idr (first_mb 0, slice_type 7, pps 0, frame_num 0, idr_pic_id
// = index & 1, flags 0, slice_qp_delta 0, deblocking off): (bits, length)
HD inline void slice_header(int index, uint32_t& val, int& len) {
  val = 0;
  len = 0;
  auto app = [&](uint32_t v, int n) {
    val = (val << n) | v;
    len += n;
  };
  auto ueh = [&](uint32_t v) {
    const uint32_t x = v + 1;
    const int l = 32 - clz32(x);
    app(0, l - 1);
    app(x, l);
  };
  ueh(0);
  ueh(7);
  ueh(0);
  app(0, 4);
  ueh(uint32_t(index & 1));
  app(0, 1);
  app(0, 1);
  app(1, 1);   // se(0)
  ueh(1);
}

// ---- workspace layout (device or host): per picture planes, TotalCoeff, levels, info, bits
struct Layout {
  size_t y, c, tcy, tcc, lv, info, bits, per_pic;
  HD Layout(int W16, int H16) {
    const int mbw = W16 / 16, mbh = H16 / 16, nmb = mbw * mbh;
    y = (size_t)W16 * H16;
    c = y / 4;
    tcy = (size_t)16 * nmb;
    tcc = (size_t)4 * nmb;
    lv = (size_t)nmb * kLevels * 2;
    info = (size_t)nmb * 4;
    bits = (size_t)nmb * 4;
    per_pic = y + 2 * c + tcy + 2 * tcc + lv + info + bits;
    per_pic = (per_pic + 255) & ~(size_t)255;
  }
};

HD inline Pic make_pic(uint8_t* pic_ws, const Layout& Lo, const uint8_t* sy, const uint8_t* scb,
                       const uint8_t* scr, int f, int W16, int H16, int qp) {
  Pic p;
  uint8_t* b = pic_ws;
  p.sy = sy + (size_t)f * Lo.y;
  p.sc[0] = scb + (size_t)f * Lo.c;
  p.sc[1] = scr + (size_t)f * Lo.c;
  p.lv = reinterpret_cast<int16_t*>(b);  b += Lo.lv;      // 2-byte aligned first
  p.info = reinterpret_cast<uint32_t*>(b);  b += Lo.info;
  p.bits = reinterpret_cast<uint32_t*>(b);  b += Lo.bits;
  p.ry = b;  b += Lo.y;
  p.rc[0] = b;  b += Lo.c;
  p.rc[1] = b;  b += Lo.c;
  p.tcy = b;  b += Lo.tcy;
  p.tcc[0] = b;  b += Lo.tcc;
  p.tcc[1] = b;
  p.W = W16;
  p.mbw = W16 / 16;
  p.mbh = H16 / 16;
  p.qp = qp;
  return p;
}

}  // namespace h264g

using namespace h264g;

// meta (int64): [0 .. F] byte offset of each picture's RBSP in `out` (4-byte aligned; [F] = total),
// [F + 1] error flags (1 = level escape out of range, 2 = capacity), [F + 2 .. 2F + 2) RBSP bits
// (slice header + macroblocks, without the stop bit)
struct EncArgs {
  const uint8_t* y;
  const uint8_t* cb;
  const uint8_t* cr;
  uint8_t* ws;
  uint32_t* out;
  long long* meta;
  long long cap;
  int F, W16, H16, qp;
  int agent_sync;
  uint32_t* dbg;
  int dbg_mb;
};

// diagonal hand-off between the analyse kernel's waves: 1 = agent-scope release / acquire around the
// barrier (the acquire invalidates the CU's vector L1, so a neighbour's reconstruction written by
// another lane is never read from a stale line), 0 = the plain workgroup barrier (A/B)
static int g_h264_agent_sync = 1;
ARB_API void arb_set_h264_sync(int v) { g_h264_agent_sync = v; }
// diagnostics: the chroma predictor state of macroblock `mb` of picture 0 goes to `buf` (>= 128 dwords;
// device memory for the GPU launch, host memory for arb_h264_intra_host); nullptr = off
static uint32_t* g_h264_dbg = nullptr;
static int g_h264_dbg_mb = -1;
ARB_API void arb_h264_debug(void* buf, int mb) {
  g_h264_dbg = static_cast<uint32_t*>(buf);
  g_h264_dbg_mb = mb;
}

__global__ void __launch_bounds__(128) h264_analyse_kernel(EncArgs a) {
  __shared__ uint32_t work[kWork * 128];
  const WBuf wk{work + threadIdx.x, 128};
  const Layout Lo(a.W16, a.H16);
  const Pic p = make_pic(a.ws + (size_t)blockIdx.x * Lo.per_pic, Lo, a.y, a.cb, a.cr, blockIdx.x, a.W16, a.H16, a.qp);
  for (int d = 0; d < p.mbw + p.mbh - 1; ++d) {
    const int lo = d - (p.mbw - 1) > 0 ? d - (p.mbw - 1) : 0;
    const int hi = d < p.mbh - 1 ? d : p.mbh - 1;
    for (int my = lo + (int)threadIdx.x; my <= hi; my += blockDim.x) {
      const int mx = d - my;
      analyse_mb(p, mx, my, wk,
                 (a.dbg && blockIdx.x == 0 && my * p.mbw + mx == a.dbg_mb) ? a.dbg : nullptr);
    }
    // this diagonal's reconstruction / TotalCoeff before the next one reads them
    if (a.agent_sync) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    } else {
      __syncthreads();
    }
  }
}

// CAVLC bit count of every macroblock (one lane each: off the analyse kernel's serial diagonal path)
__global__ void __launch_bounds__(256) h264_count_kernel(EncArgs a) {
  const Layout Lo(a.W16, a.H16);
  const int mbw = a.W16 / 16, nmb = mbw * (a.H16 / 16);
  const long long i = blockIdx.x * 256LL + threadIdx.x;
  if (i >= (long long)a.F * nmb) return;
  const int f = (int)(i / nmb), mb = (int)(i % nmb);
  const Pic p = make_pic(a.ws + (size_t)f * Lo.per_pic, Lo, a.y, a.cb, a.cr, f, a.W16, a.H16, a.qp);
  Count c;
  mb_syntax(c, p, mb % mbw, mb / mbw);
  p.bits[mb] = c.n;
  if (c.err) atomicOr(reinterpret_cast<unsigned long long*>(a.meta + a.F + 1), 1ull);
}

// per picture: macroblock bit offsets (exclusive prefix after the slice header), RBSP bits
__global__ void __launch_bounds__(1024) h264_scan_kernel(EncArgs a) {
  __shared__ uint32_t part[1024];
  const Layout Lo(a.W16, a.H16);
  const Pic p = make_pic(a.ws + (size_t)blockIdx.x * Lo.per_pic, Lo, a.y, a.cb, a.cr, blockIdx.x, a.W16, a.H16, a.qp);
  const int nmb = p.mbw * p.mbh, t = threadIdx.x;
  const int per = (nmb + 1023) / 1024, b0 = t * per, b1 = b0 + per < nmb ? b0 + per : nmb;
  uint32_t sum = 0;
  for (int i = b0; i < b1; ++i) sum += p.bits[i];
  part[t] = sum;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {   // inclusive Hillis-Steele scan
    const uint32_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t hv;
  int hl;
  slice_header(blockIdx.x, hv, hl);
  uint32_t run = (uint32_t)hl + (t ? part[t - 1] : 0);
  for (int i = b0; i < b1; ++i) {
    const uint32_t n = p.bits[i];
    p.bits[i] = run;
    run += n;
  }
  if (t == 1023) a.meta[a.F + 2 + blockIdx.x] = (long long)hl + part[1023];
}

// one wave: picture byte offsets, capacity check
__global__ void __launch_bounds__(64) h264_frames_kernel(EncArgs a) {
  if (threadIdx.x != 0) return;
  long long base = 0;
  for (int f = 0; f < a.F; ++f) {
    a.meta[f] = base;
    const long long bits = a.meta[a.F + 2 + f];
    base += ((bits + 1 + 31) / 32) * 4;   // + the stop bit, whole words
  }
  a.meta[a.F] = base;
  if (base > a.cap) a.meta[a.F + 1] |= 2;
}

__global__ void __launch_bounds__(256) h264_zero_kernel(EncArgs a) {
  if (a.meta[a.F + 1]) return;
  const long long words = a.meta[a.F] / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < words; i += (long long)gridDim.x * 256) a.out[i] = 0;
}

// one lane per macroblock; lane 0 of each picture also writes the slice header and the stop bit
__global__ void __launch_bounds__(256) h264_write_kernel(EncArgs a) {
  if (a.meta[a.F + 1]) return;
  const Layout Lo(a.W16, a.H16);
  const int mbw = a.W16 / 16, nmb = mbw * (a.H16 / 16);
  const long long i = blockIdx.x * 256LL + threadIdx.x;
  if (i >= (long long)a.F * nmb) return;
  const int f = (int)(i / nmb), mb = (int)(i % nmb);
  const Pic p = make_pic(a.ws + (size_t)f * Lo.per_pic, Lo, a.y, a.cb, a.cr, f, a.W16, a.H16, a.qp);
  uint32_t* out = a.out + a.meta[f] / 4;
  Put s(out, p.bits[mb]);
  mb_syntax(s, p, mb % mbw, mb / mbw);
  s.finish();
  if (mb == 0) {
    uint32_t hv;
    int hl;
    slice_header(f, hv, hl);
    or_word(out, bswap32(hv << (32 - hl)));
    const long long sb = a.meta[a.F + 2 + f];
    or_word(out + sb / 32, bswap32(1u << (31 - (int)(sb & 31))));
  }
}

static bool enc_shape_ok(int F, int W16, int H16, int qp) {
  return F > 0 && W16 >= 16 && H16 >= 16 && W16 % 16 == 0 && H16 % 16 == 0 && qp >= 0 && qp <= 51 &&
         (long long)(W16 / 16) * (H16 / 16) <= (1 << 22);
}

ARB_API size_t arb_h264_intra_workspace(int F, int W16, int H16) {
  if (!enc_shape_ok(F, W16, H16, 0)) return 0;
  return (size_t)F * Layout(W16, H16).per_pic;
}

// y [F, H16, W16], cb / cr [F, H16 / 2, W16 / 2] (macroblock-padded 4:2:0, device) -> out (device,
// cap bytes, 4-byte aligned) + meta (device int64 [2F + 2], zeroed here).  The host reads meta,
// then out[meta[f] .. meta[f] + (meta[F + 2 + f] + 8) / 8) is picture f's RBSP.
ARB_API int arb_h264_intra_encode(const void* y, const void* cb, const void* cr, int F, int W16, int H16, int qp,
                                  void* ws, void* out, long long cap, void* meta, hipStream_t stream) {
  if (!enc_shape_ok(F, W16, H16, qp) || cap < 0) return -1;
  EncArgs a{(const uint8_t*)y, (const uint8_t*)cb, (const uint8_t*)cr, (uint8_t*)ws, (uint32_t*)out,
            (long long*)meta, cap, F, W16, H16, qp, g_h264_agent_sync, g_h264_dbg, g_h264_dbg_mb};
  hipError_t e = hipMemsetAsync(meta, 0, sizeof(long long) * (2 * (size_t)F + 2), stream);
  if (e != hipSuccess) return (int)e;
  const long long lanes = (long long)F * (W16 / 16) * (H16 / 16);
  const unsigned mb_blocks = (unsigned)((lanes + 255) / 256);
  h264_analyse_kernel<<<F, 128, 0, stream>>>(a);
  h264_count_kernel<<<mb_blocks, 256, 0, stream>>>(a);
  h264_scan_kernel<<<F, 1024, 0, stream>>>(a);
  h264_frames_kernel<<<1, 64, 0, stream>>>(a);
  h264_zero_kernel<<<512, 256, 0, stream>>>(a);
  h264_write_kernel<<<mb_blocks, 256, 0, stream>>>(a);
  return (int)hipGetLastError();
}

// The same functions on the CPU (raster order, one picture after another): tests without a GPU.
// Host pointers; out must hold cap bytes; meta as above.
ARB_API int arb_h264_intra_host(const void* y, const void* cb, const void* cr, int F, int W16, int H16, int qp,
                                void* out, long long cap, long long* meta, void* ws_out) {
  if (!enc_shape_ok(F, W16, H16, qp) || cap < 0) return -1;
  const Layout Lo(W16, H16);
  std::vector<uint8_t> ws(Lo.per_pic);
  std::vector<uint32_t> work(kWork);
  const int mbw = W16 / 16, mbh = H16 / 16, nmb = mbw * mbh;
  for (int i = 0; i < 2 * F + 2; ++i) meta[i] = 0;
  long long base = 0;
  std::memset(out, 0, (size_t)cap);
  for (int f = 0; f < F; ++f) {
    std::fill(ws.begin(), ws.end(), 0);
    Pic p = make_pic(ws.data(), Lo, (const uint8_t*)y, (const uint8_t*)cb, (const uint8_t*)cr, f, W16, H16, qp);
    int err = 0;
    for (int my = 0; my < mbh; ++my)
      for (int mx = 0; mx < mbw; ++mx) {
        analyse_mb(p, mx, my, WBuf{work.data(), 1},
                   (g_h264_dbg && f == 0 && my * mbw + mx == g_h264_dbg_mb) ? g_h264_dbg : nullptr);
        Count c;
        mb_syntax(c, p, mx, my);
        p.bits[my * mbw + mx] = c.n;
        err |= c.err;
      }
    if (err) meta[F + 1] |= 1;
    uint32_t hv;
    int hl;
    slice_header(f, hv, hl);
    uint32_t run = (uint32_t)hl;
    for (int i = 0; i < nmb; ++i) {
      const uint32_t n = p.bits[i];
      p.bits[i] = run;
      run += n;
    }
    meta[f] = base;
    meta[F + 2 + f] = run;
    const long long bytes = (((long long)run + 1 + 31) / 32) * 4;
    if (base + bytes > cap) {
      meta[F + 1] |= 2;
      return 0;
    }
    uint32_t* o = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(out) + base);
    for (int i = 0; i < nmb; ++i) {
      Put s(o, p.bits[i]);
      mb_syntax(s, p, i % mbw, i / mbw);
      s.finish();
    }
    or_word(o, bswap32(hv << (32 - hl)));
    or_word(o + run / 32, bswap32(1u << (31 - (int)(run & 31))));
    base += bytes;
    if (ws_out) std::memcpy(static_cast<uint8_t*>(ws_out) + (size_t)f * Lo.per_pic, ws.data(), Lo.per_pic);
  }
  meta[F] = base;
  return 0;
}
