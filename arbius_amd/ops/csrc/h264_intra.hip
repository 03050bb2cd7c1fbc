// H.264 avc-intra encoder on the GPU: the same bytes as native/src/h264.cpp encode_idr (one IDR
// slice per picture, Intra_16x16 + chroma modes by SAD, dead-zone quantisation at a fixed QP,
// CAVLC, deblocking off), so a video task's MP4 (robust_video_matting out-1.mp4,
// /root/reference/templates/robust_video_matting.json:1-31) no longer costs ~17 ms of host CPU per
// 1080p frame.  The host keeps only emulation prevention and the MP4 mux.
//
// Work split (one launch each, all on the caller's stream):
//   analyse  one workgroup per picture walks the macroblock anti-diagonals (mx + my = d): an
//            Intra_16x16 macroblock reads only its left / top / top-left neighbours' reconstruction,
//            so every macroblock of a diagonal is independent.  Four lanes per macroblock (MbLane)
//            run the encoder's decisions (mode SADs, forward transform, quantisation,
//            reconstruction); levels, modes and TotalCoeff go to a workspace.
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
// on the CPU in raster order, the 4 lanes' phases one after another (tests/test_h264_gpu_algo.py
// compares its NALs with the native encoder on a machine without a GPU); the GPU path is checked
// against the native encoder by tests/test_h264_gpu.py.  Integer arithmetic only: nothing here
// depends on evaluation order.
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
HD inline int byte_of(const WBuf& s, int i) { return int((s[i >> 2] >> (8 * (i & 3))) & 255u); }
// acc + sum |a.byte[k] - b.byte[k]| (v_sad_u8 on the device: 4 samples per instruction; the mode
// decisions' SADs are integer sums, so the two forms are the same number)
HD inline uint32_t sad4(uint32_t a, uint32_t b, uint32_t acc) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_sad_u8(a, b, acc);
#else
  for (int k = 0; k < 4; ++k) {
    const int d = int((a >> (8 * k)) & 255u) - int((b >> (8 * k)) & 255u);
    acc += uint32_t(d < 0 ? -d : d);
  }
  return acc;
#endif
}

// Intra_16x16 predictor (8.3.3): the neighbours, the DC value and the plane parameters; V / H / DC
// samples are the neighbours / dc themselves, plane(x, y) the plane sample
struct Pred16 {
  int top[16], left[16], dc, a, b, c;
  HD int plane(int x, int y) const { return plane_px(a + b * (x - 7) + c * (y - 7) + 16); }
};
// Intra chroma 8x8 predictor (8.3.4): neighbours and plane parameters (the per-quadrant DC values of
// a lane's half are MbLane::cdq)
struct PredC {
  int top[8], left[8], a, b, c;
  HD int plane(int x, int y) const { return plane_px(a + b * (x - 3) + c * (y - 3) + 16); }
};

// One 4x4 block's residual (source - prediction, a row of `n` samples per picture row: 16 luma, 8
// chroma), forward transform and AC quantisation: the DC coefficient is returned, the 15 AC levels
// (zig-zag positions 1..15) go to ac.  The reconstruction recomputes them (ALU) instead of reading
// back the levels it stored (a global-memory round trip per block on the serial diagonal path).
template <int n>
HD inline int block_ac(const WBuf& s, const WBuf& pr, int bx, int by, int q6, int f, int qbits, int* ac) {
  int res[16], w4[16];
#pragma unroll
  for (int y = 0; y < 4; ++y)
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int i = n * (4 * by + y) + 4 * bx + x;
      res[4 * y + x] = byte_of(s, i) - byte_of(pr, i);
    }
  fwd4x4(res, w4);
#pragma unroll
  for (int k = 0; k < 15; ++k) {
    const int r = kZigzag[k + 1];
    ac[k] = quant(w4[r], kMF[q6][pos_class(r)], f, qbits);
  }
  return w4[0];
}

// ---- the per-macroblock decisions, levels and reconstruction (native encode_mb), by 4 lanes
//
// Lane q of a macroblock owns luma quadrant q (8x8 samples = 4x4 blocks 4q..4q+3 in blkIdx order) and
// half h = q & 1 of chroma component c = q >> 1 (rows 4h..4h+3 = 4x4 blocks 2h, 2h+1).  Three phases,
// a mailbox exchange between them (16 dwords per lane):
//   A  neighbours, predictor parameters, partial SADs of the 4 luma / 4 chroma modes over its samples
//   B  modes from the summed SADs; its blocks' prediction, residual, transform, AC levels; block DCs
//   C  luma / chroma DC transform + levels from all blocks' DCs (every lane, redundantly); the
//      reconstruction of its blocks; lane 0 writes the macroblock's DC levels and mode / cbp word.
// On the GPU the 4 lanes are neighbours in one wave and the phases are separated by an LDS fence; on
// the host (arb_h264_intra_host) the phases run lane after lane - the same functions, the same bytes.
constexpr int kMail = 16;      // mailbox dwords per lane: SADs 0..7, luma DCs 8..11, chroma DCs 12..13, flags 14
// work dwords per lane: luma src 16 | luma pred 16 | chroma src 8 | chroma pred 8 | dequantised luma DCs 16 |
// dequantised chroma DCs 4 (per-lane indexing goes through this buffer: indexing a private array by the
// lane's quadrant would put the lane's state in scratch memory)
constexpr int kLaneWork = 68;

HD inline uint32_t pack4(int a, int b, int c, int d) {
  return uint32_t(a) | uint32_t(b) << 8 | uint32_t(c) << 16 | uint32_t(d) << 24;
}

struct MbLane {
  Pic p;
  int mx, my, q, c, h;
  bool L, T, TL;
  WBuf s, pr, sc, pc;   // luma quadrant src / pred (8 rows x 2 dwords), chroma half src / pred (4 x 2)
  uint32_t* mail;       // the macroblock's mailbox: dword j of lane l at mail[j * mail_stride + l]
  int mail_stride;      // >= 4 (the 4 lanes' copies of one dword are adjacent)
  Pred16 P;
  PredC C;
  uint32_t t4[4], ct2[2], t4q[2];
  int tq[8], lq[8], clq[4], cdq[2];   // this lane's part of the neighbours (no per-lane array indexing)
  const uint8_t* rcc;                 // component c's reconstruction, source, TotalCoeff planes
  const uint8_t* scc;
  uint8_t* tccc;
  int mode, cmode;

  HD uint32_t& box(int lane, int j) const { return mail[j * mail_stride + lane]; }

  HD void init(const Pic& pic, int mx_, int my_, int q_, const WBuf& wk, uint32_t* mail_, int mstride) {
    p = pic; mx = mx_; my = my_; q = q_; c = q >> 1; h = q & 1;
    L = mx > 0; T = my > 0; TL = L && T;
    s = wk; pr = wk.at(16); sc = wk.at(32); pc = wk.at(40);
    mail = mail_; mail_stride = mstride;
    rcc = c ? p.rc[1] : p.rc[0];
    scc = c ? p.sc[1] : p.sc[0];
    tccc = c ? p.tcc[1] : p.tcc[0];
  }

  // ---- A: predictors and partial SADs
  HD void phase_a() {
    const int W = p.W, Wc = W / 2, x0 = 16 * mx, y0 = 16 * my, cx0 = 8 * mx, cy0 = 8 * my;
#pragma unroll
    for (int k = 0; k < 4; ++k) t4[k] = T ? ld32(p.ry + (size_t)(y0 - 1) * W + x0 + 4 * k) : 0u;
    int tl = TL ? p.ry[(size_t)(y0 - 1) * W + x0 - 1] : 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      P.top[i] = int((t4[i >> 2] >> (8 * (i & 3))) & 255u);
      P.left[i] = L ? p.ry[(size_t)(y0 + i) * W + x0 - 1] : 0;
    }
    {
      int st = 0, sl = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) { st += P.top[i]; sl += P.left[i]; }
      P.dc = (L && T) ? (st + sl + 16) >> 5 : L ? (sl + 8) >> 4 : T ? (st + 8) >> 4 : 128;
      int H = 0, V = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int t1 = 6 - i < 0 ? tl : P.top[6 - i], l1 = 6 - i < 0 ? tl : P.left[6 - i];
        H += (i + 1) * (P.top[8 + i] - t1);
        V += (i + 1) * (P.left[8 + i] - l1);
      }
      P.a = 16 * (P.left[15] + P.top[15]);
      P.b = (5 * H + 32) >> 6;
      P.c = (5 * V + 32) >> 6;
    }
    const int qx = q & 1, qy = q >> 1;
#pragma unroll
    for (int k = 0; k < 2; ++k) t4q[k] = T ? ld32(p.ry + (size_t)(y0 - 1) * W + x0 + 8 * qx + 4 * k) : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      tq[k] = int((t4q[k >> 2] >> (8 * (k & 3))) & 255u);
      lq[k] = L ? p.ry[(size_t)(y0 + 8 * qy + k) * W + x0 - 1] : 0;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int k = 0; k < 2; ++k) s[2 * r + k] = ld32(p.sy + (size_t)(y0 + 8 * qy + r) * W + x0 + 8 * qx + 4 * k);
    uint32_t sv = 0, sh = 0, sd = 0, sp = 0;
    const uint32_t dv = uint32_t(P.dc) * 0x01010101u;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int y = 8 * qy + r;
      const uint32_t lv4 = uint32_t(lq[r]) * 0x01010101u;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const uint32_t si = s[2 * r + k];
        const int x = 8 * qx + 4 * k;
        sv = sad4(si, t4q[k], sv);
        sh = sad4(si, lv4, sh);
        sd = sad4(si, dv, sd);
        sp = sad4(si, pack4(P.plane(x, y), P.plane(x + 1, y), P.plane(x + 2, y), P.plane(x + 3, y)), sp);
      }
    }
    // chroma component c
    {
      const uint8_t* r = rcc;
      int ctl = TL ? r[(size_t)(cy0 - 1) * Wc + cx0 - 1] : 0;
#pragma unroll
      for (int k = 0; k < 2; ++k) ct2[k] = T ? ld32(r + (size_t)(cy0 - 1) * Wc + cx0 + 4 * k) : 0u;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        C.top[i] = int((ct2[i >> 2] >> (8 * (i & 3))) & 255u);
        C.left[i] = L ? r[(size_t)(cy0 + i) * Wc + cx0 - 1] : 0;
      }
      int H = 0, V = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t1 = 2 - i < 0 ? ctl : C.top[2 - i], l1 = 2 - i < 0 ? ctl : C.left[2 - i];
        H += (i + 1) * (C.top[4 + i] - t1);
        V += (i + 1) * (C.left[4 + i] - l1);
      }
      C.a = 16 * (C.left[7] + C.top[7]);
      C.b = (34 * H + 32) >> 6;
      C.c = (34 * V + 32) >> 6;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int k = 0; k < 2; ++k) sc[2 * rr + k] = ld32(scc + (size_t)(cy0 + 4 * h + rr) * Wc + cx0 + 4 * k);
#pragma unroll
      for (int k = 0; k < 4; ++k) clq[k] = L ? r[(size_t)(cy0 + 4 * h + k) * Wc + cx0 - 1] : 0;
      // the DC predictions of this half's two 4x4 quadrants (bx = k, by = h), from the sums
      int sl0 = 0, sl1 = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) { sl0 += C.left[i]; sl1 += C.left[4 + i]; }
      const int sl = h ? sl1 : sl0;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        int st = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) st += C.top[4 * k + i];
        int v = 128;
        if (k == h) {
          if (T && L) v = (st + sl + 4) >> 3;
          else if (L) v = (sl + 2) >> 2;
          else if (T) v = (st + 2) >> 2;
        } else if (k == 1) {
          if (T) v = (st + 2) >> 2;
          else if (L) v = (sl + 2) >> 2;
        } else {
          if (L) v = (sl + 2) >> 2;
          else if (T) v = (st + 2) >> 2;
        }
        cdq[k] = v;
      }
    }
    uint32_t cd = 0, ch = 0, cv = 0, cpl = 0;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int y = 4 * h + rr;
      const uint32_t lv4 = uint32_t(clq[rr]) * 0x01010101u;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const uint32_t si = sc[2 * rr + k];
        const int x = 4 * k;
        cd = sad4(si, uint32_t(cdq[k]) * 0x01010101u, cd);
        ch = sad4(si, lv4, ch);
        cv = sad4(si, ct2[k], cv);
        cpl = sad4(si, pack4(C.plane(x, y), C.plane(x + 1, y), C.plane(x + 2, y), C.plane(x + 3, y)), cpl);
      }
    }
    box(q, 0) = sv; box(q, 1) = sh; box(q, 2) = sd; box(q, 3) = sp;
    box(q, 4) = cd; box(q, 5) = ch; box(q, 6) = cv; box(q, 7) = cpl;
  }

  // ---- B: modes, prediction, AC levels of this lane's blocks, block DCs to the mailbox
  HD void phase_b() {
    uint32_t sum[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int l = 0; l < 4; ++l)
#pragma unroll
      for (int j = 0; j < 8; ++j) sum[j] += box(l, j);
    int best = 1 << 30;   // candidates in mode order, ties to the lowest mode
    mode = 2;
    if (T) { best = int(sum[0]); mode = 0; }
    if (L && int(sum[1]) < best) { best = int(sum[1]); mode = 1; }
    if (int(sum[2]) < best) { best = int(sum[2]); mode = 2; }
    if (TL && int(sum[3]) < best) { best = int(sum[3]); mode = 3; }
    int cbest = int(sum[4]);
    cmode = 0;
    if (L && int(sum[5]) < cbest) { cbest = int(sum[5]); cmode = 1; }
    if (T && int(sum[6]) < cbest) { cbest = int(sum[6]); cmode = 2; }
    if (TL && int(sum[7]) < cbest) { cbest = int(sum[7]); cmode = 3; }
    // this lane's prediction (quadrant / chroma half), one loop per mode: static indices only
    const int qx = q & 1, qy = q >> 1;
    if (mode == 0) {
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int k = 0; k < 2; ++k) pr[2 * r + k] = t4q[k];
    } else if (mode == 1) {
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int k = 0; k < 2; ++k) pr[2 * r + k] = uint32_t(lq[r]) * 0x01010101u;
    } else if (mode == 2) {
#pragma unroll
      for (int i = 0; i < 16; ++i) pr[i] = uint32_t(P.dc) * 0x01010101u;
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int x = 8 * qx + 4 * k, y = 8 * qy + r;
          pr[2 * r + k] = pack4(P.plane(x, y), P.plane(x + 1, y), P.plane(x + 2, y), P.plane(x + 3, y));
        }
    }
    if (cmode == 0) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int k = 0; k < 2; ++k) pc[2 * rr + k] = uint32_t(cdq[k]) * 0x01010101u;
    } else if (cmode == 1) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int k = 0; k < 2; ++k) pc[2 * rr + k] = uint32_t(clq[rr]) * 0x01010101u;
    } else if (cmode == 2) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int k = 0; k < 2; ++k) pc[2 * rr + k] = ct2[k];
    } else {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int x = 4 * k, y = 4 * h + rr;
          pc[2 * rr + k] = pack4(C.plane(x, y), C.plane(x + 1, y), C.plane(x + 2, y), C.plane(x + 3, y));
        }
    }
    const int qp = p.qp, qp6 = qp % 6, qbits = 15 + qp / 6, fq = (1 << qbits) / 3;
    const int qpc = kChromaQp[qp], qc6 = qpc % 6, qcbits = 15 + qpc / 6, fqc = (1 << qcbits) / 3;
    int16_t* lv = p.lv + (size_t)(my * p.mbw + mx) * kLevels;
    uint32_t flags = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // luma blocks 4q + j: (j & 1, j >> 1) inside the quadrant
      const int blk = 4 * q + j;
      int ac[15];
      box(q, 8 + j) = uint32_t(block_ac<8>(s, pr, j & 1, j >> 1, qp6, fq, qbits, ac));
      int tc = 0;
#pragma unroll
      for (int k = 0; k < 15; ++k) {
        lv[kLvAc + 15 * blk + k] = (int16_t)ac[k];
        tc += ac[k] != 0;
      }
      p.tcy[(size_t)(4 * my + kBlkY[blk]) * 4 * p.mbw + 4 * mx + kBlkX[blk]] = (uint8_t)tc;
      flags |= uint32_t(tc != 0) << j;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {   // chroma blocks 2h + j of component c: (j, 0) inside the half
      const int cblk = 2 * h + j;
      int ac[15];
      box(q, 12 + j) = uint32_t(block_ac<8>(sc, pc, j, 0, qc6, fqc, qcbits, ac));
      int tc = 0;
#pragma unroll
      for (int k = 0; k < 15; ++k) {
        lv[kLvCac + 60 * c + 15 * cblk + k] = (int16_t)ac[k];
        tc += ac[k] != 0;
      }
      tccc[(size_t)(2 * my + h) * 2 * p.mbw + 2 * mx + j] = (uint8_t)tc;
      flags |= uint32_t(tc != 0) << (4 + j);
    }
    box(q, 14) = flags;
  }

  // ---- C: DC levels from every block's DC, reconstruction of this lane's blocks
  HD void phase_c() {
    const int qp = p.qp, qp6 = qp % 6, qbits = 15 + qp / 6, fq = (1 << qbits) / 3;
    const int qpc = kChromaQp[qp], qc6 = qpc % 6, qcbits = 15 + qpc / 6, fqc = (1 << qcbits) / 3;
    int dcm[16];
    uint32_t any_ac = 0, c_any_ac = 0;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int blk = 4 * l + j;
        dcm[4 * kBlkY[blk] + kBlkX[blk]] = int(box(l, 8 + j));
      }
      any_ac |= box(l, 14) & 15u;
      c_any_ac |= (box(l, 14) >> 4) & 3u;
    }
    int hd[16], dc[16];
    hadamard4(dcm, hd);
#pragma unroll
    for (int k = 0; k < 16; ++k) dc[k] = quant(hd[kZigzag[k]] / 2, kMF[qp6][0], 2 * fq, qbits + 1);
    int cdc[2][4], c_any_dc = 0;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int d0 = int(box(2 * cc, 12)), d1 = int(box(2 * cc, 13)), d2 = int(box(2 * cc + 1, 12)),
                d3 = int(box(2 * cc + 1, 13));
      const int hh[4] = {d0 + d1 + d2 + d3, d0 - d1 + d2 - d3, d0 + d1 - d2 - d3, d0 - d1 - d2 + d3};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        cdc[cc][k] = quant(hh[k], kMF[qc6][0], 2 * fqc, qcbits + 1);
        c_any_dc |= cdc[cc][k];
      }
    }
    const int cbp_chroma = c_any_ac ? 2 : c_any_dc ? 1 : 0;
    const int mb = my * p.mbw + mx;
    int16_t* lv = p.lv + (size_t)mb * kLevels;
    if (q == 0) {
#pragma unroll
      for (int k = 0; k < 16; ++k) lv[k] = (int16_t)dc[k];
#pragma unroll
      for (int cc = 0; cc < 2; ++cc)
#pragma unroll
        for (int k = 0; k < 4; ++k) lv[kLvCdc + 4 * cc + k] = (int16_t)cdc[cc][k];
      p.info[mb] = uint32_t(mode) | uint32_t(cmode) << 2 | uint32_t(cbp_chroma) << 4 | uint32_t(any_ac != 0) << 6;
    }
    // luma reconstruction of blocks 4q .. 4q + 3 (native recon_luma16)
    const int W = p.W, x0 = 16 * mx, y0 = 16 * my, qx = q & 1, qy = q >> 1;
    {
      int cz[16], fdc[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) cz[kZigzag[k]] = dc[k];
      hadamard4(cz, fdc);
      const WBuf wf = s.at(48);   // this lane's copy of the 16 dequantisation inputs, indexed by quadrant
#pragma unroll
      for (int k = 0; k < 16; ++k) wf[k] = uint32_t(fdc[k]);
      const int ls = 16 * kV[qp6][0];
      const Dq dq(qp);
      const uint32_t nz = box(q, 14);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int fv = int(wf[8 * qy + 2 * qx + 4 * (j >> 1) + (j & 1)]);   // fdc[4 by + bx] of block 4q + j
        int d[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) d[k] = 0;
        d[0] = qp >= 36 ? fv * ls * (1 << (qp / 6 - 6)) : (fv * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
        int ac[15] = {0}, any = 0;
        if ((nz >> j) & 1) block_ac<8>(s, pr, j & 1, j >> 1, qp6, fq, qbits, ac);
#pragma unroll
        for (int k = 0; k < 15; ++k) {
          const int r = kZigzag[k + 1];
          d[r] = dq(ac[k], r);
          any |= ac[k];
        }
        int r16[16];
        if (any) {
          inv4x4(d, r16);
        } else {
          const int v = (d[0] + 32) >> 6;
#pragma unroll
          for (int k = 0; k < 16; ++k) r16[k] = v;
        }
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int ly = 4 * (j >> 1) + y;   // row inside the quadrant
          const uint32_t pw = pr[2 * ly + (j & 1)];
          uint32_t v = 0;
#pragma unroll
          for (int x = 0; x < 4; ++x)
            v |= uint32_t(clip255(int((pw >> (8 * x)) & 255u) + sat16(r16[4 * y + x]))) << (8 * x);
          *reinterpret_cast<uint32_t*>(p.ry + (size_t)(y0 + 8 * qy + ly) * W + x0 + 8 * qx + 4 * (j & 1)) = v;
        }
      }
    }
    // chroma reconstruction of blocks 2h, 2h + 1 of component c (native recon_chroma)
    {
      const int Wc = W / 2, cx0 = 8 * mx, cy0 = 8 * my;
      const WBuf wc = s.at(64);   // component c's 4 dequantisation inputs (both computed, c's kept)
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const int* q4 = cdc[cc];
        if (cc == c) {
          wc[0] = uint32_t(q4[0] + q4[1] + q4[2] + q4[3]);
          wc[1] = uint32_t(q4[0] - q4[1] + q4[2] - q4[3]);
          wc[2] = uint32_t(q4[0] + q4[1] - q4[2] - q4[3]);
          wc[3] = uint32_t(q4[0] - q4[1] - q4[2] + q4[3]);
        }
      }
      const int ls = 16 * kV[qc6][0];
      const Dq dq(qpc);
      const uint32_t nz = box(q, 14) >> 4;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int cblk = 2 * h + j;
        int d[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) d[k] = 0;
        d[0] = (int(wc[2 * h + j]) * ls * (1 << (qpc / 6))) >> 5;
        int ac[15] = {0}, any = 0;
        if ((nz >> j) & 1) block_ac<8>(sc, pc, j, 0, qc6, fqc, qcbits, ac);
#pragma unroll
        for (int k = 0; k < 15; ++k) {
          const int r = kZigzag[k + 1];
          d[r] = dq(ac[k], r);
          any |= ac[k];
        }
        int r16[16];
        if (any) {
          inv4x4(d, r16);
        } else {
          const int v = (d[0] + 32) >> 6;
#pragma unroll
          for (int k = 0; k < 16; ++k) r16[k] = v;
        }
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const uint32_t pw = pc[2 * y + j];
          uint32_t v = 0;
#pragma unroll
          for (int x = 0; x < 4; ++x)
            v |= uint32_t(clip255(int((pw >> (8 * x)) & 255u) + sat16(r16[4 * y + x]))) << (8 * x);
          *reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(rcc) + (size_t)(cy0 + 4 * h + y) * Wc + cx0 + 4 * j) = v;
        }
      }
    }
  }
};

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
};

// diagonal hand-off between the analyse kernel's waves: 0 = the workgroup barrier (all waves of the
// workgroup share one CU and its vector L1, so workgroup scope makes a neighbour's reconstruction
// visible), 1 = agent-scope release / acquire around it (L2 write-back + L1 invalidate per diagonal,
// A/B: the same bytes, profiles/r6/h264/)
static int g_h264_agent_sync = 0;
ARB_API void arb_set_h264_sync(int v) { g_h264_agent_sync = v; }

// 80 macroblocks x 4 lanes per pass: a 1080p anti-diagonal holds <= 68 macroblocks
constexpr int kAnalyseThreads = 320;

// the mailbox writes of the other 3 lanes (same wave) are visible: one wave's LDS operations complete
// in order, so this only has to keep the compiler from moving LDS accesses across it
__device__ __forceinline__ void lane_exchange() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

__global__ void __launch_bounds__(kAnalyseThreads) h264_analyse_kernel(EncArgs a) {
  __shared__ uint32_t work[kLaneWork * kAnalyseThreads];
  __shared__ uint32_t mail[kMail * kAnalyseThreads];
  const int t = threadIdx.x, slot = t >> 2, q = t & 3;
  const WBuf wk{work + t, kAnalyseThreads};
  const Layout Lo(a.W16, a.H16);
  const Pic p = make_pic(a.ws + (size_t)blockIdx.x * Lo.per_pic, Lo, a.y, a.cb, a.cr, blockIdx.x, a.W16, a.H16, a.qp);
  for (int d = 0; d < p.mbw + p.mbh - 1; ++d) {
    const int lo = d - (p.mbw - 1) > 0 ? d - (p.mbw - 1) : 0;
    const int hi = d < p.mbh - 1 ? d : p.mbh - 1;
    for (int base = 0; base <= hi - lo; base += kAnalyseThreads / 4) {
      const int my = lo + base + slot;
      const bool active = my <= hi;
      MbLane ln;
      if (active) {
        ln.init(p, d - my, my, q, wk, mail + 4 * slot, kAnalyseThreads);
        ln.phase_a();
      }
      lane_exchange();
      if (active) ln.phase_b();
      lane_exchange();
      if (active) ln.phase_c();
      lane_exchange();
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
            (long long*)meta, cap, F, W16, H16, qp, g_h264_agent_sync};
  hipError_t e = hipMemsetAsync(meta, 0, sizeof(long long) * (2 * (size_t)F + 2), stream);
  if (e != hipSuccess) return (int)e;
  const long long lanes = (long long)F * (W16 / 16) * (H16 / 16);
  const unsigned mb_blocks = (unsigned)((lanes + 255) / 256);
  h264_analyse_kernel<<<F, kAnalyseThreads, 0, stream>>>(a);
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
  std::vector<uint32_t> work(4 * kLaneWork), mail(4 * kMail);
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
        MbLane ln[4];   // the 4 lanes of the GPU kernel, phase after phase
        for (int q = 0; q < 4; ++q) ln[q].init(p, mx, my, q, WBuf{work.data() + q, 4}, mail.data(), 4);
        for (int q = 0; q < 4; ++q) ln[q].phase_a();
        for (int q = 0; q < 4; ++q) ln[q].phase_b();
        for (int q = 0; q < 4; ++q) ln[q].phase_c();
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
