// Deterministic H.264 Constrained-Baseline codec (CAVLC), see h264.h.
//
// Why it exists (SURVEY.md §2.6(c,d)): the video templates (/root/reference/templates/zeroscopev2xl.json:1,
// robust_video_matting.json:6-31) return out-1.mp4 whose CID is the solution, so the encoder must be a
// pure function of the frames on every node, and there is no ffmpeg / libx264 in the image; the matting
// template's input_video has to be decoded without one too.
//
// Encoder: IPPP GOPs.  I macroblocks choose the Intra_16x16 luma / chroma mode by SAD (SSE2 psadbw,
// integer, ties -> lowest mode); P macroblocks a quarter-sample motion vector by a fixed search order
// (P_L0_16x16 / P_Skip); forward core transform + Hadamard DC, dead-zone quantisation at a fixed QP,
// CAVLC over a non-zero bit mask; in-loop deblocking ON.  The reconstruction is the normative decoding
// process (ITU-T H.264 8.3-8.7) shared with the decoder below, so the encoder's reference pictures are
// every decoder's output, bit for bit; slices encode in parallel (same bytes at any thread count).
//
// Decoder (input_video): SPS / PPS, IDR and non-IDR I and P slices, CAVLC, I_PCM / I_16x16 / I_NxN /
// P partitions with quarter-sample MC, multiple reference frames with list modification and MMCO,
// in-loop deblocking (wavefront-parallel), multiple slices, 4:2:0 8-bit.  CABAC, B slices, High-profile
// tools (8x8 transform), weighted prediction and long-term references throw: the node then skips the
// task as undecodable (never marks it invalid: another miner's decoder may read it).
#include "h264.h"

#include <emmintrin.h>   // SSE2 (x86-64 baseline): psadbw for the mode-decision SADs

#include <algorithm>
#include <atomic>
#include <cstring>
#include <memory>
#include <utility>
#include <thread>
#include <stdexcept>

namespace h264 {
namespace {

// ------------------------------------------------------------------------------------ bit I/O
struct BitWriter {
  std::string out;
  uint64_t acc = 0;   // pending bits: the low n bits of acc, MSB first
  int n = 0;          // < 32 between calls: full 32-bit words are flushed as they complete
  void put(uint32_t v, int len) {  // len <= 32
    if (len == 0) return;
    acc = (acc << len) | (len == 32 ? v : (v & ((1u << len) - 1)));
    n += len;
    if (n >= 32) {
      n -= 32;
      const uint32_t w = uint32_t(acc >> n);
      const char b[4] = {char(w >> 24), char(w >> 16), char(w >> 8), char(w)};
      out.append(b, 4);
    }
  }
  void flush_bytes() {
    while (n >= 8) {
      n -= 8;
      out.push_back(char((acc >> n) & 0xFF));
    }
  }
  void ue(uint32_t v) {
    const uint32_t x = v + 1;
    const int len = 32 - __builtin_clz(x);
    put(0, len - 1);
    put(x, len);
  }
  void se(int v) { ue(v > 0 ? 2u * v - 1 : 2u * uint32_t(-v)); }
  void trailing() {  // rbsp_trailing_bits
    put(1, 1);
    if (n & 7) put(0, 8 - (n & 7));
    flush_bytes();
  }
  bool aligned() const { return (n & 7) == 0; }
  void align_zero() {
    if (n & 7) put(0, 8 - (n & 7));
  }
};

struct BitReader {
  const uint8_t* p;
  size_t nbits, pos = 0;
  BitReader(const std::string& rbsp) : p(reinterpret_cast<const uint8_t*>(rbsp.data())), nbits(rbsp.size() * 8) {}
  uint32_t peek(int len) const {  // len <= 24, zero bits past the end
    uint32_t v = 0;
    size_t byte = pos >> 3;
    const int shift = int(pos & 7);
    uint32_t w = 0;
    for (int i = 0; i < 4; ++i) w = (w << 8) | (byte + i < nbits / 8 ? p[byte + i] : 0);
    v = (w << shift) >> (32 - len);
    return v;
  }
  uint32_t u(int len) {
    if (len == 0) return 0;
    if (pos + len > nbits) throw std::runtime_error("h264: bitstream overrun");
    uint32_t v = 0;
    while (len > 16) {
      v = (v << 16) | peek(16);
      pos += 16;
      len -= 16;
    }
    v = (v << len) | peek(len);
    pos += len;
    return v;
  }
  void skip(int len) {
    if (pos + len > nbits) throw std::runtime_error("h264: bitstream overrun");
    pos += len;
  }
  uint32_t ue() {
    const uint32_t w = peek(24);
    if (w >= (1u << 12)) {                 // fewer than 12 leading zeros: the whole code is in w
      const int lz = __builtin_clz(w) - 8, len = 2 * lz + 1;
      if (pos + size_t(len) > nbits) throw std::runtime_error("h264: bitstream overrun");
      pos += size_t(len);
      return (w >> (24 - len)) - 1;
    }
    int lz = 0;
    while (u(1) == 0) {
      if (++lz > 31) throw std::runtime_error("h264: bad exp-golomb code");
    }
    return lz ? ((1u << lz) - 1 + u(lz)) : 0;
  }
  int se() {
    const uint32_t k = ue();
    return (k & 1) ? int((k + 1) >> 1) : -int(k >> 1);
  }
  bool byte_aligned() const { return (pos & 7) == 0; }
  bool more_rbsp_data() const {
    // true unless only the rbsp_stop_one_bit and alignment zeros remain
    if (pos >= nbits) return false;
    size_t last = nbits;
    while (last > 0 && !((p[(last - 1) >> 3] >> (7 - ((last - 1) & 7))) & 1)) --last;
    return last > 0 && pos < last - 1;
  }
};

void append_emulation_prevented(std::string& out, const char* p, size_t n) {
  // copy runs up to each 00 00 pair (rare in coded data), then apply the 00 00 0x -> 00 00 03 0x rule
  out.reserve(out.size() + n + n / 64 + 4);
  size_t i = 0;
  int zeros = 0;
  while (i < n) {
    if (zeros == 0) {   // fast path: jump to the next zero byte
      const void* z = std::memchr(p + i, 0, n - i);
      const size_t j = z ? size_t(static_cast<const char*>(z) - p) : n;
      out.append(p + i, j - i);
      i = j;
      if (i == n) break;
    }
    const unsigned char b = static_cast<unsigned char>(p[i]);
    if (zeros >= 2 && b <= 3) {
      out.push_back(3);
      zeros = 0;
    }
    out.push_back(char(b));
    zeros = b == 0 ? zeros + 1 : 0;
    ++i;
  }
}

std::string add_emulation_prevention(const std::string& rbsp) {
  std::string out;
  append_emulation_prevented(out, rbsp.data(), rbsp.size());
  return out;
}

std::string strip_emulation_prevention(const uint8_t* d, size_t n) {
  std::string out;
  out.reserve(n);
  int zeros = 0;
  for (size_t i = 0; i < n; ++i) {
    if (zeros >= 2 && d[i] == 3) {
      zeros = 0;
      continue;
    }
    out.push_back(char(d[i]));
    zeros = d[i] == 0 ? zeros + 1 : 0;
  }
  return out;
}

// ------------------------------------------------------------------------------------ tables
// coeff_token (Table 9-5) indexed [nC class][TotalCoeff * 4 + TrailingOnes]: code length / value
const uint8_t kCoeffTokenLen[4][68] = {
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
const uint8_t kCoeffTokenBits[4][68] = {
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
// chroma DC (nC = -1, 4:2:0), [TotalCoeff * 4 + TrailingOnes], TotalCoeff <= 4
const uint8_t kChromaDcTokenLen[20] = {2, 0, 0, 0, 6, 1, 0, 0, 6, 6, 3, 0, 6, 7, 7, 6, 6, 8, 8, 7};
const uint8_t kChromaDcTokenBits[20] = {1, 0, 0, 0, 7, 1, 0, 0, 4, 6, 1, 0, 3, 3, 2, 5, 2, 3, 2, 0};

// total_zeros for 4x4 blocks (Tables 9-7, 9-8), [TotalCoeff - 1][total_zeros]
const uint8_t kTotalZerosLen[15][16] = {
    {1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9}, {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6},
    {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6},       {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5},
    {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5},             {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6},
    {6, 5, 3, 3, 3, 2, 3, 4, 3, 6},                   {6, 4, 5, 3, 2, 2, 3, 3, 6},
    {6, 6, 4, 2, 2, 3, 2, 5},                         {5, 5, 3, 2, 2, 2, 4},
    {4, 4, 3, 3, 1, 3},                               {4, 4, 2, 1, 3},
    {3, 3, 1, 2},                                     {2, 2, 1},
    {1, 1},
};
const uint8_t kTotalZerosBits[15][16] = {
    {1, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 1}, {7, 6, 5, 4, 3, 5, 4, 3, 2, 3, 2, 3, 2, 1, 0},
    {5, 7, 6, 5, 4, 3, 4, 3, 2, 3, 2, 1, 1, 0},       {3, 7, 5, 4, 6, 5, 4, 3, 3, 2, 2, 1, 0},
    {5, 4, 3, 7, 6, 5, 4, 3, 2, 1, 1, 0},             {1, 1, 7, 6, 5, 4, 3, 2, 1, 1, 0},
    {1, 1, 5, 4, 3, 3, 2, 1, 1, 0},                   {1, 1, 1, 3, 3, 2, 2, 1, 0},
    {1, 0, 1, 3, 2, 1, 1, 1},                         {1, 0, 1, 3, 2, 1, 1},
    {0, 1, 1, 2, 1, 3},                               {0, 1, 1, 1, 1},
    {0, 1, 1, 1},                                     {0, 1, 1},
    {0, 1},
};
// total_zeros for 4:2:0 chroma DC (Table 9-9a), [TotalCoeff - 1][total_zeros]
const uint8_t kChromaDcTotalZerosLen[3][4] = {{1, 2, 3, 3}, {1, 2, 2, 0}, {1, 1, 0, 0}};
const uint8_t kChromaDcTotalZerosBits[3][4] = {{1, 1, 1, 0}, {1, 1, 0, 0}, {1, 0, 0, 0}};
// run_before (Table 9-10), [min(zerosLeft, 7) - 1][run_before]
const uint8_t kRunLen[7][15] = {
    {1, 1}, {1, 2, 2}, {2, 2, 2, 2}, {2, 2, 2, 3, 3}, {2, 2, 3, 3, 3, 3}, {2, 3, 3, 3, 3, 3, 3},
    {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11},
};
const uint8_t kRunBits[7][15] = {
    {1, 0}, {1, 1, 0}, {3, 2, 1, 0}, {3, 2, 1, 1, 0}, {3, 2, 3, 2, 1, 0}, {3, 0, 1, 3, 2, 5, 4},
    {7, 6, 5, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1},
};
// coded_block_pattern me(v) for Intra_4x4 (Table 9-4), codeNum -> cbp
const uint8_t kIntraCbp[48] = {47, 31, 15, 0,  23, 27, 29, 30, 7,  11, 13, 14, 39, 43, 45, 46,
                               16, 3,  5,  10, 12, 19, 21, 26, 28, 35, 37, 42, 44, 1,  2,  4,
                               8,  17, 18, 20, 24, 6,  9,  22, 25, 32, 33, 34, 36, 40, 38, 41};

// frame zig-zag scan: coefficient index -> raster position (row * 4 + col) in the 4x4 block
const uint8_t kZigzag[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
// luma4x4BlkIdx -> (x, y) in 4-sample units inside the macroblock
const uint8_t kBlkX[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
const uint8_t kBlkY[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};
// dequantisation normAdjust4x4 v (8.5.9) and the matching forward multipliers, [qp % 6][class]
// class: 0 = (even, even) positions, 1 = (odd, odd), 2 = mixed
const int kV[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
const int kMF[6][3] = {{13107, 5243, 8066}, {11916, 4660, 7490}, {10082, 4194, 6554},
                       {9362, 3647, 5825},  {8192, 3355, 5243}, {7282, 2893, 4559}};
const uint8_t kChromaQp[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
                               18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33,
                               34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};

inline int pos_class(int r) {
  const int i = r >> 2, j = r & 3;
  return ((i & 1) == 0 && (j & 1) == 0) ? 0 : ((i & 1) && (j & 1)) ? 1 : 2;
}
inline int level_scale(int qp6, int r) { return 16 * kV[qp6][pos_class(r)]; }  // flat weights
inline uint8_t clip255(int v) { return uint8_t(v < 0 ? 0 : v > 255 ? 255 : v); }

// ---- VLC decode lookup (code value left-aligned in `bits` bits -> (symbol, length))
struct Vlc {
  int bits = 0;
  std::vector<int16_t> sym;
  std::vector<uint8_t> len;
  void build(int maxbits, const uint8_t* lens, const uint8_t* codes, int n) {
    bits = maxbits;
    sym.assign(size_t(1) << bits, -1);
    len.assign(size_t(1) << bits, 0);
    for (int s = 0; s < n; ++s) {
      const int l = lens[s];
      if (l == 0) continue;
      const uint32_t base = uint32_t(codes[s]) << (bits - l);
      for (uint32_t k = 0; k < (1u << (bits - l)); ++k) {
        if (sym[base + k] != -1) throw std::logic_error("h264: VLC table is not prefix-free");
        sym[base + k] = int16_t(s);
        len[base + k] = uint8_t(l);
      }
    }
  }
  int read(BitReader& br) const {
    const uint32_t v = br.peek(bits);
    if (sym[v] < 0) throw std::runtime_error("h264: invalid VLC code");
    br.skip(len[v]);
    return sym[v];
  }
};

struct Tables {
  Vlc coeff_token[4], chroma_dc_token, total_zeros[15], chroma_dc_total_zeros[3], run[7];
  Tables() {
    for (int t = 0; t < 4; ++t) coeff_token[t].build(16, kCoeffTokenLen[t], kCoeffTokenBits[t], 68);
    chroma_dc_token.build(8, kChromaDcTokenLen, kChromaDcTokenBits, 20);
    for (int t = 0; t < 15; ++t) total_zeros[t].build(9, kTotalZerosLen[t], kTotalZerosBits[t], 16 - t);
    for (int t = 0; t < 3; ++t)
      chroma_dc_total_zeros[t].build(3, kChromaDcTotalZerosLen[t], kChromaDcTotalZerosBits[t], 4 - t);
    for (int t = 0; t < 7; ++t) run[t].build(11, kRunLen[t], kRunBits[t], t < 6 ? t + 2 : 15);
  }
};
const Tables& tables() {
  static const Tables t;
  return t;
}

// ------------------------------------------------------------------------------------ transforms
void fwd4x4(const int* x, int* out) {  // core transform Cf X Cf^T (exact integer)
  int t[16];
  for (int i = 0; i < 4; ++i) {  // rows
    const int* r = x + 4 * i;
    const int s03 = r[0] + r[3], d03 = r[0] - r[3], s12 = r[1] + r[2], d12 = r[1] - r[2];
    t[4 * i + 0] = s03 + s12;
    t[4 * i + 1] = 2 * d03 + d12;
    t[4 * i + 2] = s03 - s12;
    t[4 * i + 3] = d03 - 2 * d12;
  }
  for (int j = 0; j < 4; ++j) {  // columns
    const int s03 = t[j] + t[12 + j], d03 = t[j] - t[12 + j], s12 = t[4 + j] + t[8 + j], d12 = t[4 + j] - t[8 + j];
    out[j] = s03 + s12;
    out[4 + j] = 2 * d03 + d12;
    out[8 + j] = s03 - s12;
    out[12 + j] = d03 - 2 * d12;
  }
}

// 8.5.12.2: rows first (each horizontal row), then columns, r = (h + 32) >> 6
void inv4x4(const int* d, int* r) {
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

void hadamard4(const int* c, int* f) {  // H c H, H = [[1,1,1,1],[1,1,-1,-1],[1,-1,-1,1],[1,-1,1,-1]]
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

// AC / non-DC scaling (8.5.12.1), qp >= 24 shifts left (written as a multiply: the spec's << of a
// negative value is x * 2^n, which C++17 leaves undefined; >> stays the arithmetic shift)
inline int dequant(int c, int qp, int r) {
  const int ls = level_scale(qp % 6, r);
  return qp >= 24 ? c * ls * (1 << (qp / 6 - 4)) : (c * ls + (1 << (3 - qp / 6))) >> (4 - qp / 6);
}

// ------------------------------------------------------------------------------------ prediction
struct Nb {            // neighbouring samples of a block
  bool left = false, top = false, topleft = false, topright = false;
};

// Intra_16x16 (8.3.3), mode 0 V, 1 H, 2 DC, 3 plane.  pl = picture plane, stride
void pred16(const uint8_t* pl, int stride, int x0, int y0, const Nb& nb, int mode, uint8_t* out) {
  const uint8_t* top = pl + (y0 - 1) * stride + x0;
  auto L = [&](int y) { return int(pl[(y0 + y) * stride + x0 - 1]); };
  if (mode == 0) {
    for (int y = 0; y < 16; ++y) std::memcpy(out + 16 * y, top, 16);
  } else if (mode == 1) {
    for (int y = 0; y < 16; ++y) std::memset(out + 16 * y, L(y), 16);
  } else if (mode == 2) {
    int s = 0, v = 128;
    if (nb.left && nb.top) {
      for (int i = 0; i < 16; ++i) s += top[i] + L(i);
      v = (s + 16) >> 5;
    } else if (nb.left) {
      for (int i = 0; i < 16; ++i) s += L(i);
      v = (s + 8) >> 4;
    } else if (nb.top) {
      for (int i = 0; i < 16; ++i) s += top[i];
      v = (s + 8) >> 4;
    }
    std::memset(out, v, 256);
  } else {
    auto T = [&](int x) { return x < 0 ? int(pl[(y0 - 1) * stride + x0 - 1]) : int(top[x]); };
    auto Lp = [&](int y) { return y < 0 ? int(pl[(y0 - 1) * stride + x0 - 1]) : L(y); };
    int H = 0, V = 0;
    for (int i = 0; i < 8; ++i) {
      H += (i + 1) * (T(8 + i) - T(6 - i));
      V += (i + 1) * (Lp(8 + i) - Lp(6 - i));
    }
    const int a = 16 * (L(15) + T(15)), b = (5 * H + 32) >> 6, c = (5 * V + 32) >> 6;
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) out[16 * y + x] = clip255((a + b * (x - 7) + c * (y - 7) + 16) >> 5);
  }
}

// Intra chroma 8x8 for 4:2:0 (8.3.4), mode 0 DC, 1 H, 2 V, 3 plane
void pred_chroma(const uint8_t* pl, int stride, int x0, int y0, const Nb& nb, int mode, uint8_t* out) {
  const uint8_t* top = pl + (y0 - 1) * stride + x0;
  auto L = [&](int y) { return int(pl[(y0 + y) * stride + x0 - 1]); };
  if (mode == 0) {
    for (int by = 0; by < 2; ++by)
      for (int bx = 0; bx < 2; ++bx) {
        int st = 0, sl = 0;
        if (nb.top)
          for (int i = 0; i < 4; ++i) st += top[4 * bx + i];
        if (nb.left)
          for (int i = 0; i < 4; ++i) sl += L(4 * by + i);
        int v = 128;
        if ((bx == 0 && by == 0) || (bx == 1 && by == 1)) {
          if (nb.top && nb.left) v = (st + sl + 4) >> 3;
          else if (nb.left) v = (sl + 2) >> 2;
          else if (nb.top) v = (st + 2) >> 2;
        } else if (bx == 1 && by == 0) {
          if (nb.top) v = (st + 2) >> 2;
          else if (nb.left) v = (sl + 2) >> 2;
        } else {
          if (nb.left) v = (sl + 2) >> 2;
          else if (nb.top) v = (st + 2) >> 2;
        }
        for (int y = 0; y < 4; ++y) std::memset(out + 8 * (4 * by + y) + 4 * bx, v, 4);
      }
  } else if (mode == 1) {
    for (int y = 0; y < 8; ++y) std::memset(out + 8 * y, L(y), 8);
  } else if (mode == 2) {
    for (int y = 0; y < 8; ++y) std::memcpy(out + 8 * y, top, 8);
  } else {
    auto T = [&](int x) { return x < 0 ? int(pl[(y0 - 1) * stride + x0 - 1]) : int(top[x]); };
    auto Lp = [&](int y) { return y < 0 ? int(pl[(y0 - 1) * stride + x0 - 1]) : L(y); };
    int H = 0, V = 0;
    for (int i = 0; i < 4; ++i) {
      H += (i + 1) * (T(4 + i) - T(2 - i));
      V += (i + 1) * (Lp(4 + i) - Lp(2 - i));
    }
    const int a = 16 * (L(7) + T(7)), b = (34 * H + 32) >> 6, c = (34 * V + 32) >> 6;
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) out[8 * y + x] = clip255((a + b * (x - 3) + c * (y - 3) + 16) >> 5);
  }
}

// Intra_4x4 (8.3.1.2): p[-1..7, -1] in t[0..8] (t[0] = top-left), p[-1, 0..3] in l[0..3]
void pred4(const int* t, const int* l, int mode, bool has_top, bool has_left, int* out) {
  auto P = [&](int x, int y) -> int {  // p[x, y] with x or y == -1
    if (y == -1) return t[x + 1];
    return l[y];
  };
  for (int y = 0; y < 4; ++y)
    for (int x = 0; x < 4; ++x) {
      int v = 0;
      switch (mode) {
        case 0: v = P(x, -1); break;
        case 1: v = P(-1, y); break;
        case 2: {
          int s = 0;
          if (has_top && has_left) {
            for (int i = 0; i < 4; ++i) s += P(i, -1) + P(-1, i);
            v = (s + 4) >> 3;
          } else if (has_left) {
            for (int i = 0; i < 4; ++i) s += P(-1, i);
            v = (s + 2) >> 2;
          } else if (has_top) {
            for (int i = 0; i < 4; ++i) s += P(i, -1);
            v = (s + 2) >> 2;
          } else {
            v = 128;
          }
          break;
        }
        case 3:  // diagonal down left
          if (x == 3 && y == 3) v = (P(6, -1) + 3 * P(7, -1) + 2) >> 2;
          else v = (P(x + y, -1) + 2 * P(x + y + 1, -1) + P(x + y + 2, -1) + 2) >> 2;
          break;
        case 4:  // diagonal down right
          if (x > y) v = (P(x - y - 2, -1) + 2 * P(x - y - 1, -1) + P(x - y, -1) + 2) >> 2;
          else if (x < y) v = (P(-1, y - x - 2) + 2 * P(-1, y - x - 1) + P(-1, y - x) + 2) >> 2;
          else v = (P(0, -1) + 2 * P(-1, -1) + P(-1, 0) + 2) >> 2;
          break;
        case 5: {  // vertical right
          const int z = 2 * x - y;
          if (z >= 0 && !(z & 1)) v = (P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 1) >> 1;
          else if (z >= 0) v = (P(x - (y >> 1) - 2, -1) + 2 * P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 2) >> 2;
          else if (z == -1) v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2;
          else v = (P(-1, y - 1) + 2 * P(-1, y - 2) + P(-1, y - 3) + 2) >> 2;
          break;
        }
        case 6: {  // horizontal down
          const int z = 2 * y - x;
          if (z >= 0 && !(z & 1)) v = (P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 1) >> 1;
          else if (z >= 0) v = (P(-1, y - (x >> 1) - 2) + 2 * P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 2) >> 2;
          else if (z == -1) v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2;
          else v = (P(x - 1, -1) + 2 * P(x - 2, -1) + P(x - 3, -1) + 2) >> 2;
          break;
        }
        case 7:  // vertical left
          if (!(y & 1)) v = (P(x + (y >> 1), -1) + P(x + (y >> 1) + 1, -1) + 1) >> 1;
          else v = (P(x + (y >> 1), -1) + 2 * P(x + (y >> 1) + 1, -1) + P(x + (y >> 1) + 2, -1) + 2) >> 2;
          break;
        default: {  // 8: horizontal up
          const int z = x + 2 * y;
          if (z <= 4 && !(z & 1)) v = (P(-1, y + (x >> 1)) + P(-1, y + (x >> 1) + 1) + 1) >> 1;
          else if (z < 5) v = (P(-1, y + (x >> 1)) + 2 * P(-1, y + (x >> 1) + 1) + P(-1, y + (x >> 1) + 2) + 2) >> 2;
          else if (z == 5) v = (P(-1, 2) + 3 * P(-1, 3) + 2) >> 2;
          else v = P(-1, 3);
          break;
        }
      }
      out[4 * y + x] = v;
    }
}

// ------------------------------------------------------------------------------------ CAVLC
void write_block(BitWriter& bw, const int* coef, int max_num, int nC) {
  int levels[16], runs[16], tc = 0;
  // non-zero mask of the max_num (4 / 15 / 16) levels, then a reverse walk over its set bits:
  // runs[k] = zeros just below level k (the gap to the next set bit)
  uint32_t nzm = 0;
  for (int i = 0; i < max_num; ++i) nzm |= uint32_t(coef[i] != 0) << i;
  const int last = nzm ? 31 - __builtin_clz(nzm) : -1;
  for (uint32_t m = nzm; m;) {
    const int i = 31 - __builtin_clz(m);
    m &= ~(1u << i);
    levels[tc] = coef[i];
    runs[tc++] = m ? i - 1 - (31 - __builtin_clz(m)) : i;
  }
  const int total_zeros = last + 1 - tc;
  int t1 = 0;
  while (t1 < tc && t1 < 3 && (levels[t1] == 1 || levels[t1] == -1)) ++t1;
  if (nC == -1) {
    bw.put(kChromaDcTokenBits[tc * 4 + t1], kChromaDcTokenLen[tc * 4 + t1]);
  } else {
    const int t = nC < 2 ? 0 : nC < 4 ? 1 : nC < 8 ? 2 : 3;
    bw.put(kCoeffTokenBits[t][tc * 4 + t1], kCoeffTokenLen[t][tc * 4 + t1]);
  }
  if (tc == 0) return;
  uint32_t signs = 0;
  for (int k = 0; k < t1; ++k) signs = (signs << 1) | uint32_t(levels[k] < 0);
  bw.put(signs, t1);
  int sl = (tc > 10 && t1 < 3) ? 1 : 0;
  for (int k = t1; k < tc; ++k) {
    const int lv = levels[k];
    int code = lv > 0 ? 2 * lv - 2 : -2 * lv - 1;
    if (k == t1 && t1 < 3) code -= 2;
    // level_prefix (leading zeros + 1) and level_suffix written as one field
    if (sl == 0) {
      if (code < 14) {
        bw.put(1, code + 1);
      } else if (code < 30) {
        bw.put(16 | uint32_t(code - 14), 19);
      } else {
        if (code - 30 >= 4096) throw std::logic_error("h264: level out of range");
        bw.put(4096 | uint32_t(code - 30), 28);
      }
    } else {
      if (code < (15 << sl)) {
        bw.put((1u << sl) | uint32_t(code & ((1 << sl) - 1)), (code >> sl) + 1 + sl);
      } else {
        if (code - (15 << sl) >= 4096) throw std::logic_error("h264: level out of range");
        bw.put(4096 | uint32_t(code - (15 << sl)), 28);
      }
    }
    if (sl == 0) sl = 1;
    if ((lv < 0 ? -lv : lv) > (3 << (sl - 1)) && sl < 6) ++sl;
  }
  if (tc < max_num) {
    if (nC == -1) bw.put(kChromaDcTotalZerosBits[tc - 1][total_zeros], kChromaDcTotalZerosLen[tc - 1][total_zeros]);
    else bw.put(kTotalZerosBits[tc - 1][total_zeros], kTotalZerosLen[tc - 1][total_zeros]);
  }
  int zl = total_zeros;
  for (int k = 0; k < tc - 1 && zl > 0; ++k) {
    const int t = std::min(zl, 7) - 1;
    bw.put(kRunBits[t][runs[k]], kRunLen[t][runs[k]]);
    zl -= runs[k];
  }
}

// returns TotalCoeff; coef[0..max_num) filled (zeros elsewhere)
int read_block(BitReader& br, int* coef, int max_num, int nC) {
  const Tables& T = tables();
  for (int i = 0; i < max_num; ++i) coef[i] = 0;
  int sym;
  if (nC == -1) sym = T.chroma_dc_token.read(br);
  else sym = T.coeff_token[nC < 2 ? 0 : nC < 4 ? 1 : nC < 8 ? 2 : 3].read(br);
  const int tc = sym >> 2, t1 = sym & 3;
  if (tc == 0) return 0;
  if (tc > max_num) throw std::runtime_error("h264: TotalCoeff exceeds block size");
  int levels[16];
  for (int k = 0; k < t1; ++k) levels[k] = br.u(1) ? -1 : 1;
  int sl = (tc > 10 && t1 < 3) ? 1 : 0;
  for (int k = t1; k < tc; ++k) {
    int prefix = 0;
    while (br.u(1) == 0) {
      if (++prefix > 24) throw std::runtime_error("h264: bad level_prefix");
    }
    const int ssize = (prefix == 14 && sl == 0) ? 4 : prefix >= 15 ? prefix - 3 : sl;
    int code = (std::min(15, prefix) << sl) + (ssize ? int(br.u(ssize)) : 0);
    if (prefix >= 15 && sl == 0) code += 15;
    if (prefix >= 16) code += (1 << (prefix - 3)) - 4096;
    if (k == t1 && t1 < 3) code += 2;
    const int lv = (code & 1) ? (-code - 1) >> 1 : (code + 2) >> 1;
    levels[k] = lv;
    if (sl == 0) sl = 1;
    if ((lv < 0 ? -lv : lv) > (3 << (sl - 1)) && sl < 6) ++sl;
  }
  int tz = 0;
  if (tc < max_num) tz = nC == -1 ? T.chroma_dc_total_zeros[tc - 1].read(br) : T.total_zeros[tc - 1].read(br);
  if (tz + tc > max_num) throw std::runtime_error("h264: total_zeros out of range");
  int idx = tz + tc - 1, zl = tz;
  for (int k = 0; k < tc; ++k) {
    int run = 0;
    if (k < tc - 1 && zl > 0) run = T.run[std::min(zl, 7) - 1].read(br);
    else if (k == tc - 1) run = zl;
    if (run > zl) throw std::runtime_error("h264: run_before out of range");
    coef[idx] = levels[k];
    idx -= 1 + run;
    zl -= run;
  }
  return tc;
}

// ------------------------------------------------------------------------------------ picture state
struct Frame {
  int mbw, mbh, W, H;
  std::vector<uint8_t> y, cb, cr;
  std::vector<uint8_t> tc_y, tc_cb, tc_cr;   // TotalCoeff per 4x4 block (nC prediction, deblocking bS 2)
  std::vector<int> slice;                    // slice id per macroblock (-1: not decoded yet)
  std::vector<int8_t> i4mode;                // Intra4x4PredMode per 4x4 block, -1 = not I_NxN
  // inter state per 4x4 luma block: motion vector (quarter samples), ref_idx (-1: intra / none)
  // and the identity of the reference picture (deblocking compares pictures, not indices)
  std::vector<int16_t> mvx, mvy;
  std::vector<int8_t> ref;
  std::vector<int> refpic;
  std::vector<uint8_t> intra, mbqp;          // per macroblock: intra flag, QP_Y (0 for I_PCM)
  bool constrained_intra = false;            // PPS constrained_intra_pred_flag
  Frame(int mbw_, int mbh_) : mbw(mbw_), mbh(mbh_), W(16 * mbw_), H(16 * mbh_) {
    y.assign(size_t(W) * H, 0);
    cb.assign(size_t(W / 2) * (H / 2), 0);
    cr.assign(cb.size(), 0);
    tc_y.assign(size_t(4 * mbw) * 4 * mbh, 0);
    tc_cb.assign(size_t(2 * mbw) * 2 * mbh, 0);
    tc_cr.assign(tc_cb.size(), 0);
    slice.assign(size_t(mbw) * mbh, -1);
    i4mode.assign(tc_y.size(), -1);
    mvx.assign(tc_y.size(), 0);
    mvy.assign(tc_y.size(), 0);
    ref.assign(tc_y.size(), -1);
    refpic.assign(tc_y.size(), -1);
    intra.assign(size_t(mbw) * mbh, 1);
    mbqp.assign(size_t(mbw) * mbh, 0);
  }
  bool avail(int mx, int my, int cur_slice) const {
    return mx >= 0 && my >= 0 && mx < mbw && my < mbh && slice[size_t(my) * mbw + mx] == cur_slice;
  }
  // neighbour availability for INTRA prediction: with constrained_intra_pred, inter neighbours
  // do not count (8.3.1.2 / 8.3.3 / 8.3.4)
  bool avail_intra(int mx, int my, int cur_slice) const {
    return avail(mx, my, cur_slice) && (!constrained_intra || intra[size_t(my) * mbw + mx]);
  }
  Nb nb(int mx, int my, int s) const {
    Nb n;
    n.left = avail_intra(mx - 1, my, s);
    n.top = avail_intra(mx, my - 1, s);
    n.topleft = avail_intra(mx - 1, my - 1, s);
    n.topright = avail_intra(mx + 1, my - 1, s);
    return n;
  }
  // nC for a 4x4 block at (bx, by) in block units of a plane with `per` blocks per MB side
  int nc(const std::vector<uint8_t>& tcs, int bx, int by, int per, int s) const {
    const int stride = per * mbw;
    const bool a = bx % per ? true : avail(bx / per - 1, by / per, s);
    const bool b = by % per ? true : avail(bx / per, by / per - 1, s);
    const int na = a ? tcs[size_t(by) * stride + bx - 1] : 0, nb_ = b ? tcs[size_t(by - 1) * stride + bx] : 0;
    if (a && b) return (na + nb_ + 1) >> 1;
    return a ? na : b ? nb_ : 0;
  }
};

// Reconstruction of an Intra_16x16 macroblock from its levels (normative, shared enc/dec).
// dc: 16 levels in scan order; ac[blk][0..14]: levels of scan positions 1..15 (blkIdx order)
// AC dequantisation of one QP as a table: dequant(c, qp, r) == (c * mul[r] + add) >> sh (qp >= 24:
// c * ls * 2^n == c * (ls << n), add = sh = 0) - the same integers, without the per-coefficient
// position class / qp split.
struct AcDequant {
  int mul[16], add, sh;
  explicit AcDequant(int qp) {
    const int q6 = qp / 6;
    for (int r = 0; r < 16; ++r) mul[r] = qp >= 24 ? level_scale(qp % 6, r) * (1 << (q6 - 4)) : level_scale(qp % 6, r);
    add = qp >= 24 ? 0 : 1 << (3 - q6);
    sh = qp >= 24 ? 0 : 4 - q6;
  }
  int operator()(int c, int r) const { return (c * mul[r] + add) >> sh; }
};

// Residual of one 4x4 block into an n x n int16 residual plane (saturated to int16: pred + r is
// clipped to [0, 255] afterwards, and any |r| beyond the int16 range clips to the same 0 / 255).
// A block whose only non-zero coefficient is the DC has the constant residual (d0 + 32) >> 6
// (inv4x4's rows and columns pass d0 through unchanged).
inline int16_t sat16(int v) { return int16_t(v < -32768 ? -32768 : v > 32767 ? 32767 : v); }
inline void put_residual(int16_t* rs, int n, int bx, int by, int* d, bool any_ac) {
  int16_t* o = rs + n * 4 * by + 4 * bx;
  if (!any_ac) {
    const int16_t v = sat16((d[0] + 32) >> 6);
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) o[n * y + x] = v;
    return;
  }
  int r[16];
  inv4x4(d, r);
  for (int y = 0; y < 4; ++y)
    for (int x = 0; x < 4; ++x) o[n * y + x] = sat16(r[4 * y + x]);
}
// dst = clip255(pred + rs) over a 16 x 16 (n = 16) or 8 x 8 (n = 8) block: saturating int16 adds
// and an unsigned-saturating pack, the same values as the scalar clip.
inline void add_residual(uint8_t* dst, int dstride, const uint8_t* pred, const int16_t* rs, int n) {
  const __m128i z = _mm_setzero_si128();
  for (int y = 0; y < n; ++y) {
    const int16_t* r = rs + n * y;
    if (n == 16) {
      const __m128i p = _mm_loadu_si128(reinterpret_cast<const __m128i*>(pred + 16 * y));
      const __m128i r0 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(r));
      const __m128i r1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(r + 8));
      const __m128i lo = _mm_adds_epi16(_mm_unpacklo_epi8(p, z), r0);
      const __m128i hi = _mm_adds_epi16(_mm_unpackhi_epi8(p, z), r1);
      _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + size_t(y) * dstride), _mm_packus_epi16(lo, hi));
    } else {
      const __m128i p = _mm_loadl_epi64(reinterpret_cast<const __m128i*>(pred + 8 * y));
      const __m128i lo = _mm_adds_epi16(_mm_unpacklo_epi8(p, z), _mm_loadu_si128(reinterpret_cast<const __m128i*>(r)));
      _mm_storel_epi64(reinterpret_cast<__m128i*>(dst + size_t(y) * dstride), _mm_packus_epi16(lo, lo));
    }
  }
}

void recon_luma16(Frame& f, int mx, int my, const uint8_t* pred, const int* dc, const int (*ac)[15], int qp) {
  int c[16], fdc[16];
  for (int k = 0; k < 16; ++k) c[kZigzag[k]] = dc[k];
  hadamard4(c, fdc);
  const int ls = level_scale(qp % 6, 0);
  const AcDequant dq(qp);
  alignas(16) int16_t rs[256];
  for (int blk = 0; blk < 16; ++blk) {
    const int bx = kBlkX[blk], by = kBlkY[blk];
    const int fv = fdc[4 * by + bx];
    int d[16] = {0};
    d[0] = qp >= 36 ? fv * ls * (1 << (qp / 6 - 6)) : (fv * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    int any = 0;   // a zero level dequantises to 0 ((0 * mul + add) >> sh, add < 2^sh): no branch
    for (int k = 0; k < 15; ++k) {
      const int rp = kZigzag[k + 1];
      d[rp] = dq(ac[blk][k], rp);
      any |= ac[blk][k];
    }
    put_residual(rs, 16, bx, by, d, any != 0);
  }
  add_residual(f.y.data() + size_t(my * 16) * f.W + mx * 16, f.W, pred, rs, 16);
}

// chroma component: dc[4] raster (blkIdx) order, ac[4][15]
void recon_chroma(std::vector<uint8_t>& pl, int Wc, int mx, int my, const uint8_t* pred, const int* dc,
                  const int (*ac)[15], int qpc) {
  const int f0 = dc[0] + dc[1] + dc[2] + dc[3], f1 = dc[0] - dc[1] + dc[2] - dc[3];
  const int f2 = dc[0] + dc[1] - dc[2] - dc[3], f3 = dc[0] - dc[1] - dc[2] + dc[3];
  const int fv[4] = {f0, f1, f2, f3};
  const int ls = level_scale(qpc % 6, 0);
  const AcDequant dq(qpc);
  alignas(16) int16_t rs[64];
  for (int blk = 0; blk < 4; ++blk) {
    const int bx = blk & 1, by = blk >> 1;
    int d[16] = {0};
    d[0] = (fv[blk] * ls * (1 << (qpc / 6))) >> 5;
    int any = 0;
    for (int k = 0; k < 15; ++k) {
      const int rp = kZigzag[k + 1];
      d[rp] = dq(ac[blk][k], rp);
      any |= ac[blk][k];
    }
    put_residual(rs, 8, bx, by, d, any != 0);
  }
  add_residual(pl.data() + size_t(my * 8) * Wc + mx * 8, Wc, pred, rs, 8);
}

// ------------------------------------------------------------------------------------ inter (P) tools
// coded_block_pattern me(v) for Inter macroblocks (Table 9-4), codeNum -> cbp
const uint8_t kInterCbp[48] = {0,  16, 1,  2,  4,  8,  32, 3,  5,  10, 12, 15, 47, 7,  11, 13,
                               14, 6,  9,  31, 35, 37, 42, 44, 33, 34, 36, 40, 39, 43, 45, 46,
                               17, 18, 20, 24, 19, 21, 26, 28, 23, 27, 29, 30, 22, 25, 38, 41};

inline int tap6(int a, int b, int c, int d, int e, int f) { return a - 5 * b + 20 * c + 20 * d - 5 * e + f; }

// Luma inter prediction (8.4.2.2.1) of a w x h block whose top-left integer position is (x0, y0),
// motion vector (mvx, mvy) in quarter samples; reference samples outside the picture are the
// nearest edge sample.  The half-sample values b / h / j come from the unclipped 6-tap sums of a
// (w + 5) x (h + 5) window; quarter samples average the two nearest (8-251..8-261).
void mc_luma(const Frame& r, int x0, int y0, int mvx, int mvy, int w, int h, uint8_t* out, int ostride) {
  const int xi = x0 + (mvx >> 2), yi = y0 + (mvy >> 2), xf = mvx & 3, yf = mvy & 3;
  if (xf == 0 && yf == 0) {                         // full-sample vector: a (clamped) copy
    if (xi >= 0 && yi >= 0 && xi + w <= r.W && yi + h <= r.H) {
      for (int j = 0; j < h; ++j) std::memcpy(out + j * ostride, r.y.data() + size_t(yi + j) * r.W + xi, size_t(w));
    } else {
      for (int j = 0; j < h; ++j) {
        const uint8_t* row = r.y.data() + size_t(std::clamp(yi + j, 0, r.H - 1)) * r.W;
        for (int i = 0; i < w; ++i) out[j * ostride + i] = row[std::clamp(xi + i, 0, r.W - 1)];
      }
    }
    return;
  }
  int win[21][22];                                  // rows yi-2 .. yi+h+2, cols xi-2 .. xi+w+3
  if (xi - 2 >= 0 && yi - 2 >= 0 && xi + w + 3 < r.W && yi + h + 2 < r.H) {
    for (int j = 0; j < h + 5; ++j) {
      const uint8_t* row = r.y.data() + size_t(yi - 2 + j) * r.W + xi - 2;
      for (int i = 0; i < w + 6; ++i) win[j][i] = row[i];
    }
  } else {
    for (int j = 0; j < h + 5; ++j) {
      const uint8_t* row = r.y.data() + size_t(std::clamp(yi - 2 + j, 0, r.H - 1)) * r.W;
      for (int i = 0; i < w + 6; ++i) win[j][i] = row[std::clamp(xi - 2 + i, 0, r.W - 1)];
    }
  }
  const int cs = yf * 4 + xf;
  const bool use_b = cs == 1 || cs == 2 || cs == 3 || cs == 5 || cs == 6 || cs == 7 || cs >= 13;
  const bool use_j = cs == 6 || cs == 9 || cs == 10 || cs == 11 || cs == 14;
  const bool use_h =
      cs == 4 || cs == 5 || cs == 7 || cs == 8 || cs == 9 || cs == 11 || cs == 12 || cs == 13 || cs == 15;
  auto clip = [](int v) { return v < 0 ? 0 : v > 255 ? 255 : v; };
  // b1[j][i]: unclipped horizontal half sample (i + 1/2, j - 2) for window rows j = 0 .. h+4
  int b1[21][16], bq[17][16], hq[16][17], jq[16][16];
  if (use_b || use_j) {
    const int j0 = use_j ? 0 : 2, j1 = use_j ? h + 5 : h + 3;
    for (int j = j0; j < j1; ++j)
      for (int i = 0; i < w; ++i)
        b1[j][i] = tap6(win[j][i], win[j][i + 1], win[j][i + 2], win[j][i + 3], win[j][i + 4], win[j][i + 5]);
    for (int j = 0; j <= h; ++j)                    // b at rows 0 .. h (row h: the "s" samples below)
      for (int i = 0; i < w; ++i) bq[j][i] = clip((b1[j + 2][i] + 16) >> 5);
  }
  if (use_h)
    for (int j = 0; j < h; ++j)                     // h at cols 0 .. w (col w: the "m" samples right)
      for (int i = 0; i <= w; ++i)
        hq[j][i] = clip((tap6(win[j][i + 2], win[j + 1][i + 2], win[j + 2][i + 2], win[j + 3][i + 2], win[j + 4][i + 2],
                              win[j + 5][i + 2]) + 16) >> 5);
  if (use_j)
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i)
        jq[j][i] =
            clip((tap6(b1[j][i], b1[j + 1][i], b1[j + 2][i], b1[j + 3][i], b1[j + 4][i], b1[j + 5][i]) + 512) >> 10);
  auto G = [&](int i, int j) { return win[j + 2][i + 2]; };
  auto run = [&](auto fn) {
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i) out[j * ostride + i] = uint8_t(fn(i, j));
  };
  switch (cs) {
    case 1: run([&](int i, int j) { return (G(i, j) + bq[j][i] + 1) >> 1; }); break;            // a
    case 2: run([&](int i, int j) { return bq[j][i]; }); break;                                   // b
    case 3: run([&](int i, int j) { return (G(i + 1, j) + bq[j][i] + 1) >> 1; }); break;        // c
    case 4: run([&](int i, int j) { return (G(i, j) + hq[j][i] + 1) >> 1; }); break;            // d
    case 5: run([&](int i, int j) { return (bq[j][i] + hq[j][i] + 1) >> 1; }); break;           // e
    case 6: run([&](int i, int j) { return (bq[j][i] + jq[j][i] + 1) >> 1; }); break;           // f
    case 7: run([&](int i, int j) { return (bq[j][i] + hq[j][i + 1] + 1) >> 1; }); break;       // g
    case 8: run([&](int i, int j) { return hq[j][i]; }); break;                                   // h
    case 9: run([&](int i, int j) { return (hq[j][i] + jq[j][i] + 1) >> 1; }); break;           // i
    case 10: run([&](int i, int j) { return jq[j][i]; }); break;                                  // j
    case 11: run([&](int i, int j) { return (jq[j][i] + hq[j][i + 1] + 1) >> 1; }); break;      // k
    case 12: run([&](int i, int j) { return (G(i, j + 1) + hq[j][i] + 1) >> 1; }); break;       // n
    case 13: run([&](int i, int j) { return (hq[j][i] + bq[j + 1][i] + 1) >> 1; }); break;      // p
    case 14: run([&](int i, int j) { return (jq[j][i] + bq[j + 1][i] + 1) >> 1; }); break;      // q
    default: run([&](int i, int j) { return (hq[j][i + 1] + bq[j + 1][i] + 1) >> 1; }); break; // r
  }
}

// Chroma inter prediction (8.4.2.2.2), 4:2:0 frame: eighth-sample bilinear, vector = the luma one
void mc_chroma(const std::vector<uint8_t>& pl, int Wc, int Hc, int x0, int y0, int mvx, int mvy, int w, int h,
               uint8_t* out, int ostride) {
  const int xi = x0 + (mvx >> 3), yi = y0 + (mvy >> 3), xf = mvx & 7, yf = mvy & 7;
  auto P = [&](int x, int y) { return int(pl[size_t(std::clamp(y, 0, Hc - 1)) * Wc + std::clamp(x, 0, Wc - 1)]); };
  for (int j = 0; j < h; ++j)
    for (int i = 0; i < w; ++i) {
      const int x = xi + i, y = yi + j;
      out[j * ostride + i] = uint8_t(((8 - xf) * (8 - yf) * P(x, y) + xf * (8 - yf) * P(x + 1, y) +
                                      (8 - xf) * yf * P(x, y + 1) + xf * yf * P(x + 1, y + 1) + 32) >> 6);
    }
}

// Motion vector prediction (8.4.1.3) inside macroblock (mx, my).  `done` marks the 4x4 blocks of the
// current macroblock whose motion is already known (partitions decoded earlier in the macroblock).
struct MvPred {
  const Frame& f;
  int mx, my, slice;
  uint16_t done = 0;
  struct N {
    bool avail;
    int ref, x, y;
  };
  N at(int bx, int by) const {            // 4x4 block (bx, by) in MB-relative 4x4 units
    N n{false, -1, 0, 0};
    if (bx >= 0 && bx < 4 && by >= 0 && by < 4) {
      if (!(done >> (by * 4 + bx) & 1)) return n;
    } else {
      const int nmx = mx + (bx < 0 ? -1 : bx > 3 ? 1 : 0), nmy = my + (by < 0 ? -1 : by > 3 ? 1 : 0);
      if (by >= 0 && by < 4 && bx > 3) return n;             // right neighbour: not decoded yet
      if (by > 3) return n;
      if (!f.avail(nmx, nmy, slice)) return n;
    }
    const int gx = 4 * mx + bx, gy = 4 * my + by;
    const size_t i = size_t(gy) * 4 * f.mbw + gx;
    n.avail = true;
    n.ref = f.ref[i];
    if (n.ref >= 0) {
      n.x = f.mvx[i];
      n.y = f.mvy[i];
    }
    return n;
  }
  static int med(int a, int b, int c) { return std::max(std::min(a, b), std::min(std::max(a, b), c)); }
  // shape: 0 generic, 1 16x8 upper, 2 16x8 lower, 3 8x16 left, 4 8x16 right
  void pred(int bx, int by, int bw, int ref, int shape, int& px, int& py) const {
    N A = at(bx - 1, by), Bn = at(bx, by - 1), C = at(bx + bw, by - 1);
    if (!C.avail) C = at(bx - 1, by - 1);
    if (shape == 1 && Bn.ref == ref) { px = Bn.x; py = Bn.y; return; }
    if (shape == 2 && A.ref == ref) { px = A.x; py = A.y; return; }
    if (shape == 3 && A.ref == ref) { px = A.x; py = A.y; return; }
    if (shape == 4 && C.ref == ref) { px = C.x; py = C.y; return; }
    if (!Bn.avail && !C.avail && A.avail) Bn = C = A;
    const int m = (A.ref == ref) + (Bn.ref == ref) + (C.ref == ref);
    if (m == 1) {
      const N& s = A.ref == ref ? A : Bn.ref == ref ? Bn : C;
      px = s.x;
      py = s.y;
      return;
    }
    px = med(A.x, Bn.x, C.x);
    py = med(A.y, Bn.y, C.y);
  }
  void skip(int& px, int& py) const {    // P_Skip (8.4.1.1)
    const N A = at(-1, 0), Bn = at(0, -1);
    if (!A.avail || !Bn.avail || (A.ref == 0 && A.x == 0 && A.y == 0) || (Bn.ref == 0 && Bn.x == 0 && Bn.y == 0)) {
      px = py = 0;
      return;
    }
    pred(0, 0, 4, 0, 0, px, py);
  }
};

// Assign one (sub-)partition's motion (4x4-block rectangle) and mark it known for later predictions
inline void set_motion(Frame& f, MvPred& mp, int mx, int my, int bx, int by, int bw, int bh, int ref, int refpic,
                       int mvx, int mvy) {
  for (int y = by; y < by + bh; ++y)
    for (int x = bx; x < bx + bw; ++x) {
      const size_t i = size_t(4 * my + y) * 4 * f.mbw + 4 * mx + x;
      f.ref[i] = int8_t(ref);
      f.refpic[i] = refpic;
      f.mvx[i] = int16_t(mvx);
      f.mvy[i] = int16_t(mvy);
      mp.done |= uint16_t(1u << (y * 4 + x));
    }
}

// Residual of an inter / Intra_4x4-style macroblock: coef[blk][16] in scan order (blkIdx order)
void recon_luma4x4(Frame& f, int mx, int my, const uint8_t* pred, const int (*coef)[16], int qp) {
  for (int blk = 0; blk < 16; ++blk) {
    const int bx = kBlkX[blk], by = kBlkY[blk];
    int d[16] = {0}, r[16] = {0};
    bool any = false;
    for (int k = 0; k < 16; ++k)
      if (coef[blk][k]) {
        const int rp = kZigzag[k];
        d[rp] = dequant(coef[blk][k], qp, rp);
        any = true;
      }
    if (any) inv4x4(d, r);
    uint8_t* dst = f.y.data() + size_t(my * 16 + 4 * by) * f.W + mx * 16 + 4 * bx;
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) dst[y * f.W + x] = clip255(pred[16 * (4 * by + y) + 4 * bx + x] + r[4 * y + x]);
  }
}

// ------------------------------------------------------------------------------------ deblocking (8.7)
const uint8_t kAlpha[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,   0,   0,   0,   4,   4,
                            5,  6,  7,  8,  9,  10, 12, 13, 15, 17, 20, 22,  25,  28,  32,  36,  40,  45,
                            50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
const uint8_t kBeta[52] = {0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  0,  0,  2,  2,
                           2, 3, 3, 3, 3, 4, 4, 4, 6,  6,  7,  7,  8,  8,  9,  9,  10, 10,
                           11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
const uint8_t kTc0[52][3] = {
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 1},
    {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1},
    {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 2, 3}, {1, 2, 3}, {2, 2, 3}, {2, 2, 4}, {2, 3, 4},
    {2, 3, 4}, {3, 3, 5}, {3, 4, 6}, {3, 4, 6}, {4, 5, 7}, {4, 5, 8}, {4, 6, 9}, {5, 7, 10}, {6, 8, 11},
    {6, 8, 13}, {7, 10, 14}, {8, 11, 16}, {9, 12, 18}, {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

struct SliceDb {           // per-slice deblocking controls
  int idc = 1, offa = 0, offb = 0;
};

// one edge position: p[i] = *(p0 - i * step) (i = 0..3), q[i] = *(q0 + i * step)
inline void filter_px(uint8_t* q0, int step, int bS, int alpha, int beta, int tc0, bool luma) {
  const int p0 = q0[-step], p1 = q0[-2 * step], q0v = q0[0], q1 = q0[step];
  if (!(std::abs(p0 - q0v) < alpha && std::abs(p1 - p0) < beta && std::abs(q1 - q0v) < beta)) return;
  if (bS < 4) {
    int tc = tc0;
    int ap = 0, aq = 0, p2 = 0, q2 = 0;
    if (luma) {
      p2 = q0[-3 * step];
      q2 = q0[2 * step];
      ap = std::abs(p2 - p0);
      aq = std::abs(q2 - q0v);
      tc += (ap < beta) + (aq < beta);
    } else {
      tc += 1;
    }
    const int delta = std::clamp((((q0v - p0) * 4) + (p1 - q1) + 4) >> 3, -tc, tc);
    q0[-step] = clip255(p0 + delta);
    q0[0] = clip255(q0v - delta);
    if (luma) {
      if (ap < beta) q0[-2 * step] = uint8_t(p1 + std::clamp((p2 + ((p0 + q0v + 1) >> 1) - (p1 * 2)) >> 1, -tc0, tc0));
      if (aq < beta) q0[step] = uint8_t(q1 + std::clamp((q2 + ((p0 + q0v + 1) >> 1) - (q1 * 2)) >> 1, -tc0, tc0));
    }
    return;
  }
  if (!luma) {
    q0[-step] = uint8_t((2 * p1 + p0 + q1 + 2) >> 2);
    q0[0] = uint8_t((2 * q1 + q0v + p1 + 2) >> 2);
    return;
  }
  const int p2 = q0[-3 * step], p3 = q0[-4 * step], q2 = q0[2 * step], q3 = q0[3 * step];
  const int ap = std::abs(p2 - p0), aq = std::abs(q2 - q0v);
  const bool strong = std::abs(p0 - q0v) < ((alpha >> 2) + 2);
  if (ap < beta && strong) {
    q0[-step] = uint8_t((p2 + 2 * p1 + 2 * p0 + 2 * q0v + q1 + 4) >> 3);
    q0[-2 * step] = uint8_t((p2 + p1 + p0 + q0v + 2) >> 2);
    q0[-3 * step] = uint8_t((2 * p3 + 3 * p2 + p1 + p0 + q0v + 4) >> 3);
  } else {
    q0[-step] = uint8_t((2 * p1 + p0 + q1 + 2) >> 2);
  }
  if (aq < beta && strong) {
    q0[0] = uint8_t((p1 + 2 * p0 + 2 * q0v + 2 * q1 + q2 + 4) >> 3);
    q0[step] = uint8_t((p0 + q0v + q1 + q2 + 2) >> 2);
    q0[2 * step] = uint8_t((2 * q3 + 3 * q2 + q1 + q0v + p0 + 4) >> 3);
  } else {
    q0[0] = uint8_t((2 * q1 + q0v + p1 + 2) >> 2);
  }
}

// boundary strength between 4x4 luma blocks p and q (absolute 4x4 coordinates)
inline int bs_of(const Frame& f, int pbx, int pby, int qbx, int qby, bool mb_edge) {
  const int pm = (pby / 4) * f.mbw + pbx / 4, qm = (qby / 4) * f.mbw + qbx / 4;
  if (f.intra[pm] || f.intra[qm]) return mb_edge ? 4 : 3;
  const size_t pi = size_t(pby) * 4 * f.mbw + pbx, qi = size_t(qby) * 4 * f.mbw + qbx;
  if (f.tc_y[pi] || f.tc_y[qi]) return 2;
  if (f.refpic[pi] != f.refpic[qi] || std::abs(f.mvx[pi] - f.mvx[qi]) >= 4 || std::abs(f.mvy[pi] - f.mvy[qi]) >= 4)
    return 1;
  return 0;
}

// The in-loop deblocking filter over a whole decoded picture, macroblocks in raster order (luma,
// then chroma; vertical edges, then horizontal ones), on the unfiltered reconstruction.
void deblock(Frame& f, const std::vector<SliceDb>& sl, int chroma_qp_offset, int threads) {
  const int Wc = f.W / 2;
  auto filter_mb = [&](int mx, int my) {
      const int mb = my * f.mbw + mx, sid = f.slice[mb];
      const SliceDb& d = sl[sid];
      if (d.idc == 1) return;
      const bool left = mx > 0 && (d.idc != 2 || f.slice[mb - 1] == sid);
      const bool top = my > 0 && (d.idc != 2 || f.slice[mb - f.mbw] == sid);
      for (int dir = 0; dir < 2; ++dir) {                   // 0: vertical edges, 1: horizontal edges
        for (int e = 0; e < 4; ++e) {
          if (e == 0 && !(dir == 0 ? left : top)) continue;
          int bS[4];
          bool any = false;
          for (int k = 0; k < 4; ++k) {
            const int qbx = 4 * mx + (dir == 0 ? e : k), qby = 4 * my + (dir == 0 ? k : e);
            const int pbx = dir == 0 ? qbx - 1 : qbx, pby = dir == 0 ? qby : qby - 1;
            bS[k] = bs_of(f, pbx, pby, qbx, qby, e == 0);
            any |= bS[k] != 0;
          }
          if (!any) continue;
          const int pmb = e == 0 ? (dir == 0 ? mb - 1 : mb - f.mbw) : mb;
          const int qpav = (f.mbqp[pmb] + f.mbqp[mb] + 1) >> 1;
          const int ia = std::clamp(qpav + d.offa, 0, 51), ib = std::clamp(qpav + d.offb, 0, 51);
          const int alpha = kAlpha[ia], beta = kBeta[ib];
          // luma: 16 samples along the edge
          for (int k = 0; k < 16; ++k) {
            const int bsk = bS[k / 4];
            if (!bsk) continue;
            const int x = 16 * mx + (dir == 0 ? 4 * e : k), y = 16 * my + (dir == 0 ? k : 4 * e);
            filter_px(f.y.data() + size_t(y) * f.W + x, dir == 0 ? 1 : f.W, bsk, alpha, beta,
                      bsk < 4 ? kTc0[ia][bsk - 1] : 0, true);
          }
          // chroma: the luma edges 0 and 8 map to chroma edges 0 and 4
          if (e & 1) continue;
          const int qpp = kChromaQp[std::clamp(f.mbqp[pmb] + chroma_qp_offset, 0, 51)];
          const int qpq = kChromaQp[std::clamp(f.mbqp[mb] + chroma_qp_offset, 0, 51)];
          const int qpc = (qpp + qpq + 1) >> 1;
          const int ca = std::clamp(qpc + d.offa, 0, 51), cbb = std::clamp(qpc + d.offb, 0, 51);
          for (std::vector<uint8_t>* pl : {&f.cb, &f.cr})
            for (int k = 0; k < 8; ++k) {
              const int bsk = bS[k / 2];
              if (!bsk) continue;
              const int x = 8 * mx + (dir == 0 ? 2 * e : k), y = 8 * my + (dir == 0 ? k : 2 * e);
              filter_px(pl->data() + size_t(y) * Wc + x, dir == 0 ? 1 : Wc, bsk, kAlpha[ca], kBeta[cbb],
                        bsk < 4 ? kTc0[ca][bsk - 1] : 0, false);
            }
        }
      }
  };
  // Raster order, or a wavefront over macroblock rows: a macroblock's edges touch samples that the
  // macroblocks left of it and up to one column right of it in the row above filter first, so
  // row y may filter column x once row y-1 has finished column x+1 - the same result as raster order.
  if (threads <= 1 || f.mbh < 2) {
    for (int my = 0; my < f.mbh; ++my)
      for (int mx = 0; mx < f.mbw; ++mx) filter_mb(mx, my);
    return;
  }
  std::vector<std::atomic<int>> progress(static_cast<size_t>(f.mbh));
  for (auto& a : progress) a.store(0);
  const int nt = std::min(threads, f.mbh);
  auto worker = [&](int t) {
    for (int my = t; my < f.mbh; my += nt)
      for (int mx = 0; mx < f.mbw; ++mx) {
        if (my > 0) {
          const int need = std::min(f.mbw, mx + 2);
          while (progress[size_t(my - 1)].load(std::memory_order_acquire) < need) std::this_thread::yield();
        }
        filter_mb(mx, my);
        progress[size_t(my)].store(mx + 1, std::memory_order_release);
      }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(worker, t);
  worker(0);
  for (auto& th : pool) th.join();
}

struct RefPic {                   // a decoded, deblocked picture in the DPB
  std::shared_ptr<const Frame> f;
  int id = -1, frame_num = 0;
};

// RefPicList0 of a P slice (8.2.4.2.1 + 8.2.4.3.1): short-term references by descending PicNum,
// then the modifications, truncated to num_ref_idx_l0_active (missing entries stay empty)
std::vector<RefPic> ref_list0(const std::vector<RefPic>& dpb, int cur, int max_fn,
                              const std::vector<std::pair<int, int>>& mods, int n_active) {
  auto picnum = [&](const RefPic& r) { return r.frame_num > cur ? r.frame_num - max_fn : r.frame_num; };
  std::vector<RefPic> list = dpb;
  std::stable_sort(list.begin(), list.end(), [&](const RefPic& a, const RefPic& b) { return picnum(a) > picnum(b); });
  int pred = cur;
  for (size_t m = 0; m < mods.size(); ++m) {
    const int diff = mods[m].second + 1;
    int nowrap = mods[m].first == 0 ? pred - diff : pred + diff;
    if (nowrap < 0) nowrap += max_fn;
    if (nowrap >= max_fn) nowrap -= max_fn;
    pred = nowrap;
    const int pn = nowrap > cur ? nowrap - max_fn : nowrap;
    auto it = std::find_if(list.begin(), list.end(), [&](const RefPic& r) { return picnum(r) == pn; });
    if (it == list.end()) throw std::runtime_error("h264: reference list modification names no picture");
    const RefPic r = *it;
    list.erase(it);
    list.insert(list.begin() + std::ptrdiff_t(std::min(m, list.size())), r);
  }
  list.resize(size_t(n_active));
  return list;
}

// Reference marking after a reference picture (8.2.5.3 sliding window / 8.2.5.4 MMCO 1 and 5);
// the picture then joins the DPB.  Returns the frame_num later pictures continue from.
int mark_reference(std::vector<RefPic>& dpb, RefPic pic, int max_fn, int max_refs, bool adaptive,
                   const std::vector<std::pair<int, int>>& mmco) {
  const int cur = pic.frame_num;
  auto picnum = [&](const RefPic& r) { return r.frame_num > cur ? r.frame_num - max_fn : r.frame_num; };
  bool cleared = false;
  if (adaptive) {
    for (const auto& op : mmco) {
      if (op.first == 1) {
        const int pn = cur - (op.second + 1);
        dpb.erase(std::remove_if(dpb.begin(), dpb.end(), [&](const RefPic& r) { return picnum(r) == pn; }), dpb.end());
      } else {
        dpb.clear();
        cleared = true;
      }
    }
  } else if (int(dpb.size()) >= max_refs) {
    dpb.erase(std::min_element(dpb.begin(), dpb.end(),
                               [&](const RefPic& a, const RefPic& b) { return picnum(a) < picnum(b); }));
  }
  if (int(dpb.size()) >= max_refs) throw std::runtime_error("h264: too many reference pictures");
  if (cleared) pic.frame_num = 0;
  dpb.push_back(pic);
  return pic.frame_num;
}

void mark_intra(Frame& f, int mx, int my) {
  for (int y = 0; y < 4; ++y)
    for (int x = 0; x < 4; ++x) {
      const size_t i = size_t(4 * my + y) * 4 * f.mbw + 4 * mx + x;
      f.ref[i] = -1;
      f.refpic[i] = -1;
      f.mvx[i] = f.mvy[i] = 0;
    }
  f.intra[size_t(my) * f.mbw + mx] = 1;
}

// inter prediction of the whole macroblock from its (already assigned) 4x4 motion
void predict_inter(const Frame& f, const std::vector<RefPic>& list, int mx, int my, uint8_t* py, uint8_t* pcb,
                   uint8_t* pcr) {
  // every sample depends only on its position and its block's (ref, mv), so runs of equal motion
  // are predicted as one larger block: 16x16, else per 8x8 quadrant, else per 4x4
  auto idx = [&](int bx, int by) { return size_t(4 * my + by) * 4 * f.mbw + 4 * mx + bx; };
  auto same = [&](int bx, int by, int n) {
    const size_t a = idx(bx, by);
    for (int y = by; y < by + n; ++y)
      for (int x = bx; x < bx + n; ++x) {
        const size_t b = idx(x, y);
        if (f.ref[b] != f.ref[a] || f.mvx[b] != f.mvx[a] || f.mvy[b] != f.mvy[a]) return false;
      }
    return true;
  };
  auto block = [&](int bx, int by, int n) {
    const size_t i = idx(bx, by);
    const Frame& r = *list[size_t(f.ref[i])].f;
    mc_luma(r, 16 * mx + 4 * bx, 16 * my + 4 * by, f.mvx[i], f.mvy[i], 4 * n, 4 * n, py + 16 * 4 * by + 4 * bx, 16);
    mc_chroma(r.cb, r.W / 2, r.H / 2, 8 * mx + 2 * bx, 8 * my + 2 * by, f.mvx[i], f.mvy[i], 2 * n, 2 * n,
              pcb + 8 * 2 * by + 2 * bx, 8);
    mc_chroma(r.cr, r.W / 2, r.H / 2, 8 * mx + 2 * bx, 8 * my + 2 * by, f.mvx[i], f.mvy[i], 2 * n, 2 * n,
              pcr + 8 * 2 * by + 2 * bx, 8);
  };
  if (same(0, 0, 4)) {
    block(0, 0, 4);
    return;
  }
  for (int q = 0; q < 4; ++q) {
    const int qx = 2 * (q & 1), qy = 2 * (q >> 1);
    if (same(qx, qy, 2)) {
      block(qx, qy, 2);
      continue;
    }
    for (int k = 0; k < 4; ++k) block(qx + (k & 1), qy + (k >> 1), 1);
  }
}

// ------------------------------------------------------------------------------------ encoder
inline int quant(int w, int mf, int f, int qbits) {
  const int a = w < 0 ? -w : w;
  int z = (a * mf + f) >> qbits;   // |w| * mf < 2^31 for 8-bit residuals (luma DC: 32640 x 13107)
  z = std::min(z, 2047);
  return w < 0 ? -z : z;
}

// Sum of absolute differences of an n x n source block against a packed n x n prediction, n = 8
// or 16: one psadbw per row (integer: the same value as the scalar sum).
inline int hsum_sad(__m128i acc) { return _mm_cvtsi128_si32(acc) + _mm_cvtsi128_si32(_mm_srli_si128(acc, 8)); }
int sad(const uint8_t* src, int stride, const uint8_t* pred, int n) {
  __m128i acc = _mm_setzero_si128();
  if (n == 16) {
    for (int y = 0; y < 16; ++y)
      acc = _mm_add_epi64(acc, _mm_sad_epu8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(src + y * stride)),
                                            _mm_loadu_si128(reinterpret_cast<const __m128i*>(pred + 16 * y))));
  } else {
    for (int y = 0; y < n; ++y)
      acc = _mm_add_epi64(acc, _mm_sad_epu8(_mm_loadl_epi64(reinterpret_cast<const __m128i*>(src + y * stride)),
                                            _mm_loadl_epi64(reinterpret_cast<const __m128i*>(pred + n * y))));
  }
  return hsum_sad(acc);
}

// SAD of a 16x16 source block against Intra_16x16 mode 0 / 1 / 2 (V / H / DC) without building
// the prediction: row y is compared against the top row, the broadcast left sample or the DC.
int sad16_mode(const uint8_t* src, int stride, const uint8_t* pl, int pstride, int x0, int y0, const Nb& nb, int mode) {
  __m128i acc = _mm_setzero_si128();
  if (mode == 0) {
    const __m128i top = _mm_loadu_si128(reinterpret_cast<const __m128i*>(pl + (y0 - 1) * pstride + x0));
    for (int y = 0; y < 16; ++y)
      acc = _mm_add_epi64(acc, _mm_sad_epu8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(src + y * stride)), top));
  } else if (mode == 1) {
    for (int y = 0; y < 16; ++y)
      acc = _mm_add_epi64(acc, _mm_sad_epu8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(src + y * stride)),
                                            _mm_set1_epi8(char(pl[(y0 + y) * pstride + x0 - 1]))));
  } else {
    uint8_t dc[256];
    pred16(pl, pstride, x0, y0, nb, 2, dc);
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(dc));
    for (int y = 0; y < 16; ++y)
      acc = _mm_add_epi64(acc, _mm_sad_epu8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(src + y * stride)), v));
  }
  return hsum_sad(acc);
}

void encode_mb(BitWriter& bw, Frame& f, const uint8_t* sy, const uint8_t* scb, const uint8_t* scr, int mx, int my,
               int qp, int slice_id = 0, int type_offset = 0) {
  const Nb nb = f.nb(mx, my, slice_id);
  const int W = f.W, Wc = f.W / 2;
  // ---- luma mode
  uint8_t pred[256], best[256];
  int mode = 2, best_sad = 1 << 30;
  const uint8_t* src = sy + size_t(my * 16) * W + mx * 16;
  for (int m : {0, 1, 2, 3}) {
    if ((m == 0 && !nb.top) || (m == 1 && !nb.left) || (m == 3 && !(nb.top && nb.left && nb.topleft))) continue;
    int s;
    if (m < 3) {
      s = sad16_mode(src, W, f.y.data(), W, mx * 16, my * 16, nb, m);
    } else {
      pred16(f.y.data(), W, mx * 16, my * 16, nb, m, pred);
      s = sad(src, W, pred, 16);
    }
    if (s < best_sad) {
      best_sad = s;
      mode = m;
    }
  }
  if (mode == 3) std::memcpy(best, pred, 256);
  else pred16(f.y.data(), W, mx * 16, my * 16, nb, mode, best);
  // ---- luma residual -> levels
  const int qp6 = qp % 6, qbits = 15 + qp / 6, fq = (1 << qbits) / 3;
  int W4[16][16], dcm[16], ac[16][15];
  alignas(16) int16_t rsd[256];   // src - pred, 16 x 16 (one unpack + subtract per 8 samples)
  {
    const __m128i z = _mm_setzero_si128();
    for (int y = 0; y < 16; ++y) {
      const __m128i sv = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + size_t(y) * W));
      const __m128i pv = _mm_loadu_si128(reinterpret_cast<const __m128i*>(best + 16 * y));
      const __m128i lo = _mm_sub_epi16(_mm_unpacklo_epi8(sv, z), _mm_unpacklo_epi8(pv, z));
      const __m128i hi = _mm_sub_epi16(_mm_unpackhi_epi8(sv, z), _mm_unpackhi_epi8(pv, z));
      _mm_store_si128(reinterpret_cast<__m128i*>(rsd + 16 * y), lo);
      _mm_store_si128(reinterpret_cast<__m128i*>(rsd + 16 * y + 8), hi);
    }
  }
  for (int blk = 0; blk < 16; ++blk) {
    const int bx = kBlkX[blk], by = kBlkY[blk];
    int res[16];
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) res[4 * y + x] = rsd[16 * (4 * by + y) + 4 * bx + x];
    fwd4x4(res, W4[blk]);
    dcm[4 * by + bx] = W4[blk][0];
  }
  int hd[16], dc[16];
  hadamard4(dcm, hd);
  bool any_ac = false;
  for (int k = 0; k < 16; ++k) dc[k] = quant(hd[kZigzag[k]] / 2, kMF[qp6][0], 2 * fq, qbits + 1);
  int mfz[15];   // quantiser multiplier per scan position 1..15
  for (int k = 0; k < 15; ++k) mfz[k] = kMF[qp6][pos_class(kZigzag[k + 1])];
  for (int blk = 0; blk < 16; ++blk) {
    int zz[15], nz = 0;   // scan order first, so the quantiser loop is contiguous (vectorised)
    for (int k = 0; k < 15; ++k) zz[k] = W4[blk][kZigzag[k + 1]];
    for (int k = 0; k < 15; ++k) {
      ac[blk][k] = quant(zz[k], mfz[k], fq, qbits);
      nz |= ac[blk][k];
    }
    any_ac |= nz != 0;
  }
  const int cbp_luma = any_ac ? 15 : 0;
  if (!any_ac) std::memset(ac, 0, sizeof(ac));
  // ---- chroma
  const int qpc = kChromaQp[qp], qc6 = qpc % 6, qcbits = 15 + qpc / 6, fqc = (1 << qcbits) / 3;
  const uint8_t* csrc[2] = {scb + size_t(my * 8) * Wc + mx * 8, scr + size_t(my * 8) * Wc + mx * 8};
  std::vector<uint8_t>* cpl[2] = {&f.cb, &f.cr};
  uint8_t cpred[2][64];
  int cmode = 0, cbest = 1 << 30;
  for (int m : {0, 1, 2, 3}) {
    if ((m == 1 && !nb.left) || (m == 2 && !nb.top) || (m == 3 && !(nb.top && nb.left && nb.topleft))) continue;
    uint8_t p[2][64];
    int s = 0;
    for (int c = 0; c < 2; ++c) {
      pred_chroma(cpl[c]->data(), Wc, mx * 8, my * 8, nb, m, p[c]);
      s += sad(csrc[c], Wc, p[c], 8);
    }
    if (s < cbest) {
      cbest = s;
      cmode = m;
      std::memcpy(cpred, p, sizeof(p));
    }
  }
  int cdc[2][4], cac[2][4][15], mfc[15];
  for (int k = 0; k < 15; ++k) mfc[k] = kMF[qc6][pos_class(kZigzag[k + 1])];
  bool c_any_dc = false, c_any_ac = false;
  for (int c = 0; c < 2; ++c) {
    int Wb[4][16];
    for (int blk = 0; blk < 4; ++blk) {
      const int bx = blk & 1, by = blk >> 1;
      int res[16];
      for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x)
          res[4 * y + x] = int(csrc[c][(4 * by + y) * Wc + 4 * bx + x]) - int(cpred[c][8 * (4 * by + y) + 4 * bx + x]);
      fwd4x4(res, Wb[blk]);
      int zz[15], nz = 0;
      for (int k = 0; k < 15; ++k) zz[k] = Wb[blk][kZigzag[k + 1]];
      for (int k = 0; k < 15; ++k) {
        cac[c][blk][k] = quant(zz[k], mfc[k], fqc, qcbits);
        nz |= cac[c][blk][k];
      }
      c_any_ac |= nz != 0;
    }
    const int d0 = Wb[0][0], d1 = Wb[1][0], d2 = Wb[2][0], d3 = Wb[3][0];
    const int h[4] = {d0 + d1 + d2 + d3, d0 - d1 + d2 - d3, d0 + d1 - d2 - d3, d0 - d1 - d2 + d3};
    for (int k = 0; k < 4; ++k) {
      cdc[c][k] = quant(h[k], kMF[qc6][0], 2 * fqc, qcbits + 1);
      c_any_dc |= cdc[c][k] != 0;
    }
  }
  const int cbp_chroma = c_any_ac ? 2 : c_any_dc ? 1 : 0;
  if (cbp_chroma < 2) std::memset(cac, 0, sizeof(cac));
  // ---- syntax
  bw.ue(type_offset + 1 + mode + 4 * cbp_chroma + (cbp_luma ? 12 : 0));
  bw.ue(cmode);
  bw.se(0);  // mb_qp_delta
  write_block(bw, dc, 16, f.nc(f.tc_y, 4 * mx, 4 * my, 4, slice_id));
  for (int blk = 0; blk < 16; ++blk) {
    const int bx = 4 * mx + kBlkX[blk], by = 4 * my + kBlkY[blk];
    int tc = 0;
    if (cbp_luma) {
      write_block(bw, ac[blk], 15, f.nc(f.tc_y, bx, by, 4, slice_id));
      for (int k = 0; k < 15; ++k) tc += ac[blk][k] != 0;
    }
    f.tc_y[size_t(by) * 4 * f.mbw + bx] = uint8_t(tc);
  }
  if (cbp_chroma)
    for (int c = 0; c < 2; ++c) write_block(bw, cdc[c], 4, -1);
  for (int c = 0; c < 2; ++c) {
    std::vector<uint8_t>& tcs = c ? f.tc_cr : f.tc_cb;
    for (int blk = 0; blk < 4; ++blk) {
      const int bx = 2 * mx + (blk & 1), by = 2 * my + (blk >> 1);
      int tc = 0;
      if (cbp_chroma == 2) {
        write_block(bw, cac[c][blk], 15, f.nc(tcs, bx, by, 2, slice_id));
        for (int k = 0; k < 15; ++k) tc += cac[c][blk][k] != 0;
      }
      tcs[size_t(by) * 2 * f.mbw + bx] = uint8_t(tc);
    }
  }
  // ---- reconstruction (the decoder's output)
  // (slice-parallel callers pre-set the slice ids: no write then, so other slices may read them)
  if (f.slice[size_t(my) * f.mbw + mx] != slice_id) f.slice[size_t(my) * f.mbw + mx] = slice_id;
  f.mbqp[size_t(my) * f.mbw + mx] = uint8_t(qp);
  for (int b = 0; b < 16; ++b) f.i4mode[size_t(4 * my + b / 4) * 4 * f.mbw + 4 * mx + b % 4] = -1;
  recon_luma16(f, mx, my, best, dc, ac, qp);
  for (int c = 0; c < 2; ++c) recon_chroma(*cpl[c], Wc, mx, my, cpred[c], cdc[c], cac[c], qpc);
}


// ------------------------------------------------------------------------------------ P encoder
const int kLambda16[52] = {4,   4,   5,   5,   6,   7,   7,   8,   9,   10,  12,  13,  15,  17,  19,  21,  23,  26,
                           30,  33,  37,  42,  47,  53,  59,  66,  74,  83,  94,  105, 118, 132, 149, 167, 187, 210,
                           236, 265, 297, 334, 375, 421, 472, 530, 595, 668, 749, 841, 944, 1060, 1189, 1335};

inline int ue_bits(uint32_t v) {
  int n = 0;
  for (uint32_t x = v + 1; x > 1; x >>= 1) ++n;
  return 2 * n + 1;
}
inline int se_bits(int v) { return ue_bits(v > 0 ? uint32_t(2 * v - 1) : uint32_t(-2 * v)); }

template <class Fn>
void parallel_for(int n, int threads, Fn fn) {
  const int nt = std::max(1, std::min(threads, n));
  std::vector<std::thread> pool;
  std::vector<std::string> errs(static_cast<size_t>(nt));
  auto work = [&](int t) {
    try {
      for (int i = t; i < n; i += nt) fn(i);
    } catch (const std::exception& e) {
      errs[size_t(t)] = e.what();
    }
  };
  for (int t = 1; t < nt; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  for (auto& e : errs)
    if (!e.empty()) throw std::runtime_error(e);
}

// Half-sample planes of a reference picture with a `pad`-sample margin (the decoder's clamped-
// coordinate 6-tap values, so quarter samples from them equal mc_luma's): motion search only.
struct HalfPel {
  int W = 0, H = 0, pad = 0, stride = 0;
  std::vector<uint8_t> g, b, h, j;
  void build(const Frame& r, int pad_, int threads) {
    W = r.W;
    H = r.H;
    pad = pad_;
    stride = W + 2 * pad;
    const int rows = H + 2 * pad;
    // edge-replicated copy with 3 more samples of margin: every tap is a plain load, and rows or
    // columns outside the picture equal the clamped ones (so do the sums built from them)
    const int e = pad + 3, es = W + 2 * e, erows = H + 2 * e;
    std::vector<uint8_t> ext(size_t(es) * erows);
    for (int yy = 0; yy < erows; ++yy) {
      const uint8_t* src = r.y.data() + size_t(std::clamp(yy - e, 0, H - 1)) * W;
      uint8_t* d = ext.data() + size_t(yy) * es;
      std::memset(d, src[0], size_t(e));
      std::memcpy(d + e, src, size_t(W));
      std::memset(d + e + W, src[W - 1], size_t(e));
    }
    auto X = [&](int x, int y) { return int(ext[size_t(y + e) * es + x + e]); };
    g.assign(size_t(stride) * rows, 0);
    b = h = j = g;
    auto clip = [](int v) { return uint8_t(v < 0 ? 0 : v > 255 ? 255 : v); };
    // unclipped horizontal sums for rows -pad-2 .. H+pad+2 (j's vertical taps reach 3 rows out)
    const int b1rows = rows + 5;
    std::vector<int> b1(size_t(stride) * b1rows);
    const int bands = std::max(1, threads) * 4;
    parallel_for(bands, threads, [&](int t) {
      for (int k = t * b1rows / bands; k < (t + 1) * b1rows / bands; ++k) {
        const int yy = k - pad - 2;
        int* o = b1.data() + size_t(k) * stride;
        for (int xx = -pad; xx < W + pad; ++xx)
          o[xx + pad] = tap6(X(xx - 2, yy), X(xx - 1, yy), X(xx, yy), X(xx + 1, yy), X(xx + 2, yy), X(xx + 3, yy));
      }
    });
    parallel_for(bands, threads, [&](int t) {
      for (int yy = -pad + t * rows / bands; yy < -pad + (t + 1) * rows / bands; ++yy) {
        const int* r0 = b1.data() + size_t(yy + pad) * stride;   // b1 row yy - 2
        const size_t o0 = size_t(yy + pad) * stride;
        for (int xx = -pad; xx < W + pad; ++xx) {
          const size_t o = o0 + xx + pad;
          const int c = xx + pad;
          g[o] = uint8_t(X(xx, yy));
          b[o] = clip((r0[2 * stride + c] + 16) >> 5);
          h[o] = clip(
              (tap6(X(xx, yy - 2), X(xx, yy - 1), X(xx, yy), X(xx, yy + 1), X(xx, yy + 2), X(xx, yy + 3)) + 16) >> 5);
          j[o] = clip((tap6(r0[c], r0[stride + c], r0[2 * stride + c], r0[3 * stride + c], r0[4 * stride + c],
                            r0[5 * stride + c]) + 512) >> 10);
        }
      }
    });
  }
  // SAD of the 16x16 source block against the prediction at integer position (x0, y0) + quarter
  // vector (mvx, mvy): every quarter sample is the rounded mean of two planes (8-250..8-261; full
  // and half positions average a plane with itself).  The caller keeps the block in the margin.
  int sad16(const uint8_t* src, int sstride, int x0, int y0, int mvx, int mvy) const {
    const int X0 = x0 + (mvx >> 2), Y0 = y0 + (mvy >> 2), cs = (mvy & 3) * 4 + (mvx & 3);
    struct Pair { char a; int ax, ay; char b; int bx, by; };
    static const Pair kCases[16] = {{'g', 0, 0, 'g', 0, 0}, {'g', 0, 0, 'b', 0, 0}, {'b', 0, 0, 'b', 0, 0},
                                    {'g', 1, 0, 'b', 0, 0}, {'g', 0, 0, 'h', 0, 0}, {'b', 0, 0, 'h', 0, 0},
                                    {'b', 0, 0, 'j', 0, 0}, {'b', 0, 0, 'h', 1, 0}, {'h', 0, 0, 'h', 0, 0},
                                    {'h', 0, 0, 'j', 0, 0}, {'j', 0, 0, 'j', 0, 0}, {'j', 0, 0, 'h', 1, 0},
                                    {'g', 0, 1, 'h', 0, 0}, {'h', 0, 0, 'b', 0, 1}, {'j', 0, 0, 'b', 0, 1},
                                    {'h', 1, 0, 'b', 0, 1}};
    const Pair& pc = kCases[cs];
    auto plane = [&](char c) -> const std::vector<uint8_t>& { return c == 'g' ? g : c == 'b' ? b : c == 'h' ? h : j; };
    const uint8_t* A = plane(pc.a).data() + size_t(Y0 + pc.ay + pad) * stride + X0 + pc.ax + pad;
    const uint8_t* B = plane(pc.b).data() + size_t(Y0 + pc.by + pad) * stride + X0 + pc.bx + pad;
    int s = 0;
    for (int yy = 0; yy < 16; ++yy) {
      const uint8_t* a = A + size_t(yy) * stride;
      const uint8_t* bb = B + size_t(yy) * stride;
      const uint8_t* q = src + size_t(yy) * sstride;
      for (int xx = 0; xx < 16; ++xx) s += std::abs(int(q[xx]) - ((int(a[xx]) + int(bb[xx]) + 1) >> 1));
    }
    return s;
  }
};

struct Lcg {                   // deterministic decisions of the scripted (decoder-coverage) mode
  uint32_t s;
  uint32_t next() {
    s = s * 1664525u + 1013904223u;
    return s >> 8;
  }
  int below(int n) { return int(next() % uint32_t(n)); }
};

// residual of an inter macroblock -> levels (inter dead zone 1/6), cbp; returns cbp
int quant_inter(const uint8_t* sy, int W, const uint8_t* const* csrc, int Wc, const uint8_t* py,
                const uint8_t (*pc)[64],
                int qp, int qpc, int (*coef)[16], int (*cdc)[4], int (*cac)[4][15]) {
  const int qp6 = qp % 6, qbits = 15 + qp / 6, fq = (1 << qbits) / 6;
  int cbp = 0;
  for (int blk = 0; blk < 16; ++blk) {
    const int bx = kBlkX[blk], by = kBlkY[blk];
    int res[16], w[16];
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x)
        res[4 * y + x] = int(sy[(4 * by + y) * W + 4 * bx + x]) - int(py[16 * (4 * by + y) + 4 * bx + x]);
    fwd4x4(res, w);
    bool any = false;
    for (int k = 0; k < 16; ++k) {
      const int rp = kZigzag[k];
      coef[blk][k] = quant(w[rp], kMF[qp6][pos_class(rp)], fq, qbits);
      any |= coef[blk][k] != 0;
    }
    if (any) cbp |= 1 << (blk / 4);
  }
  for (int blk = 0; blk < 16; ++blk)
    if (!(cbp & (1 << (blk / 4)))) std::memset(coef[blk], 0, sizeof(int) * 16);
  const int qc6 = qpc % 6, qcbits = 15 + qpc / 6, fqc = (1 << qcbits) / 6;
  bool c_dc = false, c_ac = false;
  for (int c = 0; c < 2; ++c) {
    int Wb[4][16];
    for (int blk = 0; blk < 4; ++blk) {
      const int bx = blk & 1, by = blk >> 1;
      int res[16];
      for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x)
          res[4 * y + x] = int(csrc[c][(4 * by + y) * Wc + 4 * bx + x]) - int(pc[c][8 * (4 * by + y) + 4 * bx + x]);
      fwd4x4(res, Wb[blk]);
      for (int k = 0; k < 15; ++k) {
        const int rp = kZigzag[k + 1];
        cac[c][blk][k] = quant(Wb[blk][rp], kMF[qc6][pos_class(rp)], fqc, qcbits);
        c_ac |= cac[c][blk][k] != 0;
      }
    }
    const int d0 = Wb[0][0], d1 = Wb[1][0], d2 = Wb[2][0], d3 = Wb[3][0];
    const int hd[4] = {d0 + d1 + d2 + d3, d0 - d1 + d2 - d3, d0 + d1 - d2 - d3, d0 - d1 - d2 + d3};
    for (int k = 0; k < 4; ++k) {
      cdc[c][k] = quant(hd[k], kMF[qc6][0], 2 * fqc, qcbits + 1);
      c_dc |= cdc[c][k] != 0;
    }
  }
  const int cbp_chroma = c_ac ? 2 : c_dc ? 1 : 0;
  if (cbp_chroma < 2) std::memset(cac, 0, sizeof(int) * 120);
  if (cbp_chroma == 0) std::memset(cdc, 0, sizeof(int) * 8);
  return cbp | (cbp_chroma << 4);
}

// cbp -> me(v) codeNum for inter macroblocks
int inter_cbp_code(int cbp) {
  for (int k = 0; k < 48; ++k)
    if (kInterCbp[k] == cbp) return k;
  return 0;
}

// residual syntax of an inter macroblock (the cbp, qp delta and blocks) + TotalCoeff bookkeeping
void write_inter_residual(BitWriter& bw, Frame& f, int mx, int my, int cbp, int qp_delta, const int (*coef)[16],
                          const int (*cdc)[4], const int (*cac)[4][15], int slice_id) {
  bw.ue(uint32_t(inter_cbp_code(cbp)));
  if (cbp) bw.se(qp_delta);
  for (int blk = 0; blk < 16; ++blk) {
    const int bx = 4 * mx + kBlkX[blk], by = 4 * my + kBlkY[blk];
    int tc = 0;
    if (cbp & (1 << (blk / 4))) {
      write_block(bw, coef[blk], 16, f.nc(f.tc_y, bx, by, 4, slice_id));
      for (int k = 0; k < 16; ++k) tc += coef[blk][k] != 0;
    }
    f.tc_y[size_t(by) * 4 * f.mbw + bx] = uint8_t(tc);
  }
  if (cbp >> 4)
    for (int c = 0; c < 2; ++c) write_block(bw, cdc[c], 4, -1);
  for (int c = 0; c < 2; ++c) {
    std::vector<uint8_t>& tcs = c ? f.tc_cr : f.tc_cb;
    for (int blk = 0; blk < 4; ++blk) {
      const int bx = 2 * mx + (blk & 1), by = 2 * my + (blk >> 1);
      int tc = 0;
      if ((cbp >> 4) == 2) {
        write_block(bw, cac[c][blk], 15, f.nc(tcs, bx, by, 2, slice_id));
        for (int k = 0; k < 15; ++k) tc += cac[c][blk][k] != 0;
      }
      tcs[size_t(by) * 2 * f.mbw + bx] = uint8_t(tc);
    }
  }
}

struct PEncCtx {
  const uint8_t *y, *cb, *cr;
  int qp;
  const std::vector<RefPic>& list;             // RefPicList0 as the decoder will build it
  const std::vector<const HalfPel*>& hp;       // half-sample planes per list entry (production search)
  uint32_t seed;                                // 0: production decisions; else scripted
};

// prediction of a macroblock from its assigned motion into py / pc (the decoder's own MC)
void inter_pred_mb(const Frame& f, const std::vector<RefPic>& list, int mx, int my, bool uniform, uint8_t* py,
                   uint8_t (*pc)[64]) {
  if (uniform) {
    const size_t i = size_t(4 * my) * 4 * f.mbw + 4 * mx;
    const Frame& r = *list[size_t(f.ref[i])].f;
    mc_luma(r, 16 * mx, 16 * my, f.mvx[i], f.mvy[i], 16, 16, py, 16);
    mc_chroma(r.cb, r.W / 2, r.H / 2, 8 * mx, 8 * my, f.mvx[i], f.mvy[i], 8, 8, pc[0], 8);
    mc_chroma(r.cr, r.W / 2, r.H / 2, 8 * mx, 8 * my, f.mvx[i], f.mvy[i], 8, 8, pc[1], 8);
  } else {
    predict_inter(f, list, mx, my, py, pc[0], pc[1]);
  }
}

// Production motion search for one 16x16 macroblock (ref 0): integer diamond around the predictor
// and zero, then half- and quarter-sample refinement; cost = SAD + lambda * mvd bits.
void search16(const PEncCtx& c, const Frame& f, int mx, int my, int pmx, int pmy, int& bmx, int& bmy) {
  const HalfPel& hp = *c.hp[0];
  const int W = f.W, x0 = 16 * mx, y0 = 16 * my, lam = kLambda16[c.qp];
  const uint8_t* src = c.y + size_t(y0) * W + x0;
  const int lo_x = 4 * (-x0 - hp.pad + 2), hi_x = 4 * (W + hp.pad - 19 - x0);
  const int lo_y = 4 * (-y0 - hp.pad + 2), hi_y = 4 * (f.H + hp.pad - 19 - y0);
  auto cost = [&](int vx, int vy) {
    if (vx < lo_x || vx > hi_x || vy < lo_y || vy > hi_y) return 1 << 30;
    return hp.sad16(src, W, x0, y0, vx, vy) * 16 + lam * (se_bits(vx - pmx) + se_bits(vy - pmy));
  };
  int best = 1 << 30;
  auto consider = [&](int vx, int vy) {
    const int cst = cost(vx, vy);
    if (cst < best) {
      best = cst;
      bmx = vx;
      bmy = vy;
    }
  };
  bmx = bmy = 0;
  consider(0, 0);
  consider(pmx & ~3, pmy & ~3);
  for (int it = 0; it < 24; ++it) {                    // integer small diamond
    const int cx = bmx, cy = bmy;
    for (const auto& d : {std::pair<int, int>{-4, 0}, {4, 0}, {0, -4}, {0, 4}}) consider(cx + d.first, cy + d.second);
    if (cx == bmx && cy == bmy) break;
  }
  for (int step : {2, 1}) {                             // half, then quarter samples
    const int cx = bmx, cy = bmy;
    for (int dy = -step; dy <= step; dy += step)
      for (int dx = -step; dx <= step; dx += step)
        if (dx || dy) consider(cx + dx, cy + dy);
  }
}

// One P slice (macroblocks [first, last)) into bw; updates f (motion, recon before deblocking)
void encode_p_slice_data(BitWriter& bw, Frame& f, const PEncCtx& c, int first, int last, int slice_id, Lcg& rng) {
  const int W = f.W, Wc = f.W / 2, nref = int(c.list.size());
  int qp = c.qp, run = 0;
  for (int mb = first; mb < last; ++mb) {
    const int mx = mb % f.mbw, my = mb / f.mbw;
    const uint8_t* sy = c.y + size_t(16 * my) * W + 16 * mx;
    const uint8_t* csrc[2] = {c.cb + size_t(8 * my) * Wc + 8 * mx, c.cr + size_t(8 * my) * Wc + 8 * mx};
    MvPred mp{f, mx, my, slice_id};
    int coef[16][16], cdc[2][4], cac[2][4][15];
    uint8_t py[256], pc[2][64];
    int kind;                   // 0 skip, 1 16x16, 2 16x8, 3 8x16, 4 8x8, 5 8x8ref0, 6 intra
    if (c.seed) {
      const int r = rng.below(16);
      kind = r < 3 ? 0 : r < 6 ? 1 : r < 8 ? 2 : r < 10 ? 3 : r < 13 ? 4 : r < 14 ? (nref > 1 ? 5 : 4) : 6;
    } else {
      kind = -1;
    }
    // ---- production: skip test, then search; intra when clearly better
    int smx = 0, smy = 0;
    mp.skip(smx, smy);
    if (kind < 0) {
      set_motion(f, mp, mx, my, 0, 0, 4, 4, 0, c.list[0].id, smx, smy);
      inter_pred_mb(f, c.list, mx, my, true, py, pc);
      const int qpc = kChromaQp[qp];
      const int cbp = quant_inter(sy, W, csrc, Wc, py, pc, qp, qpc, coef, cdc, cac);
      if (cbp == 0) {
        kind = 0;
      } else {
        mp.done = 0;
        int pmx, pmy, bmx, bmy;
        mp.pred(0, 0, 4, 0, 0, pmx, pmy);
        search16(c, f, mx, my, pmx, pmy, bmx, bmy);
        set_motion(f, mp, mx, my, 0, 0, 4, 4, 0, c.list[0].id, bmx, bmy);
        inter_pred_mb(f, c.list, mx, my, true, py, pc);
        const int inter_sad = sad(sy, W, py, 16);
        // intra 16x16 DC / V / H / plane estimate on the current (unfiltered) reconstruction
        const Nb nb = f.nb(mx, my, slice_id);
        int intra_sad = 1 << 30;
        uint8_t ip[256];
        for (int m : {0, 1, 2, 3}) {
          if ((m == 0 && !nb.top) || (m == 1 && !nb.left) || (m == 3 && !(nb.top && nb.left && nb.topleft))) continue;
          pred16(f.y.data(), W, mx * 16, my * 16, nb, m, ip);
          intra_sad = std::min(intra_sad, sad(sy, W, ip, 16));
        }
        kind = intra_sad + 16 * 24 < inter_sad ? 6 : 1;
      }
    }
    if (kind == 0) {                                     // P_Skip
      mp.done = 0;
      set_motion(f, mp, mx, my, 0, 0, 4, 4, 0, c.list[0].id, smx, smy);
      inter_pred_mb(f, c.list, mx, my, true, py, pc);
      std::memset(coef, 0, sizeof(coef));
      std::memset(cdc, 0, sizeof(cdc));
      std::memset(cac, 0, sizeof(cac));
      for (int b = 0; b < 16; ++b) {
        const size_t i = size_t(4 * my + b / 4) * 4 * f.mbw + 4 * mx + b % 4;
        f.tc_y[i] = 0;
        f.i4mode[i] = -1;
      }
      for (int b = 0; b < 4; ++b) {
        const size_t i = size_t(2 * my + b / 2) * 2 * f.mbw + 2 * mx + b % 2;
        f.tc_cb[i] = f.tc_cr[i] = 0;
      }
      recon_luma4x4(f, mx, my, py, coef, qp);
      const int qpc = kChromaQp[qp];
      for (int cc = 0; cc < 2; ++cc) recon_chroma(cc ? f.cr : f.cb, Wc, mx, my, pc[cc], cdc[cc], cac[cc], qpc);
      f.intra[mb] = 0;
      f.mbqp[mb] = uint8_t(qp);
      ++run;
      continue;
    }
    bw.ue(uint32_t(run));
    run = 0;
    if (kind == 6) {                                     // Intra_16x16 in a P slice (mb_type 5 + I type)
      mark_intra(f, mx, my);
      encode_mb(bw, f, c.y, c.cb, c.cr, mx, my, qp, slice_id, 5);
      continue;
    }
    // ---- inter syntax: partitions, then refs, then mvds (motion assigned in decoding order)
    mp.done = 0;
    const int mb_type = kind - 1;                        // 0 16x16, 1 16x8, 2 8x16, 3 8x8, 4 8x8ref0
    bw.ue(uint32_t(mb_type));
    auto rnd_mv = [&](int p) { return p + rng.below(97) - 48; };
    auto clamp_mv = [&](int v, int lo, int hi) { return std::clamp(v, lo, hi); };
    if (mb_type <= 2) {
      const int np = mb_type == 0 ? 1 : 2;
      int refs[2] = {0, 0};
      if (c.seed)
        for (int p = 0; p < np; ++p) refs[p] = rng.below(nref);
      if (nref > 1)
        for (int p = 0; p < np; ++p) {
          if (nref == 2) bw.put(refs[p] ? 0u : 1u, 1);
          else bw.ue(uint32_t(refs[p]));
        }
      for (int p = 0; p < np; ++p) {
        int bx = 0, by = 0, bwid = 4, bh = 4, shape = 0;
        if (mb_type == 1) { by = 2 * p; bh = 2; shape = 1 + p; }
        if (mb_type == 2) { bx = 2 * p; bwid = 2; shape = 3 + p; }
        int pmx, pmy, vx, vy;
        mp.pred(bx, by, bwid, refs[p], shape, pmx, pmy);
        if (c.seed) {
          vx = clamp_mv(rnd_mv(pmx), -4 * (16 * mx + 40), 4 * (W - 16 * mx + 24));
          vy = clamp_mv(rnd_mv(pmy), -4 * (16 * my + 40), 4 * (f.H - 16 * my + 24));
        } else {
          vx = f.mvx[size_t(4 * my) * 4 * f.mbw + 4 * mx];   // the searched vector (kept by set_motion)
          vy = f.mvy[size_t(4 * my) * 4 * f.mbw + 4 * mx];
        }
        bw.se(vx - pmx);
        bw.se(vy - pmy);
        set_motion(f, mp, mx, my, bx, by, bwid, bh, refs[p], c.list[size_t(refs[p])].id, vx, vy);
      }
    } else {
      int sub[4], refs[4] = {0, 0, 0, 0};
      for (int s = 0; s < 4; ++s) {
        sub[s] = rng.below(4);
        bw.ue(uint32_t(sub[s]));
      }
      if (mb_type == 3 && nref > 1)
        for (int s = 0; s < 4; ++s) {
          refs[s] = rng.below(nref);
          if (nref == 2) bw.put(refs[s] ? 0u : 1u, 1);
          else bw.ue(uint32_t(refs[s]));
        }
      for (int s = 0; s < 4; ++s) {
        const int sx = 2 * (s & 1), sy2 = 2 * (s >> 1);
        const int n = sub[s] == 0 ? 1 : sub[s] == 3 ? 4 : 2;
        const int pw = sub[s] == 0 || sub[s] == 1 ? 2 : 1, ph = sub[s] == 0 || sub[s] == 2 ? 2 : 1;
        for (int k = 0; k < n; ++k) {
          const int bx = sx + (sub[s] == 2 || sub[s] == 3 ? (k & 1) : 0);
          const int by = sy2 + (sub[s] == 1 ? k : sub[s] == 3 ? (k >> 1) : 0);
          int pmx, pmy;
          mp.pred(bx, by, pw, refs[s], 0, pmx, pmy);
          const int vx = clamp_mv(rnd_mv(pmx), -4 * (16 * mx + 40), 4 * (W - 16 * mx + 24));
          const int vy = clamp_mv(rnd_mv(pmy), -4 * (16 * my + 40), 4 * (f.H - 16 * my + 24));
          bw.se(vx - pmx);
          bw.se(vy - pmy);
          set_motion(f, mp, mx, my, bx, by, pw, ph, refs[s], c.list[size_t(refs[s])].id, vx, vy);
        }
      }
    }
    int qp_delta = 0;
    inter_pred_mb(f, c.list, mx, my, mb_type == 0, py, pc);
    if (c.seed) qp_delta = rng.below(4) == 0 ? rng.below(9) - 4 : 0;
    int qpm = std::clamp(qp + qp_delta, 0, 51);
    int cbp = quant_inter(sy, W, csrc, Wc, py, pc, qpm, kChromaQp[qpm], coef, cdc, cac);
    if (!cbp) qpm = qp;                                  // no mb_qp_delta without residual
    write_inter_residual(bw, f, mx, my, cbp, qpm - qp, coef, cdc, cac, slice_id);
    qp = qpm;
    for (int b = 0; b < 16; ++b) f.i4mode[size_t(4 * my + b / 4) * 4 * f.mbw + 4 * mx + b % 4] = -1;
    recon_luma4x4(f, mx, my, py, coef, qp);
    const int qpc = kChromaQp[qp];
    for (int cc = 0; cc < 2; ++cc) recon_chroma(cc ? f.cr : f.cb, Wc, mx, my, pc[cc], cdc[cc], cac[cc], qpc);
    f.intra[mb] = 0;
    f.mbqp[mb] = uint8_t(qp);
  }
  if (run) bw.ue(uint32_t(run));
}

void write_sps(BitWriter& s, int width, int height, int max_refs = 1) {
  const int mbw = (width + 15) / 16, mbh = (height + 15) / 16;
  s.put(66, 8);    // profile_idc: Baseline
  s.put(0xC0, 8);  // constraint_set0/1 -> Constrained Baseline
  s.put(51, 8);    // level_idc
  s.ue(0);         // seq_parameter_set_id
  s.ue(0);         // log2_max_frame_num_minus4
  s.ue(2);         // pic_order_cnt_type
  s.ue(uint32_t(max_refs));  // max_num_ref_frames
  s.put(0, 1);     // gaps_in_frame_num_value_allowed_flag
  s.ue(mbw - 1);
  s.ue(mbh - 1);
  s.put(1, 1);  // frame_mbs_only_flag
  s.put(1, 1);  // direct_8x8_inference_flag
  const int cr = (mbw * 16 - width) / 2, cbm = (mbh * 16 - height) / 2;
  if (cr || cbm) {
    s.put(1, 1);
    s.ue(0);
    s.ue(cr);
    s.ue(0);
    s.ue(cbm);
  } else {
    s.put(0, 1);
  }
  s.put(0, 1);  // vui_parameters_present_flag
  s.trailing();
}

}  // namespace

void parameter_sets(int width, int height, int qp, std::string& sps, std::string& pps, int max_refs) {
  if (max_refs < 1 || max_refs > 16) throw std::invalid_argument("h264: max_refs must be in [1, 16]");
  BitWriter s;
  write_sps(s, width, height, max_refs);
  sps = std::string(1, char(0x67)) + add_emulation_prevention(s.out);
  BitWriter p;
  p.ue(0);  // pic_parameter_set_id
  p.ue(0);  // seq_parameter_set_id
  p.put(0, 1);  // entropy_coding_mode_flag: CAVLC
  p.put(0, 1);  // bottom_field_pic_order_in_frame_present_flag
  p.ue(0);      // num_slice_groups_minus1
  p.ue(0);
  p.ue(0);      // num_ref_idx_l0/l1_default_active_minus1
  p.put(0, 1);
  p.put(0, 2);  // weighted_pred_flag, weighted_bipred_idc
  p.se(qp - 26);  // pic_init_qp_minus26
  p.se(0);        // pic_init_qs_minus26
  p.se(0);        // chroma_qp_index_offset
  p.put(1, 1);    // deblocking_filter_control_present_flag
  p.put(0, 1);    // constrained_intra_pred_flag
  p.put(0, 1);    // redundant_pic_cnt_present_flag
  p.trailing();
  pps = std::string(1, char(0x68)) + add_emulation_prevention(p.out);
}

std::string rbsp_to_nal(uint8_t nal_header, const uint8_t* rbsp, size_t n) {
  std::string out(1, char(nal_header));
  append_emulation_prevented(out, reinterpret_cast<const char*>(rbsp), n);
  return out;
}

std::string encode_idr(const uint8_t* y, const uint8_t* cb, const uint8_t* cr, int W, int H, int qp, int idr_pic_id,
                       uint8_t* recon_y, uint8_t* recon_cb, uint8_t* recon_cr) {
  if (W % 16 || H % 16 || W <= 0 || H <= 0) throw std::invalid_argument("h264: W, H must be positive multiples of 16");
  if (qp < 0 || qp > 51) throw std::invalid_argument("h264: qp must be in [0, 51]");
  Frame f(W / 16, H / 16);
  BitWriter bw;
  bw.ue(0);               // first_mb_in_slice
  bw.ue(7);               // slice_type: I (all slices of the picture)
  bw.ue(0);               // pic_parameter_set_id
  bw.put(0, 4);           // frame_num
  bw.ue(idr_pic_id & 1);  // idr_pic_id
  bw.put(0, 1);           // no_output_of_prior_pics_flag
  bw.put(0, 1);           // long_term_reference_flag
  bw.se(0);               // slice_qp_delta (pic_init_qp carries the QP)
  bw.ue(1);               // disable_deblocking_filter_idc: off -> recon is the output
  for (int my = 0; my < f.mbh; ++my)
    for (int mx = 0; mx < f.mbw; ++mx) encode_mb(bw, f, y, cb, cr, mx, my, qp);
  bw.trailing();
  if (recon_y) {
    std::memcpy(recon_y, f.y.data(), f.y.size());
    std::memcpy(recon_cb, f.cb.data(), f.cb.size());
    std::memcpy(recon_cr, f.cr.data(), f.cr.size());
  }
  return std::string(1, char(0x65)) + add_emulation_prevention(bw.out);
}

namespace {

void write_slice_header(BitWriter& bw, int first_mb, bool idr, bool p, int frame_num, int idr_pic_id, int nal_ref_idc,
                        int nref_active, const std::vector<std::pair<int, int>>& mods, const SliceDb& db) {
  bw.ue(uint32_t(first_mb));
  bw.ue(p ? 5 : 7);                    // slice_type: every slice of the picture has this type
  bw.ue(0);                            // pic_parameter_set_id
  bw.put(uint32_t(frame_num) & 15u, 4);
  if (idr) bw.ue(uint32_t(idr_pic_id & 1));
  if (p) {
    if (nref_active != 1) {
      bw.put(1, 1);                    // num_ref_idx_active_override_flag
      bw.ue(uint32_t(nref_active - 1));
    } else {
      bw.put(0, 1);
    }
    bw.put(mods.empty() ? 0u : 1u, 1);  // ref_pic_list_modification_flag_l0
    if (!mods.empty()) {
      for (const auto& m : mods) {
        bw.ue(uint32_t(m.first));
        bw.ue(uint32_t(m.second));
      }
      bw.ue(3);
    }
  }
  if (nal_ref_idc) {
    if (idr) {
      bw.put(0, 1);                    // no_output_of_prior_pics_flag
      bw.put(0, 1);                    // long_term_reference_flag
    } else {
      bw.put(0, 1);                    // adaptive_ref_pic_marking_mode_flag: sliding window
    }
  }
  bw.se(0);                            // slice_qp_delta
  bw.ue(uint32_t(db.idc));
  if (db.idc != 1) {
    bw.se(db.offa / 2);
    bw.se(db.offb / 2);
  }
}

}  // namespace

std::vector<EncodedPicture> encode_stream(int F, int W, int H, const StreamOptions& o, const LoadFn& load) {
  if (W % 16 || H % 16 || W <= 0 || H <= 0) throw std::invalid_argument("h264: W, H must be positive multiples of 16");
  if (o.qp < 0 || o.qp > 51) throw std::invalid_argument("h264: qp must be in [0, 51]");
  if (o.gop < 1 || o.max_refs < 1 || o.max_refs > 16 || o.rows_per_slice < 1)
    throw std::invalid_argument("h264: bad stream options");
  const int mbw = W / 16, mbh = H / 16, nmb = mbw * mbh, max_fn = 16;
  std::vector<EncodedPicture> out(static_cast<size_t>(F));
  std::vector<RefPic> dpb;
  std::vector<std::pair<int, std::shared_ptr<HalfPel>>> planes;   // RefPic id -> half-sample planes
  std::vector<uint8_t> y(size_t(W) * H), cb(size_t(W) * H / 4), cr(cb.size());
  Lcg rng{o.seed * 2654435761u + 12345u};
  int prev_ref_fn = 0, next_id = 1, gop_idx = -1;
  for (int i = 0; i < F; ++i) {
    load(i, y.data(), cb.data(), cr.data());
    const bool idr = i % o.gop == 0;
    if (idr) {
      ++gop_idx;
      dpb.clear();
      planes.clear();
      prev_ref_fn = 0;
    }
    const int frame_num = idr ? 0 : (prev_ref_fn + 1) % max_fn;
    const int nal_ref_idc = idr ? 3 : (o.seed && rng.below(5) == 0) ? 0 : 2;
    auto f = std::make_shared<Frame>(mbw, mbh);
    // slices: production = fixed bands of MB rows (a function of the size only); scripted = random cuts
    std::vector<int> cuts{0};
    if (o.seed) {
      const int extra = rng.below(3);
      for (int k = 0; k < extra; ++k) cuts.push_back(1 + rng.below(std::max(1, nmb - 1)));
      std::sort(cuts.begin(), cuts.end());
      cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
    } else {
      for (int r = o.rows_per_slice; r < mbh; r += o.rows_per_slice) cuts.push_back(r * mbw);
    }
    cuts.push_back(nmb);
    const int ns = int(cuts.size()) - 1;
    for (int sl = 0; sl < ns; ++sl)
      for (int m = cuts[size_t(sl)]; m < cuts[size_t(sl) + 1]; ++m) f->slice[size_t(m)] = sl;
    std::vector<SliceDb> dbs(static_cast<size_t>(ns));
    std::vector<std::vector<std::pair<int, int>>> mods(static_cast<size_t>(ns));
    std::vector<int> nactive(static_cast<size_t>(ns), 1);
    std::vector<uint32_t> seeds(static_cast<size_t>(ns), 0);
    for (int sl = 0; sl < ns; ++sl) {
      if (o.seed) {
        dbs[size_t(sl)] = SliceDb{rng.below(3), 2 * (rng.below(5) - 2), 2 * (rng.below(5) - 2)};
        seeds[size_t(sl)] = rng.next() | 1u;
        if (!idr) {
          nactive[size_t(sl)] = 1 + rng.below(int(dpb.size()));
          if (dpb.size() >= 2 && rng.below(2)) {
            // move the second most recent reference to the front
            std::vector<RefPic> l = ref_list0(dpb, frame_num, max_fn, {}, int(dpb.size()));
            const int pn = l[1].frame_num > frame_num ? l[1].frame_num - max_fn : l[1].frame_num;
            mods[size_t(sl)].emplace_back(0, frame_num - pn - 1);
          }
        }
      } else {
        dbs[size_t(sl)] = SliceDb{0, 0, 0};
      }
    }
    std::vector<std::string> nals(static_cast<size_t>(ns));
    std::vector<std::vector<RefPic>> lists(static_cast<size_t>(ns));
    std::vector<std::vector<const HalfPel*>> hps(static_cast<size_t>(ns));
    if (!idr) {
      for (int sl = 0; sl < ns; ++sl) {
        lists[size_t(sl)] = ref_list0(dpb, frame_num, max_fn, mods[size_t(sl)], nactive[size_t(sl)]);
        for (const RefPic& r : lists[size_t(sl)])
          for (auto& pp : planes)
            if (pp.first == r.id) hps[size_t(sl)].push_back(pp.second.get());
      }
    }
    parallel_for(ns, o.threads, [&](int sl) {
      BitWriter bw;
      write_slice_header(bw, cuts[size_t(sl)], idr, !idr, frame_num, gop_idx, nal_ref_idc, nactive[size_t(sl)],
                         mods[size_t(sl)], dbs[size_t(sl)]);
      if (idr) {
        for (int m = cuts[size_t(sl)]; m < cuts[size_t(sl) + 1]; ++m)
          encode_mb(bw, *f, y.data(), cb.data(), cr.data(), m % mbw, m / mbw, o.qp, sl, 0);
      } else {
        Lcg srng{seeds[size_t(sl)]};
        const PEncCtx c{y.data(), cb.data(), cr.data(), o.qp, lists[size_t(sl)], hps[size_t(sl)], o.seed};
        encode_p_slice_data(bw, *f, c, cuts[size_t(sl)], cuts[size_t(sl) + 1], sl, srng);
      }
      bw.trailing();
      const char hdr = char(idr ? 0x65 : (nal_ref_idc << 5) | 1);
      nals[size_t(sl)] = std::string(1, hdr) + add_emulation_prevention(bw.out);
    });
    deblock(*f, dbs, 0, o.threads);
    EncodedPicture& ep = out[size_t(i)];
    ep.nals = std::move(nals);
    if (o.keep_recon) {
      ep.y = f->y;
      ep.cb = f->cb;
      ep.cr = f->cr;
    }
    if (nal_ref_idc) {
      const int id = next_id++;
      prev_ref_fn = mark_reference(dpb, RefPic{f, id, frame_num}, max_fn, o.max_refs, false, {});
      planes.erase(std::remove_if(planes.begin(), planes.end(),
                                  [&](const std::pair<int, std::shared_ptr<HalfPel>>& pp) {
                                    return std::none_of(dpb.begin(), dpb.end(),
                                                         [&](const RefPic& r) { return r.id == pp.first; });
                                  }),
                   planes.end());
      if (!o.seed) {                       // production search reads half-sample planes of ref 0
        auto hp = std::make_shared<HalfPel>();
        hp->build(*f, 32, o.threads);
        planes.emplace_back(id, hp);
      }
    }
  }
  return out;
}

bool tables_prefix_free() {
  try {
    (void)tables();
  } catch (const std::logic_error&) {
    return false;
  }
  // me(v) intra cbp table must be a permutation of 0..47
  bool seen[48] = {false};
  for (int v : kIntraCbp) {
    if (v >= 48 || seen[v]) return false;
    seen[v] = true;
  }
  return true;
}

// ------------------------------------------------------------------------------------ decoder
namespace {

struct Sps {
  bool ok = false;
  int mbw = 0, mbh = 0, log2_max_frame_num = 4, poc_type = 0, log2_max_poc_lsb = 4, max_refs = 1;
  bool delta_pic_order_always_zero = false, gaps_allowed = false;
  int crop_l = 0, crop_r = 0, crop_t = 0, crop_b = 0;
};
struct Pps {
  bool ok = false;
  int sps_id = 0, init_qp = 26, chroma_qp_offset = 0, num_ref_default = 1;
  bool bottom_field_pic_order = false, deblocking_control = false, redundant_pic_cnt = false;
  bool weighted_pred = false, constrained_intra = false;
};

Sps parse_sps(BitReader& br) {
  Sps s;
  const int profile = int(br.u(8));
  br.u(8);  // constraint flags + reserved
  br.u(8);  // level
  const uint32_t id = br.ue();
  if (id != 0) throw std::runtime_error("h264: only seq_parameter_set_id 0 is supported");
  if (profile == 100 || profile == 110 || profile == 122 || profile == 244 || profile == 44 || profile == 83 ||
      profile == 86 || profile == 118 || profile == 128)
    throw std::runtime_error("h264: High / scalable profiles are not supported (Baseline only)");
  const uint32_t lmf = br.ue(), poc_type = br.ue();
  if (lmf > 12 || poc_type > 2) throw std::runtime_error("h264: SPS field out of range");
  s.log2_max_frame_num = int(lmf) + 4;
  s.poc_type = int(poc_type);
  if (s.poc_type == 0) {
    const uint32_t lpl = br.ue();
    if (lpl > 12) throw std::runtime_error("h264: SPS field out of range");
    s.log2_max_poc_lsb = int(lpl) + 4;
  } else if (s.poc_type == 1) {
    s.delta_pic_order_always_zero = br.u(1);
    br.se();
    br.se();
    const uint32_t n = br.ue();
    if (n > 255) throw std::runtime_error("h264: SPS field out of range");
    for (uint32_t i = 0; i < n; ++i) br.se();
  }
  const uint32_t refs = br.ue();
  if (refs > 16) throw std::runtime_error("h264: max_num_ref_frames out of range");
  s.max_refs = std::max(1, int(refs));
  s.gaps_allowed = br.u(1);
  const uint32_t mbw = br.ue(), mbh = br.ue();
  if (mbw >= 256 || mbh >= 256 || (uint64_t(mbw) + 1) * (mbh + 1) > 36864)   // <= 4096 x 2304 (level 5.1)
    throw std::runtime_error("h264: picture too large");
  s.mbw = int(mbw) + 1;
  s.mbh = int(mbh) + 1;
  if (!br.u(1)) throw std::runtime_error("h264: interlaced (frame_mbs_only_flag = 0) is not supported");
  br.u(1);  // direct_8x8_inference_flag
  if (br.u(1)) {
    const uint32_t l = br.ue(), r = br.ue(), t = br.ue(), b = br.ue();
    if (2 * (uint64_t(l) + r) >= uint64_t(16) * s.mbw || 2 * (uint64_t(t) + b) >= uint64_t(16) * s.mbh)
      throw std::runtime_error("h264: bad cropping window");
    s.crop_l = int(l);
    s.crop_r = int(r);
    s.crop_t = int(t);
    s.crop_b = int(b);
  }
  s.ok = true;
  return s;
}

Pps parse_pps(BitReader& br) {
  Pps p;
  if (br.ue() != 0) throw std::runtime_error("h264: only pic_parameter_set_id 0 is supported");
  if (br.ue() != 0) throw std::runtime_error("h264: only seq_parameter_set_id 0 is supported");
  p.sps_id = 0;
  if (br.u(1)) throw std::runtime_error("h264: CABAC is not supported");
  p.bottom_field_pic_order = br.u(1);
  if (br.ue() != 0) throw std::runtime_error("h264: slice groups (FMO) are not supported");
  const uint32_t l0 = br.ue();
  br.ue();
  if (l0 > 31) throw std::runtime_error("h264: PPS field out of range");
  p.num_ref_default = int(l0) + 1;
  p.weighted_pred = br.u(1);
  br.u(2);
  const int64_t init_qp = 26 + int64_t(br.se());   // int64: a hostile se() must not overflow
  br.se();
  const int64_t cqo = br.se();
  if (init_qp < 0 || init_qp > 51 || cqo < -12 || cqo > 12) throw std::runtime_error("h264: PPS field out of range");
  p.init_qp = int(init_qp);
  p.chroma_qp_offset = int(cqo);
  p.deblocking_control = br.u(1);
  p.constrained_intra = br.u(1);
  p.redundant_pic_cnt = br.u(1);
  if (br.more_rbsp_data()) throw std::runtime_error("h264: PPS extensions (8x8 transform) are not supported");
  p.ok = true;
  return p;
}

// Parsed slice header (7.3.3) - the part the picture level needs before the macroblocks
struct SliceHdr {
  int first_mb = 0, slice_type = 2, frame_num = 0, nal_type = 5, nal_ref_idc = 0;
  int num_ref_active = 1, qp = 26;
  SliceDb db;
  std::vector<std::pair<int, int>> list_mods;    // (modification_of_pic_nums_idc, abs_diff_pic_num_minus1)
  std::vector<std::pair<int, int>> mmco;         // (op, difference_of_pic_nums_minus1)
  bool adaptive_marking = false;
};

SliceHdr parse_slice_header(BitReader& br, int nal_type, int nal_ref_idc, const Sps& sps, const Pps& pps, int nmb) {
  SliceHdr h;
  h.nal_type = nal_type;
  h.nal_ref_idc = nal_ref_idc;
  // untrusted input: range-check every exp-golomb value as uint32 before it becomes an index
  const uint32_t first_mb_u = br.ue();
  if (first_mb_u >= uint32_t(nmb)) throw std::runtime_error("h264: first_mb_in_slice out of range");
  h.first_mb = int(first_mb_u);
  h.slice_type = int(br.ue() % 5);
  if (h.slice_type != 2 && h.slice_type != 0)
    throw std::runtime_error("h264: only I and P slices are supported (no B/SP/SI)");
  if (nal_type == 5 && h.slice_type != 2) throw std::runtime_error("h264: IDR picture with a P slice");
  br.ue();  // pps id (checked == 0 by the PPS parser's single-PPS rule)
  h.frame_num = int(br.u(sps.log2_max_frame_num));
  if (nal_type == 5) br.ue();  // idr_pic_id
  if (sps.poc_type == 0) {
    br.u(sps.log2_max_poc_lsb);
    if (pps.bottom_field_pic_order) br.se();
  } else if (sps.poc_type == 1 && !sps.delta_pic_order_always_zero) {
    br.se();
    if (pps.bottom_field_pic_order) br.se();
  }
  if (pps.redundant_pic_cnt && br.ue() != 0) throw std::runtime_error("h264: redundant pictures are not supported");
  h.num_ref_active = pps.num_ref_default;
  if (h.slice_type == 0) {
    if (br.u(1)) {                                  // num_ref_idx_active_override_flag
      const uint32_t n = br.ue();
      if (n > 15) throw std::runtime_error("h264: num_ref_idx_l0_active out of range");
      h.num_ref_active = int(n) + 1;
    }
    if (br.u(1)) {                                  // ref_pic_list_modification_flag_l0
      for (int guard = 0;; ++guard) {
        if (guard > 32) throw std::runtime_error("h264: too many reference list modifications");
        const uint32_t idc = br.ue();
        if (idc == 3) break;
        if (idc > 2) throw std::runtime_error("h264: bad modification_of_pic_nums_idc");
        if (idc == 2) throw std::runtime_error("h264: long-term references are not supported");
        const uint32_t v = br.ue();
        if (v > (1u << 16)) throw std::runtime_error("h264: abs_diff_pic_num out of range");
        h.list_mods.emplace_back(int(idc), int(v));
      }
    }
    if (pps.weighted_pred) throw std::runtime_error("h264: weighted prediction is not supported");
  }
  if (nal_ref_idc) {
    if (nal_type == 5) {
      br.u(1);                                      // no_output_of_prior_pics_flag
      if (br.u(1)) throw std::runtime_error("h264: long-term references are not supported");
    } else if (br.u(1)) {
      h.adaptive_marking = true;
      for (int guard = 0;; ++guard) {
        if (guard > 64) throw std::runtime_error("h264: too many memory management operations");
        const uint32_t op = br.ue();
        if (op == 0) break;
        if (op != 1 && op != 5) throw std::runtime_error("h264: long-term memory management is not supported");
        int v = 0;
        if (op == 1) {
          const uint32_t d = br.ue();
          if (d > (1u << 16)) throw std::runtime_error("h264: difference_of_pic_nums out of range");
          v = int(d);
        }
        h.mmco.emplace_back(int(op), v);
      }
    }
  }
  const int64_t qp0 = pps.init_qp + int64_t(br.se());
  if (qp0 < 0 || qp0 > 51) throw std::runtime_error("h264: slice QP out of range");
  h.qp = int(qp0);
  h.db = SliceDb{0, 0, 0};
  if (pps.deblocking_control) {
    const uint32_t idc = br.ue();
    if (idc > 2) throw std::runtime_error("h264: bad disable_deblocking_filter_idc");
    h.db.idc = int(idc);
    if (idc != 1) {
      const int64_t a = br.se(), b = br.se();
      if (a < -6 || a > 6 || b < -6 || b > 6) throw std::runtime_error("h264: deblocking offsets out of range");
      h.db.offa = int(a) * 2;
      h.db.offb = int(b) * 2;
    }
  }
  return h;
}

struct SliceCtx {
  const Pps& pps;
  const SliceHdr& hdr;
  const std::vector<RefPic>& list;   // RefPicList0 (P slices)
  int slice_id;
};

int read_te(BitReader& br, int range) {    // te(v), range = num_ref_idx_active - 1 >= 1
  if (range == 1) return br.u(1) ? 0 : 1;
  const uint32_t v = br.ue();
  if (v > uint32_t(range)) throw std::runtime_error("h264: ref_idx out of range");
  return int(v);
}

// luma / chroma residual of a non-Intra_16x16 macroblock (cbp-driven), TotalCoeff tables updated
void read_residual(BitReader& br, Frame& f, int mx, int my, int cbp, int (*coef)[16], int (*cdc)[4],
                   int (*cac)[4][15], int slice_id) {
  const int cbp_luma = cbp & 15, cbp_chroma = cbp >> 4;
  std::memset(coef, 0, sizeof(int) * 256);
  for (int blk = 0; blk < 16; ++blk) {
    const int bx = 4 * mx + kBlkX[blk], by = 4 * my + kBlkY[blk];
    int tc = 0;
    if (cbp_luma & (1 << (blk / 4))) tc = read_block(br, coef[blk], 16, f.nc(f.tc_y, bx, by, 4, slice_id));
    f.tc_y[size_t(by) * 4 * f.mbw + bx] = uint8_t(tc);
  }
  std::memset(cdc, 0, sizeof(int) * 8);
  std::memset(cac, 0, sizeof(int) * 120);
  if (cbp_chroma)
    for (int c = 0; c < 2; ++c) read_block(br, cdc[c], 4, -1);
  for (int c = 0; c < 2; ++c) {
    std::vector<uint8_t>& tcs = c ? f.tc_cr : f.tc_cb;
    for (int blk = 0; blk < 4; ++blk) {
      const int bx = 2 * mx + (blk & 1), by = 2 * my + (blk >> 1);
      int tc = 0;
      if (cbp_chroma == 2) tc = read_block(br, cac[c][blk], 15, f.nc(tcs, bx, by, 2, slice_id));
      tcs[size_t(by) * 2 * f.mbw + bx] = uint8_t(tc);
    }
  }
}

// Intra macroblock (mb_type in I-slice numbering 0..25) at (mx, my)
void decode_intra_mb(BitReader& br, Frame& f, int mx, int my, uint32_t mb_type, int& qp, const Pps& pps,
                     int slice_id) {
  const Nb nb = f.nb(mx, my, slice_id);
  const int Wc = f.W / 2;
  auto qp_delta = [&](int q) {
    const int64_t d = br.se();
    if (d < -26 || d > 25) throw std::runtime_error("h264: mb_qp_delta out of range");
    return (q + int(d) + 52) % 52;
  };
  mark_intra(f, mx, my);
  if (mb_type == 25) {  // I_PCM
    while (!br.byte_aligned()) br.u(1);
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) f.y[size_t(my * 16 + y) * f.W + mx * 16 + x] = uint8_t(br.u(8));
    for (auto* pl : {&f.cb, &f.cr})
      for (int y = 0; y < 8; ++y)
        for (int x = 0; x < 8; ++x) (*pl)[size_t(my * 8 + y) * Wc + mx * 8 + x] = uint8_t(br.u(8));
    for (int b = 0; b < 16; ++b) {
      const size_t i = size_t(4 * my + b / 4) * 4 * f.mbw + 4 * mx + b % 4;
      f.tc_y[i] = 16;
      f.i4mode[i] = -1;
    }
    for (int b = 0; b < 4; ++b) {
      const size_t i = size_t(2 * my + b / 2) * 2 * f.mbw + 2 * mx + b % 2;
      f.tc_cb[i] = f.tc_cr[i] = 16;
    }
    f.mbqp[size_t(my) * f.mbw + mx] = 0;     // deblocking treats I_PCM as QP 0
    return;
  }
  if (mb_type >= 1 && mb_type <= 24) {  // I_16x16
    const int mode = int(mb_type - 1) % 4, cbp_chroma = (int(mb_type - 1) / 4) % 3;
    const int cbp_luma = mb_type >= 13 ? 15 : 0;
    const uint32_t cmode_u = br.ue();
    if (cmode_u > 3) throw std::runtime_error("h264: bad intra_chroma_pred_mode");
    const int cmode = int(cmode_u);
    qp = qp_delta(qp);
    if ((mode == 0 && !nb.top) || (mode == 1 && !nb.left) || (mode == 3 && !(nb.top && nb.left && nb.topleft)))
      throw std::runtime_error("h264: Intra_16x16 mode uses unavailable samples");
    int dc[16], ac[16][15];
    std::memset(ac, 0, sizeof(ac));
    read_block(br, dc, 16, f.nc(f.tc_y, 4 * mx, 4 * my, 4, slice_id));
    for (int blk = 0; blk < 16; ++blk) {
      const int bx = 4 * mx + kBlkX[blk], by = 4 * my + kBlkY[blk];
      int tc = 0;
      if (cbp_luma) tc = read_block(br, ac[blk], 15, f.nc(f.tc_y, bx, by, 4, slice_id));
      f.tc_y[size_t(by) * 4 * f.mbw + bx] = uint8_t(tc);
      f.i4mode[size_t(by) * 4 * f.mbw + bx] = -1;
    }
    uint8_t pred[256];
    pred16(f.y.data(), f.W, mx * 16, my * 16, nb, mode, pred);
    recon_luma16(f, mx, my, pred, dc, ac, qp);
    int cdc[2][4] = {{0}}, cac[2][4][15];
    std::memset(cac, 0, sizeof(cac));
    if (cbp_chroma)
      for (int c = 0; c < 2; ++c) read_block(br, cdc[c], 4, -1);
    for (int c = 0; c < 2; ++c) {
      std::vector<uint8_t>& tcs = c ? f.tc_cr : f.tc_cb;
      for (int blk = 0; blk < 4; ++blk) {
        const int bx = 2 * mx + (blk & 1), by = 2 * my + (blk >> 1);
        int tc = 0;
        if (cbp_chroma == 2) tc = read_block(br, cac[c][blk], 15, f.nc(tcs, bx, by, 2, slice_id));
        tcs[size_t(by) * 2 * f.mbw + bx] = uint8_t(tc);
      }
    }
    if ((cmode == 1 && !nb.left) || (cmode == 2 && !nb.top) || (cmode == 3 && !(nb.top && nb.left && nb.topleft)))
      throw std::runtime_error("h264: chroma mode uses unavailable samples");
    const int qpc = kChromaQp[std::clamp(qp + pps.chroma_qp_offset, 0, 51)];
    for (int c = 0; c < 2; ++c) {
      std::vector<uint8_t>& pl = c ? f.cr : f.cb;
      uint8_t cp[64];
      pred_chroma(pl.data(), Wc, mx * 8, my * 8, nb, cmode, cp);
      recon_chroma(pl, Wc, mx, my, cp, cdc[c], cac[c], qpc);
    }
    f.mbqp[size_t(my) * f.mbw + mx] = uint8_t(qp);
    return;
  }
  if (mb_type != 0) throw std::runtime_error("h264: macroblock type out of range");
  // I_NxN (intra 4x4)
  int modes[16];
  for (int blk = 0; blk < 16; ++blk) {
    const int bx = 4 * mx + kBlkX[blk], by = 4 * my + kBlkY[blk];
    const bool ia = kBlkX[blk] ? true : nb.left, ib = kBlkY[blk] ? true : nb.top;
    int pred_mode = 2;
    if (ia && ib) {
      const int ma = f.i4mode[size_t(by) * 4 * f.mbw + bx - 1], mb_ = f.i4mode[size_t(by - 1) * 4 * f.mbw + bx];
      pred_mode = std::min(ma < 0 ? 2 : ma, mb_ < 0 ? 2 : mb_);
    }
    int m = pred_mode;
    if (!br.u(1)) {
      const int rem = int(br.u(3));
      m = rem < pred_mode ? rem : rem + 1;
    }
    modes[blk] = m;
    f.i4mode[size_t(by) * 4 * f.mbw + bx] = int8_t(m);
  }
  const uint32_t cmode_u = br.ue();
  if (cmode_u > 3) throw std::runtime_error("h264: bad intra_chroma_pred_mode");
  const int cmode = int(cmode_u);
  const uint32_t cbp_code = br.ue();
  if (cbp_code > 47) throw std::runtime_error("h264: bad coded_block_pattern");
  const int cbp = kIntraCbp[cbp_code];
  if (cbp) qp = qp_delta(qp);
  int coef[16][16], cdc[2][4], cac[2][4][15];
  read_residual(br, f, mx, my, cbp, coef, cdc, cac, slice_id);
  // luma reconstruction block by block (later blocks predict from earlier ones)
  for (int blk = 0; blk < 16; ++blk) {
    const int lx = 4 * kBlkX[blk], ly = 4 * kBlkY[blk];
    const int x0 = mx * 16 + lx, y0 = my * 16 + ly;
    const bool has_left = lx ? true : nb.left, has_top = ly ? true : nb.top;
    bool has_tl = (lx && ly) ? true : (lx ? nb.top : (ly ? nb.left : nb.topleft));
    bool has_tr;
    if (ly == 0) has_tr = lx < 12 ? nb.top : nb.topright;
    else if (lx == 12) has_tr = false;
    else {
      const int bxr = kBlkX[blk] + 1, byr = kBlkY[blk] - 1;
      int idx = 0;
      for (int k = 0; k < 16; ++k)
        if (kBlkX[k] == bxr && kBlkY[k] == byr) idx = k;
      has_tr = idx < blk;
    }
    const int m = modes[blk];
    if (((m == 0 || m == 3 || m == 7) && !has_top) || ((m == 1 || m == 8) && !has_left) ||
        ((m == 4 || m == 5 || m == 6) && !(has_top && has_left && has_tl)))
      throw std::runtime_error("h264: Intra_4x4 mode uses unavailable samples");
    int t[9] = {0}, l[4] = {0};
    if (has_tl) t[0] = f.y[size_t(y0 - 1) * f.W + x0 - 1];
    if (has_top) {
      for (int i = 0; i < 4; ++i) t[1 + i] = f.y[size_t(y0 - 1) * f.W + x0 + i];
      for (int i = 4; i < 8; ++i) t[1 + i] = has_tr ? f.y[size_t(y0 - 1) * f.W + x0 + i] : t[4];
    }
    if (has_left)
      for (int i = 0; i < 4; ++i) l[i] = f.y[size_t(y0 + i) * f.W + x0 - 1];
    int p[16], d[16], r[16];
    pred4(t, l, m, has_top, has_left, p);
    for (int k = 0; k < 16; ++k) {
      const int rp = kZigzag[k];
      d[rp] = coef[blk][k] ? dequant(coef[blk][k], qp, rp) : 0;
    }
    inv4x4(d, r);
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) f.y[size_t(y0 + y) * f.W + x0 + x] = clip255(p[4 * y + x] + r[4 * y + x]);
  }
  if ((cmode == 1 && !nb.left) || (cmode == 2 && !nb.top) || (cmode == 3 && !(nb.top && nb.left && nb.topleft)))
    throw std::runtime_error("h264: chroma mode uses unavailable samples");
  const int qpc = kChromaQp[std::clamp(qp + pps.chroma_qp_offset, 0, 51)];
  for (int c = 0; c < 2; ++c) {
    std::vector<uint8_t>& pl = c ? f.cr : f.cb;
    uint8_t cp[64];
    pred_chroma(pl.data(), Wc, mx * 8, my * 8, nb, cmode, cp);
    recon_chroma(pl, Wc, mx, my, cp, cdc[c], cac[c], qpc);
  }
  f.mbqp[size_t(my) * f.mbw + mx] = uint8_t(qp);
}

void recon_inter(Frame& f, const SliceCtx& sc, int mx, int my, const int (*coef)[16], const int (*cdc)[4],
                 const int (*cac)[4][15], int qp) {
  uint8_t py[256], pc[2][64];
  predict_inter(f, sc.list, mx, my, py, pc[0], pc[1]);
  recon_luma4x4(f, mx, my, py, coef, qp);
  const int qpc = kChromaQp[std::clamp(qp + sc.pps.chroma_qp_offset, 0, 51)];
  for (int c = 0; c < 2; ++c) recon_chroma(c ? f.cr : f.cb, f.W / 2, mx, my, pc[c], cdc[c], cac[c], qpc);
  f.intra[size_t(my) * f.mbw + mx] = 0;
  f.mbqp[size_t(my) * f.mbw + mx] = uint8_t(qp);
}

void decode_skip(Frame& f, const SliceCtx& sc, int mx, int my, int qp) {
  MvPred mp{f, mx, my, sc.slice_id};
  int px, py;
  mp.skip(px, py);
  if (sc.list.empty() || !sc.list[0].f) throw std::runtime_error("h264: P_Skip without a reference picture");
  set_motion(f, mp, mx, my, 0, 0, 4, 4, 0, sc.list[0].id, px, py);
  int coef[16][16] = {{0}}, cdc[2][4] = {{0}}, cac[2][4][15];
  std::memset(cac, 0, sizeof(cac));
  for (int y = 0; y < 4; ++y)
    for (int x = 0; x < 4; ++x) f.tc_y[size_t(4 * my + y) * 4 * f.mbw + 4 * mx + x] = 0;
  for (int y = 0; y < 2; ++y)
    for (int x = 0; x < 2; ++x) f.tc_cb[size_t(2 * my + y) * 2 * f.mbw + 2 * mx + x] =
        f.tc_cr[size_t(2 * my + y) * 2 * f.mbw + 2 * mx + x] = 0;
  for (int b = 0; b < 16; ++b) f.i4mode[size_t(4 * my + b / 4) * 4 * f.mbw + 4 * mx + b % 4] = -1;
  recon_inter(f, sc, mx, my, coef, cdc, cac, qp);
}

// P macroblock types 0..4 (Table 7-13): partitions, sub-partitions, ref_idx, mvd, cbp, residual
void decode_inter_mb(BitReader& br, Frame& f, const SliceCtx& sc, int mx, int my, uint32_t mb_type, int& qp) {
  const int nref = sc.hdr.num_ref_active;
  MvPred mp{f, mx, my, sc.slice_id};
  auto need_ref = [&](int r) {
    if (size_t(r) >= sc.list.size() || !sc.list[size_t(r)].f)
      throw std::runtime_error("h264: ref_idx names no reference picture");
    return sc.list[size_t(r)].id;
  };
  auto mvd = [&]() {
    const int64_t x = br.se(), y = br.se();
    if (x < -8192 || x > 8191 || y < -2048 || y > 2047) throw std::runtime_error("h264: mvd out of range");
    return std::make_pair(int(x), int(y));
  };
  auto add_mv = [](int p, int d, int lo, int hi) {
    const int v = p + d;
    if (v < lo || v > hi) throw std::runtime_error("h264: motion vector out of range");
    return v;
  };
  if (mb_type <= 2) {
    const int nparts = mb_type == 0 ? 1 : 2;
    int refs[2] = {0, 0};
    for (int p = 0; p < nparts; ++p) refs[p] = nref > 1 ? read_te(br, nref - 1) : 0;
    for (int p = 0; p < nparts; ++p) {
      const auto d = mvd();
      int bx = 0, by = 0, bw = 4, bh = 4, shape = 0;
      if (mb_type == 1) { by = 2 * p; bh = 2; shape = 1 + p; }
      if (mb_type == 2) { bx = 2 * p; bw = 2; shape = 3 + p; }
      int px, py;
      mp.pred(bx, by, bw, refs[p], shape, px, py);
      set_motion(f, mp, mx, my, bx, by, bw, bh, refs[p], need_ref(refs[p]), add_mv(px, d.first, -8192, 8191),
                 add_mv(py, d.second, -2048, 2047));
    }
  } else if (mb_type <= 4) {
    int sub[4], refs[4] = {0, 0, 0, 0};
    for (int s = 0; s < 4; ++s) {
      const uint32_t t = br.ue();
      if (t > 3) throw std::runtime_error("h264: bad sub_mb_type");
      sub[s] = int(t);
    }
    if (mb_type == 3 && nref > 1)
      for (int s = 0; s < 4; ++s) refs[s] = read_te(br, nref - 1);
    for (int s = 0; s < 4; ++s) {
      const int sx = 2 * (s & 1), sy = 2 * (s >> 1);
      const int n = sub[s] == 0 ? 1 : sub[s] == 3 ? 4 : 2;
      const int pw = sub[s] == 0 || sub[s] == 1 ? 2 : 1, ph = sub[s] == 0 || sub[s] == 2 ? 2 : 1;
      for (int k = 0; k < n; ++k) {
        const auto d = mvd();
        const int bx = sx + (sub[s] == 2 || sub[s] == 3 ? (k & 1) : 0);
        const int by = sy + (sub[s] == 1 ? k : sub[s] == 3 ? (k >> 1) : 0);
        int px, py;
        mp.pred(bx, by, pw, refs[s], 0, px, py);
        set_motion(f, mp, mx, my, bx, by, pw, ph, refs[s], need_ref(refs[s]), add_mv(px, d.first, -8192, 8191),
                   add_mv(py, d.second, -2048, 2047));
      }
    }
  } else {
    throw std::runtime_error("h264: P macroblock type out of range");
  }
  const uint32_t cbp_code = br.ue();
  if (cbp_code > 47) throw std::runtime_error("h264: bad coded_block_pattern");
  const int cbp = kInterCbp[cbp_code];
  if (cbp) {
    const int64_t d = br.se();
    if (d < -26 || d > 25) throw std::runtime_error("h264: mb_qp_delta out of range");
    qp = (qp + int(d) + 52) % 52;
  }
  int coef[16][16], cdc[2][4], cac[2][4][15];
  read_residual(br, f, mx, my, cbp, coef, cdc, cac, sc.slice_id);
  for (int b = 0; b < 16; ++b) f.i4mode[size_t(4 * my + b / 4) * 4 * f.mbw + 4 * mx + b % 4] = -1;
  recon_inter(f, sc, mx, my, coef, cdc, cac, qp);
}

// Macroblocks of one slice: [first_mb, end_mb), f.slice already holds the slice id over that range
// (slices of a picture decode concurrently; neighbours in other slices are never read).
void decode_slice_data(BitReader& br, Frame& f, const SliceCtx& sc, int end_mb, std::vector<uint8_t>& done) {
  const int nmb = f.mbw * f.mbh;
  const bool p_slice = sc.hdr.slice_type == 0;
  int qp = sc.hdr.qp;
  int mb = sc.hdr.first_mb;
  auto claim = [&](int m) {
    if (m >= nmb) throw std::runtime_error("h264: slice data past the last macroblock");
    if (m >= end_mb) throw std::runtime_error("h264: slice overlaps the next slice");
    done[size_t(m)] = 1;
  };
  bool more = true;
  while (more) {
    if (p_slice) {
      const uint32_t run = br.ue();
      if (run > uint32_t(nmb - mb)) throw std::runtime_error("h264: mb_skip_run out of range");
      for (uint32_t i = 0; i < run; ++i, ++mb) {
        claim(mb);
        decode_skip(f, sc, mb % f.mbw, mb / f.mbw, qp);
      }
      if (run > 0 && !br.more_rbsp_data()) break;
    }
    claim(mb);
    const int mx = mb % f.mbw, my = mb / f.mbw;
    const uint32_t mb_type = br.ue();
    if (p_slice && mb_type < 5) {
      decode_inter_mb(br, f, sc, mx, my, mb_type, qp);
    } else {
      const uint32_t it = p_slice ? mb_type - 5 : mb_type;
      if (it > 25) throw std::runtime_error("h264: macroblock type not allowed in this slice");
      decode_intra_mb(br, f, mx, my, it, qp, sc.pps, sc.slice_id);
    }
    ++mb;
    more = br.more_rbsp_data();
  }
}

}  // namespace

void decode(const std::vector<std::string>& nals, int threads, const LayoutFn& on_layout, const PictureSink& sink,
            std::vector<SideInfo>* side, uint64_t max_samples) {
  // Pass 1 (sequential): parameter sets and the split into pictures (a picture starts at a slice with
  // first_mb_in_slice == 0), grouped into coded video sequences from IDR to IDR.  Pass 2: every
  // sequence decodes in order (P pictures reference earlier ones); sequences run in parallel.
  struct Pic {
    Sps sps;
    Pps pps;
    std::vector<std::pair<int, std::string>> slices;  // (nal header byte, rbsp)
  };
  Sps sps;
  Pps pps;
  std::vector<std::vector<Pic>> seqs;
  size_t npics = 0;
  for (const std::string& nal : nals) {
    if (nal.empty()) continue;
    const uint8_t h = uint8_t(nal[0]);
    if (h & 0x80) throw std::runtime_error("h264: forbidden_zero_bit set");
    const int type = h & 0x1F;
    std::string rbsp = strip_emulation_prevention(reinterpret_cast<const uint8_t*>(nal.data()) + 1, nal.size() - 1);
    if (type == 7) {
      BitReader br(rbsp);
      sps = parse_sps(br);
    } else if (type == 8) {
      BitReader br(rbsp);
      pps = parse_pps(br);
    } else if (type == 5 || type == 1) {
      if (!sps.ok || !pps.ok) throw std::runtime_error("h264: slice before SPS/PPS");
      BitReader peek(rbsp);
      if (peek.ue() == 0) {
        if (type == 5 || seqs.empty()) seqs.emplace_back();
        seqs.back().push_back(Pic{sps, pps, {}});
        ++npics;
      }
      if (seqs.empty() || seqs.back().empty())
        throw std::runtime_error("h264: slice of a picture without its first macroblock");
      seqs.back().back().slices.emplace_back(h, std::move(rbsp));
    } else if (type == 9 || type == 6 || type == 10 || type == 11 || type == 12) {
      // access unit delimiter, SEI, end of sequence / stream, filler: ignored
    } else {
      throw std::runtime_error("h264: unsupported NAL unit type " + std::to_string(type));
    }
  }
  // untrusted input: a few bits per macroblock can declare huge pictures, so bound what decoding
  // may allocate: 4K per picture via the SPS limits, max_samples luma samples in total (default
  // 2^30: ~1.6 GB of 4:2:0 planes or ~3.2 GB of RGB, about 17 s of 1080p at 30 fps)
  uint64_t samples = 0;
  for (const auto& sq : seqs)
    for (const Pic& j : sq) samples += uint64_t(j.sps.mbw) * j.sps.mbh * 256;
  if (samples > max_samples) throw std::runtime_error("h264: video too large to decode");
  std::vector<size_t> base(seqs.size(), 0);
  for (size_t s = 1; s < seqs.size(); ++s) base[s] = base[s - 1] + seqs[s - 1].size();
  std::vector<std::pair<int, int>> crops;
  for (const auto& sq : seqs)
    for (const Pic& j : sq) {
      const int cw = 16 * j.sps.mbw - 2 * (j.sps.crop_l + j.sps.crop_r);
      const int ch = 16 * j.sps.mbh - 2 * (j.sps.crop_t + j.sps.crop_b);
      if (cw <= 0 || ch <= 0) throw std::runtime_error("h264: bad cropping window");
      crops.emplace_back(cw, ch);
    }
  if (on_layout) on_layout(crops);
  if (side) side->assign(npics, SideInfo{});
  std::vector<std::string> errors(seqs.size());
  int inner_threads = 1;                  // slices of one picture in parallel when sequences are few
  auto run_seq = [&](size_t s) {
    std::vector<RefPic> dpb;              // short-term reference pictures
    int prev_ref_frame_num = 0, next_id = 1;
    for (size_t k = 0; k < seqs[s].size(); ++k) {
      const Pic& j = seqs[s][k];
      auto f = std::make_shared<Frame>(j.sps.mbw, j.sps.mbh);
      f->constrained_intra = j.pps.constrained_intra;
      const int nmb = f->mbw * f->mbh, max_fn = 1 << j.sps.log2_max_frame_num;
      // slice headers first (picture-level state, ranges), then the slices' macroblocks in parallel
      const size_t ns = j.slices.size();
      std::vector<SliceHdr> hdrs;
      std::vector<BitReader> readers;
      hdrs.reserve(ns);
      readers.reserve(ns);
      for (size_t si = 0; si < ns; ++si) {
        const auto& sl = j.slices[si];
        readers.emplace_back(sl.second);
        hdrs.push_back(parse_slice_header(readers.back(), sl.first & 0x1F, (sl.first >> 5) & 3, j.sps, j.pps, nmb));
        if (si > 0 && hdrs[si].first_mb <= hdrs[si - 1].first_mb)
          throw std::runtime_error("h264: slices out of order (arbitrary slice order is not supported)");
        if (si > 0 && (hdrs[si].nal_type != hdrs[0].nal_type || hdrs[si].frame_num != hdrs[0].frame_num ||
                       (hdrs[si].nal_ref_idc != 0) != (hdrs[0].nal_ref_idc != 0)))
          throw std::runtime_error("h264: slices of one picture disagree");
      }
      const SliceHdr& first = hdrs[0];
      if (first.nal_type == 5) {
        dpb.clear();
        prev_ref_frame_num = 0;
      } else if (first.frame_num != prev_ref_frame_num && first.frame_num != (prev_ref_frame_num + 1) % max_fn &&
                 !j.sps.gaps_allowed) {
        throw std::runtime_error("h264: gap in frame_num (lost reference pictures)");
      }
      std::vector<SliceDb> dbs;
      std::vector<std::vector<RefPic>> lists(ns);
      for (size_t si = 0; si < ns; ++si) {
        dbs.push_back(hdrs[si].db);
        if (hdrs[si].slice_type == 0)
          lists[si] = ref_list0(dpb, hdrs[si].frame_num, max_fn, hdrs[si].list_mods, hdrs[si].num_ref_active);
        const int end = si + 1 < ns ? hdrs[si + 1].first_mb : nmb;
        for (int m = hdrs[si].first_mb; m < end; ++m) f->slice[size_t(m)] = int(si);
      }
      std::vector<uint8_t> done(size_t(nmb), 0);
      parallel_for(int(ns), inner_threads, [&](int si) {
        const SliceCtx sc{j.pps, hdrs[size_t(si)], lists[size_t(si)], si};
        const int end = size_t(si) + 1 < ns ? hdrs[size_t(si) + 1].first_mb : nmb;
        decode_slice_data(readers[size_t(si)], *f, sc, end, done);
      });
      for (uint8_t d : done)
        if (!d) throw std::runtime_error("h264: picture has undecoded macroblocks");
      const size_t idx = base[s] + k;
      if (side) {                                   // test hook: the unfiltered picture + filter inputs
        SideInfo& si = (*side)[idx];
        si.y = f->y;
        si.cb = f->cb;
        si.cr = f->cr;
        si.mvx.assign(f->mvx.begin(), f->mvx.end());
        si.mvy.assign(f->mvy.begin(), f->mvy.end());
        si.refpic = f->refpic;
        si.nonzero.assign(f->tc_y.begin(), f->tc_y.end());
        si.intra = f->intra;
        si.qp = f->mbqp;
        si.slice = f->slice;
        for (const SliceDb& d : dbs) si.deblock.push_back({d.idc, d.offa, d.offb});
        si.chroma_qp_offset = j.pps.chroma_qp_offset;
      }
      deblock(*f, dbs, j.pps.chroma_qp_offset, inner_threads);
      {
        Picture p;
        p.w16 = f->W;
        p.h16 = f->H;
        p.crop_w = crops[idx].first;
        p.crop_h = crops[idx].second;
        p.y = f->y;
        p.cb = f->cb;
        p.cr = f->cr;
        sink(idx, std::move(p), inner_threads);
      }
      if (first.nal_ref_idc)
        prev_ref_frame_num = mark_reference(dpb, RefPic{f, next_id++, first.frame_num}, max_fn, j.sps.max_refs,
                                            first.adaptive_marking, first.mmco);
    }
  };
  auto work = [&](int t, int nt) {
    for (size_t s = size_t(t); s < seqs.size(); s += size_t(nt)) {
      try {
        run_seq(s);
      } catch (const std::exception& e) {
        errors[s] = e.what();
      }
    }
  };
  const int nt = std::max(1, std::min<int>(threads, (int)seqs.size()));
  inner_threads = std::max(1, threads / nt);
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work, t, nt);
  work(0, nt);
  for (auto& th : pool) th.join();
  for (auto& e : errors)
    if (!e.empty()) throw std::runtime_error(e);
}

std::vector<Picture> decode(const std::vector<std::string>& nals, int threads) {
  std::vector<Picture> out;
  decode(
      nals, threads, [&](const std::vector<std::pair<int, int>>& crops) { out.resize(crops.size()); },
      [&](size_t i, Picture&& p, int) { out[i] = std::move(p); }, nullptr, kDefaultMaxSamples);
  return out;
}

}  // namespace h264
