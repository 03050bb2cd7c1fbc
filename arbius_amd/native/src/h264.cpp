// Deterministic H.264 Constrained-Baseline intra codec (CAVLC), see h264.h.
//
// Why it exists (SURVEY.md §2.6(c,d), VERDICT r1 "Harden video input and shrink video output"):
// the video templates (/root/reference/templates/zeroscopev2xl.json:1,
// robust_video_matting.json:6-31) return out-1.mp4 whose CID is the solution, so the encoder
// must be a pure function of the frames on every node, and there is no ffmpeg / libx264 in the
// image.  Round 1 wrote raw I_PCM macroblocks (~149 MB per 1080p 48-frame clip); this codec
// writes I_16x16 macroblocks with the integer 4x4 transform at a fixed QP, which is ~10-40x
// smaller and still decodable by every H.264 decoder (Constrained Baseline, CAVLC, deblocking
// disabled in the slice header so the reconstruction is exactly the decoder's output).
//
// Encoder: per macroblock the Intra_16x16 luma mode (V / H / DC / plane) and the chroma mode
// (DC / H / V / plane) are chosen by SAD over the source (integer, ties -> lowest mode);
// forward core transform + Hadamard DC, dead-zone quantisation (intra rounding 1/3), coded
// block patterns from the quantised levels; the reconstruction is the normative decoding
// process (ITU-T H.264 8.3.3, 8.3.4, 8.5.10-8.5.12) shared with the decoder below, so the
// encoder's recon == any decoder's output, bit for bit.
//
// Decoder: SPS/PPS/IDR + non-IDR I slices, CAVLC, I_PCM / I_16x16 / I_NxN (intra 4x4), multiple
// slices, 4:2:0 8-bit, deblocking disabled.  Everything else throws (the node then marks the
// task's input undecodable instead of failing the solve).
#include "h264.h"

#include <algorithm>
#include <cstring>
#include <memory>
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

std::string add_emulation_prevention(const std::string& rbsp) {
  // copy runs up to each 00 00 pair (rare in coded data), then apply the 00 00 0x -> 00 00 03 0x rule
  std::string out;
  out.reserve(rbsp.size() + rbsp.size() / 64 + 4);
  const char* p = rbsp.data();
  const size_t n = rbsp.size();
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
  int levels[16], runs[16], tc = 0, last = max_num - 1;
  while (last >= 0 && !coef[last]) --last;
  int zeros = 0;
  for (int i = last; i >= 0; --i) {   // reverse scan: runs[k] = zeros just below level k
    if (coef[i]) {
      if (tc) runs[tc - 1] = zeros;
      levels[tc++] = coef[i];
      zeros = 0;
    } else {
      ++zeros;
    }
  }
  if (tc) runs[tc - 1] = zeros;
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
  std::vector<uint8_t> tc_y, tc_cb, tc_cr;   // TotalCoeff per 4x4 block (nC prediction)
  std::vector<int> slice;                    // slice id per macroblock (-1: not decoded yet)
  std::vector<int8_t> i4mode;                // Intra4x4PredMode per 4x4 block, -1 = not I_NxN
  Frame(int mbw_, int mbh_) : mbw(mbw_), mbh(mbh_), W(16 * mbw_), H(16 * mbh_) {
    y.assign(size_t(W) * H, 0);
    cb.assign(size_t(W / 2) * (H / 2), 0);
    cr.assign(cb.size(), 0);
    tc_y.assign(size_t(4 * mbw) * 4 * mbh, 0);
    tc_cb.assign(size_t(2 * mbw) * 2 * mbh, 0);
    tc_cr.assign(tc_cb.size(), 0);
    slice.assign(size_t(mbw) * mbh, -1);
    i4mode.assign(tc_y.size(), -1);
  }
  bool avail(int mx, int my, int cur_slice) const {
    return mx >= 0 && my >= 0 && mx < mbw && my < mbh && slice[size_t(my) * mbw + mx] == cur_slice;
  }
  Nb nb(int mx, int my, int s) const {
    Nb n;
    n.left = avail(mx - 1, my, s);
    n.top = avail(mx, my - 1, s);
    n.topleft = avail(mx - 1, my - 1, s);
    n.topright = avail(mx + 1, my - 1, s);
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
void recon_luma16(Frame& f, int mx, int my, const uint8_t* pred, const int* dc, const int (*ac)[15], int qp) {
  int c[16], fdc[16];
  for (int k = 0; k < 16; ++k) c[kZigzag[k]] = dc[k];
  hadamard4(c, fdc);
  const int ls = level_scale(qp % 6, 0);
  for (int blk = 0; blk < 16; ++blk) {
    const int bx = kBlkX[blk], by = kBlkY[blk];
    const int fv = fdc[4 * by + bx];
    int d[16] = {0}, r[16];
    d[0] = qp >= 36 ? fv * ls * (1 << (qp / 6 - 6)) : (fv * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    for (int k = 0; k < 15; ++k) {
      const int rp = kZigzag[k + 1];
      if (ac[blk][k]) d[rp] = dequant(ac[blk][k], qp, rp);
    }
    inv4x4(d, r);
    uint8_t* dst = f.y.data() + size_t(my * 16 + 4 * by) * f.W + mx * 16 + 4 * bx;
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) dst[y * f.W + x] = clip255(pred[16 * (4 * by + y) + 4 * bx + x] + r[4 * y + x]);
  }
}

// chroma component: dc[4] raster (blkIdx) order, ac[4][15]
void recon_chroma(std::vector<uint8_t>& pl, int Wc, int mx, int my, const uint8_t* pred, const int* dc,
                  const int (*ac)[15], int qpc) {
  const int f0 = dc[0] + dc[1] + dc[2] + dc[3], f1 = dc[0] - dc[1] + dc[2] - dc[3];
  const int f2 = dc[0] + dc[1] - dc[2] - dc[3], f3 = dc[0] - dc[1] - dc[2] + dc[3];
  const int fv[4] = {f0, f1, f2, f3};
  const int ls = level_scale(qpc % 6, 0);
  for (int blk = 0; blk < 4; ++blk) {
    const int bx = blk & 1, by = blk >> 1;
    int d[16] = {0}, r[16];
    d[0] = (fv[blk] * ls * (1 << (qpc / 6))) >> 5;
    for (int k = 0; k < 15; ++k) {
      const int rp = kZigzag[k + 1];
      if (ac[blk][k]) d[rp] = dequant(ac[blk][k], qpc, rp);
    }
    inv4x4(d, r);
    uint8_t* dst = pl.data() + size_t(my * 8 + 4 * by) * Wc + mx * 8 + 4 * bx;
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) dst[y * Wc + x] = clip255(pred[8 * (4 * by + y) + 4 * bx + x] + r[4 * y + x]);
  }
}

// ------------------------------------------------------------------------------------ encoder
inline int quant(int w, int mf, int f, int qbits) {
  const int a = w < 0 ? -w : w;
  int z = (a * mf + f) >> qbits;   // |w| * mf < 2^31 for 8-bit residuals (luma DC: 32640 x 13107)
  z = std::min(z, 2047);
  return w < 0 ? -z : z;
}

int sad(const uint8_t* src, int stride, const uint8_t* pred, int n) {
  int s = 0;
  for (int y = 0; y < n; ++y)
    for (int x = 0; x < n; ++x) s += std::abs(int(src[y * stride + x]) - int(pred[n * y + x]));
  return s;
}

void encode_mb(BitWriter& bw, Frame& f, const uint8_t* sy, const uint8_t* scb, const uint8_t* scr, int mx, int my,
               int qp) {
  const Nb nb = f.nb(mx, my, 0);
  const int W = f.W, Wc = f.W / 2;
  // ---- luma mode
  uint8_t pred[256], best[256];
  int mode = 2, best_sad = 1 << 30;
  const uint8_t* src = sy + size_t(my * 16) * W + mx * 16;
  for (int m : {0, 1, 2, 3}) {
    if ((m == 0 && !nb.top) || (m == 1 && !nb.left) || (m == 3 && !(nb.top && nb.left && nb.topleft))) continue;
    pred16(f.y.data(), W, mx * 16, my * 16, nb, m, pred);
    const int s = sad(src, W, pred, 16);
    if (s < best_sad) {
      best_sad = s;
      mode = m;
      std::memcpy(best, pred, 256);
    }
  }
  // ---- luma residual -> levels
  const int qp6 = qp % 6, qbits = 15 + qp / 6, fq = (1 << qbits) / 3;
  int W4[16][16], dcm[16], ac[16][15];
  for (int blk = 0; blk < 16; ++blk) {
    const int bx = kBlkX[blk], by = kBlkY[blk];
    int res[16];
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x)
        res[4 * y + x] = int(src[(4 * by + y) * W + 4 * bx + x]) - int(best[16 * (4 * by + y) + 4 * bx + x]);
    fwd4x4(res, W4[blk]);
    dcm[4 * by + bx] = W4[blk][0];
  }
  int hd[16], dc[16];
  hadamard4(dcm, hd);
  bool any_ac = false;
  for (int k = 0; k < 16; ++k) dc[k] = quant(hd[kZigzag[k]] / 2, kMF[qp6][0], 2 * fq, qbits + 1);
  for (int blk = 0; blk < 16; ++blk)
    for (int k = 0; k < 15; ++k) {
      const int rp = kZigzag[k + 1];
      ac[blk][k] = quant(W4[blk][rp], kMF[qp6][pos_class(rp)], fq, qbits);
      any_ac |= ac[blk][k] != 0;
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
  int cdc[2][4], cac[2][4][15];
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
      for (int k = 0; k < 15; ++k) {
        const int rp = kZigzag[k + 1];
        cac[c][blk][k] = quant(Wb[blk][rp], kMF[qc6][pos_class(rp)], fqc, qcbits);
        c_any_ac |= cac[c][blk][k] != 0;
      }
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
  bw.ue(1 + mode + 4 * cbp_chroma + (cbp_luma ? 12 : 0));
  bw.ue(cmode);
  bw.se(0);  // mb_qp_delta
  write_block(bw, dc, 16, f.nc(f.tc_y, 4 * mx, 4 * my, 4, 0));
  for (int blk = 0; blk < 16; ++blk) {
    const int bx = 4 * mx + kBlkX[blk], by = 4 * my + kBlkY[blk];
    int tc = 0;
    if (cbp_luma) {
      write_block(bw, ac[blk], 15, f.nc(f.tc_y, bx, by, 4, 0));
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
        write_block(bw, cac[c][blk], 15, f.nc(tcs, bx, by, 2, 0));
        for (int k = 0; k < 15; ++k) tc += cac[c][blk][k] != 0;
      }
      tcs[size_t(by) * 2 * f.mbw + bx] = uint8_t(tc);
    }
  }
  // ---- reconstruction (the decoder's output)
  f.slice[size_t(my) * f.mbw + mx] = 0;
  recon_luma16(f, mx, my, best, dc, ac, qp);
  for (int c = 0; c < 2; ++c) recon_chroma(*cpl[c], Wc, mx, my, cpred[c], cdc[c], cac[c], qpc);
}

void write_sps(BitWriter& s, int width, int height) {
  const int mbw = (width + 15) / 16, mbh = (height + 15) / 16;
  s.put(66, 8);    // profile_idc: Baseline
  s.put(0xC0, 8);  // constraint_set0/1 -> Constrained Baseline
  s.put(51, 8);    // level_idc
  s.ue(0);         // seq_parameter_set_id
  s.ue(0);         // log2_max_frame_num_minus4
  s.ue(2);         // pic_order_cnt_type
  s.ue(1);         // max_num_ref_frames
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

void parameter_sets(int width, int height, int qp, std::string& sps, std::string& pps) {
  BitWriter s;
  write_sps(s, width, height);
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
  int mbw = 0, mbh = 0, log2_max_frame_num = 4, poc_type = 0, log2_max_poc_lsb = 4;
  bool delta_pic_order_always_zero = false;
  int crop_l = 0, crop_r = 0, crop_t = 0, crop_b = 0;
};
struct Pps {
  bool ok = false;
  int sps_id = 0, init_qp = 26, chroma_qp_offset = 0;
  bool bottom_field_pic_order = false, deblocking_control = false, redundant_pic_cnt = false;
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
    throw std::runtime_error("h264: High / scalable profiles are not supported (Constrained Baseline intra only)");
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
    for (uint32_t i = 0; i < n; ++i) br.se();
  }
  br.ue();    // max_num_ref_frames
  br.u(1);    // gaps
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
  br.ue();
  br.ue();
  br.u(1);
  br.u(2);
  const int64_t init_qp = 26 + int64_t(br.se());   // int64: a hostile se() must not overflow
  br.se();
  const int64_t cqo = br.se();
  if (init_qp < 0 || init_qp > 51 || cqo < -12 || cqo > 12) throw std::runtime_error("h264: PPS field out of range");
  p.init_qp = int(init_qp);
  p.chroma_qp_offset = int(cqo);
  if (p.init_qp < 0 || p.init_qp > 51 || p.chroma_qp_offset < -12 || p.chroma_qp_offset > 12)
    throw std::runtime_error("h264: PPS field out of range");
  p.deblocking_control = br.u(1);
  br.u(1);  // constrained_intra_pred_flag (intra-only streams: no effect)
  p.redundant_pic_cnt = br.u(1);
  if (br.more_rbsp_data()) throw std::runtime_error("h264: PPS extensions (8x8 transform) are not supported");
  p.ok = true;
  return p;
}

void decode_slice(BitReader& br, int nal_type, int nal_ref_idc, const Sps& sps, const Pps& pps, Frame& f,
                  int slice_id) {
  // untrusted input: range-check every exp-golomb value as uint32 before it becomes an index
  const uint32_t first_mb_u = br.ue();
  if (first_mb_u >= uint32_t(f.mbw) * uint32_t(f.mbh)) throw std::runtime_error("h264: first_mb_in_slice out of range");
  const int first_mb = int(first_mb_u);
  const int slice_type = int(br.ue() % 5);
  if (slice_type != 2) throw std::runtime_error("h264: only I slices are supported (no P/B/SP/SI)");
  br.ue();  // pps id
  br.u(sps.log2_max_frame_num);
  if (nal_type == 5) br.ue();  // idr_pic_id
  if (sps.poc_type == 0) {
    br.u(sps.log2_max_poc_lsb);
    if (pps.bottom_field_pic_order) br.se();
  } else if (sps.poc_type == 1 && !sps.delta_pic_order_always_zero) {
    br.se();
    if (pps.bottom_field_pic_order) br.se();
  }
  if (pps.redundant_pic_cnt) br.ue();
  if (nal_ref_idc) {
    if (nal_type == 5) {
      br.u(1);
      br.u(1);
    } else if (br.u(1)) {
      for (;;) {
        const uint32_t op = br.ue();
        if (op == 0) break;
        if (op == 1 || op == 3) br.ue();
        if (op == 2) br.ue();
        if (op == 3 || op == 6) br.ue();
        if (op == 4) br.ue();
      }
    }
  }
  const int64_t qp0 = pps.init_qp + int64_t(br.se());
  if (qp0 < 0 || qp0 > 51) throw std::runtime_error("h264: slice QP out of range");
  int qp = int(qp0);
  auto qp_delta = [&](int q) {
    const int d = br.se();
    if (d < -26 || d > 25) throw std::runtime_error("h264: mb_qp_delta out of range");
    return (q + d + 52) % 52;
  };
  if (pps.deblocking_control) {
    const uint32_t idc = br.ue();
    if (idc != 1)
      throw std::runtime_error("h264: in-loop deblocking is not supported (disable_deblocking_filter_idc != 1)");
  } else {
    throw std::runtime_error("h264: in-loop deblocking is not supported (no deblocking control in the PPS)");
  }
  const int nmb = f.mbw * f.mbh;
  const int Wc = f.W / 2;
  for (int mb = first_mb; mb < nmb; ++mb) {
    const int mx = mb % f.mbw, my = mb / f.mbw;
    if (f.slice[mb] != -1) throw std::runtime_error("h264: macroblock decoded twice");
    f.slice[mb] = slice_id;
    const Nb nb = f.nb(mx, my, slice_id);
    const uint32_t mb_type = br.ue();
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
    } else if (mb_type >= 1 && mb_type <= 24) {  // I_16x16
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
      // chroma
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
    } else if (mb_type == 0) {  // I_NxN (intra 4x4)
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
      const int cbp = kIntraCbp[cbp_code], cbp_luma = cbp & 15, cbp_chroma = cbp >> 4;
      if (cbp) qp = qp_delta(qp);
      int coef[16][16];
      std::memset(coef, 0, sizeof(coef));
      for (int blk = 0; blk < 16; ++blk) {
        const int bx = 4 * mx + kBlkX[blk], by = 4 * my + kBlkY[blk];
        int tc = 0;
        if (cbp_luma & (1 << (blk / 4))) tc = read_block(br, coef[blk], 16, f.nc(f.tc_y, bx, by, 4, slice_id));
        f.tc_y[size_t(by) * 4 * f.mbw + bx] = uint8_t(tc);
      }
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
    } else {
      throw std::runtime_error("h264: macroblock type not allowed in an I slice");
    }
    if (!br.more_rbsp_data()) break;
  }
}

}  // namespace

std::vector<Picture> decode(const std::vector<std::string>& nals, int threads) {
  // Pass 1 (sequential): parameter sets and the split into pictures (a picture starts at a slice
  // with first_mb_in_slice == 0).  Pass 2: pictures are intra-only and independent -> parallel.
  struct Job {
    Sps sps;
    Pps pps;
    std::vector<std::pair<int, std::string>> slices;  // (nal header byte, rbsp)
  };
  Sps sps;
  Pps pps;
  std::vector<Job> jobs;
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
      if (peek.ue() == 0) jobs.push_back(Job{sps, pps, {}});
      if (jobs.empty()) throw std::runtime_error("h264: slice of a picture without its first macroblock");
      jobs.back().slices.emplace_back(h, std::move(rbsp));
    } else if (type == 9 || type == 6 || type == 10 || type == 11 || type == 12) {
      // access unit delimiter, SEI, end of sequence / stream, filler: ignored
    } else {
      throw std::runtime_error("h264: unsupported NAL unit type " + std::to_string(type));
    }
  }
  // untrusted input: a few bits per macroblock can declare huge pictures, so bound what decoding
  // may allocate (4K per picture via the SPS limits, 2^31 luma samples - ~3.2 GB of 4:2:0 - in total)
  uint64_t samples = 0;
  for (const Job& j : jobs) samples += uint64_t(j.sps.mbw) * j.sps.mbh * 256;
  if (samples > (uint64_t(1) << 31)) throw std::runtime_error("h264: video too large to decode");
  std::vector<Picture> out(jobs.size());
  std::vector<std::string> errors(jobs.size());
  auto work = [&](int t, int nt) {
    for (size_t i = t; i < jobs.size(); i += nt) {
      try {
        const Job& j = jobs[i];
        Frame f(j.sps.mbw, j.sps.mbh);
        int slice_id = 0;
        for (const auto& sl : j.slices) {
          BitReader br(sl.second);
          decode_slice(br, sl.first & 0x1F, (sl.first >> 5) & 3, j.sps, j.pps, f, slice_id++);
        }
        for (int s : f.slice)
          if (s < 0) throw std::runtime_error("h264: picture has undecoded macroblocks");
        Picture& p = out[i];
        p.w16 = f.W;
        p.h16 = f.H;
        p.crop_w = f.W - 2 * (j.sps.crop_l + j.sps.crop_r);
        p.crop_h = f.H - 2 * (j.sps.crop_t + j.sps.crop_b);
        if (p.crop_w <= 0 || p.crop_h <= 0) throw std::runtime_error("h264: bad cropping window");
        p.y = std::move(f.y);
        p.cb = std::move(f.cb);
        p.cr = std::move(f.cr);
      } catch (const std::exception& e) {
        errors[i] = e.what();
      }
    }
  };
  const int nt = std::max(1, std::min<int>(threads, (int)jobs.size()));
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work, t, nt);
  work(0, nt);
  for (auto& th : pool) th.join();
  for (auto& e : errors)
    if (!e.empty()) throw std::runtime_error(e);
  return out;
}

}  // namespace h264
