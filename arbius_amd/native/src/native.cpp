// arbius_amd._native: CPU-side hot paths of the node runtime.
//
//  * keccak256          - Ethereum keccak (padding 0x01), used for task ids,
//                         commitments, selectors, tx hashes (hashlib has none);
//  * png_encode         - deterministic PNG (filter 0 rows + a segmented parallel zlib stream):
//                         byte-identical to utils/png.py (same zlib, same params),
//                         without the Python-side row copy;
//  * secp256k1_*        - ECDSA signing (RFC 6979, constant-time in the key), public key,
//                         ecrecover (secp256k1.cpp);
//  * pcm_slice_body     - the H.264 I_PCM macroblock payload of one picture for
//                         utils/mp4.py: RGB -> BT.601 YCbCr 4:2:0 (integer) and the
//                         macroblock raster, multi-threaded over macroblock rows
//                         (zeroscope 1024x576x24f: ~1 s in numpy, ~20 ms here).
//
// Everything is a pure function of its input (no time, no thread-count dependence:
// each thread writes a disjoint, precomputed byte range).
#include "h264.h"
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <zlib.h>

#include "secp256k1.h"

#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <functional>
#include <cstdint>
#include <cstring>
#include <exception>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

// ------------------------------------------------------------------------------------ keccak
static const uint64_t RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int ROTC[25] = {0, 36, 3, 41, 18, 1, 44, 10, 45, 2, 62, 6, 43,   // [x*5+y]
                             15, 61, 28, 55, 25, 21, 56, 27, 20, 39, 8, 14};

static inline uint64_t rol(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }

static void keccak_f(uint64_t s[25]) {  // s[x + 5y]
  for (int round = 0; round < 24; ++round) {
    uint64_t c[5], d[5], b[25];
    for (int x = 0; x < 5; ++x) c[x] = s[x] ^ s[x + 5] ^ s[x + 10] ^ s[x + 15] ^ s[x + 20];
    for (int x = 0; x < 5; ++x) d[x] = c[(x + 4) % 5] ^ rol(c[(x + 1) % 5], 1);
    for (int i = 0; i < 25; ++i) s[i] ^= d[i % 5];
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) b[y + 5 * ((2 * x + 3 * y) % 5)] = rol(s[x + 5 * y], ROTC[x * 5 + y]);
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) s[x + 5 * y] = b[x + 5 * y] ^ ((~b[(x + 1) % 5 + 5 * y]) & b[(x + 2) % 5 + 5 * y]);
    s[0] ^= RC[round];
  }
}

static std::string keccak256_raw(const uint8_t* p, size_t n) {
  const size_t rate = 136;
  uint64_t s[25] = {0};
  std::vector<uint8_t> blk(rate);
  size_t off = 0;
  bool done = false;
  while (!done) {
    size_t take = std::min(rate, n - off);
    std::memset(blk.data(), 0, rate);
    std::memcpy(blk.data(), p + off, take);
    off += take;
    if (take < rate) {  // final (padded) block
      blk[take] ^= 0x01;
      blk[rate - 1] ^= 0x80;
      done = true;
    }
    for (size_t i = 0; i < rate / 8; ++i) {
      uint64_t w;
      std::memcpy(&w, blk.data() + 8 * i, 8);
      s[i] ^= w;
    }
    keccak_f(s);
  }
  std::string out(32, '\0');
  std::memcpy(&out[0], s, 32);
  return out;
}

static py::bytes keccak256(py::bytes data) {
  std::string d = data;
  std::string h;
  {
    py::gil_scoped_release nogil;
    h = keccak256_raw(reinterpret_cast<const uint8_t*>(d.data()), d.size());
  }
  return py::bytes(h);
}

// ------------------------------------------------------------------------------------ PNG
static void put_be32(std::string& s, uint32_t v) {
  char b[4] = {char(v >> 24), char(v >> 16), char(v >> 8), char(v)};
  s.append(b, 4);
}

static void png_chunk(std::string& out, const char* tag, const std::string& body) {
  put_be32(out, (uint32_t)body.size());
  std::string tb(tag, 4);
  tb += body;
  out += tb;
  put_be32(out, (uint32_t)crc32(0L, reinterpret_cast<const Bytef*>(tb.data()), (uInt)tb.size()));
}

// Deterministic parallel zlib stream (pigz layout): the input is cut into PNG_SEG-byte segments at
// fixed offsets, each segment is raw-deflated on its own thread with the previous 32 KiB of input as
// its preset dictionary and ends on a sync flush (the last one with BFINAL), and the zlib header and
// the Adler-32 of the whole input wrap the concatenation.  The bytes depend only on the input, the
// level and PNG_SEG - never on the thread count - and decode with any inflater; a 768x768 RGB image
// is 14 segments (~4 ms on 8 threads instead of ~30 ms single-stream at level 6).
#define PNG_SEG (128 * 1024)
static std::string deflate_segment(const uint8_t* data, size_t n, const uint8_t* dict, size_t dn, int level,
                                   bool last) {
  z_stream zs;
  std::memset(&zs, 0, sizeof zs);
  if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK)
    throw std::runtime_error("deflateInit2 failed");
  if (dn && deflateSetDictionary(&zs, dict, (uInt)dn) != Z_OK) throw std::runtime_error("deflateSetDictionary");
  std::string out(deflateBound(&zs, n) + 16, '\0');
  zs.next_in = const_cast<Bytef*>(data);
  zs.avail_in = (uInt)n;
  zs.next_out = reinterpret_cast<Bytef*>(&out[0]);
  zs.avail_out = (uInt)out.size();
  const int r = deflate(&zs, last ? Z_FINISH : Z_SYNC_FLUSH);
  if (r != (last ? Z_STREAM_END : Z_OK) || zs.avail_in != 0) {
    deflateEnd(&zs);
    throw std::runtime_error("deflate segment failed");
  }
  out.resize(out.size() - zs.avail_out);
  deflateEnd(&zs);
  return out;
}

static std::string zlib_segmented(const uint8_t* data, size_t n, int level) {
  const size_t nseg = n == 0 ? 1 : (n + PNG_SEG - 1) / PNG_SEG;
  std::vector<std::string> parts(nseg);
  auto work = [&](size_t i) {
    const size_t off = i * PNG_SEG, len = std::min((size_t)PNG_SEG, n - off);
    const size_t dn = std::min(off, (size_t)32768);
    parts[i] = deflate_segment(data + off, len, data + off - dn, dn, level, i + 1 == nseg);
  };
  const size_t nt = std::min(nseg, (size_t)std::max(1u, std::min(8u, std::thread::hardware_concurrency())));
  // an exception must not escape a std::thread (std::terminate would abort the whole GPU worker):
  // each thread keeps its first failure and the caller rethrows it after the join
  std::vector<std::exception_ptr> errs(nt);
  auto lane = [&](size_t t) {
    try {
      for (size_t i = t; i < nseg; i += nt) work(i);
    } catch (...) {
      errs[t] = std::current_exception();
    }
  };
  std::vector<std::thread> th;
  for (size_t t = 1; t < nt; ++t) th.emplace_back(lane, t);
  lane(0);
  for (auto& t : th) t.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
  // zlib header: CM 8 / CINFO 7, FLEVEL as zlib's own compress2 writes it, FCHECK
  const int flevel = level == 1 ? 0 : level < 6 && level >= 0 ? 1 : level == 6 || level == -1 ? 2 : 3;
  const unsigned hdr = (0x78u << 8) | (unsigned)(flevel << 6);
  std::string z;
  z.push_back((char)0x78);
  z.push_back((char)((hdr | (31 - hdr % 31)) & 0xff));
  for (auto& p : parts) z += p;
  const uint32_t ad = (uint32_t)adler32(adler32(0L, Z_NULL, 0), data, (uInt)n);
  put_be32(z, ad);
  return z;
}

static py::bytes png_encode(py::array_t<uint8_t, py::array::c_style | py::array::forcecast> img, int level) {
  auto b = img.request();
  if (b.ndim != 2 && b.ndim != 3) throw std::invalid_argument("png_encode: [H, W] or [H, W, C]");
  const size_t h = b.shape[0], w = b.shape[1], c = b.ndim == 3 ? b.shape[2] : 1;
  int color;
  switch (c) {
    case 1: color = 0; break;
    case 3: color = 2; break;
    case 4: color = 6; break;
    default: throw std::invalid_argument("png_encode: C must be 1, 3 or 4");
  }
  const uint8_t* src = static_cast<const uint8_t*>(b.ptr);
  std::string out;
  {
    py::gil_scoped_release nogil;
    const size_t row = 1 + w * c;
    std::vector<uint8_t> raw(h * row);
    for (size_t y = 0; y < h; ++y) {
      raw[y * row] = 0;  // filter type 0
      std::memcpy(&raw[y * row + 1], src + y * w * c, w * c);
    }
    const std::string z = zlib_segmented(raw.data(), raw.size(), level);
    out = "\x89PNG\r\n\x1a\n";
    std::string ihdr;
    put_be32(ihdr, (uint32_t)w);
    put_be32(ihdr, (uint32_t)h);
    ihdr.push_back(8);
    ihdr.push_back((char)color);
    ihdr.append(3, '\0');
    png_chunk(out, "IHDR", ihdr);
    png_chunk(out, "IDAT", z);
    png_chunk(out, "IEND", std::string());
  }
  return py::bytes(out);
}

// ------------------------------------------------------------------------------------ H.264 I_PCM
static inline uint8_t clip1(int v) { return (uint8_t)std::min(254, std::max(1, v)); }

// frame: uint8 [H, W, 3] with H, W multiples of 16.  Returns the macroblock payload of the
// slice: MB0 samples (its mb_type/alignment are in the Python-built header) followed by
// (0x0D 0x00 + samples) for every later macroblock; 386 bytes per macroblock minus 2.
static py::bytes pcm_slice_body(py::array_t<uint8_t, py::array::c_style | py::array::forcecast> frame, int threads) {
  auto b = frame.request();
  if (b.ndim != 3 || b.shape[2] != 3) throw std::invalid_argument("pcm_slice_body: [H, W, 3]");
  const int H = (int)b.shape[0], W = (int)b.shape[1];
  if (H % 16 || W % 16) throw std::invalid_argument("pcm_slice_body: H, W must be multiples of 16");
  const uint8_t* src = static_cast<const uint8_t*>(b.ptr);
  const int mbw = W / 16, mbh = H / 16;
  const size_t nmb = (size_t)mbw * mbh;
  std::string out(nmb * 386 - 2, '\0');
  {
    py::gil_scoped_release nogil;
    auto work = [&](int r0, int r1) {
      for (int my = r0; my < r1; ++my) {
        for (int mx = 0; mx < mbw; ++mx) {
          const size_t idx = (size_t)my * mbw + mx;
          uint8_t* dst = reinterpret_cast<uint8_t*>(&out[0]) + (idx == 0 ? 0 : idx * 386 - 2);
          if (idx != 0) {
            *dst++ = 0x0D;
            *dst++ = 0x00;
          }
          for (int y = 0; y < 16; ++y) {
            const uint8_t* p = src + ((size_t)(my * 16 + y) * W + mx * 16) * 3;
            for (int x = 0; x < 16; ++x) {
              const int r = p[3 * x], g = p[3 * x + 1], bl = p[3 * x + 2];
              dst[y * 16 + x] = clip1(((66 * r + 129 * g + 25 * bl + 128) >> 8) + 16);
            }
          }
          uint8_t* cb = dst + 256;
          uint8_t* cr = dst + 320;
          for (int y = 0; y < 8; ++y) {
            const uint8_t* p0 = src + ((size_t)(my * 16 + 2 * y) * W + mx * 16) * 3;
            const uint8_t* p1 = p0 + (size_t)W * 3;
            for (int x = 0; x < 8; ++x) {
              const int r = p0[6 * x] + p0[6 * x + 3] + p1[6 * x] + p1[6 * x + 3];
              const int g = p0[6 * x + 1] + p0[6 * x + 4] + p1[6 * x + 1] + p1[6 * x + 4];
              const int bl = p0[6 * x + 2] + p0[6 * x + 5] + p1[6 * x + 2] + p1[6 * x + 5];
              cb[y * 8 + x] = clip1(((-38 * r - 74 * g + 112 * bl + 512) >> 10) + 128);
              cr[y * 8 + x] = clip1(((112 * r - 94 * g - 18 * bl + 512) >> 10) + 128);
            }
          }
        }
      }
    };
    int nt = std::max(1, std::min(threads, mbh));
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t) {
      const int r0 = mbh * t / nt, r1 = mbh * (t + 1) / nt;
      pool.emplace_back(work, r0, r1);
    }
    for (auto& th : pool) th.join();
  }
  return py::bytes(out);
}


// ------------------------------------------------------------------------------------ H.264 CAVLC
// RGB -> 4:2:0 (the same integer BT.601 conversion as pcm_slice_body / mp4.rgb_to_yuv420) of an
// H x W frame edge-replicated to H16 x W16 (whole macroblocks; the SPS crops it back)
// RGB -> 4:2:0 at macroblock-padded size (rows / columns past H / W replicate the last one).  Per
// row: the columns inside the picture run as a plain stride-3 loop (no per-sample clamping, so
// the compiler vectorises it), the padding columns reuse the last sample.
static void rgb_to_420(const uint8_t* src, int H, int W, int H16, int W16, uint8_t* y, uint8_t* cb, uint8_t* cr) {
  auto row = [&](int r) { return src + (size_t)std::min(r, H - 1) * W * 3; };
  for (int r = 0; r < H16; ++r) {
    const uint8_t* p = row(r);
    uint8_t* o = y + (size_t)r * W16;
    for (int x = 0; x < W; ++x)
      o[x] = clip1(((66 * p[3 * x] + 129 * p[3 * x + 1] + 25 * p[3 * x + 2] + 128) >> 8) + 16);
    for (int x = W; x < W16; ++x) o[x] = o[W - 1];
  }
  const int Wc = W16 / 2, Wi = W / 2;   // chroma columns whose 2x2 source lies inside the picture
  for (int r = 0; r < H16 / 2; ++r) {
    const uint8_t *p0 = row(2 * r), *p1 = row(2 * r + 1);
    uint8_t *ob = cb + (size_t)r * Wc, *orr = cr + (size_t)r * Wc;
    for (int x = 0; x < Wi; ++x) {
      const uint8_t *a = p0 + 6 * x, *c = p1 + 6 * x;
      const int rr = a[0] + a[3] + c[0] + c[3], g = a[1] + a[4] + c[1] + c[4], bl = a[2] + a[5] + c[2] + c[5];
      ob[x] = clip1(((-38 * rr - 74 * g + 112 * bl + 512) >> 10) + 128);
      orr[x] = clip1(((112 * rr - 94 * g - 18 * bl + 512) >> 10) + 128);
    }
    for (int x = Wi; x < Wc; ++x) {       // odd W / padding: clamp the source columns
      const int x0 = std::min(2 * x, W - 1), x1 = std::min(2 * x + 1, W - 1);
      const uint8_t *a = p0 + 3 * x0, *b = p0 + 3 * x1, *c = p1 + 3 * x0, *d = p1 + 3 * x1;
      const int rr = a[0] + b[0] + c[0] + d[0], g = a[1] + b[1] + c[1] + d[1], bl = a[2] + b[2] + c[2] + d[2];
      ob[x] = clip1(((-38 * rr - 74 * g + 112 * bl + 512) >> 10) + 128);
      orr[x] = clip1(((112 * rr - 94 * g - 18 * bl + 512) >> 10) + 128);
    }
  }
}

// nice > 0: every item runs on a spawned thread that first lowers its own scheduling priority
// (Linux setpriority on the thread id; raising nice needs no privilege) and the caller only joins.
// A background encode then yields the CPU to the threads that feed the GPU (the next clip's
// host<->device staging copies) instead of time-slicing with them.
static void run_parallel(int n, int threads, const std::function<void(int)>& fn, int nice = 0) {
  std::vector<std::string> errors(n);
  auto work = [&](int t, int nt) {
    if (nice > 0) setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), nice);
    for (int i = t; i < n; i += nt) {
      try {
        fn(i);
      } catch (const std::exception& e) {
        errors[i] = e.what();
      }
    }
  };
  const int nt = std::max(1, std::min(threads, n));
  std::vector<std::thread> pool;
  for (int t = nice > 0 ? 0 : 1; t < nt; ++t) pool.emplace_back(work, t, nt);
  if (nice <= 0) work(0, nt);
  for (auto& th : pool) th.join();
  for (auto& e : errors)
    if (!e.empty()) throw std::runtime_error(e);
}

// frames uint8 [F, H, W, 3] -> (sps, pps, [IDR NAL per frame]); frames are independent pictures,
// so they are encoded in parallel (the output does not depend on the thread count).
static py::tuple h264_encode_rgb(py::array_t<uint8_t, py::array::c_style | py::array::forcecast> frames, int qp,
                                 int threads, int nice) {
  auto b = frames.request();
  if (b.ndim != 4 || b.shape[3] != 3 || b.shape[0] < 1 || b.shape[1] < 1 || b.shape[2] < 1)
    throw std::invalid_argument("h264_encode_rgb: frames [F, H, W, 3]");
  const int F = (int)b.shape[0], H = (int)b.shape[1], W = (int)b.shape[2];
  const int H16 = (H + 15) / 16 * 16, W16 = (W + 15) / 16 * 16;
  const uint8_t* src = static_cast<const uint8_t*>(b.ptr);
  std::vector<std::string> nals(F);
  std::string sps, pps;
  h264::parameter_sets(W, H, qp, sps, pps);
  {
    py::gil_scoped_release nogil;
    run_parallel(F, threads, [&](int i) {
      std::vector<uint8_t> y((size_t)H16 * W16), cb((size_t)H16 * W16 / 4), cr((size_t)H16 * W16 / 4);
      rgb_to_420(src + (size_t)i * H * W * 3, H, W, H16, W16, y.data(), cb.data(), cr.data());
      nals[i] = h264::encode_idr(y.data(), cb.data(), cr.data(), W16, H16, qp, i, nullptr, nullptr, nullptr);
    }, nice);
  }
  py::list out;
  for (auto& n : nals) out.append(py::bytes(n));
  return py::make_tuple(py::bytes(sps), py::bytes(pps), out);
}

using u8arr = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;

// Macroblock-padded 4:2:0 planes y [F, H16, W16], cb / cr [F, H16 / 2, W16 / 2] of an H x W picture
// (the GPU's rgb_to_yuv420 output, same samples as rgb_to_420) -> (sps, pps, [IDR NAL per frame]):
// h264_encode_rgb without the host colour conversion.  Same bytes for the same planes.
static py::tuple h264_encode_yuv420_frames(u8arr y, u8arr cb, u8arr cr, int W, int H, int qp, int threads,
                                           int nice) {
  auto by = y.request(), bcb = cb.request(), bcr = cr.request();
  const int H16 = (H + 15) / 16 * 16, W16 = (W + 15) / 16 * 16;
  if (W < 1 || H < 1 || by.ndim != 3 || bcb.ndim != 3 || bcr.ndim != 3 || by.shape[1] != H16 || by.shape[2] != W16 ||
      bcb.shape[0] != by.shape[0] || bcr.shape[0] != by.shape[0] || bcb.shape[1] != H16 / 2 ||
      bcb.shape[2] != W16 / 2 || bcr.shape[1] != H16 / 2 || bcr.shape[2] != W16 / 2 || by.shape[0] < 1)
    throw std::invalid_argument("h264_encode_yuv420_frames: y [F, H16, W16], cb / cr [F, H16/2, W16/2]");
  const int F = (int)by.shape[0];
  const uint8_t* py_ = static_cast<const uint8_t*>(by.ptr);
  const uint8_t* pcb = static_cast<const uint8_t*>(bcb.ptr);
  const uint8_t* pcr = static_cast<const uint8_t*>(bcr.ptr);
  const size_t ly = (size_t)H16 * W16, lc = ly / 4;
  std::vector<std::string> nals(F);
  std::string sps, pps;
  h264::parameter_sets(W, H, qp, sps, pps);
  {
    py::gil_scoped_release nogil;
    run_parallel(F, threads, [&](int i) {
      nals[i] = h264::encode_idr(py_ + i * ly, pcb + i * lc, pcr + i * lc, W16, H16, qp, i, nullptr, nullptr, nullptr);
    }, nice);
  }
  py::list out;
  for (auto& n : nals) out.append(py::bytes(n));
  return py::make_tuple(py::bytes(sps), py::bytes(pps), out);
}

// The GPU intra encoder's output (ops/csrc/h264_intra.hip) -> IDR NAL units: buf holds every
// picture's RBSP at meta[f] (bytes), meta[F + 2 + f] RBSP bits before the stop bit (the layout of
// arb_h264_intra_encode / arb_h264_intra_host).  Same NALs as h264_encode_yuv420_frames.
static py::list h264_nals_from_rbsp(py::array_t<uint8_t, py::array::c_style> buf,
                                    py::array_t<int64_t, py::array::c_style> meta, int F, int threads) {
  auto bb = buf.request(), bm = meta.request();
  if (F < 1 || bm.ndim != 1 || bm.shape[0] < 2 * F + 2 || bb.ndim != 1)
    throw std::invalid_argument("h264_nals_from_rbsp: meta [2F + 2] int64, buf 1-D uint8");
  const int64_t* m = static_cast<const int64_t*>(bm.ptr);
  const uint8_t* b = static_cast<const uint8_t*>(bb.ptr);
  if (m[F + 1] != 0) throw std::runtime_error("h264_nals_from_rbsp: the encoder flagged an error");
  for (int f = 0; f < F; ++f) {
    const int64_t bytes = (m[F + 2 + f] + 8) / 8;
    if (m[f] < 0 || m[F + 2 + f] < 0 || m[f] + bytes > (int64_t)bb.shape[0])
      throw std::invalid_argument("h264_nals_from_rbsp: picture outside buf");
  }
  std::vector<std::string> nals(F);
  {
    py::gil_scoped_release nogil;
    run_parallel(F, threads, [&](int f) {
      nals[f] = h264::rbsp_to_nal(0x65, b + m[f], (size_t)((m[F + 2 + f] + 8) / 8));
    });
  }
  py::list out;
  for (auto& n : nals) out.append(py::bytes(n));
  return out;
}

// the host conversion on its own (tests: the GPU planes equal these)
static py::tuple rgb_to_yuv420_planes(u8arr frames) {
  auto b = frames.request();
  if (b.ndim != 4 || b.shape[3] != 3 || b.shape[0] < 1 || b.shape[1] < 1 || b.shape[2] < 1)
    throw std::invalid_argument("rgb_to_yuv420_planes: frames [F, H, W, 3]");
  const int F = (int)b.shape[0], H = (int)b.shape[1], W = (int)b.shape[2];
  const int H16 = (H + 15) / 16 * 16, W16 = (W + 15) / 16 * 16;
  u8arr y({F, H16, W16}), cb({F, H16 / 2, W16 / 2}), cr({F, H16 / 2, W16 / 2});
  const uint8_t* src = static_cast<const uint8_t*>(b.ptr);
  for (int i = 0; i < F; ++i)
    rgb_to_420(src + (size_t)i * H * W * 3, H, W, H16, W16, y.mutable_data() + (size_t)i * H16 * W16,
               cb.mutable_data() + (size_t)i * H16 * W16 / 4, cr.mutable_data() + (size_t)i * H16 * W16 / 4);
  return py::make_tuple(y, cb, cr);
}

// One picture from 4:2:0 planes -> (IDR NAL, recon Y, recon Cb, recon Cr) (tests: recon == decoder output)
static py::tuple h264_encode_yuv(u8arr y, u8arr cb, u8arr cr, int qp, int idr_pic_id) {
  auto by = y.request(), bcb = cb.request(), bcr = cr.request();
  if (by.ndim != 2 || bcb.ndim != 2 || bcr.ndim != 2) throw std::invalid_argument("h264_encode_yuv: 2-D planes");
  const int H = (int)by.shape[0], W = (int)by.shape[1];
  if (bcb.shape[0] != H / 2 || bcb.shape[1] != W / 2 || bcr.shape[0] != H / 2 || bcr.shape[1] != W / 2)
    throw std::invalid_argument("h264_encode_yuv: chroma planes must be [H/2, W/2]");
  u8arr ry({H, W}), rcb({H / 2, W / 2}), rcr({H / 2, W / 2});
  std::string nal = h264::encode_idr(static_cast<const uint8_t*>(by.ptr), static_cast<const uint8_t*>(bcb.ptr),
                                     static_cast<const uint8_t*>(bcr.ptr), W, H, qp, idr_pic_id, ry.mutable_data(),
                                     rcb.mutable_data(), rcr.mutable_data());
  return py::make_tuple(py::bytes(nal), ry, rcb, rcr);
}

static py::tuple h264_parameter_sets(int width, int height, int qp, int max_refs) {
  std::string sps, pps;
  h264::parameter_sets(width, height, qp, sps, pps, max_refs);
  return py::make_tuple(py::bytes(sps), py::bytes(pps));
}

static py::list nal_lists(const std::vector<h264::EncodedPicture>& pics) {
  py::list out;
  for (const auto& p : pics) {
    py::list n;
    for (const auto& s : p.nals) n.append(py::bytes(s));
    out.append(n);
  }
  return out;
}

// frames uint8 [F, H, W, 3] -> (sps, pps, [[slice NALs] per picture]): IPPP stream (IDR every
// `gop` pictures), each picture's row-band slices encoded in parallel.  The colour conversion
// runs per picture inside the encoder's loader (no whole-clip YUV copy).
static py::tuple h264_encode_rgb_stream(py::array_t<uint8_t, py::array::c_style | py::array::forcecast> frames,
                                        int qp, int gop, int threads, int rows_per_slice) {
  auto b = frames.request();
  if (b.ndim != 4 || b.shape[3] != 3 || b.shape[0] < 1 || b.shape[1] < 1 || b.shape[2] < 1)
    throw std::invalid_argument("h264_encode_rgb_stream: frames [F, H, W, 3]");
  const int F = (int)b.shape[0], H = (int)b.shape[1], W = (int)b.shape[2];
  const int H16 = (H + 15) / 16 * 16, W16 = (W + 15) / 16 * 16;
  const uint8_t* src = static_cast<const uint8_t*>(b.ptr);
  std::string sps, pps;
  h264::parameter_sets(W, H, qp, sps, pps, 1);
  h264::StreamOptions o;
  o.qp = qp;
  o.gop = gop;
  o.threads = threads;
  o.rows_per_slice = rows_per_slice;
  std::vector<h264::EncodedPicture> pics;
  {
    py::gil_scoped_release nogil;
    pics = h264::encode_stream(F, W16, H16, o, [&](int i, uint8_t* y, uint8_t* cb, uint8_t* cr) {
      rgb_to_420(src + (size_t)i * H * W * 3, H, W, H16, W16, y, cb, cr);
    });
  }
  return py::make_tuple(py::bytes(sps), py::bytes(pps), nal_lists(pics));
}

// 4:2:0 planes [F, H, W] / [F, H/2, W/2] -> ([[NAL]], recon Y, Cb, Cr) (tests: recon == decoder
// output; seed != 0 = the randomised decoder-coverage mode)
static py::tuple h264_encode_yuv_stream(u8arr y, u8arr cb, u8arr cr, int qp, int gop, uint32_t seed, int max_refs,
                                        int threads, int rows_per_slice) {
  auto by = y.request(), bcb = cb.request(), bcr = cr.request();
  if (by.ndim != 3 || bcb.ndim != 3 || bcr.ndim != 3) throw std::invalid_argument("h264_encode_yuv_stream: [F, H, W]");
  const int F = (int)by.shape[0], H = (int)by.shape[1], W = (int)by.shape[2];
  if (bcb.shape[0] != F || bcr.shape[0] != F || bcb.shape[1] != H / 2 || bcb.shape[2] != W / 2 ||
      bcr.shape[1] != H / 2 || bcr.shape[2] != W / 2)
    throw std::invalid_argument("h264_encode_yuv_stream: chroma planes must be [F, H/2, W/2]");
  h264::StreamOptions o;
  o.qp = qp;
  o.gop = gop;
  o.seed = seed;
  o.max_refs = max_refs;
  o.threads = threads;
  o.rows_per_slice = rows_per_slice;
  o.keep_recon = true;
  const uint8_t *py_ = static_cast<const uint8_t*>(by.ptr), *pcb = static_cast<const uint8_t*>(bcb.ptr),
                *pcr = static_cast<const uint8_t*>(bcr.ptr);
  const size_t ny = (size_t)H * W, nc = ny / 4;
  std::vector<h264::EncodedPicture> pics;
  {
    py::gil_scoped_release nogil;
    pics = h264::encode_stream(F, W, H, o, [&](int i, uint8_t* yy, uint8_t* cbb, uint8_t* crr) {
      std::memcpy(yy, py_ + i * ny, ny);
      std::memcpy(cbb, pcb + i * nc, nc);
      std::memcpy(crr, pcr + i * nc, nc);
    });
  }
  u8arr ry({F, H, W}), rcb({F, H / 2, W / 2}), rcr({F, H / 2, W / 2});
  for (int i = 0; i < F; ++i) {
    std::memcpy(ry.mutable_data() + i * ny, pics[i].y.data(), ny);
    std::memcpy(rcb.mutable_data() + i * nc, pics[i].cb.data(), nc);
    std::memcpy(rcr.mutable_data() + i * nc, pics[i].cr.data(), nc);
  }
  return py::make_tuple(nal_lists(pics), ry, rcb, rcr);
}

template <class T>
static py::array_t<T> vec_array(const std::vector<T>& v) {
  py::array_t<T> a((py::ssize_t)v.size());
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

// NAL units (no start codes) -> [(Y, Cb, Cr, (crop_w, crop_h))]; raises ValueError outside the subset.
// with_side=True (tests) appends a dict of the deblocking filter's inputs per picture.
static py::list h264_decode(const std::vector<std::string>& nals, int threads, bool with_side, uint64_t max_samples) {
  std::vector<h264::Picture> pics;
  std::vector<h264::SideInfo> side;
  {
    py::gil_scoped_release nogil;
    try {
      h264::decode(
          nals, threads, [&](const std::vector<std::pair<int, int>>& crops) { pics.resize(crops.size()); },
          [&](size_t i, h264::Picture&& p, int) { pics[i] = std::move(p); }, with_side ? &side : nullptr,
          max_samples);
    } catch (const std::runtime_error& e) {
      py::gil_scoped_acquire gil;
      throw py::value_error(e.what());
    }
  }
  py::list out;
  for (size_t k = 0; k < pics.size(); ++k) {
    const auto& p = pics[k];
    u8arr y({p.h16, p.w16}), cb({p.h16 / 2, p.w16 / 2}), cr({p.h16 / 2, p.w16 / 2});
    std::memcpy(y.mutable_data(), p.y.data(), p.y.size());
    std::memcpy(cb.mutable_data(), p.cb.data(), p.cb.size());
    std::memcpy(cr.mutable_data(), p.cr.data(), p.cr.size());
    if (!with_side) {
      out.append(py::make_tuple(y, cb, cr, py::make_tuple(p.crop_w, p.crop_h)));
      continue;
    }
    const auto& s = side[k];
    py::dict d;
    d["y"] = vec_array(s.y);
    d["cb"] = vec_array(s.cb);
    d["cr"] = vec_array(s.cr);
    d["mvx"] = vec_array(s.mvx);
    d["mvy"] = vec_array(s.mvy);
    d["refpic"] = vec_array(s.refpic);
    d["nonzero"] = vec_array(s.nonzero);
    d["intra"] = vec_array(s.intra);
    d["qp"] = vec_array(s.qp);
    d["slice"] = vec_array(s.slice);
    d["deblock"] = s.deblock;
    d["chroma_qp_offset"] = s.chroma_qp_offset;
    out.append(py::make_tuple(y, cb, cr, py::make_tuple(p.crop_w, p.crop_h), d));
  }
  return out;
}

// NAL units -> uint8 RGB [F, crop_h, crop_w, 3]: the integer BT.601 inverse of rgb_to_420 (the
// reference is video_io.yuv420_to_rgb: nearest chroma upsampling, clipped).  The output is
// allocated once from the stream's layout and every picture is converted as soon as it is decoded,
// so no plane copy of the whole clip is ever held.
static u8arr h264_decode_rgb(const std::vector<std::string>& nals, int threads, uint64_t max_samples) {
  uint8_t* dst = nullptr;
  int F = 0, H = 0, W = 0;
  std::string layout_err;
  {
    py::gil_scoped_release nogil;
    try {
      h264::decode(
          nals, threads,
          [&](const std::vector<std::pair<int, int>>& crops) {
            if (crops.empty()) throw std::runtime_error("no pictures in the H.264 stream");
            W = crops[0].first;
            H = crops[0].second;
            for (auto& c : crops)
              if (c.first != W || c.second != H) throw std::runtime_error("pictures of different sizes");
            F = (int)crops.size();
            dst = new uint8_t[(size_t)F * H * W * 3];
          },
          [&](size_t i, h264::Picture&& p, int free_threads) {
            uint8_t* o = dst + i * (size_t)H * W * 3;
            const int bands = std::max(1, std::min(free_threads, H / 16));
            run_parallel(bands, bands, [&](int band) {
             for (int r = band * H / bands; r < (band + 1) * H / bands; ++r)
              for (int x = 0; x < W; ++x) {
                const int c = int(p.y[(size_t)r * p.w16 + x]) - 16;
                const int d = int(p.cb[(size_t)(r / 2) * (p.w16 / 2) + x / 2]) - 128;
                const int e = int(p.cr[(size_t)(r / 2) * (p.w16 / 2) + x / 2]) - 128;
                uint8_t* q = o + ((size_t)r * W + x) * 3;
                q[0] = (uint8_t)std::min(255, std::max(0, (298 * c + 409 * e + 128) >> 8));
                q[1] = (uint8_t)std::min(255, std::max(0, (298 * c - 100 * d - 208 * e + 128) >> 8));
                q[2] = (uint8_t)std::min(255, std::max(0, (298 * c + 516 * d + 128) >> 8));
              }
            });
          },
          nullptr, max_samples);
    } catch (const std::runtime_error& e) {
      delete[] dst;
      py::gil_scoped_acquire gil;
      throw py::value_error(e.what());
    }
  }
  py::capsule owner(dst, [](void* ptr) { delete[] static_cast<uint8_t*>(ptr); });
  return u8arr({F, H, W, 3}, dst, owner);
}

static py::bytes as_bytes32(const py::bytes& b, const char* what) {
  std::string s = b;
  if (s.size() != 32) throw std::invalid_argument(std::string(what) + " must be 32 bytes");
  return b;
}

static py::tuple py_secp_sign(const py::bytes& hash, const py::bytes& priv) {
  std::string h = as_bytes32(hash, "hash"), k = as_bytes32(priv, "private key");
  uint8_t r[32], s[32];
  int rec;
  {
    py::gil_scoped_release nogil;
    rec = secp256k1_sign((const uint8_t*)h.data(), (const uint8_t*)k.data(), r, s);
  }
  std::fill(k.begin(), k.end(), 0);
  if (rec < 0) throw std::invalid_argument("invalid secp256k1 private key");
  return py::make_tuple(py::bytes((const char*)r, 32), py::bytes((const char*)s, 32), rec);
}

static py::bytes py_secp_pubkey(const py::bytes& priv) {
  std::string k = as_bytes32(priv, "private key");
  uint8_t out[64];
  const int rc = secp256k1_pubkey((const uint8_t*)k.data(), out);
  std::fill(k.begin(), k.end(), 0);
  if (rc) throw std::invalid_argument("invalid secp256k1 private key");
  return py::bytes((const char*)out, 64);
}

static py::object py_secp_recover(const py::bytes& hash, const py::bytes& r, const py::bytes& s, int rec) {
  std::string h = as_bytes32(hash, "hash"), rr = as_bytes32(r, "r"), ss = as_bytes32(s, "s");
  uint8_t out[64];
  if (secp256k1_recover((const uint8_t*)h.data(), (const uint8_t*)rr.data(), (const uint8_t*)ss.data(), rec, out))
    return py::none();
  return py::bytes((const char*)out, 64);
}

static py::bytes py_sha256(const py::bytes& data) {
  std::string d = data;
  uint8_t out[32];
  sha256_digest((const uint8_t*)d.data(), d.size(), out);
  return py::bytes((const char*)out, 32);
}

PYBIND11_MODULE(_native, m) {
  m.def("secp256k1_sign", &py_secp_sign, "ECDSA sign (RFC 6979, low-s) -> (r, s, recid)");
  m.def("secp256k1_pubkey", &py_secp_pubkey, "uncompressed public key X||Y");
  m.def("secp256k1_recover", &py_secp_recover, "ecrecover -> X||Y or None");
  m.def("sha256", &py_sha256, "SHA-256 (the RFC 6979 HMAC's hash; checked against hashlib)");
  m.doc() = "arbius_amd native CPU runtime (keccak256, PNG, H.264 CAVLC codec, secp256k1)";
  m.def("keccak256", &keccak256, "Ethereum keccak-256");
  m.def("png_encode", &png_encode, py::arg("img"), py::arg("level") = 6, "deterministic filter-0 PNG");
  m.def("deflate_id", [] {
    // the deflate linked into THIS module (static libz.a, private symbols): its header and runtime
    // versions must agree, or a foreign libz has been interposed
    if (std::strcmp(zlibVersion(), ZLIB_VERSION) != 0)
      return std::string("zlib-mismatch-") + zlibVersion() + "-vs-" + ZLIB_VERSION;
    return std::string("zlib-") + ZLIB_VERSION;
  }, "identity of the deflate implementation behind png_encode");
  m.def("pcm_slice_body", &pcm_slice_body, py::arg("frame"), py::arg("threads") = 8,
        "H.264 I_PCM macroblock payload of one RGB frame");
  m.def("h264_encode_yuv420_frames", &h264_encode_yuv420_frames, py::arg("y"), py::arg("cb"), py::arg("cr"),
        py::arg("width"), py::arg("height"), py::arg("qp"), py::arg("threads") = 8, py::arg("nice") = 0);
  m.def("h264_nals_from_rbsp", &h264_nals_from_rbsp, py::arg("buf"), py::arg("meta"), py::arg("frames"),
        py::arg("threads") = 4, "GPU intra encoder RBSPs -> IDR NALs (emulation prevention)");
  m.def("rgb_to_yuv420_planes", &rgb_to_yuv420_planes, py::arg("frames"));
  m.def("h264_encode_rgb", &h264_encode_rgb, py::arg("frames"), py::arg("qp"), py::arg("threads") = 8,
        py::arg("nice") = 0, "H.264 CAVLC intra: RGB frames [F, H, W, 3] -> (sps, pps, [IDR NAL]); nice > 0 runs "
        "the encode threads at that lower priority");
  m.def("h264_encode_yuv", &h264_encode_yuv, py::arg("y"), py::arg("cb"), py::arg("cr"), py::arg("qp"),
        py::arg("idr_pic_id") = 0, "one 4:2:0 picture -> (IDR NAL, recon Y, Cb, Cr)");
  m.def("h264_parameter_sets", &h264_parameter_sets, py::arg("width"), py::arg("height"), py::arg("qp"),
        py::arg("max_refs") = 1, "(sps, pps) NALs of the CAVLC streams");
  m.def("h264_encode_rgb_stream", &h264_encode_rgb_stream, py::arg("frames"), py::arg("qp"), py::arg("gop"),
        py::arg("threads") = 8, py::arg("rows_per_slice") = 4,
        "H.264 CAVLC IPPP: RGB frames [F, H, W, 3] -> (sps, pps, [[slice NALs] per picture])");
  m.def("h264_encode_yuv_stream", &h264_encode_yuv_stream, py::arg("y"), py::arg("cb"), py::arg("cr"), py::arg("qp"),
        py::arg("gop"), py::arg("seed") = 0, py::arg("max_refs") = 1, py::arg("threads") = 4,
        py::arg("rows_per_slice") = 4, "4:2:0 pictures -> ([[NAL]], recon Y, Cb, Cr)");
  m.def("h264_decode", &h264_decode, py::arg("nals"), py::arg("threads") = 8, py::arg("with_side") = false,
        py::arg("max_samples") = h264::kDefaultMaxSamples,
        "decode Constrained Baseline CAVLC NAL units -> [(Y, Cb, Cr, (w, h)[, side info])]");
  m.def("h264_decode_rgb", &h264_decode_rgb, py::arg("nals"), py::arg("threads") = 8,
        py::arg("max_samples") = h264::kDefaultMaxSamples,
        "decode Constrained Baseline CAVLC NAL units -> uint8 RGB [F, H, W, 3] (cropped)");
  m.def("h264_tables_ok", &h264::tables_prefix_free, "every CAVLC VLC table is prefix-free");
}
