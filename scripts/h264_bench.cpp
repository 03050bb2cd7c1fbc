// Single-thread timing of the intra (IDR) H.264 encoder on synthetic 1080p pictures.
//
// The RVM output path encodes every 1080p frame as one I_16x16 IDR picture (utils/mp4.py
// "avc-intra"), so this loop is the CPU cost per output frame.  Prints ms/frame and an FNV-1a
// hash of all NAL bytes: an encoder optimisation must leave the hash unchanged.
//
//   g++ -O3 -std=c++17 -pthread -I arbius_amd/native/src scripts/h264_bench.cpp
//       arbius_amd/native/src/h264.cpp -o build/h264_bench && build/h264_bench [frames]
#include <algorithm>
#include <chrono>
#include <ctime>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "h264.h"

// argv[2] (optional): raw 1920x1088 4:2:0 pictures (Y, Cb, Cr planes back to back) to cycle
// through instead of the synthetic ones, e.g. real matting output converted by the probe script.
int main(int argc, char** argv) {
  const int F = argc > 1 ? std::atoi(argv[1]) : 8;
  const int W = 1920, H = 1088, Wc = W / 2, Hc = H / 2;
  std::vector<uint8_t> y((size_t)W * H), cb((size_t)Wc * Hc), cr((size_t)Wc * Hc);
  std::vector<uint8_t> file;
  if (argc > 2) {
    FILE* fp = std::fopen(argv[2], "rb");
    if (!fp) return 1;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof(buf), fp)) > 0) file.insert(file.end(), buf, buf + n);
    std::fclose(fp);
  }
  const size_t pic = y.size() + cb.size() + cr.size();
  const int nfile = (int)(file.size() / pic);
  uint32_t rng = 12345u;
  auto rnd = [&]() { rng = rng * 1664525u + 1013904223u; return (rng >> 24) & 15; };
  uint64_t h = 1469598103934665603ull;
  size_t bytes = 0;
  double secs = 0;
  for (int f = 0; f < F; ++f) {
    if (nfile > 0) {
      const uint8_t* p = file.data() + (size_t)(f % nfile) * pic;
      std::copy(p, p + y.size(), y.begin());
      std::copy(p + y.size(), p + y.size() + cb.size(), cb.begin());
      std::copy(p + y.size() + cb.size(), p + pic, cr.begin());
    } else {
    // smooth shading + a moving edge + low-amplitude grain: a matted subject over a flat screen
    for (int r = 0; r < H; ++r)
      for (int c = 0; c < W; ++c) {
        const bool subj = (c - 960 - 6 * f) * (c - 960 - 6 * f) + (r - 540) * (r - 540) < 300 * 300;
        const int v = subj ? 90 + (int)(60 * std::sin((r + c + 3 * f) * 0.02)) + (int)rnd() : 150;
        y[(size_t)r * W + c] = (uint8_t)v;
      }
    for (int r = 0; r < Hc; ++r)
      for (int c = 0; c < Wc; ++c) {
        cb[(size_t)r * Wc + c] = (uint8_t)(44 + ((r * 3 + c + f) & 7));
        cr[(size_t)r * Wc + c] = (uint8_t)(21 + ((r + c * 2) & 3));
      }
    }
    timespec a, b;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &a);   // thread CPU time: robust to preemption on a busy host
    const std::string nal = h264::encode_idr(y.data(), cb.data(), cr.data(), W, H, 20, f, nullptr, nullptr, nullptr);
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &b);
    secs += (b.tv_sec - a.tv_sec) + 1e-9 * (b.tv_nsec - a.tv_nsec);
    bytes += nal.size();
    for (unsigned char ch : nal) h = (h ^ ch) * 1099511628211ull;
  }
  std::printf("{\"frames\": %d, \"ms_per_frame\": %.2f, \"bytes\": %zu, \"fnv\": \"%016llx\"}\n", F,
              1e3 * secs / F, bytes, (unsigned long long)h);
  return 0;
}
