// Deterministic H.264 Constrained-Baseline intra codec (CAVLC) for the video templates'
// out-1.mp4 (zeroscopev2xl / damo / robust_video_matting) and their input_video.
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <utility>
#include <vector>

namespace h264 {

struct Picture {          // decoded 4:2:0 planes at macroblock-padded size
  int w16 = 0, h16 = 0;   // luma size in samples (multiples of 16)
  int crop_w = 0, crop_h = 0;
  std::vector<uint8_t> y, cb, cr;
};

// One IDR access unit (a single NAL: header byte + emulation-prevented slice RBSP) of I_16x16
// macroblocks at constant qp from 4:2:0 planes (W, H multiples of 16).  When recon_* are
// non-null they receive the decoder-side reconstruction (what every conforming decoder outputs).
std::string encode_idr(const uint8_t* y, const uint8_t* cb, const uint8_t* cr, int W, int H, int qp,
                       int idr_pic_id, uint8_t* recon_y, uint8_t* recon_cb, uint8_t* recon_cr);

// A NAL unit (header byte + emulation-prevented payload) from a finished RBSP, e.g. the GPU
// encoder's slices (ops/csrc/h264_intra.hip): encode_idr's bytes for the same RBSP.
std::string rbsp_to_nal(uint8_t nal_header, const uint8_t* rbsp, size_t n);

// SPS + PPS NALs (header byte included, no start code) matching encode_idr's / encode_stream's slices.
void parameter_sets(int width, int height, int qp, std::string& sps, std::string& pps, int max_refs = 1);

// IPPP stream: an IDR every `gop` pictures, P pictures in between (P_Skip / P_L0_16x16 from a
// quarter-sample motion search, Intra_16x16 where cheaper), deblocking on, slices of
// `rows_per_slice` macroblock rows encoded in parallel (the slicing depends on the size only, so
// the bytes never depend on `threads`).  seed != 0 is the decoder-coverage mode: random partitions
// (16x8 / 8x16 / 8x8 + sub-partitions), vectors, reference indices among `max_refs`, list
// modifications, non-reference pictures, slice cuts, deblocking controls and QP deltas.
struct StreamOptions {
  int qp = 20, gop = 30, max_refs = 1, rows_per_slice = 4, threads = 1;
  uint32_t seed = 0;
  bool keep_recon = false;
};
struct EncodedPicture {
  std::vector<std::string> nals;              // one NAL per slice
  std::vector<uint8_t> y, cb, cr;             // deblocked reconstruction when keep_recon
};
using LoadFn = std::function<void(int index, uint8_t* y, uint8_t* cb, uint8_t* cr)>;
std::vector<EncodedPicture> encode_stream(int F, int W, int H, const StreamOptions& opts, const LoadFn& load);

// Decode a sequence of NAL units: Constrained Baseline CAVLC - SPS / PPS, I and P slices (I_PCM,
// I_16x16, I_NxN, P_Skip, P_L0 16x16 / 16x8 / 8x16 / 8x8 with sub-partitions, multiple short-term
// references, list modification, sliding-window / MMCO 1+5 marking), in-loop deblocking.
// Coded video sequences (IDR to IDR) decode in parallel on `threads` threads.  Throws
// std::runtime_error on anything outside that subset (B slices, CABAC, FMO, interlace, long-term
// references, weighted prediction, 8x8 transform, non-4:2:0) so callers can reject the input.
std::vector<Picture> decode(const std::vector<std::string>& nals, int threads = 1);

// Streaming form: on_layout gets every picture's crop size before any decoding (so a caller can
// allocate its output once), sink gets each picture as soon as it is decoded (from worker threads,
// each index once; threads_free = how many threads the sink may use itself).  side (tests)
// receives every picture's unfiltered reconstruction and the deblocking filter's inputs.
struct SideInfo {
  std::vector<uint8_t> y, cb, cr;             // before the deblocking filter
  std::vector<int> mvx, mvy, refpic;          // per 4x4 luma block
  std::vector<int> nonzero;                   // TotalCoeff per 4x4 luma block
  std::vector<uint8_t> intra, qp;             // per macroblock
  std::vector<int> slice;                     // per macroblock
  std::vector<std::vector<int>> deblock;      // per slice: (disable_deblocking_filter_idc, 2*alpha, 2*beta offsets)
  int chroma_qp_offset = 0;
};
using LayoutFn = std::function<void(const std::vector<std::pair<int, int>>& crops)>;
using PictureSink = std::function<void(size_t index, Picture&& picture, int threads_free)>;
constexpr uint64_t kDefaultMaxSamples = uint64_t(1) << 30;   // total luma samples a stream may decode to
void decode(const std::vector<std::string>& nals, int threads, const LayoutFn& on_layout, const PictureSink& sink,
            std::vector<SideInfo>* side = nullptr, uint64_t max_samples = kDefaultMaxSamples);

// Table sanity: every VLC table is prefix-free (checked by tests/test_video.py).
bool tables_prefix_free();

}  // namespace h264
