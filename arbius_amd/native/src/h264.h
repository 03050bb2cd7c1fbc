// Deterministic H.264 Constrained-Baseline intra codec (CAVLC) for the video templates'
// out-1.mp4 (zeroscopev2xl / damo / robust_video_matting) and their input_video.
#pragma once
#include <cstdint>
#include <string>
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

// SPS + PPS NALs (header byte included, no start code) matching encode_idr's slices.
void parameter_sets(int width, int height, int qp, std::string& sps, std::string& pps);

// Decode a sequence of NAL units (SPS / PPS / intra slices; CAVLC; I_PCM, I_16x16 and I_NxN
// macroblocks, deblocking disabled); pictures decode in parallel on `threads` threads.  Throws
// std::runtime_error on anything outside that subset (P/B slices, CABAC, FMO, deblocking on,
// non-4:2:0) so callers can reject the input.
std::vector<Picture> decode(const std::vector<std::string>& nals, int threads = 1);

// Table sanity: every VLC table is prefix-free (checked by tests/test_video.py).
bool tables_prefix_free();

}  // namespace h264
