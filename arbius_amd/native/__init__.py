"""Native C++ CPU runtime of the node (``src/native.cpp``): keccak256, deterministic
PNG, H.264 I_PCM payload and the CAVLC intra codec (``src/h264.cpp``),
secp256k1 ECDSA.  Built in-tree by ``python -m arbius_amd.native.build``
(``__graft_entry__.build()``); every function has a byte-identical Python
reference that tests compare against.  When the extension is not built the
names are absent and callers use their Python reference (``loaded`` is False)."""
try:
    from ._native import (deflate_id, h264_decode, h264_decode_rgb, h264_encode_rgb, h264_encode_rgb_stream,  # noqa: F401
                          h264_encode_yuv, h264_encode_yuv420_frames, h264_encode_yuv_stream, h264_nals_from_rbsp,
                          h264_parameter_sets,
                          h264_tables_ok, keccak256, pcm_slice_body, png_encode, rgb_to_yuv420_planes,
                          secp256k1_pubkey,
                          secp256k1_recover, secp256k1_sign, sha256)
    loaded = True
except ImportError:  # not built (CPU-only checkout before build())
    loaded = False
