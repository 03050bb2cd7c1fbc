// secp256k1 ECDSA (RFC 6979, low-s, recovery id) for the node's transaction signer; see secp256k1.cpp.
#pragma once
#include <cstddef>
#include <cstdint>

// -> recovery id (0..3) or -1 on an invalid key
int secp256k1_sign(const uint8_t hash[32], const uint8_t priv[32], uint8_t r_out[32], uint8_t s_out[32]);
// uncompressed public key X || Y (64 bytes); 0 ok, -1 invalid key
int secp256k1_pubkey(const uint8_t priv[32], uint8_t out[64]);
// ecrecover: 0 ok, -1 invalid signature
int secp256k1_recover(const uint8_t hash[32], const uint8_t r[32], const uint8_t s[32], int rec, uint8_t out[64]);
void sha256_digest(const uint8_t* data, size_t n, uint8_t out[32]);
