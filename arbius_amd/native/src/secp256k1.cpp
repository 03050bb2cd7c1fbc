// secp256k1 ECDSA for the node's transaction signer (SURVEY.md §2.6(e) "secp256k1 ECDSA signing with
// RFC6979 nonces"; chain/tx.py).  The private key and the nonce never steer a branch or an address:
//
//  * field / scalar arithmetic on 4x64-bit limbs with fixed-count loops, reductions by the special
//    forms P = 2^256 - 0x1000003D1 and N = 2^256 - NC, final corrections by masks;
//  * points in projective coordinates with the COMPLETE addition law for a = 0 curves
//    (Renes-Costello-Batina 2016, Alg. 7): one formula for every pair of inputs, doubling and the
//    identity included - no special-case branches;
//  * scalar multiplication by a fixed 4-bit window: 64 x (4 doublings + 1 addition), the window's
//    table entry picked by scanning all 16 entries with masks;
//  * inversions by Fermat exponentiation (fixed public exponents).
// RFC 6979 nonces use HMAC-SHA256 (implemented here).  Only public values branch (the rejection
// loop of RFC 6979 on a nonce >= N, low-s normalisation of the public signature).
// Outputs are bit-identical to chain/secp256k1.py (tests/test_native.py compares both).
#include "secp256k1.h"

#include <cstring>

namespace secp {

typedef unsigned __int128 u128;
typedef uint64_t u64;

// ------------------------------------------------------------------------------------- SHA-256
namespace sha {
static const uint32_t K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
    0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
    0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
    0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
    0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
    0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
    0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};
static inline uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

struct Ctx {
  uint32_t h[8];
  uint8_t buf[64];
  size_t nbuf;
  uint64_t total;
};
static void init(Ctx& c) {
  static const uint32_t H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(c.h, H0, sizeof(H0));
  c.nbuf = 0;
  c.total = 0;
}
static void block(Ctx& c, const uint8_t* p) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 |
                                      (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
    const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = c.h[0], b = c.h[1], cc = c.h[2], d = c.h[3], e = c.h[4], f = c.h[5], g = c.h[6], h = c.h[7];
  for (int i = 0; i < 64; ++i) {
    const uint32_t t1 = h + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
    const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & cc) ^ (b & cc));
    h = g; g = f; f = e; e = d + t1; d = cc; cc = b; b = a; a = t1 + t2;
  }
  c.h[0] += a; c.h[1] += b; c.h[2] += cc; c.h[3] += d; c.h[4] += e; c.h[5] += f; c.h[6] += g; c.h[7] += h;
}
static void update(Ctx& c, const uint8_t* p, size_t n) {
  c.total += n;
  while (n) {
    const size_t k = (64 - c.nbuf) < n ? (64 - c.nbuf) : n;
    memcpy(c.buf + c.nbuf, p, k);
    c.nbuf += k; p += k; n -= k;
    if (c.nbuf == 64) { block(c, c.buf); c.nbuf = 0; }
  }
}
static void final(Ctx& c, uint8_t out[32]) {
  const uint64_t bits = c.total * 8;
  const uint8_t one = 0x80, zero = 0;
  update(c, &one, 1);
  while (c.nbuf != 56) update(c, &zero, 1);
  uint8_t len[8];
  for (int i = 0; i < 8; ++i) len[i] = (uint8_t)(bits >> (56 - 8 * i));
  update(c, len, 8);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(c.h[i] >> 24); out[4 * i + 1] = (uint8_t)(c.h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(c.h[i] >> 8); out[4 * i + 3] = (uint8_t)c.h[i];
  }
}
// HMAC-SHA256(key[32], m1 || m2 || m3)
static void hmac(const uint8_t key[32], const uint8_t* m1, size_t n1, const uint8_t* m2, size_t n2,
                 const uint8_t* m3, size_t n3, uint8_t out[32]) {
  uint8_t ipad[64], opad[64], inner[32];
  for (int i = 0; i < 64; ++i) {
    const uint8_t k = i < 32 ? key[i] : 0;
    ipad[i] = k ^ 0x36;
    opad[i] = k ^ 0x5c;
  }
  Ctx c;
  init(c); update(c, ipad, 64); update(c, m1, n1); update(c, m2, n2); update(c, m3, n3); final(c, inner);
  init(c); update(c, opad, 64); update(c, inner, 32); final(c, out);
}
}  // namespace sha

// ---------------------------------------------------------------------------------- field mod P
struct fe { u64 v[4]; };
static const u64 PC = 0x1000003D1ULL;   // 2^256 - P
static const fe FP = {{0xFFFFFFFEFFFFFC2FULL, ~0ULL, ~0ULL, ~0ULL}};

static inline void csub(u64 s[4], const u64 m[4], u64 extra_top) {
  // s := (extra_top * 2^256 + s) >= m ? s - m : s    (extra_top in {0, 1})
  u64 d[4];
  u64 borrow = 0;
  for (int i = 0; i < 4; ++i) {
    const u128 t = (u128)s[i] - m[i] - borrow;
    d[i] = (u64)t;
    borrow = (u64)(t >> 64) & 1;
  }
  const u64 take = extra_top | (borrow ^ 1);      // 1 -> take d
  const u64 mask = 0 - take;
  for (int i = 0; i < 4; ++i) s[i] = (d[i] & mask) | (s[i] & ~mask);
}

static inline fe fe_from_reduced8(const u64 t[8]) {
  u64 s[4];
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)t[i] + (u128)t[4 + i] * PC;
    s[i] = (u64)c;
    c >>= 64;
  }
  const u64 top = (u64)c;                          // < 2^34
  c = (u128)s[0] + (u128)top * PC;
  s[0] = (u64)c; c >>= 64;
  for (int i = 1; i < 4; ++i) { c += s[i]; s[i] = (u64)c; c >>= 64; }
  const u64 carry = (u64)c;                        // 0 / 1: 2^256 == PC (mod P)
  c = (u128)s[0] + (u128)(carry * PC);
  s[0] = (u64)c; c >>= 64;
  for (int i = 1; i < 4; ++i) { c += s[i]; s[i] = (u64)c; c >>= 64; }
  csub(s, FP.v, 0);
  fe r;
  memcpy(r.v, s, sizeof(s));
  return r;
}

static inline fe fe_mul(const fe& a, const fe& b) {
  u64 t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c += (u128)a.v[i] * b.v[j] + t[i + j];
      t[i + j] = (u64)c;
      c >>= 64;
    }
    t[i + 4] = (u64)c;
  }
  return fe_from_reduced8(t);
}
static inline fe fe_add(const fe& a, const fe& b) {
  fe r;
  u128 c = 0;
  for (int i = 0; i < 4; ++i) { c += (u128)a.v[i] + b.v[i]; r.v[i] = (u64)c; c >>= 64; }
  csub(r.v, FP.v, (u64)c);
  return r;
}
static inline fe fe_sub(const fe& a, const fe& b) {
  fe r;
  u64 borrow = 0;
  for (int i = 0; i < 4; ++i) {
    const u128 t = (u128)a.v[i] - b.v[i] - borrow;
    r.v[i] = (u64)t;
    borrow = (u64)(t >> 64) & 1;
  }
  const u64 mask = 0 - borrow;                      // add P back on underflow
  u128 c = 0;
  for (int i = 0; i < 4; ++i) { c += (u128)r.v[i] + (FP.v[i] & mask); r.v[i] = (u64)c; c >>= 64; }
  return r;
}
static inline fe fe_small(u64 k) { fe r = {{k, 0, 0, 0}}; return r; }

// a^e for a public exponent e (fixed pattern: square every bit, multiply where e has a 1)
static fe fe_pow(const fe& a, const u64 e[4]) {
  fe r = fe_small(1);
  for (int i = 255; i >= 0; --i) {
    r = fe_mul(r, r);
    if ((e[i >> 6] >> (i & 63)) & 1) r = fe_mul(r, a);
  }
  return r;
}
static fe fe_inv(const fe& a) {
  const u64 e[4] = {0xFFFFFFFEFFFFFC2DULL, ~0ULL, ~0ULL, ~0ULL};      // P - 2
  return fe_pow(a, e);
}
static fe fe_sqrt_candidate(const fe& a) {
  const u64 e[4] = {0xFFFFFFFFBFFFFF0CULL, ~0ULL, ~0ULL, 0x3FFFFFFFFFFFFFFFULL};   // (P + 1) / 4
  return fe_pow(a, e);
}
static bool fe_eq(const fe& a, const fe& b) {
  u64 d = 0;
  for (int i = 0; i < 4; ++i) d |= a.v[i] ^ b.v[i];
  return d == 0;
}

// ------------------------------------------------------------------------------ scalars mod N
static const u64 NN[4] = {0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, ~0ULL};
static const u64 NC[3] = {0x402DA1732FC9BEBFULL, 0x4551231950B75FC4ULL, 0x1ULL};   // 2^256 - N

// acc[0..na) += x[0..nx) * y[0..ny)   (fixed sizes -> fixed instruction count)
static inline void mac(u64* acc, int na, const u64* x, int nx, const u64* y, int ny) {
  for (int i = 0; i < nx; ++i) {
    u128 c = 0;
    for (int j = 0; j < ny; ++j) {
      c += (u128)x[i] * y[j] + acc[i + j];
      acc[i + j] = (u64)c;
      c >>= 64;
    }
    for (int k = i + ny; k < na; ++k) {
      c += acc[k];
      acc[k] = (u64)c;
      c >>= 64;
    }
  }
}

static void sc_reduce8(const u64 t[8], u64 r[4]) {
  u64 a[8] = {t[0], t[1], t[2], t[3], 0, 0, 0, 0};
  mac(a, 8, t + 4, 4, NC, 3);                       // < 2^386
  u64 b[8] = {a[0], a[1], a[2], a[3], 0, 0, 0, 0};
  mac(b, 8, a + 4, 4, NC, 3);                       // a[4..] < 2^130 -> b < 2^260
  u64 c[8] = {b[0], b[1], b[2], b[3], 0, 0, 0, 0};
  mac(c, 8, b + 4, 4, NC, 3);                       // b[4] < 2^4 -> c < 2^256 + 2^133
  u64 s[4] = {c[0], c[1], c[2], c[3]};
  csub(s, NN, c[4] & 1);
  csub(s, NN, 0);
  memcpy(r, s, 32);
}
static void sc_mul(const u64 a[4], const u64 b[4], u64 r[4]) {
  u64 t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  mac(t, 8, a, 4, b, 4);
  sc_reduce8(t, r);
}
static void sc_add(const u64 a[4], const u64 b[4], u64 r[4]) {
  u128 c = 0;
  for (int i = 0; i < 4; ++i) { c += (u128)a[i] + b[i]; r[i] = (u64)c; c >>= 64; }
  csub(r, NN, (u64)c);
}
static void sc_inv(const u64 a[4], u64 r[4]) {
  const u64 e[4] = {0xBFD25E8CD036413FULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, ~0ULL};   // N - 2
  u64 x[4] = {1, 0, 0, 0};
  for (int i = 255; i >= 0; --i) {
    sc_mul(x, x, x);
    u64 y[4];
    sc_mul(x, a, y);
    const u64 mask = 0 - ((e[i >> 6] >> (i & 63)) & 1);
    for (int k = 0; k < 4; ++k) x[k] = (y[k] & mask) | (x[k] & ~mask);
  }
  memcpy(r, x, 32);
}
static bool sc_is_zero(const u64 a[4]) { return (a[0] | a[1] | a[2] | a[3]) == 0; }
static bool sc_lt_n(const u64 a[4]) {              // a < N (public use only)
  for (int i = 3; i >= 0; --i) {
    if (a[i] < NN[i]) return true;
    if (a[i] > NN[i]) return false;
  }
  return false;
}

static void be_to_limbs(const uint8_t b[32], u64 r[4]) {
  for (int i = 0; i < 4; ++i) {
    u64 v = 0;
    for (int j = 0; j < 8; ++j) v = (v << 8) | b[(3 - i) * 8 + j];
    r[i] = v;
  }
}
static void limbs_to_be(const u64 a[4], uint8_t b[32]) {
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) b[(3 - i) * 8 + j] = (uint8_t)(a[i] >> (56 - 8 * j));
}

// ------------------------------------------------------------------------------------- points
struct pt { fe X, Y, Z; };                  // projective; identity = (0 : 1 : 0)
static const fe B3 = {{21, 0, 0, 0}};        // 3 * b, b = 7

// complete addition, a = 0 (Renes-Costello-Batina 2016, Algorithm 7)
static pt pt_add(const pt& p, const pt& q) {
  fe t0 = fe_mul(p.X, q.X), t1 = fe_mul(p.Y, q.Y), t2 = fe_mul(p.Z, q.Z);
  fe t3 = fe_add(p.X, p.Y), t4 = fe_add(q.X, q.Y);
  t3 = fe_mul(t3, t4);
  t4 = fe_add(t0, t1);
  t3 = fe_sub(t3, t4);
  t4 = fe_add(p.Y, p.Z);
  fe X3 = fe_add(q.Y, q.Z);
  t4 = fe_mul(t4, X3);
  X3 = fe_add(t1, t2);
  t4 = fe_sub(t4, X3);
  X3 = fe_add(p.X, p.Z);
  fe Y3 = fe_add(q.X, q.Z);
  X3 = fe_mul(X3, Y3);
  Y3 = fe_add(t0, t2);
  Y3 = fe_sub(X3, Y3);
  X3 = fe_add(t0, t0);
  t0 = fe_add(X3, t0);
  t2 = fe_mul(B3, t2);
  fe Z3 = fe_add(t1, t2);
  t1 = fe_sub(t1, t2);
  Y3 = fe_mul(B3, Y3);
  X3 = fe_mul(t4, Y3);
  t2 = fe_mul(t3, t1);
  X3 = fe_sub(t2, X3);
  Y3 = fe_mul(Y3, t0);
  t1 = fe_mul(t1, Z3);
  Y3 = fe_add(t1, Y3);
  t0 = fe_mul(t0, t3);
  Z3 = fe_mul(Z3, t4);
  Z3 = fe_add(Z3, t0);
  return pt{X3, Y3, Z3};
}

static pt pt_identity() { return pt{fe_small(0), fe_small(1), fe_small(0)}; }

// k * P, fixed 4-bit window, constant-time table selection
static pt pt_mul(const pt& P, const u64 k[4]) {
  pt tab[16];
  tab[0] = pt_identity();
  tab[1] = P;
  for (int i = 2; i < 16; ++i) tab[i] = pt_add(tab[i - 1], P);
  pt R = pt_identity();
  for (int w = 63; w >= 0; --w) {
    for (int d = 0; d < 4; ++d) R = pt_add(R, R);
    const u64 digit = (k[w >> 4] >> ((w & 15) * 4)) & 15;
    pt T = pt_identity();
    for (u64 i = 0; i < 16; ++i) {
      const u64 eq = ((i ^ digit) - 1) >> 63;     // 1 iff i == digit
      const u64 m = 0 - eq;
      for (int l = 0; l < 4; ++l) {
        T.X.v[l] = (tab[i].X.v[l] & m) | (T.X.v[l] & ~m);
        T.Y.v[l] = (tab[i].Y.v[l] & m) | (T.Y.v[l] & ~m);
        T.Z.v[l] = (tab[i].Z.v[l] & m) | (T.Z.v[l] & ~m);
      }
    }
    R = pt_add(R, T);
  }
  return R;
}

static const pt G = {
    {{0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL, 0x79BE667EF9DCBBACULL}},
    {{0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL, 0x483ADA7726A3C465ULL}},
    {{1, 0, 0, 0}}};

// affine (x, y); false for the identity
static bool pt_affine(const pt& p, fe& x, fe& y) {
  if (fe_eq(p.Z, fe_small(0))) return false;
  const fe zi = fe_inv(p.Z);
  x = fe_mul(p.X, zi);
  y = fe_mul(p.Y, zi);
  return true;
}

// ------------------------------------------------------------------------------------ ECDSA
static void rfc6979(const uint8_t priv[32], const uint8_t h[32], u64 k[4]) {
  u64 hv[4];
  be_to_limbs(h, hv);
  csub(hv, NN, 0);                                   // bits2octets: h mod N
  uint8_t hb[32];
  limbs_to_be(hv, hb);
  uint8_t V[32], K[32], buf[97];
  memset(V, 1, 32);
  memset(K, 0, 32);
  const uint8_t z = 0, o = 1;
  memcpy(buf, priv, 32);
  memcpy(buf + 32, hb, 32);
  sha::hmac(K, V, 32, &z, 1, buf, 64, K);
  sha::hmac(K, V, 32, nullptr, 0, nullptr, 0, V);
  sha::hmac(K, V, 32, &o, 1, buf, 64, K);
  sha::hmac(K, V, 32, nullptr, 0, nullptr, 0, V);
  for (;;) {
    sha::hmac(K, V, 32, nullptr, 0, nullptr, 0, V);
    be_to_limbs(V, k);
    if (!sc_is_zero(k) && sc_lt_n(k)) return;       // rejection is public (probability ~2^-128)
    sha::hmac(K, V, 32, &z, 1, nullptr, 0, K);
    sha::hmac(K, V, 32, nullptr, 0, nullptr, 0, V);
  }
}

}  // namespace secp

using namespace secp;

int secp256k1_sign(const uint8_t hash[32], const uint8_t priv[32], uint8_t r_out[32], uint8_t s_out[32]) {
  u64 d[4], k[4], z[4];
  be_to_limbs(priv, d);
  if (sc_is_zero(d) || !sc_lt_n(d)) return -1;
  rfc6979(priv, hash, k);
  fe x, y;
  if (!pt_affine(pt_mul(G, k), x, y)) return -1;
  u64 r[4] = {x.v[0], x.v[1], x.v[2], x.v[3]};
  const int high = !sc_lt_n(r);                      // R.x >= N (public)
  csub(r, NN, 0);
  be_to_limbs(hash, z);
  csub(z, NN, 0);
  u64 rd[4], sum[4], ki[4], s[4];
  sc_mul(r, d, rd);
  sc_add(z, rd, sum);
  sc_inv(k, ki);
  sc_mul(ki, sum, s);
  int rec = (int)(y.v[0] & 1) | (high ? 2 : 0);
  // low-s (EIP-2): s > N/2 -> N - s   (s is public)
  static const u64 HALF[4] = {0xDFE92F46681B20A0ULL, 0x5D576E7357A4501DULL, 0xFFFFFFFFFFFFFFFFULL,
                              0x7FFFFFFFFFFFFFFFULL};
  bool gt = false;
  for (int i = 3; i >= 0; --i) {
    if (s[i] != HALF[i]) { gt = s[i] > HALF[i]; break; }
  }
  if (gt) {
    u64 borrow = 0;
    for (int i = 0; i < 4; ++i) {
      const u128 t = (u128)NN[i] - s[i] - borrow;
      s[i] = (u64)t;
      borrow = (u64)(t >> 64) & 1;
    }
    rec ^= 1;
  }
  limbs_to_be(r, r_out);
  limbs_to_be(s, s_out);
  return rec;
}

int secp256k1_pubkey(const uint8_t priv[32], uint8_t out[64]) {
  u64 d[4];
  be_to_limbs(priv, d);
  if (sc_is_zero(d) || !sc_lt_n(d)) return -1;
  fe x, y;
  if (!pt_affine(pt_mul(G, d), x, y)) return -1;
  limbs_to_be(x.v, out);
  limbs_to_be(y.v, out + 32);
  return 0;
}

int secp256k1_recover(const uint8_t hash[32], const uint8_t r_in[32], const uint8_t s_in[32], int rec,
                      uint8_t out[64]) {
  u64 r[4], s[4], z[4];
  be_to_limbs(r_in, r);
  be_to_limbs(s_in, s);
  if (sc_is_zero(r) || sc_is_zero(s) || !sc_lt_n(r) || !sc_lt_n(s)) return -1;
  fe x;
  memcpy(x.v, r, 32);
  if (rec & 2) {                                     // x = r + N (< P)
    u128 c = 0;
    for (int i = 0; i < 4; ++i) { c += (u128)x.v[i] + NN[i]; x.v[i] = (u64)c; c >>= 64; }
    if (c) return -1;
  }
  const fe alpha = fe_add(fe_mul(fe_mul(x, x), x), fe_small(7));
  fe beta = fe_sqrt_candidate(alpha);
  if (!fe_eq(fe_mul(beta, beta), alpha)) return -1;
  if ((beta.v[0] & 1) != (u64)(rec & 1)) beta = fe_sub(fe_small(0), beta);
  const pt R = {x, beta, fe_small(1)};
  be_to_limbs(hash, z);
  csub(z, NN, 0);
  u64 ri[4], u1[4], u2[4], nz[4];
  sc_inv(r, ri);
  // u1 = -z / r, u2 = s / r
  if (sc_is_zero(z)) {
    memset(nz, 0, sizeof(nz));
  } else {
    u64 borrow = 0;
    for (int i = 0; i < 4; ++i) {
      const u128 t = (u128)NN[i] - z[i] - borrow;
      nz[i] = (u64)t;
      borrow = (u64)(t >> 64) & 1;
    }
  }
  sc_mul(nz, ri, u1);
  sc_mul(s, ri, u2);
  fe qx, qy;
  if (!pt_affine(pt_add(pt_mul(G, u1), pt_mul(R, u2)), qx, qy)) return -1;
  limbs_to_be(qx.v, out);
  limbs_to_be(qy.v, out + 32);
  return 0;
}

void sha256_digest(const uint8_t* data, size_t n, uint8_t out[32]) {
  sha::Ctx c;
  sha::init(c);
  sha::update(c, data, n);
  sha::final(c, out);
}
