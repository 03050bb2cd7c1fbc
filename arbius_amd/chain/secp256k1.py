"""secp256k1 ECDSA for Ethereum transactions: deterministic RFC 6979 nonces,
low-s normalisation, recovery id, public-key recovery (ecrecover) and address
derivation (no Ethereum library exists in this image).

``sign`` / ``pubkey`` / ``recover`` run the native C++ implementation
(``native/src/secp256k1.cpp``: complete projective formulas, fixed-window
constant-time scalar multiplication - the private key never steers a branch) when
the extension is built.  The pure-Python Jacobian double-and-add below is the
variable-time reference the native code is tested against (tests/test_native.py);
it signs only when the extension is missing (CPU checkout before build()).
"""
from __future__ import annotations

import hashlib
import hmac
from typing import Optional, Tuple

from ..utils.keccak import keccak256

P = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
G = (GX, GY, 1)


def _inv(a, m=P):
    return pow(a, m - 2, m)


def _jdouble(p):
    x, y, z = p
    if y == 0:
        return (0, 0, 0)
    ysq = (y * y) % P
    s = (4 * x * ysq) % P
    m = (3 * x * x) % P
    nx = (m * m - 2 * s) % P
    ny = (m * (s - nx) - 8 * ysq * ysq) % P
    nz = (2 * y * z) % P
    return (nx, ny, nz)


def _jadd(p, q):
    if p[2] == 0:
        return q
    if q[2] == 0:
        return p
    x1, y1, z1 = p
    x2, y2, z2 = q
    z1s, z2s = (z1 * z1) % P, (z2 * z2) % P
    u1, u2 = (x1 * z2s) % P, (x2 * z1s) % P
    s1, s2 = (y1 * z2s * z2) % P, (y2 * z1s * z1) % P
    if u1 == u2:
        if s1 != s2:
            return (0, 0, 0)
        return _jdouble(p)
    h = (u2 - u1) % P
    r = (s2 - s1) % P
    h2 = (h * h) % P
    h3 = (h * h2) % P
    u1h2 = (u1 * h2) % P
    nx = (r * r - h3 - 2 * u1h2) % P
    ny = (r * (u1h2 - nx) - s1 * h3) % P
    nz = (h * z1 * z2) % P
    return (nx, ny, nz)


def _jmul(p, k):
    r = (0, 0, 0)
    for bit in bin(k)[2:]:
        r = _jdouble(r)
        if bit == "1":
            r = _jadd(r, p)
    return r


def _affine(p):
    if p[2] == 0:
        return None
    zi = _inv(p[2])
    return ((p[0] * zi * zi) % P, (p[1] * zi * zi * zi) % P)


def _native():
    try:
        from .. import native
    except Exception:  # noqa: BLE001
        return None
    return native if getattr(native, "loaded", False) and hasattr(native, "secp256k1_sign") else None


def pubkey(priv: int) -> Tuple[int, int]:
    nat = _native()
    if nat is not None:
        raw = nat.secp256k1_pubkey(int(priv).to_bytes(32, "big"))
        return int.from_bytes(raw[:32], "big"), int.from_bytes(raw[32:], "big")
    return py_pubkey(priv)


def py_pubkey(priv: int) -> Tuple[int, int]:
    return _affine(_jmul(G, priv))


def address_from_pub(pub: Tuple[int, int]) -> str:
    raw = pub[0].to_bytes(32, "big") + pub[1].to_bytes(32, "big")
    return "0x" + keccak256(raw)[12:].hex()


def address_from_priv(priv) -> str:
    return address_from_pub(pubkey(_priv_int(priv)))


def _priv_int(priv) -> int:
    if isinstance(priv, int):
        return priv
    if isinstance(priv, (bytes, bytearray)):
        return int.from_bytes(priv, "big")
    return int(priv[2:] if priv.startswith("0x") else priv, 16)


def _rfc6979_k(priv: int, h: bytes) -> int:
    x = priv.to_bytes(32, "big")
    hv = (int.from_bytes(h, "big") % N).to_bytes(32, "big")
    v = b"\x01" * 32
    k = b"\x00" * 32
    k = hmac.new(k, v + b"\x00" + x + hv, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    k = hmac.new(k, v + b"\x01" + x + hv, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    while True:
        v = hmac.new(k, v, hashlib.sha256).digest()
        cand = int.from_bytes(v, "big")
        if 1 <= cand < N:
            return cand
        k = hmac.new(k, v + b"\x00", hashlib.sha256).digest()
        v = hmac.new(k, v, hashlib.sha256).digest()


def sign(msg_hash: bytes, priv) -> Tuple[int, int, int]:
    """-> (r, s, recovery_id) with low-s (EIP-2)."""
    nat = _native()
    if nat is not None:
        r, s, rec = nat.secp256k1_sign(bytes(msg_hash), _priv_int(priv).to_bytes(32, "big"))
        return int.from_bytes(r, "big"), int.from_bytes(s, "big"), rec
    return py_sign(msg_hash, priv)


def py_sign(msg_hash: bytes, priv) -> Tuple[int, int, int]:
    """Variable-time reference of ``sign`` (tests, no-extension fallback)."""
    d = _priv_int(priv)
    z = int.from_bytes(msg_hash, "big")
    k = _rfc6979_k(d, msg_hash)
    R = _affine(_jmul(G, k))
    r = R[0] % N
    s = (_inv(k, N) * (z + r * d)) % N
    rec = (R[1] & 1) | (2 if R[0] >= N else 0)
    if s > N // 2:
        s = N - s
        rec ^= 1
    return r, s, rec


def recover(msg_hash: bytes, r: int, s: int, rec: int) -> Optional[Tuple[int, int]]:
    """ecrecover: public key from a signature."""
    nat = _native()
    if nat is not None:
        raw = nat.secp256k1_recover(bytes(msg_hash), int(r).to_bytes(32, "big"), int(s).to_bytes(32, "big"), rec)
        return None if raw is None else (int.from_bytes(raw[:32], "big"), int.from_bytes(raw[32:], "big"))
    return py_recover(msg_hash, r, s, rec)


def py_recover(msg_hash: bytes, r: int, s: int, rec: int) -> Optional[Tuple[int, int]]:
    x = r + (N if rec & 2 else 0)
    alpha = (x * x * x + 7) % P
    beta = pow(alpha, (P + 1) // 4, P)
    y = beta if (beta & 1) == (rec & 1) else P - beta
    Rp = (x, y, 1)
    z = int.from_bytes(msg_hash, "big")
    rinv = _inv(r, N)
    u1 = (-z * rinv) % N
    u2 = (s * rinv) % N
    Q = _jadd(_jmul(G, u1), _jmul(Rp, u2))
    return _affine(Q)


def recover_address(msg_hash: bytes, r: int, s: int, rec: int) -> str:
    return address_from_pub(recover(msg_hash, r, s, rec))
