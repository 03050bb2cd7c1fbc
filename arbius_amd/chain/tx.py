"""RLP + Ethereum transaction signing (legacy EIP-155 and EIP-1559 type-2).

Arbitrum Nova is chain id 42170 (0xa4ba); the reference sends legacy-priced
transactions through ethers v5 with explicit gas limits (index.ts:620-739).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple, Union

from ..utils.keccak import keccak256
from . import secp256k1

RLPItem = Union[bytes, int, str, List["RLPItem"]]


def _to_bytes(x: RLPItem) -> bytes:
    if isinstance(x, bytes):
        return x
    if isinstance(x, int):
        if x == 0:
            return b""
        return x.to_bytes((x.bit_length() + 7) // 8, "big")
    if isinstance(x, str):
        h = x[2:] if x.startswith("0x") else x
        return bytes.fromhex(h)
    raise TypeError(type(x))


def _len_prefix(n: int, offset: int) -> bytes:
    if n < 56:
        return bytes([offset + n])
    ln = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([offset + 55 + len(ln)]) + ln


def rlp_encode(x: RLPItem) -> bytes:
    if isinstance(x, list):
        body = b"".join(rlp_encode(i) for i in x)
        return _len_prefix(len(body), 0xC0) + body
    b = _to_bytes(x)
    if len(b) == 1 and b[0] < 0x80:
        return b
    return _len_prefix(len(b), 0x80) + b


def rlp_decode(data: bytes):
    def dec(i):
        b0 = data[i]
        if b0 < 0x80:
            return data[i:i + 1], i + 1
        if b0 < 0xB8:
            n = b0 - 0x80
            return data[i + 1:i + 1 + n], i + 1 + n
        if b0 < 0xC0:
            ll = b0 - 0xB7
            n = int.from_bytes(data[i + 1:i + 1 + ll], "big")
            s = i + 1 + ll
            return data[s:s + n], s + n
        if b0 < 0xF8:
            n, s = b0 - 0xC0, i + 1
        else:
            ll = b0 - 0xF7
            n = int.from_bytes(data[i + 1:i + 1 + ll], "big")
            s = i + 1 + ll
        out, j = [], s
        while j < s + n:
            item, j = dec(j)
            out.append(item)
        return out, s + n

    item, end = dec(0)
    if end != len(data):
        raise ValueError("trailing bytes")
    return item


@dataclass
class Tx:
    nonce: int
    to: str
    data: bytes
    gas: int
    chain_id: int
    value: int = 0
    gas_price: Optional[int] = None          # legacy
    max_fee: Optional[int] = None            # EIP-1559
    max_priority_fee: Optional[int] = None

    def signing_hash(self) -> bytes:
        if self.max_fee is not None:
            payload = rlp_encode([self.chain_id, self.nonce, self.max_priority_fee or 0, self.max_fee, self.gas,
                                  self.to, self.value, self.data, []])
            return keccak256(b"\x02" + payload)
        return keccak256(rlp_encode([self.nonce, self.gas_price or 0, self.gas, self.to, self.value, self.data,
                                     self.chain_id, 0, 0]))

    def sign(self, priv) -> bytes:
        h = self.signing_hash()
        r, s, rec = secp256k1.sign(h, priv)
        if self.max_fee is not None:
            return b"\x02" + rlp_encode([self.chain_id, self.nonce, self.max_priority_fee or 0, self.max_fee,
                                         self.gas, self.to, self.value, self.data, [], rec, r, s])
        v = rec + 35 + 2 * self.chain_id
        return rlp_encode([self.nonce, self.gas_price or 0, self.gas, self.to, self.value, self.data, v, r, s])


def decode_raw_tx(raw: bytes) -> Tuple[dict, str]:
    """-> (fields, sender).  Used by the mock JSON-RPC node and for tests."""
    if raw[0] == 0x02:
        f = rlp_decode(raw[1:])
        chain_id, nonce, tip, fee, gas, to, value, data, _al, rec, r, s = f
        tx = Tx(int.from_bytes(nonce, "big"), "0x" + to.hex(), data, int.from_bytes(gas, "big"),
                int.from_bytes(chain_id, "big"), int.from_bytes(value, "big"), None, int.from_bytes(fee, "big"),
                int.from_bytes(tip, "big"))
        rec_id = int.from_bytes(rec, "big")
    else:
        nonce, gp, gas, to, value, data, v, r, s = rlp_decode(raw)
        vv = int.from_bytes(v, "big")
        chain_id = (vv - 35) // 2
        rec_id = vv - 35 - 2 * chain_id
        tx = Tx(int.from_bytes(nonce, "big"), "0x" + to.hex(), data, int.from_bytes(gas, "big"), chain_id,
                int.from_bytes(value, "big"), int.from_bytes(gp, "big"))
    sender = secp256k1.recover_address(tx.signing_hash(), int.from_bytes(r, "big"), int.from_bytes(s, "big"), rec_id)
    return {"nonce": tx.nonce, "to": tx.to, "data": tx.data, "gas": tx.gas, "chain_id": tx.chain_id,
            "value": tx.value, "gas_price": tx.gas_price, "max_fee": tx.max_fee,
            "hash": "0x" + keccak256(raw).hex()}, sender
