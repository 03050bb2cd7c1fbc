"""Solidity ABI codec (head/tail encoding) for the types the Engine ABI uses:
uintN/intN, address, bool, bytesN, bytes, string, T[] and tuples.

Replaces ethers v5 ``defaultAbiCoder`` / ``Interface`` (``miner/src/utils.ts:42-48``,
``miner/src/index.ts:151-159``) - no Ethereum library exists in this image.
"""
from __future__ import annotations

import re
from typing import Any, List, Sequence, Tuple

from ..utils.keccak import keccak256


def _split_types(s: str) -> List[str]:
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
            continue
        depth += ch == "("
        depth -= ch == ")"
        cur += ch
    if cur:
        out.append(cur)
    return [t.strip() for t in out]


def _is_dynamic(t: str) -> bool:
    if t in ("bytes", "string") or t.endswith("[]"):
        return True
    if t.startswith("("):
        return any(_is_dynamic(x) for x in _split_types(t[1:-1]))
    m = re.match(r"(.*)\[(\d+)\]$", t)
    if m:
        return _is_dynamic(m.group(1))
    return False


def _to_bytes(v) -> bytes:
    if isinstance(v, (bytes, bytearray)):
        return bytes(v)
    if isinstance(v, str):
        s = v[2:] if v.startswith("0x") else v
        return bytes.fromhex(s)
    raise TypeError(f"cannot convert {type(v)} to bytes")


def _enc_single(t: str, v: Any) -> bytes:
    if t.endswith("[]"):
        return len(v).to_bytes(32, "big") + encode([t[:-2]] * len(v), list(v))
    m = re.match(r"(.*)\[(\d+)\]$", t)
    if m:
        return encode([m.group(1)] * int(m.group(2)), list(v))
    if t.startswith("uint"):
        v = int(v)
        if v < 0:
            raise ValueError("negative uint")
        return v.to_bytes(32, "big")
    if t.startswith("int"):
        return int(v).to_bytes(32, "big", signed=True)
    if t == "address":
        b = _to_bytes(v)
        if len(b) != 20:
            raise ValueError("address must be 20 bytes")
        return b"\0" * 12 + b
    if t == "bool":
        return (1 if v else 0).to_bytes(32, "big")
    m = re.match(r"bytes(\d+)$", t)
    if m:
        b = _to_bytes(v)
        n = int(m.group(1))
        if len(b) != n:
            raise ValueError(f"{t} needs {n} bytes, got {len(b)}")
        return b + b"\0" * (32 - n)
    if t in ("bytes", "string"):
        b = v.encode() if (t == "string" and isinstance(v, str)) else _to_bytes(v)
        pad = (-len(b)) % 32
        return len(b).to_bytes(32, "big") + b + b"\0" * pad
    if t.endswith("[]"):
        inner = t[:-2]
        return len(v).to_bytes(32, "big") + encode([inner] * len(v), list(v))
    m = re.match(r"(.*)\[(\d+)\]$", t)
    if m:
        return encode([m.group(1)] * int(m.group(2)), list(v))
    if t.startswith("("):
        return encode(_split_types(t[1:-1]), list(v))
    raise ValueError(f"unsupported type {t}")


def encode(types: Sequence[str], values: Sequence[Any]) -> bytes:
    if len(types) != len(values):
        raise ValueError("types/values length mismatch")
    heads, tails = [], []
    head_len = sum(32 if _is_dynamic(t) else len(_enc_single(t, v)) for t, v in zip(types, values))
    for t, v in zip(types, values):
        if _is_dynamic(t):
            heads.append((head_len + sum(len(x) for x in tails)).to_bytes(32, "big"))
            tails.append(_enc_single(t, v))
        else:
            heads.append(_enc_single(t, v))
    return b"".join(heads) + b"".join(tails)


def _dec_single(t: str, data: bytes, off: int) -> Any:
    word = data[off:off + 32]
    if t.startswith("uint"):
        return int.from_bytes(word, "big")
    if t.startswith("int"):
        return int.from_bytes(word, "big", signed=True)
    if t == "address":
        return "0x" + word[12:].hex()
    if t == "bool":
        return int.from_bytes(word, "big") != 0
    m = re.match(r"bytes(\d+)$", t)
    if m:
        return "0x" + word[: int(m.group(1))].hex()
    raise ValueError(t)


def decode(types: Sequence[str], data: bytes, base: int = 0) -> List[Any]:
    out, off = [], base
    for t in types:
        if _is_dynamic(t):
            ptr = base + int.from_bytes(data[off:off + 32], "big")
            if t in ("bytes", "string"):
                n = int.from_bytes(data[ptr:ptr + 32], "big")
                raw = data[ptr + 32:ptr + 32 + n]
                out.append(raw.decode() if t == "string" else "0x" + raw.hex())
            elif t.endswith("[]"):
                n = int.from_bytes(data[ptr:ptr + 32], "big")
                out.append(decode([t[:-2]] * n, data, ptr + 32))
            elif t.startswith("("):
                out.append(tuple(decode(_split_types(t[1:-1]), data, ptr)))
            else:
                m = re.match(r"(.*)\[(\d+)\]$", t)
                out.append(decode([m.group(1)] * int(m.group(2)), data, ptr))
            off += 32
        elif t.startswith("("):
            inner = _split_types(t[1:-1])
            out.append(tuple(decode(inner, data, off)))
            off += 32 * len(inner)
        else:
            m = re.match(r"(.*)\[(\d+)\]$", t)
            if m:
                n = int(m.group(2))
                out.append(decode([m.group(1)] * n, data, off))
                off += 32 * n
            else:
                out.append(_dec_single(t, data, off))
                off += 32
    return out


def signature_types(sig: str) -> Tuple[str, List[str]]:
    name, rest = sig.split("(", 1)
    return name, _split_types(rest[:-1])


def selector(sig: str) -> bytes:
    return keccak256(sig.encode())[:4]


def topic(sig: str) -> str:
    return "0x" + keccak256(sig.encode()).hex()


def encode_call(sig: str, *args) -> bytes:
    _, types = signature_types(sig)
    return selector(sig) + encode(types, args)


def decode_call(sig: str, calldata: bytes) -> List[Any]:
    _, types = signature_types(sig)
    if calldata[:4] != selector(sig):
        raise ValueError("selector mismatch")
    return decode(types, calldata, 4)[:] if False else decode(types, calldata[4:])
