"""Offline IPFS CIDv0 computation: dag-pb / UnixFS importer semantics.

What the reference obtains from a kubo daemon / Pinata (``miner/src/ipfs.ts:11-16``:
``cidVersion 0, sha2-256, chunker size-262144, rawLeaves false``;
``wrapWithDirectory: true`` for solutions, ``:37-47``) computed locally, so a
solution CID is known the moment the PNG bytes exist (commitment can be
signalled before the pin completes).

* single chunk (<= 262144 B): leaf PBNode{Data=UnixFS{File, Data, filesize}}
  - identical to the on-chain ``IPFS.getIPFSCID`` (contract/contracts/libraries/IPFS.sol:38-65)
* multi chunk: balanced DAG, <= 174 links per node, leaves as above,
  internal nodes UnixFS{File, filesize, blocksizes[]}, links {Hash, Name "", Tsize}
* directory wrap: PBNode{Links sorted by name {Hash, Name, Tsize}, Data=UnixFS{Directory}}

PBNode serialisation order is Links (field 2) then Data (field 1), as dag-pb
requires.  ``Tsize`` = total bytes of the child's DAG.
"""
from __future__ import annotations

import os

import hashlib
from dataclasses import dataclass
from typing import Dict, Sequence, Tuple

CHUNK = 262144
MAX_LINKS = 174
B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"


def varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def b58encode(b: bytes) -> str:
    n = int.from_bytes(b, "big")
    s = ""
    while n:
        n, r = divmod(n, 58)
        s = B58[r] + s
    pad = len(b) - len(b.lstrip(b"\0"))
    return "1" * pad + s


def b58decode(s: str) -> bytes:
    n = 0
    for ch in s:
        n = n * 58 + B58.index(ch)
    body = n.to_bytes((n.bit_length() + 7) // 8, "big") if n else b""
    pad = len(s) - len(s.lstrip("1"))
    return b"\0" * pad + body


def multihash_sha256(data: bytes) -> bytes:
    return b"\x12\x20" + hashlib.sha256(data).digest()


def _field_bytes(num: int, data: bytes) -> bytes:
    return varint((num << 3) | 2) + varint(len(data)) + data


def _field_varint(num: int, v: int) -> bytes:
    return varint(num << 3) + varint(v)


def unixfs_data(type_: int, data: bytes = None, filesize: int = None, blocksizes: Sequence[int] = ()) -> bytes:
    out = _field_varint(1, type_)
    if data is not None:
        out += _field_bytes(2, data)
    if filesize is not None:
        out += _field_varint(3, filesize)
    for bs in blocksizes:
        out += _field_varint(4, bs)
    return out


@dataclass
class Link:
    hash: bytes  # multihash bytes (34)
    name: str
    tsize: int


def pb_node(links: Sequence[Link], data: bytes) -> bytes:
    out = b""
    for l in links:
        lb = _field_bytes(1, l.hash) + _field_bytes(2, l.name.encode()) + _field_varint(3, l.tsize)
        out += _field_bytes(2, lb)
    out += _field_bytes(1, data)
    return out


@dataclass
class DagResult:
    root: bytes        # root block bytes
    cid: bytes         # multihash of root (CIDv0 bytes)
    tsize: int         # cumulative DAG size
    blocks: Dict[bytes, bytes]  # multihash -> block (for MockIPFS / pinning)
    filesize: int

    @property
    def cid_str(self) -> str:
        return b58encode(self.cid)

    @property
    def cid_hex(self) -> str:
        return "0x" + self.cid.hex()


def _leaf(chunk: bytes) -> Tuple[bytes, int, int]:
    """pb_node([], unixfs_data(2, chunk, len(chunk))) assembled with ONE copy of the chunk:
    0a <len(inner)> | 08 02 12 <n> chunk 18 <n>  (PBNode.Data = UnixFS{File, Data, filesize})."""
    n = len(chunk)
    vn = varint(n)
    inner_len = 2 + 1 + len(vn) + n + 1 + len(vn)
    blk = b"".join((b"\x0a", varint(inner_len), b"\x08\x02\x12", vn, chunk, b"\x18", vn))
    return blk, n, len(blk)


def add_file(content: bytes, chunk_size: int = CHUNK) -> DagResult:
    """kubo ``add`` (balanced layout, dag-pb leaves) -> root CID."""
    blocks: Dict[bytes, bytes] = {}
    if len(content) <= chunk_size:
        blk, fsz, _ = _leaf(content)
        mh = multihash_sha256(blk)
        blocks[mh] = blk
        return DagResult(blk, mh, len(blk), blocks, fsz)

    # nodes as (mh, filesize, tsize)
    view = memoryview(content)

    def leaf_at(off):
        blk, fsz, _ = _leaf(view[off:off + chunk_size])
        return multihash_sha256(blk), blk, fsz

    offs = range(0, len(content), chunk_size)
    if len(offs) >= 32:
        # multi-MB video outputs: leaves are independent, and sha256 / the block copy release the
        # GIL, so hash them on a thread pool (map keeps the leaf order -> the same DAG bytes)
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
            done = list(ex.map(leaf_at, offs))
    else:
        done = [leaf_at(o) for o in offs]
    leaves = []
    for mh, blk, fsz in done:
        blocks[mh] = blk
        leaves.append((mh, fsz, len(blk)))

    def make_parent(children):
        links = [Link(mh, "", ts) for mh, _, ts in children]
        data = unixfs_data(2, None, sum(f for _, f, _ in children), [f for _, f, _ in children])
        blk = pb_node(links, data)
        mh = multihash_sha256(blk)
        blocks[mh] = blk
        return (mh, sum(f for _, f, _ in children), len(blk) + sum(ts for _, _, ts in children)), blk

    # balanced builder: depth-d subtrees hold MAX_LINKS**d leaves, filled left to right
    level = leaves
    root_blk = None
    while True:
        parents = []
        for i in range(0, len(level), MAX_LINKS):
            node, blk = make_parent(level[i:i + MAX_LINKS])
            parents.append(node)
            root_blk = blk
        if len(parents) == 1:
            mh, fsz, ts = parents[0]
            return DagResult(root_blk, mh, ts, blocks, fsz)
        level = parents


def wrap_directory(files: Sequence[Tuple[str, bytes]], chunk_size: int = CHUNK) -> DagResult:
    """kubo ``addAll(..., wrapWithDirectory: true)`` -> directory CID (the solution CID)."""
    blocks: Dict[bytes, bytes] = {}
    links = []
    total = 0
    for name, content in files:
        r = add_file(content, chunk_size)
        blocks.update(r.blocks)
        links.append(Link(r.cid, name, r.tsize))
        total += r.filesize
    links.sort(key=lambda l: l.name.encode())
    blk = pb_node(links, unixfs_data(1))
    mh = multihash_sha256(blk)
    blocks[mh] = blk
    return DagResult(blk, mh, len(blk) + sum(l.tsize for l in links), blocks, total)


def onchain_cid(content: bytes) -> bytes:
    """``IPFS.getIPFSCID`` (contract/contracts/libraries/IPFS.sol:38-65): single-chunk CIDv0."""
    if len(content) > 65536:
        raise ValueError("Max content size is 65536 bytes")
    return multihash_sha256(pb_node([], unixfs_data(2, content, len(content))))


def cid_str_to_hex(cid: str) -> str:
    """base58 CIDv0 -> '0x1220..' (``miner/src/models.ts:52``)."""
    return "0x" + b58decode(cid).hex()


def cid_hex_to_str(h: str) -> str:
    return b58encode(bytes.fromhex(h[2:] if h.startswith("0x") else h))


# ---------------------------------------------------------------------------------------------
# Reader: the inverse of add_file over a block store (LocalPinner.cat; the bytes behind an
# on-chain task CID when its input cannot be read from the transaction).

def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    n = shift = 0
    while True:
        if i >= len(b) or shift > 63:
            raise ValueError("truncated protobuf varint")
        c = b[i]
        i += 1
        n |= (c & 0x7F) << shift
        shift += 7
        if not c & 0x80:
            return n, i


def _pb_fields(b: bytes):
    """(field number, wire type, value) of a protobuf message (varint / length-delimited only)."""
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 2:
            n, i = _read_varint(b, i)
            if i + n > len(b):
                raise ValueError("truncated protobuf field")
            v, i = b[i:i + n], i + n
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield num, wt, v


def parse_pb_node(block: bytes) -> Tuple[list, bytes]:
    """dag-pb PBNode -> ([Link], Data bytes)."""
    links, data = [], b""
    for num, wt, v in _pb_fields(block):
        if num == 2 and wt == 2:
            h, name, ts = b"", "", 0
            for n2, w2, v2 in _pb_fields(v):
                if n2 == 1 and w2 == 2:
                    h = bytes(v2)
                elif n2 == 2 and w2 == 2:
                    name = bytes(v2).decode("utf-8", "replace")
                elif n2 == 3 and w2 == 0:
                    ts = v2
            links.append(Link(h, name, ts))
        elif num == 1 and wt == 2:
            data = bytes(v)
    return links, data


def read_file(get_block, cid: bytes, max_bytes: int = 1 << 30) -> bytes:
    """Bytes of the UnixFS file whose root multihash is ``cid``; ``get_block(mh) -> bytes``.
    Every block is checked against its multihash (a store cannot substitute content) and the
    output is capped at ``max_bytes`` (ValueError past it)."""
    out = bytearray()

    def walk(mh: bytes, depth: int):
        if depth > 16:
            raise ValueError("unixfs DAG too deep")
        blk = get_block(mh)
        if multihash_sha256(blk) != mh:
            raise ValueError("block does not match its multihash")
        links, data = parse_pb_node(blk)
        typ, chunk = None, b""
        for num, wt, v in _pb_fields(data):
            if num == 1 and wt == 0:
                typ = v
            elif num == 2 and wt == 2:
                chunk = bytes(v)
        if typ not in (0, 2):            # Raw / File only (a directory is not a task input)
            raise ValueError(f"unixfs node type {typ} is not a file")
        out.extend(chunk)
        if len(out) > max_bytes:
            raise ValueError("file exceeds the size cap")
        for l in links:
            walk(l.hash, depth + 1)

    walk(cid, 0)
    return bytes(out)
