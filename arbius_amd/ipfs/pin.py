"""IPFS pinning strategies (``miner/src/ipfs.ts``): kubo HTTP API, Pinata, and a
local content-addressed store (MockIPFS, the CPU plumbing config).

The node computes the CID itself (``unixfs.wrap_directory``) the moment the
output bytes exist, so the commitment can be signalled while the pin is still
in flight; the pin result is checked against the local CID.
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

from .unixfs import CHUNK, add_file, b58decode, b58encode, read_file, wrap_directory

KUBO_ADD_PARAMS = {"cid-version": "0", "hash": "sha2-256", "chunker": f"size-{CHUNK}", "raw-leaves": "false"}


class Pinner:
    async def pin_files(self, taskid: str, files: Sequence[Tuple[str, bytes]]) -> str:
        """Wrap ``files`` in a directory, pin, return the base58 directory CID."""
        raise NotImplementedError

    async def pin_file(self, content: bytes, name: str) -> str:
        raise NotImplementedError

    async def cat(self, cid: str, max_bytes: int) -> Optional[bytes]:
        """The bytes of a UnixFS file by base58 CIDv0, at most ``max_bytes`` (None: this strategy
        cannot read content back; the caller tries the configured gateway instead)."""
        return None

    async def close(self):
        pass


class LocalPinner(Pinner):
    """MockIPFS: blocks kept in memory (and optionally mirrored to ``root`` on disk)."""

    def __init__(self, root: Optional[str] = None):
        self.blocks: Dict[bytes, bytes] = {}
        self.pins: List[str] = []
        self.root = Path(root) if root else None
        if self.root:
            self.root.mkdir(parents=True, exist_ok=True)

    def _store(self, blocks):
        self.blocks.update(blocks)
        if self.root:
            for mh, blk in blocks.items():
                p = self.root / b58encode(mh)
                if not p.exists():
                    p.write_bytes(blk)

    async def pin_files(self, taskid, files):
        d = wrap_directory(list(files))
        self._store(d.blocks)
        self.pins.append(d.cid_str)
        return d.cid_str

    async def pin_file(self, content, name):
        r = add_file(content)
        self._store(r.blocks)
        self.pins.append(r.cid_str)
        return r.cid_str

    def block(self, cid_mh: bytes) -> bytes:
        return self.blocks[cid_mh]

    async def cat(self, cid, max_bytes):
        try:
            return read_file(self.block, b58decode(cid), max_bytes)
        except KeyError:
            return None


class KuboPinner(Pinner):
    """kubo ``/api/v0/add`` (ipfs-http-client addAll with wrapWithDirectory)."""

    def __init__(self, url: str = "http://127.0.0.1:5001", timeout: float = 120.0):
        import httpx
        self.url = url.rstrip("/")
        self.client = httpx.AsyncClient(timeout=timeout)

    async def pin_files(self, taskid, files):
        params = dict(KUBO_ADD_PARAMS, **{"wrap-with-directory": "true", "pin": "true"})
        multipart = [("file", (name, data, "application/octet-stream")) for name, data in files]
        r = await self.client.post(f"{self.url}/api/v0/add", params=params, files=multipart)
        r.raise_for_status()
        for line in r.text.strip().splitlines():
            obj = json.loads(line)
            if obj.get("Name", None) == "":
                return obj["Hash"]
        raise RuntimeError("ipfs cid extract failed")

    async def pin_file(self, content, name):
        r = await self.client.post(f"{self.url}/api/v0/add", params=dict(KUBO_ADD_PARAMS, pin="true"),
                                   files=[("file", (name, content, "application/octet-stream"))])
        r.raise_for_status()
        return json.loads(r.text.strip().splitlines()[-1])["Hash"]

    async def cat(self, cid, max_bytes):
        """``/api/v0/cat`` capped while streaming (kubo checks every block against its hash)."""
        async with self.client.stream("POST", f"{self.url}/api/v0/cat",
                                      params={"arg": cid, "length": str(max_bytes + 1)}) as r:
            r.raise_for_status()
            return await _read_capped(r, max_bytes)

    async def close(self):
        await self.client.aclose()


class PinataPinner(Pinner):
    """Pinata ``pinFileToIPFS`` multipart upload (files under ``<taskid>/<name>``)."""

    URL = "https://api.pinata.cloud/pinning/pinFileToIPFS"

    def __init__(self, jwt: str, timeout: float = 120.0):
        import httpx
        self.jwt = jwt
        self.client = httpx.AsyncClient(timeout=timeout)

    async def _post(self, multipart):
        data = {"pinataOptions": json.dumps({"cidVersion": 0})}
        r = await self.client.post(self.URL, files=multipart, data=data,
                                   headers={"Authorization": f"Bearer {self.jwt}"})
        r.raise_for_status()
        return r.json()["IpfsHash"]

    async def pin_files(self, taskid, files):
        return await self._post([("file", (f"{taskid}/{name}", data, "application/octet-stream"))
                                 for name, data in files])

    async def pin_file(self, content, name):
        return await self._post([("file", (name, content, "application/octet-stream"))])

    async def close(self):
        await self.client.aclose()


async def _read_capped(resp, max_bytes: int) -> bytes:
    buf = bytearray()
    async for chunk in resp.aiter_bytes():
        buf.extend(chunk)
        if len(buf) > max_bytes:
            raise ValueError(f"content exceeds {max_bytes} bytes")
    return bytes(buf)


def _gateway_base(gateway: str) -> str:
    """Operator-configured gateway (``mi355x.ipfs_gateway`` / ``$ARBIUS_IPFS_GATEWAY``): an
    http(s) URL without query or fragment."""
    from urllib.parse import urlsplit
    u = urlsplit(gateway)
    if u.scheme not in ("http", "https") or not u.netloc or u.query or u.fragment:
        raise ValueError(f"bad IPFS gateway URL {gateway!r}")
    return gateway.rstrip("/")


async def gateway_cat(gateway: str, cid: str, max_bytes: int, client=None, timeout: float = 60.0) -> bytes:
    """``GET <gateway>/ipfs/<cid>`` capped at ``max_bytes``.  A gateway is untrusted: callers check
    the bytes against the CID they asked for (``onchain_cid`` / ``add_file``)."""
    import httpx
    if not cid.isalnum():
        raise ValueError("CID must be base58")
    own = client is None
    client = client or httpx.AsyncClient(timeout=timeout, follow_redirects=False)
    try:
        async with client.stream("GET", f"{_gateway_base(gateway)}/ipfs/{cid}") as r:
            r.raise_for_status()
            return await _read_capped(r, max_bytes)
    finally:
        if own:
            await client.aclose()


async def pinata_gc(jwt: str, max_age_s: float = 7200.0, base: str = "https://api.pinata.cloud", client=None,
                    now: float = None) -> dict:
    """Unpin Pinata pins older than ``max_age_s`` (2 h) - the reference's (disabled)
    ``miner/src/scripts/pinata_unpin_old_files.ts`` as one pass (run it from cron /
    a loop).  Pages through ``/data/pinList?status=pinned`` and ``DELETE /pinning/unpin/<cid>``."""
    import datetime
    import time as _time

    import httpx
    own = client is None
    client = client or httpx.AsyncClient(timeout=60.0)
    hdr = {"Authorization": f"Bearer {jwt}"}
    now = _time.time() if now is None else now
    removed, kept, offset = [], 0, 0
    try:
        while True:
            r = await client.get(f"{base}/data/pinList", params={"status": "pinned", "pageLimit": 1000,
                                                                 "pageOffset": offset}, headers=hdr)
            r.raise_for_status()
            rows = r.json().get("rows", [])
            if not rows:
                break
            for row in rows:
                ts = datetime.datetime.fromisoformat(row["date_pinned"].replace("Z", "+00:00")).timestamp()
                if now - ts > max_age_s:
                    d = await client.delete(f"{base}/pinning/unpin/{row['ipfs_pin_hash']}", headers=hdr)
                    d.raise_for_status()
                    removed.append(row["ipfs_pin_hash"])
                else:
                    kept += 1
            offset += len(rows)
    finally:
        if own:
            await client.aclose()
    return {"unpinned": len(removed), "kept": kept, "cids": removed}


def make_pinner(cfg) -> Pinner:
    """From ``MiningConfig.ipfs`` (strategy http_client | pinata | local)."""
    s = cfg.ipfs.strategy
    if s == "http_client":
        return KuboPinner(cfg.ipfs.http_client.url)
    if s == "pinata":
        return PinataPinner(cfg.ipfs.pinata.jwt)
    return LocalPinner(os.environ.get("ARBIUS_LOCAL_IPFS_DIR"))
