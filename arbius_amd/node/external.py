"""Compatibility solver pools for externally served models - the reference's two
ML strategies (``miner/src/index.ts:752-877``): a Cog container's
``POST /predictions`` and the Replicate API.  Outputs are turned into the same
``Solution`` (files + locally computed directory CID) as the in-process engine.
"""
from __future__ import annotations

import base64
import logging
from typing import Dict

from .solver import Solution, solve_files

log = logging.getLogger("arbius.external")


def _filename(model) -> str:
    try:
        return model.template["output"][0]["filename"]
    except (KeyError, IndexError, TypeError):
        return "out-1.png"


class CogSolverPool:
    """``axios.post(c.ml.cog[modelid].url, {input})`` -> ``output[0]`` base64 data URI."""

    hardware = "cog"
    weights_id = "container"

    def __init__(self, urls: Dict[str, str], capacity: int = 1, timeout: float = 600.0):
        import httpx
        self.urls = {k.lower(): v for k, v in urls.items()}
        self.capacity = capacity
        self.http = httpx.AsyncClient(timeout=timeout)

    async def solve(self, model, taskid, inp) -> Solution:
        url = self.urls.get(model.id.lower())
        if url is None:
            raise RuntimeError(f"no cog url configured for model {model.id}")
        r = await self.http.post(url, json={"input": inp})
        r.raise_for_status()
        out = r.json().get("output")
        if not isinstance(out, list) or len(out) != 1:
            raise RuntimeError("cog output must be a list of length 1")  # index.ts:861-863
        data_uri = out[0]
        b64 = data_uri.split(",", 1)[1] if data_uri.startswith("data:") else data_uri
        return solve_files([(_filename(model), base64.b64decode(b64))])

    async def close(self):
        await self.http.aclose()


class ReplicateSolverPool:
    """``replicate.run(owner/model:hash, {input})`` then download the output URL."""

    API = "https://api.replicate.com/v1/predictions"
    hardware = "replicate"
    weights_id = "container"

    def __init__(self, api_token: str, capacity: int = 1, timeout: float = 600.0, poll: float = 1.0):
        import httpx
        self.token = api_token
        self.capacity = capacity
        self.poll = poll
        self.http = httpx.AsyncClient(timeout=timeout)

    async def solve(self, model, taskid, inp) -> Solution:
        import asyncio
        docker = model.template["meta"]["docker"]            # r8.im/owner/model@sha256:hash
        version = docker.split("@sha256:")[1]
        h = {"Authorization": f"Token {self.token}"}
        r = await self.http.post(self.API, json={"version": version, "input": inp}, headers=h)
        r.raise_for_status()
        pred = r.json()
        while pred.get("status") not in ("succeeded", "failed", "canceled"):
            await asyncio.sleep(self.poll)
            pred = (await self.http.get(pred["urls"]["get"], headers=h)).json()
        if pred["status"] != "succeeded":
            raise RuntimeError(f"replicate prediction {pred['status']}")
        out = pred["output"]
        url = out[0] if isinstance(out, list) else out
        data = (await self.http.get(url)).content
        return solve_files([(_filename(model), data)])

    async def close(self):
        await self.http.aclose()
