"""Model registry, task filters and template input hydration.

Semantics of ``miner/src/models.ts`` (getModelById ``:87-98``, checkModelFilter
``:100-143``, hydrateInput ``:145-220``), with the two
reference defects made opt-in:

* Q2 (``models.ts:185-189``): ``decimal`` rejected non-integral numbers;
* Q3 (``models.ts:194``): the ``max`` bound was never enforced.

``hydrate_input``'s own default is spec-correct; the node runs with ``quirks=True`` (config
``reference_hydration_quirks``, default on) so it judges inputs exactly as deployed miners do, and
never contests or solves a task on which the two modes disagree (``hydration_modes_agree``).
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, List, Optional, Tuple

from ..ipfs.unixfs import onchain_cid

TEMPLATE_DIR = Path(__file__).resolve().parent.parent / "config" / "templates"

# miner/src/config.json:1-18 (Arbitrum Nova mainnet deployment)
CHAIN_CONFIG = {
    "l1TokenAddress": "0xe3DBC4F88EAa632DDF9708732E2832EEaA6688AB",
    "baseTokenAddress": "0xe3DBC4F88EAa632DDF9708732E2832EEaA6688AB",
    "engineAddress": "0x399511EDEB7ca4A8328E801b1B3D0fe232aBc996",
    "proxyAdminAddress": "0xf70a86d51Bd88885054ea031344447d75bb4b432",
    "chainId": 42170,
}
KANDINSKY2_ID = "0x82ae0d19f32b6912204160f8d744de08265b7775d07c23b4171c94c8e2892c62"
KANDINSKY2_TEMPLATE_CID = "0x1220511fdf0e88fa9adba98a7693cca89b5d9f3181da4815b0f0500aa4315b38d17d"


def load_template(name: str) -> dict:
    return json.loads((TEMPLATE_DIR / f"{name}.json").read_text())


def template_bytes(name: str) -> bytes:
    return (TEMPLATE_DIR / f"{name}.json").read_bytes()


def template_cid(name: str) -> str:
    """On-chain template CID registered with ``registerModel`` (IPFS.sol:38-65)."""
    return "0x" + onchain_cid(template_bytes(name)).hex()


@dataclass
class MiningFilter:
    minfee: int = 0
    mintime: int = 0
    owner: Optional[str] = None


@dataclass
class Model:
    id: str
    name: str
    template: dict
    mineable: bool = True
    filters: List[MiningFilter] = field(default_factory=lambda: [MiningFilter()])
    kind: str = "image"   # image | video | matting


def default_models(ids: Optional[Dict[str, str]] = None, minfee: int = 0) -> Dict[str, Model]:
    """Known templates.  Only kandinsky2 has a mainnet id (miner/src/config.json:7-16);
    others get ids from config / registration (``ids`` name -> id).  ``minfee``: the
    ``MiningFilter.minfee`` of every model (index.ts:846-851 hard-codes 0)."""
    ids = dict(ids or {})
    ids.setdefault("kandinsky2", KANDINSKY2_ID)
    kinds = {"anythingv3": "image", "kandinsky2": "image", "zeroscopev2xl": "video", "damo": "video",
             "robust_video_matting": "matting"}
    out = {}
    for name, kind in kinds.items():
        mid = ids.get(name)
        if mid is None:
            continue
        out[mid.lower()] = Model(mid.lower(), name, load_template(name), True, [MiningFilter(minfee=int(minfee))],
                                 kind)
    return out


def get_model_by_id(models: Dict[str, Model], model_id: str) -> Optional[Model]:
    return models.get(model_id.lower())


def check_model_filter(models: Dict[str, Model], model: str, now: int, fee: int, blocktime: int,
                       owner: str) -> Tuple[bool, bool, Optional[dict]]:
    """-> (modelEnabled, filterPassed, modelTemplate)  (models.ts:100-143)."""
    m = get_model_by_id(models, model)
    if m is None:
        return False, False, None
    for f in m.filters:
        if f.owner and owner.lower() != f.owner.lower():
            continue
        if not int(fee) >= int(f.minfee):
            continue
        if f.mintime > 0 and now - int(blocktime) < f.mintime:
            continue
        return True, True, m.template
    return True, False, m.template


def _is_number(v) -> bool:
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def _js_int32_equal(v) -> bool:
    """JS ``col === (col|0)``: integral and representable as int32."""
    if not _is_number(v) or (isinstance(v, float) and not math.isfinite(v)):
        return False
    if isinstance(v, float) and not v.is_integer():
        return False
    return -(2 ** 31) <= int(v) < 2 ** 31


def hydrate_input(pre: Any, template: dict, quirks: bool = False) -> Tuple[Optional[dict], bool, str]:
    """-> (input, err, errmsg).  Output key order follows the template rows."""
    inp: Dict[str, Any] = {}
    if not isinstance(pre, dict):
        return inp, True, "input is not an object"

    def e(msg):
        return inp, True, msg

    for row in template["input"]:
        var = row["variable"]
        present = var in pre
        col = pre.get(var)
        if row.get("required") and not present:
            return e(f"input missing required field ({var})")
        if present:
            t = row["type"]
            if t in ("string", "string_enum"):
                if not isinstance(col, str):
                    return e(f"input wrong type ({var})")
            elif t in ("int", "int_enum"):
                if not _js_int32_equal(col):
                    return e(f"input wrong type ({var})")
            elif t == "decimal":
                ok = _js_int32_equal(col) if quirks else (_is_number(col) and math.isfinite(float(col)))
                if not ok:
                    return e(f"input wrong type ({var})")
            if t in ("int", "decimal"):
                lo, hi = row.get("min"), row.get("max")
                if lo is not None and col < lo:
                    return e(f"input out of bounds ({var})")
                if not quirks and hi is not None and col > hi:
                    return e(f"input out of bounds ({var})")
            if t in ("string_enum", "int_enum"):
                if col not in row["choices"] or (t == "int_enum" and isinstance(col, bool)):
                    return e(f"input not in enum ({var})")
            inp[var] = col
        else:
            inp[var] = row.get("default")
    return inp, False, ""


def hydration_modes_agree(pre: Any, template: dict) -> bool:
    """True when spec-correct and reference-quirk hydration reach the same verdict (valid or not).
    A task on which they disagree is neither solved nor marked invalid: contesting it, or voting on
    its contestation, could put this node on the slashed minority side."""
    _, e1, _ = hydrate_input(pre, template, False)
    _, e2, _ = hydrate_input(pre, template, True)
    return e1 == e2
