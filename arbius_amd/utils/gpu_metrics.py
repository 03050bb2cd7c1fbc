"""Per-GPU utilisation / memory gauges for ``/metrics``.

Read through ``amdsmi`` (sysfs / driver queries - no HIP context, so the pool's parent process,
which must never initialise the GPU before it spawns its workers, can call it).  Absent library,
driver or permission -> no gauges (an empty list), never an error on the metrics route.
"""
from __future__ import annotations

from typing import List

_STATE = {"init": None}


def _handles():
    if _STATE["init"] is False:
        return []
    try:
        import amdsmi
        if _STATE["init"] is None:
            amdsmi.amdsmi_init()
            _STATE["init"] = True
        return amdsmi.amdsmi_get_processor_handles()
    except Exception:  # noqa: BLE001 - optional telemetry
        _STATE["init"] = False
        return []


def gpu_gauges() -> List[str]:
    """Prometheus lines: gfx activity (%) and VRAM used (bytes) per GPU index."""
    lines: List[str] = []
    hs = _handles()
    if not hs:
        return lines
    import amdsmi
    act, mem = [], []
    for i, h in enumerate(hs):
        try:
            pct = float(amdsmi.amdsmi_get_gpu_activity(h)["gfx_activity"])
            act.append(f'arbius_gpu_utilization_percent{{gpu="{i}"}} {pct}')
        except Exception:  # noqa: BLE001
            pass
        try:
            used = amdsmi.amdsmi_get_gpu_vram_usage(h)["vram_used"]
            mem.append(f'arbius_gpu_vram_used_bytes{{gpu="{i}"}} {int(used) << 20}')
        except Exception:  # noqa: BLE001
            pass
    if act:
        lines += ["# TYPE arbius_gpu_utilization_percent gauge"] + act
    if mem:
        lines += ["# TYPE arbius_gpu_vram_used_bytes gauge"] + mem
    return lines
