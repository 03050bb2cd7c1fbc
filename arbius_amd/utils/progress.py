"""Progress heartbeats for hang detection (SURVEY.md §5.3 "job leases with a heartbeat; a per-GPU
watchdog that restarts the worker process on a HIP fault or hang").

Pipelines call ``beat()`` once per denoising step / video chunk.  A GPU worker process installs a
hook that stamps the current time into its slot of a shared-memory array; the pool's watchdog in
the dispatcher process kills a worker whose busy slot has not beaten for ``hang_timeout`` seconds
(a hung HIP kernel blocks the host thread at its next sync, so its beats stop) and fails its
tasks over.  With no hook installed ``beat()`` is a no-op (single-process node, tests).
"""
from __future__ import annotations

import threading
import time
from typing import Callable, Optional

_hook: Optional[Callable[[], None]] = None
_tl = threading.local()


def set_hook(fn: Optional[Callable[[], None]]) -> None:
    global _hook
    _hook = fn


def set_slot(slot: int) -> None:
    """Which task slot the calling thread serves (read by the installed hook)."""
    _tl.slot = int(slot)


def slot() -> int:
    return getattr(_tl, "slot", 0)


def beat() -> None:
    h = _hook
    if h is not None:
        h()


def shared_stamp_hook(arr, base: int) -> Callable[[], None]:
    """Hook writing ``time.time()`` into ``arr[base + slot()]`` (``arr``: a multiprocessing
    ``Array('d')`` shared with the dispatcher)."""
    def hook():
        arr[base + slot()] = time.time()
    return hook
