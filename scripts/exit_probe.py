#!/usr/bin/env python3
"""Where does a process that used graphs.task_stream crash at exit?  Prints a marker before each
teardown step (stderr, unbuffered) so the last marker names the step that faulted."""
import faulthandler
import gc
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.enable()


def mark(s):
    print(f"[exit_probe] {s}", file=sys.stderr, flush=True)


import torch  # noqa: E402

from arbius_amd.models import graphs  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "task"
dev = torch.device("cuda", 0)
streams, side = [], []
for i in range(4):
    streams.append(graphs.task_stream(dev, streams) if mode == "task" else torch.cuda.Stream(device=dev))
    if mode != "plain":
        s = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(s):
            torch.cuda._sleep(1000)
        side.append(s)
torch.cuda.synchronize()
t0 = time.perf_counter()
for s in streams:
    with torch.cuda.stream(s):
        torch.cuda._sleep(20_000_000)
torch.cuda.synchronize()
mark(f"mode {mode} 4-stream spin {1e3 * (time.perf_counter() - t0):.2f} ms stats {graphs.QUEUE_STATS}")
mark("del locals")
del streams, side, s
gc.collect()
mark("clear module state")
graphs._HELD.clear()
gc.collect()
mark("exit")
