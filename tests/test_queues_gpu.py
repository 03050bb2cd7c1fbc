"""Task streams own distinct hardware queues (models/graphs.task_stream; profiles/queues_r5_sd15.md).

HIP binds each stream to one of GPU_MAX_HW_QUEUES (4) HSA queues, and two streams on one queue run
their kernels one after the other.  ``task_stream`` measures the binding with a one-workgroup spin
kernel and only hands out streams whose spins overlap with every other live task stream.
"""
import time

import pytest
import torch

from arbius_amd.models import graphs


def test_task_stream_on_cpu_is_none():
    assert graphs.task_stream(torch.device("cpu")) is None


def _wall(streams, cycles):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in streams:
        with torch.cuda.stream(s):
            torch.cuda._sleep(cycles)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


@pytest.mark.gpu
def test_four_task_streams_run_concurrently():
    dev = torch.device("cuda", 0)
    # side streams first-used in between, the pattern that put two r5 task streams on one queue
    side = []
    streams = []
    for i in range(4):
        streams.append(graphs.task_stream(dev, streams))
        s = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(s):
            torch.cuda._sleep(1000)
        side.append(s)
    cycles = 20_000_000
    one = min(_wall([streams[0]], cycles) for _ in range(2))
    four = min(_wall(streams, cycles) for _ in range(2))
    assert four < 1.4 * one, (one, four, graphs.QUEUE_STATS)
