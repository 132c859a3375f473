"""The update graph's capture with unreachable device-holding cycles around
(GPU only): a cyclic-GC collection triggered by an allocation inside the
capture would run their finalizers -- freeing device memory, destroying a HIP
graph -- while the stream captures, which aborts the process (round 3:
``Fatal Python error: Aborted`` in test_online, the capture of
cql_impl._enqueue).  ops.graph_capture pauses the collector for the capture;
this pins it: with the collector's thresholds at 1 (a collection on every
allocation) and fifty unreachable cycles each owning a device tensor and a
CUDAGraph, no collection starts while a stream is capturing, and the update
still captures once and replays.

Reference: the Impl lifetime the fit loop drives (d3rlpy/algos/torch/
base.py:28-224, d3rlpy/base.py:624-663).
"""
import gc

import numpy as np
import pytest
import torch

from cql_helpers import HostBatch, make_batch, make_impl

pytestmark = pytest.mark.gpu


class _Node:
    pass


def _make_cycles(n):
    for _ in range(n):
        a, b = _Node(), _Node()
        a.peer, b.peer = b, a
        a.t = torch.zeros(4096, device="cuda")
        b.g = torch.cuda.CUDAGraph()


def test_no_gc_collection_inside_update_capture():
    D, A, H, N, B = 11, 3, [64, 64], 4, 32
    impl = make_impl(D, A, H, N)
    arrs = make_batch(np.random.RandomState(0), B, D, A)
    started = []

    def cb(phase, info):
        if phase == "start" and torch.cuda.is_current_stream_capturing():
            started.append(dict(info))

    gc.collect()
    old = gc.get_threshold()
    gc.callbacks.append(cb)
    gc.set_threshold(1, 1, 1)
    try:
        _make_cycles(50)  # unreachable from here on: only the collector frees them
        for _ in range(4):  # eager, capture, replays
            impl.update_step(HostBatch(*arrs), use_graph=True)
            _make_cycles(5)
        torch.cuda.synchronize()
    finally:
        gc.callbacks.remove(cb)
        gc.set_threshold(*old)
    assert not started, started
    assert len(impl._workspace(B)._graphs) == 1
    gc.collect()  # the cycles are collectable outside the capture
    torch.cuda.synchronize()
