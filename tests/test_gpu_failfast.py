"""Bounded host waits on the device (fail fast): a stream kept busy longer than the context's wait
bound makes gc_ctx_synchronize return GC_ERR_RUNTIME (RuntimeError) at the bound, and the context is
usable again once the work drains (the spin kernel exits by itself)."""

import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))

pytestmark = pytest.mark.gpu


def test_ctx_sync_times_out_then_recovers():
    from gcslam import _abi
    ctx = _abi.Context(0)
    ctx.sync()
    ctx.set_wait_timeout(0.3)
    _abi.call("gc_test_device_spin", ctx.handle, 2.0, ctx=ctx)
    t0 = time.perf_counter()
    with pytest.raises(RuntimeError, match="timed out after"):
        ctx.sync()
    dt = time.perf_counter() - t0
    assert 0.3 <= dt < 1.5, dt
    ctx.set_wait_timeout(30.0)
    ctx.sync()  # the kernel has drained: the stream is clean
    _abi.call("gc_test_device_spin", ctx.handle, 0.01, ctx=ctx)
    ctx.sync()
    ctx.close()
