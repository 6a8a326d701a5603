"""Dev probe (GPU box, round 6): can two ranks of one RCCL communicator share the one GPU of the box?
Two spawned processes, each a libgcslam context on device 0; rank 0 makes the unique id and passes it
through a queue; both gc_comm_init(2, r) and all-gather 1000 doubles (gc_comm_allgather_f64). Every
wait is bounded (gc_ctx_set_wait_timeout 20 s); the parent gives each rank 90 s. Prints what each rank
saw (RCCL may refuse two ranks on one device: ncclInvalidUsage)."""
import ctypes as C
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rank_main(r, q_id, q_out):
    sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))
    import numpy as np
    from gcslam import _abi
    from gcslam.pipeline import BatchedScanPipeline
    try:
        ctx = _abi.Context(0)
        ctx.set_wait_timeout(20.0)
        if r == 0:
            uid = BatchedScanPipeline.comm_unique_id()
            q_id.put(uid)
            q_id.put(uid)
        else:
            uid = None
        uid = q_id.get(timeout=60) if r == 1 else uid
        buf = (C.c_uint8 * _abi.GC_COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        _abi.call("gc_comm_init", ctx.handle, 2, r, C.addressof(buf), C.byref(h), ctx=ctx)
        x = np.arange(1000, dtype=np.float64) + 1000.0 * r
        ds, dr = _abi.DeviceArray.from_host(ctx, x), _abi.DeviceArray(ctx, 2000)
        _abi.call("gc_comm_allgather_f64", ctx.handle, h.value, ds.ptr, dr.ptr, 1000, ctx=ctx)
        ctx.sync()
        got = dr.download()
        ok = bool(np.array_equal(got, np.arange(2000, dtype=np.float64)))
        _abi.lib().gc_comm_destroy(h.value)
        q_out.put((r, "allgather ok" if ok else "allgather WRONG"))
    except Exception as e:  # the probe's answer
        q_out.put((r, "%s: %s" % (type(e).__name__, str(e)[:300])))


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    q_id, q_out = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, q_id, q_out)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=90)
    for p in ps:
        if p.is_alive():
            p.kill()
            print("rank still running after 90 s: killed")
    res = []
    while not q_out.empty():
        res.append(q_out.get())
    for r, msg in sorted(res):
        print("rank", r, ":", msg)
    print("exit codes", [p.exitcode for p in ps])
