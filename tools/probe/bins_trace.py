"""Dev probe (GPU box): per-workgroup timing of the last k_bins_io launch after a short bench run with
a GC_BINS_TIMING build (tools/variant.sh btime gc_points -DGC_BINS_TIMING).
Usage: python3 tools/probe/bins_trace.py <libgcslam.so> <H>"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))
sys.path.insert(0, ROOT)
from gcslam import _abi  # noqa: E402

_abi.LIB_PATH = os.path.abspath(sys.argv[1])
H = sys.argv[2]
sys.argv = ["bench.py", "--hyps", H, "--no-cpu", "--no-roofline", "--no-map", "--no-c5", "--no-extras",
            "--steps", "20", "--warmup", "5"]
import bench  # noqa: E402

bench.main()
L = _abi.lib()
n = 2048
buf = (C.c_double * (4 * n))()
L.gc_dev_bins_trace.argtypes = [C.POINTER(C.c_double), C.c_int64]
assert L.gc_dev_bins_trace(buf, n) == 0
a = np.array(buf).reshape(n, 4)
a = a[a[:, 2] > 0]
t0 = a[:, 0].min()
us = (a[:, :3] - t0) / 100.0  # 100 MHz ticks -> us
io = a[:, 3] < 0
pu = ~io
print(f"H={H}: {io.sum()} branch workgroups, {pu.sum()} pullers; launch span {us[:, 2].max():.1f} us")
if io.any():
    print(f"  branch: start {us[io, 0].min():.1f}-{us[io, 0].max():.1f}, end {us[io, 2].min():.1f}-{us[io, 2].max():.1f} us")
s, p, e, nt = us[pu, 0], us[pu, 1] - us[pu, 0], us[pu, 2], a[pu, 3]
print(f"  pullers: start {s.min():.1f} / median {np.median(s):.1f} / max {s.max():.1f} us")
print(f"  prologue: mean {p.mean():.2f} max {p.max():.2f} us")
print(f"  end: min {e.min():.1f} / p10 {np.percentile(e, 10):.1f} / median {np.median(e):.1f} / max {e.max():.1f} us")
print(f"  tasks per puller: min {nt.min():.0f} mean {nt.mean():.2f} max {nt.max():.0f}; total {nt.sum():.0f}")
late = s > np.percentile(s, 50) + 5
print(f"  pullers starting > 5 us after the median start: {late.sum()} (their start {s[late].min() if late.any() else 0:.1f}..)")
busy = (e - us[pu, 1]).sum()
span = e.max() - s.min()
print(f"  puller occupancy: busy (after prologue) {busy:.0f} WG-us of {pu.sum() * span:.0f} ({busy / (pu.sum() * span):.3f})")

# per task [start, end, puller, XCD] (t = chunk * H + hypothesis)
m = 16384
tb = (C.c_double * (4 * m))()
L.gc_dev_task_trace.argtypes = [C.POINTER(C.c_double), C.c_int64]
assert L.gc_dev_task_trace(tb, m) == 0
tk = np.array(tb).reshape(m, 4)
nT = int((tk[:, 1] > 0).sum())
tk = tk[:nT]
Hn = int(H)
st, en = (tk[:, 0] - t0) / 100.0, (tk[:, 1] - t0) / 100.0
du = en - st
ch = np.arange(nT) // Hn
print(f"  tasks {nT}, chunks {ch.max() + 1}")
for c in range(ch.max() + 1):
    sel = ch == c
    print(f"   chunk {c:3d}: dur median {np.median(du[sel]):6.1f} p90 {np.percentile(du[sel], 90):6.1f} max {du[sel].max():6.1f}"
          f"  start {st[sel].min():7.1f}-{st[sel].max():7.1f}  end max {en[sel].max():7.1f}")
xcc = tk[:, 3].astype(int)
print("  per XCD median task dur (last chunk):", [round(float(np.median(du[(xcc == x) & (ch == ch.max())])), 1) if ((xcc == x) & (ch == ch.max())).any() else None for x in range(8)])
print("  per XCD tasks:", [int((xcc == x).sum()) for x in range(8)])
last = np.argsort(en)[-12:]
for i in last:
    print(f"   late task {i}: chunk {ch[i]} start {st[i]:.1f} end {en[i]:.1f} dur {du[i]:.1f} puller {int(tk[i, 2])} xcc {xcc[i]}")

# per task [end of its first iteration, start of its epilogue] (wave 0 of the workgroup), when the build
# exports them: the task's set-up + first iteration, its other iterations, and its epilogue (record
# reduction + the next task's ticket / operands) up to the next task's start
if hasattr(L, "gc_dev_task_ep_trace"):
    eb = (C.c_double * (2 * m))()
    L.gc_dev_task_ep_trace.argtypes = [C.POINTER(C.c_double), C.c_int64]
    assert L.gc_dev_task_ep_trace(eb, m) == 0
    ep = (np.array(eb).reshape(m, 2)[:nT] - t0) / 100.0
    first, rest, epi = ep[:, 0] - st, ep[:, 1] - ep[:, 0], en - ep[:, 1]
    for c in range(ch.max() + 1):
        sel = ch == c
        print(f"   chunk {c:3d}: first iteration (+ set-up) {np.median(first[sel]):6.2f}  later iterations {np.median(rest[sel]):7.2f}"
              f"  epilogue {np.median(epi[sel]):5.2f} us (medians)")
    print(f"  all tasks: epilogue median {np.median(epi):.2f} p90 {np.percentile(epi, 90):.2f} us; first iteration median "
          f"{np.median(first):.2f} us")
# per task and wave: the end of the wave's iterations — the waves' skew at the epilogue's first barrier, and
# the epilogue proper (the last wave's arrival to the task's end)
if hasattr(L, "gc_dev_task_wv_trace"):
    wb = (C.c_double * (4 * m))()
    L.gc_dev_task_wv_trace.argtypes = [C.POINTER(C.c_double), C.c_int64]
    assert L.gc_dev_task_wv_trace(wb, m) == 0
    wvt = (np.array(wb).reshape(m, 4)[:nT] - t0) / 100.0
    skew = wvt.max(axis=1) - wvt.min(axis=1)
    proper = en - wvt.max(axis=1)
    for c in range(ch.max() + 1):
        sel = ch == c
        print(f"   chunk {c:3d}: wave skew median {np.median(skew[sel]):5.2f} p90 {np.percentile(skew[sel], 90):5.2f}"
              f"  epilogue after the last wave {np.median(proper[sel]):5.2f} us")
    print(f"  all tasks: wave skew median {np.median(skew):.2f} p90 {np.percentile(skew, 90):.2f}; epilogue proper median "
          f"{np.median(proper):.2f} p90 {np.percentile(proper, 90):.2f} us")
