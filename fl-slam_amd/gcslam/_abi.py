"""ctypes binding of libgcslam (include/gcslam.h).

The library is loaded from this package directory (built in-tree by ``make`` in
``fl-slam_amd/``). There is no fallback: if the shared object is missing or no GPU is
visible, the first call raises — the product path never computes on the CPU.
"""

from __future__ import annotations

import ctypes as C
import math
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgcslam.so")

GC_OK, GC_ERR_ARG, GC_ERR_RUNTIME = 0, 1, 2
GC_BIN_STATS = 38
GC_BIN_CERT = 8
GC_FUSED_TAU_MIN = 3e-3

_vp, _dp, _i32, _i64, _u64, _f64 = C.c_void_p, C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_double
_dptr = C.POINTER(C.c_double)

# name -> argtypes (restype int32 unless noted). Device pointers travel as c_void_p.
SIGNATURES = {
    "gc_version": [],
    "gc_device_count": [C.POINTER(C.c_int32)],
    "gc_ctx_create": [_i32, C.POINTER(_vp)],
    "gc_ctx_destroy": [_vp],
    "gc_ctx_synchronize": [_vp],
    "gc_ctx_set_wait_timeout": [_vp, _f64],
    "gc_test_bounded_wait": [_f64, _i64, _dptr],
    "gc_test_device_spin": [_vp, _f64],
    "gc_test_radix_sort": [_vp, _vp, _vp, _i64, _i64, _i32, _vp, _vp],
    "gc_buffer_alloc": [_vp, _u64, C.POINTER(_vp)],
    "gc_buffer_free": [_vp, _vp],
    "gc_ctx_trim": [_vp],
    "gc_ctx_alloc_stats": [_vp, _vp],
    "gc_buffer_upload": [_vp, _vp, _vp, _u64],
    "gc_buffer_download": [_vp, _vp, _vp, _u64],
    "gc_buffer_copy": [_vp, _vp, _vp, _u64],
    "gc_buffer_memset": [_vp, _vp, _i32, _u64],
    "gc_event_create": [_vp, C.POINTER(_vp)],
    "gc_event_destroy": [_vp],
    "gc_event_record": [_vp, _vp],
    "gc_event_elapsed_ms": [_vp, _vp, C.POINTER(C.c_float)],
    "gc_point_budget_resample": [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "gc_budget_stats": [_vp, _vp, _i64, _i64, _vp],
    "gc_deskew_constant_twist": [_vp, _i32, _i64, _vp, _vp, _vp, _f64, _f64, _vp, _vp, _vp, _vp],
    "gc_point_directions": [_vp, _i64, _vp, _dptr, _f64, _vp],
    "gc_bin_soft_assign": [_vp, _i32, _i64, _i32, _vp, _vp, _f64, _vp, _vp, _vp],
    "gc_scan_bin_moment_match": [_vp, _i32, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _dptr, _f64, _f64, _vp, _vp],
    "gc_scan_bins_fused": [_vp, _i32, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _f64, _f64, _vp, _vp, _f64, _dptr,
                           _f64, _f64, _vp, _vp, _i32],
    "gc_kappa_from_resultant_batch": [_vp, _i64, _vp, _f64, _f64, _f64, _f64, _vp],
    "gc_domain_projection_psd_batch": [_vp, _i32, _i32, _vp, _f64, _vp, _vp],
    "gc_pipeline_create": [_vp, _vp, _vp, C.POINTER(_vp)],
    "gc_pipeline_destroy": [_vp],
    "gc_pipeline_set_bins": [_vp, _vp],
    "gc_pipeline_set_beliefs": [_vp, _vp, _vp, _vp, _vp, _vp],
    "gc_pipeline_get_beliefs": [_vp, _vp, _vp, _vp, _vp, _vp],
    "gc_pipeline_set_weights": [_vp, _vp],
    "gc_pipeline_set_io_evidence": [_vp, _vp, _vp, _vp],
    "gc_pipeline_set_io_mode": [_vp, _i32],
    "gc_pipeline_stage_odom": [_vp, _i32, _vp, _vp, _vp, _vp],
    "gc_pipeline_get_io_parts": [_vp, _vp],
    "gc_pipeline_get_io_evidence": [_vp, _vp, _vp, _vp],
    "gc_io_factor_batch": [_vp, _i32, _i32, _vp, _vp],
    "gc_imu_vmf_gravity_tr_batch": [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _dptr, _f64, _f64, _f64, _vp],
    "gc_pipeline_set_iw": [_vp, _vp, _vp, _vp, _vp],
    "gc_pipeline_get_iw": [_vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "gc_pipeline_set_map": [_vp, _vp],
    "gc_pipeline_get_map": [_vp, _vp, _vp, _vp],
    "gc_pipeline_stage_scan": [_vp, _i32, _vp, _vp, _vp, _i64, _vp, _vp, _vp],
    "gc_pointcloud2_parse": [_vp, _vp, _i64, _i32, _vp, _f64, _dptr, _dptr, _vp, _vp, _vp, _vp, _vp],
    "gc_pipeline_stage_pointcloud2": [_vp, _i32, _vp, _i64, _i32, _vp, _f64, _dptr, _dptr, _vp, _vp, _vp],
    "gc_pipeline_run_scan": [_vp, _i32, _f64, _f64, _f64, _f64, _f64, _i64],
    "gc_pipeline_scan_local": [_vp, _i32, _f64, _f64, _f64, _f64, _f64, _i64],
    "gc_pipeline_partial_len": [_vp],
    "gc_pipeline_get_partial": [_vp, _vp],
    "gc_pipeline_scan_finish": [_vp, _vp],
    "gc_pipeline_get_combined": [_vp, _vp],
    "gc_pipeline_get_hyp_diag": [_vp, _vp],
    "gc_pipeline_get_hyp_conditioning": [_vp, _vp],
    "gc_pipeline_get_projection_certs": [_vp, _vp, _vp],
    "gc_pipeline_get_lpose6": [_vp, _vp],
    "gc_pipeline_get_bin_stats": [_vp, _vp, _vp, _vp],
    "gc_pipeline_get_hyp_stats": [_vp, _vp, _vp, _vp],
    "gc_pipeline_attach_comm": [_vp, _vp],
    "gc_pipeline_comm_size": [_vp],
    "gc_pipeline_attach_primitive_map": [_vp, _vp, _f64],
    "gc_pipeline_get_scan_map_pose": [_vp, _vp],
    "gc_pipeline_map_colors_stale": [_vp],
    "gc_pipeline_get_scan_map_count": [_vp, C.POINTER(C.c_int64)],
    "gc_pipeline_set_scan_map_mode": [_vp, _i32],
    "gc_pipeline_set_exchange_timing": [_vp, _i32],
    "gc_pipeline_exchange_ms": [_vp, C.POINTER(C.c_float)],
    "gc_pipeline_set_stage_timing": [_vp, _i32],
    "gc_pipeline_stage_ms": [_vp, _vp],
    "gc_pipeline_host_stats": [_vp, _vp, _i32],
    "gc_pipeline_set_inscan_certs": [_vp, _i32],
    "gc_pipeline_set_predict_route": [_vp, _i32],
    "gc_comm_unique_id": [_vp],
    "gc_comm_init": [_vp, _i32, _i32, _vp, C.POINTER(_vp)],
    "gc_comm_destroy": [_vp],
    "gc_comm_abort": [_vp],
    "gc_comm_healthy": [_vp, C.POINTER(C.c_int32)],
    "gc_comm_allgather_f64": [_vp, _vp, _vp, _vp, _i64],
    "gc_lie_batch": [_vp, _i32, _i64, _vp, _vp],
    "gc_belief_world_pose_batch": [_vp, _i32, _vp, _vp, _vp, _f64, _vp, _vp],
    "gc_spd_inverse_lifted_batch": [_vp, _i32, _i32, _vp, _f64, _vp],
    "gc_predict_diffusion_batch": [_vp, _i32, _vp, _vp, _vp, _f64, _f64, _f64, _f64, _vp, _vp, _vp],
    "gc_smooth_window_weights": [_vp, _i32, _vp, _f64, _f64, _f64, _vp],
    "gc_preintegrate_imu_batch": [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _dptr, _vp],
    "gc_imu_meas_iw_suffstats_batch": [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f64, _f64, _f64, _vp],
    "gc_matrix_fisher_batch": [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f64, _f64, _vp],
    "gc_planar_translation_batch": [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f64, _f64,
                                    _vp],
    "gc_excitation_scaling_batch": [_vp, _i32, _vp, _vp, _vp, _f64, _vp, _vp, _vp],
    "gc_fusion_scale_batch": [_vp, _i32, _vp, _f64, _f64, _f64, _f64, _vp],
    "gc_info_fusion_additive_batch": [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _f64, _vp, _vp, _vp],
    "gc_recompose_batch": [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _f64, _f64, _vp, _vp, _vp, _vp],
    "gc_anchor_drift_batch": [_vp, _i32, _vp, _vp, _vp, _vp, _f64, _vp, _vp, _vp, _vp],
    "gc_iw_process_suffstats_batch": [_vp, _i32, _vp, _vp, _vp, _vp, _f64, _vp, _vp],
    "gc_iw_process_apply": [_vp, _vp, _vp, _vp, _vp, _f64, _f64, _vp, _vp, _vp],
    "gc_iw_process_Q": [_vp, _vp, _vp, _f64, _vp],
    "gc_iw_meas_apply": [_vp, _vp, _vp, _vp, _vp, _f64, _f64, _vp, _vp, _vp],
    "gc_hypothesis_barycenter": [_vp, _i32, _vp, _vp, _vp, _vp, _f64, _f64, _f64, _vp, _vp, _vp, _vp],
    "gc_primitive_map_fuse": [_vp, _vp, _vp, _vp, _f64, _f64, _f64, _i64, _vp],
    "gc_primitive_map_record_layout": [_i32, _vp, _vp],
    "gc_copy_strided": [_vp, _vp, _i64, _vp, _i64, _i64, _i64],
    "gc_primitive_map_forget": [_vp, _vp, _i64, _i64, _f64],
    "gc_primitive_map_recency_inflate": [_vp, _vp, _i64, _i64, _i64, _f64, _f64, _vp],
    "gc_primitive_map_cull": [_vp, _vp, _i64, _i64, _f64, _i64, _vp],
    "gc_primitive_map_insert_masked": [_vp, _vp, _i64, _i64, _vp, _f64, _i64, _f64, _i64, _vp, _vp, _vp],
    "gc_primitive_map_merge_reduce": [_vp, _vp, _i64, _i64, _f64, _i32, _f64, _f64, _vp],
    "gc_extract_map_view": [_vp, _vp, _i64, _vp, _vp, _f64, _f64, _vp],
    "gc_associate_primitives_ot": [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp],
}

GC_PCFG_LEN = 22
GC_PIPE_MAX_SLOTS = 8
GC_MAP_REC = 26
GC_MAP_DER = 17
GC_IO_CERT = 10
GC_IO_PARTS = 40
GC_IO_GIVEN, GC_IO_COMPUTED = 0, 1
GC_IOF_IN = 64
GC_IOF_OUT = 484 + 22 + 16
(GC_IOF_ODOM_QUADRATIC, GC_IOF_IMU_GYRO_ROTATION, GC_IOF_IMU_PREINT_FACTOR, GC_IOF_PLANAR_Z_PRIOR,
 GC_IOF_VELOCITY_Z_PRIOR, GC_IOF_ODOM_VELOCITY, GC_IOF_ODOM_YAWRATE, GC_IOF_KINEMATIC, GC_IOF_IMU_DEPENDENCE,
 GC_IOF_ODOM_DEPENDENCE) = range(10)
GC_HYP_DIAG = 40
GC_STAGE_N = 8
GC_STAGE_NAMES = ("predict", "bins", "evidence", "combine_local", "exchange", "combine_final", "map_update", "total")
GC_HOST_STATS = 16
GC_HS_NAMES = ("scans", "scan_enqueue_ms", "scan_enqueue_max_ms", "scan_wait_ms", "scan_wait_max_ms", "stages",
               "stage_work_ms", "stage_work_max_ms", "stage_wait_ms", "stage_wait_max_ms", "host_syncs", "h2d_bytes",
               "d2h_bytes", "jit_recompiles")
GC_COMB_LEN = 484 + 22 + 22 + 6 + 16
# gc_pipeline_get_projection_certs layout (include/gcslam.h GC_PCERT_*)
GC_PCERT_SCAN = 12
GC_PCERT_BARY, GC_PCERT_PROC0, GC_PCERT_MEAS0, GC_PCERT_Q = 0, 1, 8, 11
GC_COMM_ID_BYTES = 128
GC_PRED_CERT = 8
GC_PREINT_OUT = 32
GC_MF_OUT = 66
GC_PT_OUT = 26
GC_RECOMPOSE_OUT = 19
GC_DRIFT_OUT = 3
GC_FUSION_ROW = 8
GC_FUSION_OUT = 4
GC_BARY_CERT = 16


class PipelineDims(C.Structure):
    _fields_ = [("H_total", C.c_int32), ("h_begin", C.c_int32), ("h_count", C.c_int32), ("B", C.c_int32),
                ("M", C.c_int32), ("world_size", C.c_int32), ("rank", C.c_int32), ("geom_hyps", C.c_int32),
                ("n_in_max", C.c_int64), ("n_cap", C.c_int64)]

_lib = None
_lock = threading.Lock()


def lib():
    """Load libgcslam.so (once). Raises RuntimeError if it has not been built."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(f"libgcslam.so not found at {LIB_PATH}: build it with "
                                       "`make -C fl-slam_amd` (there is no CPU fallback)")
                L = C.CDLL(LIB_PATH)
                for name, argt in SIGNATURES.items():
                    fn = getattr(L, name)
                    fn.argtypes = argt
                    fn.restype = C.c_int32
                L.gc_last_error.argtypes = [_vp]
                L.gc_last_error.restype = C.c_char_p
                _lib = L
    return _lib


def check(rc: int, ctx=None):
    if rc == GC_OK:
        return
    msg = lib().gc_last_error(ctx.handle if ctx is not None else None)
    msg = msg.decode() if msg else "unknown error"
    if rc == GC_ERR_ARG:
        raise ValueError(msg)
    raise RuntimeError(msg)


_fns = {}


def call(name: str, *args, ctx=None):
    f = _fns.get(name)
    if f is None:
        f = _fns[name] = getattr(lib(), name)
    rc = f(*args)
    if rc != GC_OK:
        check(rc, ctx)


def device_count() -> int:
    n = C.c_int32(0)
    rc = lib().gc_device_count(C.byref(n))
    return int(n.value) if rc == GC_OK else 0


class Context:
    """A HIP device + stream (gc_ctx). One per calling thread (see include/gcslam.h)."""

    def __init__(self, device: int = 0):
        h = _vp()
        check(lib().gc_ctx_create(int(device), C.byref(h)))
        self.handle = h.value
        self.device = device

    def sync(self):
        check(lib().gc_ctx_synchronize(self.handle), self)

    def alloc_stats(self) -> dict:
        """The device-buffer arena's counters (include/gcslam.h gc_ctx_alloc_stats)."""
        out = np.zeros(6, np.int64)
        check(lib().gc_ctx_alloc_stats(self.handle, out.ctypes.data), self)
        return dict(zip(("hip_mallocs", "hip_frees", "reuses", "live", "live_bytes", "cached_bytes"),
                        (int(v) for v in out)))

    def trim(self):
        """Return the arena's cached blocks to HIP."""
        check(lib().gc_ctx_trim(self.handle), self)

    def set_wait_timeout(self, seconds: float):
        """Bound of every host wait on this context (fail fast; include/gcslam.h gc_ctx_synchronize)."""
        check(lib().gc_ctx_set_wait_timeout(self.handle, float(seconds)), self)

    def close(self):
        if self.handle:
            lib().gc_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceArray:
    """A device allocation (the context's arena, include/gcslam.h gc_buffer_alloc) with a NumPy
    dtype/shape view. The device-resident drop-ins accept one wherever an array goes and return one
    with device_out=True, so a chain of operators keeps its point arrays and responsibilities in HBM
    (as the reference's jnp arrays stay on the JAX device, backend_node.py:1679-1690);
    np.asarray(d) downloads it."""

    def __init__(self, ctx: Context, shape, dtype=np.float64, _base=None, _ptr=None):
        self.ctx = ctx
        self.shape = tuple(map(int, shape)) if isinstance(shape, (tuple, list)) else (int(shape),)
        self.dtype = dtype if isinstance(dtype, np.dtype) else np.dtype(dtype)
        self.nbytes = math.prod(self.shape) * self.dtype.itemsize
        self._base = _base  # a view keeps its base alive and never frees
        if _ptr is not None:
            self.ptr = _ptr
            return
        p = _vp()
        rc = lib().gc_buffer_alloc(ctx.handle, max(self.nbytes, 16), C.byref(p))
        if rc != GC_OK:
            check(rc, ctx)
        self.ptr = p.value

    def view(self, shape, offset_elems: int = 0) -> "DeviceArray":
        """A non-owning view of (part of) this buffer with another shape (no copy)."""
        shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list)) else (shape,)))
        nb = math.prod(shape) * self.dtype.itemsize
        if offset_elems < 0 or offset_elems * self.dtype.itemsize + nb > self.nbytes:
            raise ValueError(f"view {shape} at {offset_elems} exceeds the buffer {self.shape}")
        return DeviceArray(self.ctx, shape, self.dtype, _base=self, _ptr=self.ptr + offset_elems * self.dtype.itemsize)

    @property
    def ndim(self) -> int:
        return len(self.shape)

    def __len__(self):
        return self.shape[0]

    def __array__(self, dtype=None, copy=None):
        a = self.download()
        return a if dtype is None else a.astype(dtype)

    @classmethod
    def from_host(cls, ctx: Context, arr, dtype=np.float64):
        a = np.ascontiguousarray(arr, dtype=dtype)
        d = cls(ctx, a.shape, a.dtype)
        d.upload(a)
        return d

    def upload(self, arr):
        a = np.ascontiguousarray(arr, dtype=self.dtype)
        if a.nbytes != self.nbytes:
            raise ValueError(f"upload size mismatch: {a.nbytes} vs {self.nbytes}")
        check(lib().gc_buffer_upload(self.ctx.handle, self.ptr, a.ctypes.data, a.nbytes), self.ctx)

    def download(self) -> np.ndarray:
        out = np.empty(self.shape, dtype=self.dtype)
        check(lib().gc_buffer_download(self.ctx.handle, out.ctypes.data, self.ptr, self.nbytes), self.ctx)
        return out

    def zero(self):
        check(lib().gc_buffer_memset(self.ctx.handle, self.ptr, 0, self.nbytes), self.ctx)

    def free(self):
        if self.ptr and self._base is None and self.ctx.handle:
            lib().gc_buffer_free(self.ctx.handle, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Event:
    def __init__(self, ctx: Context):
        h = _vp()
        check(lib().gc_event_create(ctx.handle, C.byref(h)), ctx)
        self.handle, self.ctx = h.value, ctx

    def record(self):
        check(lib().gc_event_record(self.ctx.handle, self.handle), self.ctx)

    def elapsed_ms(self, later: "Event") -> float:
        ms = C.c_float(0.0)
        check(lib().gc_event_elapsed_ms(self.handle, later.handle, C.byref(ms)), self.ctx)
        return float(ms.value)

    def __del__(self):
        try:
            lib().gc_event_destroy(self.handle)
        except Exception:
            pass


def device_input(ctx: Context, x, dtype=np.float64, shape=None) -> DeviceArray:
    """x as a device array of dtype (and shape, if given): a DeviceArray is used in place (a reshaped
    view when only the shape differs), anything else is uploaded into an arena buffer."""
    if isinstance(x, DeviceArray):
        if x.dtype != np.dtype(dtype):
            raise ValueError(f"device array of dtype {x.dtype}, expected {np.dtype(dtype)}")
        if shape is not None and tuple(shape) != x.shape:
            if math.prod(shape) != math.prod(x.shape):
                raise ValueError(f"device array of shape {x.shape}, expected {tuple(shape)}")
            return x.view(shape)
        return x
    a = np.ascontiguousarray(x, dtype=dtype)
    if shape is not None:
        a = a.reshape(shape)
    return DeviceArray.from_host(ctx, a, dtype)


def host(x):
    """A host NumPy view of x (downloads a DeviceArray)."""
    return x.download() if isinstance(x, DeviceArray) else np.asarray(x)


_PACK_ALIGN = 256


def _packed_offsets(nbytes):
    offs, tot = [], 0
    for nb in nbytes:
        offs.append(tot)
        tot += -(-max(int(nb), 1) // _PACK_ALIGN) * _PACK_ALIGN
    return offs, tot


def alloc_many(ctx: Context, specs):
    """Several device arrays as views of ONE arena block (one gc_buffer_alloc): specs = [(shape, dtype)
    or shape]. download_many of the views is then one copy and one wait."""
    specs = [s if (isinstance(s, tuple) and len(s) == 2 and isinstance(s[1], (type, np.dtype))) else (s, np.float64)
             for s in specs]
    shapes = [tuple(int(v) for v in (sh if isinstance(sh, (tuple, list)) else (sh,))) for sh, _ in specs]
    dts = [np.dtype(dt) for _, dt in specs]
    nbytes = [math.prod(sh) * dt.itemsize for sh, dt in zip(shapes, dts)]
    offs, tot = _packed_offsets(nbytes)
    base = DeviceArray(ctx, tot, np.uint8)
    return [DeviceArray(ctx, sh, dt, _base=base, _ptr=base.ptr + o) for sh, dt, o in zip(shapes, dts, offs)]


def upload_many(ctx: Context, arrays, dtype=np.float64):
    """Host arrays (or DeviceArrays, used in place) as device arrays: every host array is packed into
    one host buffer and one arena block, so an operator's small operands cost one upload (staged, no
    wait: gc_buffer_upload) instead of one each. dtype: one dtype for all, or a list."""
    dts = dtype if isinstance(dtype, (list, tuple)) else [dtype] * len(arrays)
    out = [None] * len(arrays)
    host_idx, host_arr = [], []
    for i, (x, dt) in enumerate(zip(arrays, dts)):
        if isinstance(x, DeviceArray):
            out[i] = device_input(ctx, x, dt)
        else:
            host_idx.append(i)
            host_arr.append(np.ascontiguousarray(x, dtype=dt))
    if host_arr:
        offs, tot = _packed_offsets([a.nbytes for a in host_arr])
        buf = np.empty(tot, np.uint8)
        for a, o in zip(host_arr, offs):
            buf[o:o + a.nbytes] = a.reshape(-1).view(np.uint8)
        base = DeviceArray(ctx, tot, np.uint8)
        base.upload(buf)
        for i, a, o in zip(host_idx, host_arr, offs):
            out[i] = DeviceArray(ctx, a.shape, a.dtype, _base=base, _ptr=base.ptr + o)
    return out


def download_many(arrays):
    """Host copies of device arrays; views of one block (alloc_many) come back with one download."""
    if not arrays:
        return []
    b0 = arrays[0]._base
    if b0 is not None and all(a._base is b0 for a in arrays):
        raw = b0.download()
        out = []
        for a in arrays:
            o = a.ptr - b0.ptr
            out.append(raw[o:o + a.nbytes].view(a.dtype).reshape(a.shape))
        return out
    return [a.download() for a in arrays]


_tls = threading.local()


def default_context() -> Context:
    """Per-thread context on GCSLAM_DEVICE (default 0)."""
    c = getattr(_tls, "ctx", None)
    if c is None:
        c = Context(int(os.environ.get("GCSLAM_DEVICE", "0")))
        _tls.ctx = c
    return c


def f64p(vals):
    """Host double[] for small by-value vector arguments (e.g. h_origin3)."""
    a = np.ascontiguousarray(vals, dtype=np.float64)
    return a, a.ctypes.data_as(_dptr)
