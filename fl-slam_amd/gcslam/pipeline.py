"""Batched per-scan driver: the reference's per-hypothesis loop, hypothesis combine and IW
apply (backend_node.py:2036-2119, pipeline.py:316-1621) as one device-resident pipeline over
this rank's shard of hypotheses (C-ABI gc_pipeline_*, include/gcslam.h).

Host code only stages inputs, launches ``run_scan`` and reads results back; every arithmetic
step runs in libgcslam on the GPU. With ``world_size > 1`` the per-scan exchange is one RCCL
all-gather of a fixed-layout partial record followed by a rank-ordered reduction, so every
rank ends the scan with a bit-identical combined belief, IW state and map.
"""

from __future__ import annotations

import ctypes as C
import weakref
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _abi
from .constants import (FORGETTING_FACTOR, GC_ALPHA_MAX, GC_ALPHA_MIN, GC_B_BINS, GC_C0_COND, GC_C_FROB,
                        GC_EPS_LIFT, GC_EPS_MASS, GC_EPS_PSD, GC_MAX_IMU_PREINT_LEN, GC_OU_DAMPING_LAMBDA,
                        GC_PLANAR_VZ_SIGMA, GC_PLANAR_Z_REF, GC_PLANAR_Z_SIGMA, GC_TAU_SOFT_ASSIGN, POWER_BETA_EXC_C, POWER_BETA_MIN, POWER_BETA_Z_C, T_BASE_LIDAR)
from .ops.binning import create_fibonacci_atlas


def shard(H_total: int, rank: int, world: int):
    """Contiguous hypothesis shard [h0, h1) of one rank."""
    return (H_total * rank) // world, (H_total * (rank + 1)) // world


@dataclass
class PipelineConfig:
    n_points_cap: int = 65536
    n_bins: int = GC_B_BINS
    imu_len: int = GC_MAX_IMU_PREINT_LEN
    tau: float = GC_TAU_SOFT_ASSIGN
    lidar_origin: tuple = tuple(T_BASE_LIDAR[:3])
    eps_psd: float = GC_EPS_PSD
    eps_lift: float = GC_EPS_LIFT
    eps_mass: float = GC_EPS_MASS
    lambda_ou: float = GC_OU_DAMPING_LAMBDA
    c_frob: float = GC_C_FROB
    forgetting_factor: float = FORGETTING_FACTOR
    weight_floor: Optional[float] = None  # default 0.01 / H (docs/GC_SLAM.md:122)
    power_beta_min: float = POWER_BETA_MIN
    power_beta_exc_c: float = POWER_BETA_EXC_C
    power_beta_z_c: float = POWER_BETA_Z_C
    alpha_min: float = GC_ALPHA_MIN
    alpha_max: float = GC_ALPHA_MAX
    c0_cond: float = GC_C0_COND
    nu_max: float = 1000.0
    planar_z_ref: float = GC_PLANAR_Z_REF
    planar_z_sigma: float = GC_PLANAR_Z_SIGMA
    planar_vz_sigma: float = GC_PLANAR_VZ_SIGMA
    imu_gravity_scale: float = 1.0

    def as_array(self, H_total: int) -> np.ndarray:
        floor = 0.01 / H_total if self.weight_floor is None else self.weight_floor
        return np.array([self.tau, *self.lidar_origin, self.eps_psd, self.eps_lift, self.eps_mass,
                         self.lambda_ou, self.c_frob, self.forgetting_factor, floor, self.power_beta_min,
                         self.power_beta_exc_c, self.power_beta_z_c, self.alpha_min, self.alpha_max,
                         self.c0_cond, self.nu_max, self.planar_z_ref, self.planar_z_sigma,
                         self.planar_vz_sigma, self.imu_gravity_scale], dtype=np.float64)


def _p(a):
    return a.ctypes.data if a is not None else None


def _f(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None and a.shape != tuple(shape):
        a = a.reshape(shape)
    return a


class BatchedScanPipeline:
    """One rank's device-resident hypothesis shard."""

    def __init__(self, H_total: int, n_in_max: int, cfg: PipelineConfig = None, rank: int = 0,
                 world_size: int = 1, ctx: _abi.Context = None, geometry_hyps: int = 0):
        """geometry_hyps > 0 sizes the bins launch's chunks as for a shard of that many hypotheses
        (e.g. H_total on every rank: per-hypothesis results then do not depend on world_size)."""
        self.cfg = cfg or PipelineConfig()
        self.ctx = ctx or _abi.default_context()
        self.H = H_total
        self.h0, self.h1 = shard(H_total, rank, world_size)
        self.Hl = self.h1 - self.h0
        self.B = self.cfg.n_bins
        self.M = self.cfg.imu_len
        self.rank, self.world = rank, world_size
        d = _abi.PipelineDims(H_total, self.h0, self.Hl, self.B, self.M, world_size, rank, int(geometry_hyps),
                              int(n_in_max), int(self.cfg.n_points_cap))
        cfgv = self.cfg.as_array(H_total)
        h = C.c_void_p()
        _abi.call("gc_pipeline_create", self.ctx.handle, C.addressof(d), cfgv.ctypes.data, C.byref(h), ctx=self.ctx)
        self.handle = h.value
        self._comm = None
        self._smap = None
        self.io_computed = True  # GC_IO_COMPUTED is the device default
        self.set_bins(create_fibonacci_atlas(self.B).dirs)
        self.set_weights(np.full(H_total, 1.0 / H_total))

    # ---------------------------------------------------------------- state in / out
    def _call(self, name, *args):
        _abi.call(name, self.handle, *args, ctx=self.ctx)

    def set_bins(self, bins):
        self._call("gc_pipeline_set_bins", _p(_f(bins, (self.B, 3))))

    def set_weights(self, w):
        self._call("gc_pipeline_set_weights", _p(_f(w, (self.H,))))

    def set_beliefs(self, X, z, L, h, stamp=None):
        """Local shard arrays: X (Hl,6), z (Hl,22), L (Hl,22,22), h (Hl,22), stamp (Hl,)."""
        stamp = np.zeros(self.Hl) if stamp is None else stamp
        self._call("gc_pipeline_set_beliefs", _p(_f(X, (self.Hl, 6))), _p(_f(z, (self.Hl, 22))),
                   _p(_f(L, (self.Hl, 22, 22))), _p(_f(h, (self.Hl, 22))), _p(_f(stamp, (self.Hl,))))

    def get_beliefs(self):
        X, z, L, h, st = (np.empty(s) for s in ((self.Hl, 6), (self.Hl, 22), (self.Hl, 22, 22), (self.Hl, 22),
                                                 (self.Hl,)))
        self._call("gc_pipeline_get_beliefs", _p(X), _p(z), _p(L), _p(h), _p(st))
        return dict(X_anchor=X, z_lin=z, L=L, h=h, stamp=st)

    def set_io_evidence(self, L, h, cert):
        """Given (synthetic) IMU/odom-branch evidence; selects GC_IO_GIVEN."""
        self._call("gc_pipeline_set_io_evidence", _p(_f(L, (self.Hl, 22, 22))), _p(_f(h, (self.Hl, 22))),
                   _p(_f(cert, (self.Hl, _abi.GC_IO_CERT))))
        self.io_computed = False

    def set_io_mode(self, computed: bool):
        self._call("gc_pipeline_set_io_mode", _abi.GC_IO_COMPUTED if computed else _abi.GC_IO_GIVEN)
        self.io_computed = bool(computed)

    def io_evidence(self):
        """(L_io (Hl,22,22), h_io (Hl,22), cert (Hl,10)) of the last scan."""
        L, h, c = np.empty((self.Hl, 22, 22)), np.empty((self.Hl, 22)), np.empty((self.Hl, _abi.GC_IO_CERT))
        self._call("gc_pipeline_get_io_evidence", _p(L), _p(h), _p(c))
        return L, h, c

    def io_parts(self):
        """(Hl, GC_IO_PARTS) IMU/odom-branch internals of the last scan (include/gcslam.h)."""
        o = np.empty((self.Hl, _abi.GC_IO_PARTS))
        self._call("gc_pipeline_get_io_parts", _p(o))
        return o

    def set_iw(self, nu_proc, Psi_proc, nu_meas, Psi_meas):
        self._call("gc_pipeline_set_iw", _p(_f(nu_proc, (7,))), _p(_f(Psi_proc, (7, 6, 6))),
                   _p(_f(nu_meas, (3,))), _p(_f(Psi_meas, (3, 3, 3))))

    def get_iw(self):
        out = [np.empty(s) for s in ((7,), (7, 6, 6), (3,), (3, 3, 3), (22, 22), (4,))]
        self._call("gc_pipeline_get_iw", *[_p(o) for o in out])
        return dict(nu_proc=out[0], Psi_proc=out[1], nu_meas=out[2], Psi_meas=out[3], Q=out[4], cert=out[5])

    def set_map(self, map_rec):
        self._call("gc_pipeline_set_map", _p(_f(map_rec, (self.B, _abi.GC_MAP_REC))))

    def get_map(self):
        m, d, x = np.empty((self.B, _abi.GC_MAP_REC)), np.empty((self.B, _abi.GC_MAP_DER)), np.empty(2)
        self._call("gc_pipeline_get_map", _p(m), _p(d), _p(x))
        return dict(map=m, derived=d, z_scale=x[0], N_dir_total=x[1])

    # ---------------------------------------------------------------- scans
    def stage_scan(self, slot: int, scan: dict):
        P = _f(scan["points"])
        n = P.shape[0]
        self._call("gc_pipeline_stage_scan", int(slot), _p(P), _p(_f(scan["timestamps"], (n,))),
                   _p(_f(scan["weights"], (n,))), n, _p(_f(scan["imu_stamps"], (self.M,))),
                   _p(_f(scan["imu_gyro"], (self.M, 3))), _p(_f(scan["imu_accel"], (self.M, 3))))
        if "odom_pose" in scan:  # odometry for the on-device IMU/odom branch (GC_IO_COMPUTED)
            self._call("gc_pipeline_stage_odom", int(slot), _p(_f(scan["odom_pose"], (6,))),
                       _p(_f(scan["odom_cov"], (6, 6))), _p(_f(scan["odom_twist"], (6,))),
                       _p(_f(scan["odom_twist_cov"], (6, 6))))

    def stage_pointcloud2(self, slot: int, msg, imu: dict, R_base_lidar, t_base_lidar):
        """Stage a slot from a PointCloud2 message (raw bytes parsed on the device,
        backend_node.py:377-468 + :1677-1690) and the slot's IMU window (imu_stamps, imu_gyro,
        imu_accel arrays of M rows)."""
        from .ops.pointcloud import field_table, header_stamp_sec
        n = int(msg.width) * int(msg.height)
        ft = field_table(msg) if n > 0 else np.full(10, -1, np.int32)
        raw = np.frombuffer(bytes(msg.data), dtype=np.uint8) if n > 0 else np.zeros(1, np.uint8)
        Ra, Rp = _abi.f64p(np.asarray(R_base_lidar, np.float64).reshape(9))
        ta, tp = _abi.f64p(np.asarray(t_base_lidar, np.float64).reshape(3))
        self._call("gc_pipeline_stage_pointcloud2", int(slot), raw.ctypes.data, n, int(msg.point_step), ft.ctypes.data,
                   header_stamp_sec(msg), Rp, tp, _p(_f(imu["imu_stamps"], (self.M,))),
                   _p(_f(imu["imu_gyro"], (self.M, 3))), _p(_f(imu["imu_accel"], (self.M, 3))))
        if "odom_pose" in imu:
            self._call("gc_pipeline_stage_odom", int(slot), _p(_f(imu["odom_pose"], (6,))),
                       _p(_f(imu["odom_cov"], (6, 6))), _p(_f(imu["odom_twist"], (6,))),
                       _p(_f(imu["odom_twist_cov"], (6, 6))))

    def run_scan(self, slot: int, scan: dict, scan_count: int):
        self._call("gc_pipeline_run_scan", int(slot), float(scan["scan_start"]), float(scan["scan_end"]),
                   float(scan["t_last"]), float(scan["t_scan"]), float(scan["dt_sec"]), int(scan_count))
        if self._smap is not None:
            self._map_updated()

    def run_scan_local(self, slot: int, scan: dict, scan_count: int):
        """a1-a15 for this rank's hypotheses and its partial record; finish with finish_scan."""
        self._call("gc_pipeline_scan_local", int(slot), float(scan["scan_start"]), float(scan["scan_end"]),
                   float(scan["t_last"]), float(scan["t_scan"]), float(scan["dt_sec"]), int(scan_count))

    def partial(self) -> np.ndarray:
        """This rank's partial record of the pending scan (RECORD layout, partial_len(B) doubles)."""
        o = np.empty(partial_len(self.B))
        self._call("gc_pipeline_get_partial", _p(o))
        return o

    def finish_scan(self, gathered: Optional[np.ndarray] = None):
        """Exchange + combine of the pending scan. gathered: (world_size, partial_len) records in
        rank order (any transport), or None for the RCCL all-gather / the single-rank record."""
        g = None if gathered is None else _f(gathered, (self.world, partial_len(self.B)))
        self._call("gc_pipeline_scan_finish", _p(g))
        if self._smap is not None:
            self._map_updated()

    def combined(self):
        o = np.empty(_abi.GC_COMB_LEN)
        self._call("gc_pipeline_get_combined", _p(o))
        c = o[528 + 6:]
        return dict(L=o[:484].reshape(22, 22), h=o[484:506], z_lin=o[506:528], X_anchor=o[528:534],
                    stamp=c[0], psd_delta=c[1], eig_min=c[2], eig_max=c[3], cond=c[4], near_null=c[5],
                    ess=c[6], support_frac=c[7], mass_eps_ratio=c[8], floor_adjustment=c[9], spread=c[10])

    def hyp_diag(self):
        o = np.empty((self.Hl, _abi.GC_HYP_DIAG))
        self._call("gc_pipeline_get_hyp_diag", _p(o))
        return o

    def set_predict_route(self, factorised: bool) -> None:
        """a2 predict route: the split route (default; predicted moments solved from Σ' directly, L_pred
        formed beside the bins) or the factorised chain in the predict kernel (include/gcslam.h)."""
        self._call("gc_pipeline_set_predict_route", 1 if factorised else 0)

    def set_inscan_certs(self, on: bool = True) -> None:
        """Compute the per-hypothesis predict / fusion ConditioningCerts inside every later scan
        (right after its evidence kernel), as the reference emits them on every call."""
        self._call("gc_pipeline_set_inscan_certs", 1 if on else 0)

    def hyp_conditioning(self):
        """(Hl, 2, 4): the ConditioningCert [eig_min, eig_max, cond, near_null_count] of each
        hypothesis's predict (L_pred, predict.py:183-188) and fusion (L_post, fusion.py:150-230)
        PSD projections of the last scan (computed inside the scan with set_inscan_certs, else on
        demand, off the scan path)."""
        o = np.empty((self.Hl, 2, 4))
        self._call("gc_pipeline_get_hyp_conditioning", _p(o))
        return o

    def projection_certs(self):
        """The reference's cert_vec [projection_delta, sym_delta, eig_min, eig_max, cond,
        near_null_count] (primitives.py:80-123) of the last scan's other PSD projections:
        hyp (Hl, B + 2, 6) = per hypothesis the B bins' Σ_p (binning.py:175-187), the MF L_rot and
        the planar L_trans (matrix_fisher_evidence.py:330, :609); scan (12, 6) = the barycenter L
        (hypothesis.py:99), the 7 process-IW blocks, the 3 measurement-IW blocks and Q
        (inverse_wishart_jax.py:67,168; measurement_noise_iw_jax.py:82). Computed inside the scan with
        set_inscan_certs, else on demand from the last scan's stored operands."""
        hyp, scan = np.empty((self.Hl, self.B + 2, 6)), np.empty((_abi.GC_PCERT_SCAN, 6))
        self._call("gc_pipeline_get_projection_certs", _p(hyp), _p(scan))
        return dict(bins=hyp[:, :self.B], mf=hyp[:, self.B], planar=hyp[:, self.B + 1],
                    barycenter=scan[_abi.GC_PCERT_BARY], iw_proc=scan[_abi.GC_PCERT_PROC0:_abi.GC_PCERT_MEAS0],
                    iw_meas=scan[_abi.GC_PCERT_MEAS0:_abi.GC_PCERT_Q], Q=scan[_abi.GC_PCERT_Q])

    def lpose6(self):
        """L_evidence[pose, pose] per hypothesis of the last scan (Hl, 6, 6)."""
        o = np.empty((self.Hl, 6, 6))
        self._call("gc_pipeline_get_lpose6", _p(o))
        return o

    def bin_stats(self):
        s, c, x = np.empty((self.Hl, self.B, 38)), np.empty((self.Hl, 8)), np.empty((self.Hl, 6))
        self._call("gc_pipeline_get_bin_stats", _p(s), _p(c), _p(x))
        return s, c, x

    def hyp_stats(self):
        """Per-hypothesis process-IW dPsi (Hl,7,6,6), measurement-IW dPsi (Hl,3,3,3) and belief
        covariance Σ = (L + ε_lift I)⁻¹ (Hl,22,22) of the last scan."""
        a, b, c = np.empty((self.Hl, 7, 6, 6)), np.empty((self.Hl, 3, 3, 3)), np.empty((self.Hl, 22, 22))
        self._call("gc_pipeline_get_hyp_stats", _p(a), _p(b), _p(c))
        return a, b, c

    # ---------------------------------------------------------------- C5 in-scan map update
    def attach_primitive_map(self, dmap, voxel_m: float = 0.1):
        """Fuse every scan into a device-resident PrimitiveMap (gcslam.primitive_map.DevicePrimitiveMap)
        in scan_finish: the budgeted points deskewed with hypothesis 0's twist, pushed to the world
        frame by its recomposed pose with pose-covariance inflation, one row per point into the slot
        of its voxel (build-defined, include/gcslam.h). dmap=None detaches."""
        self._call("gc_pipeline_attach_primitive_map", None if dmap is None else C.addressof(dmap.struct()),
                   float(voxel_m))
        self._smap = dmap  # the device arrays must outlive the attachment
        if dmap is not None:
            dmap._listeners.append(weakref.ref(self))

    def set_scan_map_mode(self, replicated: bool):
        """Which ranks run the in-scan map update: False (the default, GC_SMAP_OWNER) only the rank
        holding hypothesis 0, as the reference lets hypothesis 0 alone write the map
        (backend_node.py:2081-2083), so the other ranks' attached maps stay untouched; True
        (GC_SMAP_REPLICATED) every rank, each keeping a bit-identical replica."""
        self._call("gc_pipeline_set_scan_map_mode", 1 if replicated else 0)
        self._smap_replicated = bool(replicated)

    def scan_map_owner(self) -> bool:
        """This rank runs the in-scan map update (it holds hypothesis 0, or the mode is replicated)."""
        return self.h0 == 0 or getattr(self, "_smap_replicated", False)

    def _map_colors_stale(self):
        """The attached map's colour fields were written by a host operation (DevicePrimitiveMap
        .colors_stale): the next in-scan update recomputes every slot's colour estimate."""
        self._call("gc_pipeline_map_colors_stale")

    def _map_updated(self):
        """After a scan_finish with a map attached the map's colours are the fuse's estimate on every
        slot (the update's colour pass ran if they were stale; LiDAR rows keep them otherwise)."""
        m = getattr(self, "_smap", None)
        if m is not None and "cam_mass" in m.ptrs and self.scan_map_owner():
            m._tile_cc = [True] * m.n_tiles

    def scan_map_pose(self):
        """(z_t (6), Σ_pose (6,6), ξ_body (6)) of hypothesis 0 that the last scan's map update used."""
        o = np.empty(H0_LEN)
        self._call("gc_pipeline_get_scan_map_pose", _p(o))
        return o[0:6], o[6:42].reshape(6, 6), o[42:48]

    def scan_map_count(self) -> int:
        """Distinct map slots the last in-scan update touched."""
        n = C.c_int64(0)
        self._call("gc_pipeline_get_scan_map_count", C.byref(n))
        return int(n.value)

    # ---------------------------------------------------------------- multi-GPU
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (C.c_uint8 * _abi.GC_COMM_ID_BYTES)()
        _abi.check(_abi.lib().gc_comm_unique_id(C.addressof(buf)))
        return bytes(buf)

    def attach_comm(self, uid: bytes):
        buf = (C.c_uint8 * _abi.GC_COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        _abi.call("gc_comm_init", self.ctx.handle, self.world, self.rank, C.addressof(buf), C.byref(h), ctx=self.ctx)
        self._comm = h.value
        self._call("gc_pipeline_attach_comm", self._comm)

    def comm_size(self) -> int:
        """Size of the attached RCCL communicator (0 without one)."""
        return int(_abi.lib().gc_pipeline_comm_size(self.handle))

    def set_exchange_timing(self, on: bool = True) -> None:
        """Bracket every later scan's exchange with HIP events (off by default: each event between
        kernels costs the stream a few microseconds)."""
        self._call("gc_pipeline_set_exchange_timing", 1 if on else 0)

    def exchange_ms(self) -> float:
        """Device time of the last timed scan's exchange (all-gather or host-record upload), in ms."""
        ms = C.c_float(0.0)
        self._call("gc_pipeline_exchange_ms", C.byref(ms))
        return float(ms.value)

    # ---------------------------------------------------------------- observability
    def set_stage_timing(self, on: bool = True) -> None:
        """Record HIP events around every launch group of later scans (off by default: each event
        between kernels costs the stream ~1-5 us)."""
        self._call("gc_pipeline_set_stage_timing", 1 if on else 0)

    def stage_ms(self) -> dict:
        """Device time (ms) of each stage of the last scan finished with stage timing on
        (_abi.GC_STAGE_NAMES: predict, bins, evidence, combine_local, exchange, combine_final,
        map_update, total)."""
        o = (C.c_float * _abi.GC_STAGE_N)()
        self._call("gc_pipeline_stage_ms", C.addressof(o))
        return {f"{k}_ms": float(v) for k, v in zip(_abi.GC_STAGE_NAMES, o)}

    def host_stats(self, reset: bool = False) -> dict:
        """Host-side accounting (include/gcslam.h GC_HS_*): per-scan enqueue work vs waits on the
        device, staging work vs waits, host syncs, host<->device bytes."""
        o = np.zeros(_abi.GC_HOST_STATS)
        self._call("gc_pipeline_host_stats", _p(o), 1 if reset else 0)
        return {k: float(v) for k, v in zip(_abi.GC_HS_NAMES, o)}

    def device_runtime_cert(self, consume: bool = True):
        """DeviceRuntimeCert of the work since the last consume (backend_node.py:2182-2190 with
        consume_runtime_counters, common/runtime_counters.py:94-108): this pipeline's host syncs and
        host<->device bytes; jit_recompile_count is 0 (ahead-of-time compiled library)."""
        from .certificates import DeviceRuntimeCert
        h = self.host_stats(reset=consume)
        return DeviceRuntimeCert(host_sync_count_est=int(h["host_syncs"]),
                                 device_to_host_bytes_est=int(h["d2h_bytes"]),
                                 host_to_device_bytes_est=int(h["h2d_bytes"]),
                                 jit_recompile_count=int(h["jit_recompiles"]))

    def close(self):
        if getattr(self, "handle", None):
            _abi.lib().gc_pipeline_destroy(self.handle)
            self.handle = None
        if self._comm:
            _abi.lib().gc_comm_destroy(self._comm)
            self._comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def map_record(S_dir, S_dir_scatter, N_dir, N_pos, sum_p, sum_ppT) -> np.ndarray:
    """MapBinStats (archive/bin_atlas.py:79-98) -> (B, 26) device record layout."""
    B = np.asarray(N_dir).shape[0]
    return np.concatenate([np.asarray(S_dir).reshape(B, 3), np.asarray(S_dir_scatter).reshape(B, 9),
                           np.asarray(N_dir).reshape(B, 1), np.asarray(N_pos).reshape(B, 1),
                           np.asarray(sum_p).reshape(B, 3), np.asarray(sum_ppT).reshape(B, 9)], axis=1)


def iw_process_prior():
    """create_datasheet_process_noise_state (structures/inverse_wishart_jax.py:43-80):
    ν = p + 1.5, Ψ = Σ_prior · 0.5 on each padded 6x6 block (init-time constants)."""
    dims = np.array([3, 3, 3, 3, 3, 1, 6])
    diag = np.array([1e-4, 8.7e-7, 9.5e-5, 1e-8, 1e-6, 1e-6, 1e-8])
    Psi = np.zeros((7, 6, 6))
    for i in range(7):
        Psi[i, :dims[i], :dims[i]] = np.eye(dims[i]) * diag[i] * 0.5
    return dims + 1.5, Psi


def iw_meas_prior(lidar_sigma: float = 0.01):
    """create_datasheet_measurement_noise_state (structures/measurement_noise_iw_jax.py:37-68)."""
    return np.full(3, 4.5), np.stack([8.7e-7 * np.eye(3), 9.5e-5 * np.eye(3), lidar_sigma * np.eye(3)]) * 0.5


# Layout of the per-rank partial record exchanged once per scan (csrc/gc_pipe.h kP*).
RECORD = dict(L=(0, 484), h=(484, 506), z=(506, 528), mu=(528, 550), mu2=(550, 551), dPsiP=(551, 803),
              dnuP=(803, 810), dPsiM=(810, 837), dnuM=(837, 840), X0=(841, 847), stamp0=(847, 848))
MAP_INC0 = 848  # (B, 26) hypothesis 0's map increments, then its pose block (H0_LEN)
H0_LEN = 48     # [z_t 6, Σ_post pose block 36, ξ_body 6] of hypothesis 0 (in-scan PrimitiveMap update)


def record_h0(B: int) -> int:
    """Offset of hypothesis 0's pose block in the partial record."""
    return MAP_INC0 + 26 * B


def partial_len(B: int) -> int:
    return record_h0(B) + H0_LEN
