"""The reference node's per-scan loop over the per-operator drop-ins (backend_node.py:2036-2119 with the
legacy bin-path wiring of pipeline.py:316-1591): what ``gc_backend_node`` runs when it
keeps its own hypothesis loop and swaps ``fl_slam_poc.backend.operators`` for ``gcslam.ops``
(INTEGRATION.md §2). Every operator is one libgcslam entry; the point arrays of a hypothesis (budgeted,
deskewed, directions) and its N x B responsibilities stay in HBM between operators (``device_out``,
as the reference's jnp arrays stay on the JAX device after the one upload of backend_node.py:1679-1690),
and every device buffer comes from the context's arena (include/gcslam.h gc_buffer_alloc), so a steady
scan performs no hipMalloc / hipFree. Only the operators' certificate scalars and the 22-D beliefs cross
to the host, as in the reference's wrappers (float(...) of each cert, e.g. point_budget.py:185-200).

The host code here is the node's own glue: the 22-D embedding of the LiDAR evidence, the certificate
aggregation and power tempering (pipeline.py:1038-1117), the total trigger magnitude (pipeline.py:1211)
and the weighted IW accumulation (backend_node.py:2085-2090). The IMU/odom branch evidence is given per
hypothesis (as the batched pipeline's GC_IO_GIVEN mode); the bin map is held fixed."""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import _abi
from . import ops
from .ops import se3 as _se3
from .ops.imu_preintegration import imu_meas_iw_suffstats_batch
from .belief import BeliefGaussianInfo
from .constants import (D_Z, GC_ALPHA_MAX, GC_ALPHA_MIN, GC_CHART_ID, GC_EPS_MASS, GC_GRAVITY_W,
                        GC_TAU_SOFT_ASSIGN, POWER_BETA_EXC_C, POWER_BETA_MIN, POWER_BETA_Z_C, T_BASE_LIDAR)


@dataclass
class IOGiven:
    """One hypothesis's IMU/odom-branch evidence (pipeline.py:595-776): L, h and its certificate row
    [ess odom/imu/gyro, support odom/imu/gyro, exc_dt, exc_ex, nll, trigger] (include/gcslam.h GC_IO_CERT)."""
    L: np.ndarray
    h: np.ndarray
    cert: np.ndarray


@dataclass
class BinMap:
    """MapBinStats and its derived statistics (archive/bin_atlas.py:137-224) as the record / derived
    arrays of the batched pipeline (include/gcslam.h: map (B, 26), derived (B, 17))."""
    record: np.ndarray
    derived: np.ndarray

    @property
    def S_dir(self):
        return self.record[:, 0:3]

    @property
    def S_dir_scatter(self):
        return self.record[:, 3:12].reshape(-1, 3, 3)

    @property
    def N_dir(self):
        return self.record[:, 12]

    @property
    def N_pos(self):
        return self.record[:, 13]

    @property
    def centroid(self):
        return self.derived[:, 4:7]

    @property
    def Sigma_c(self):
        return self.derived[:, 7:16].reshape(-1, 3, 3)


def tempering_beta(L_raw, ess_total: float, exc_total: float):
    """Power tempering from the raw-evidence sentinels (pipeline.py:1070-1111)."""
    eps = GC_EPS_MASS
    dpose = float(np.linalg.norm(L_raw[15, 0:6]) + np.linalg.norm(L_raw[0:6, 15]))
    dvel = float(np.linalg.norm(L_raw[15, 6:9]) + np.linalg.norm(L_raw[6:9, 15]))
    dt_asym = min(max(abs(dvel - dpose) / (dvel + dpose + eps), 0.0), 1.0)
    z_xy = abs(L_raw[2, 2]) / (0.5 * (abs(L_raw[0, 0]) + abs(L_raw[1, 1])) + eps)
    e2x = ess_total / (exc_total + eps)
    s = min(max(dt_asym * (z_xy / (z_xy + POWER_BETA_Z_C)) * (1.0 / (1.0 + e2x / POWER_BETA_EXC_C)), 0.0), 1.0)
    return min(max(POWER_BETA_MIN + (1.0 - POWER_BETA_MIN) * s, POWER_BETA_MIN), 1.0), dt_asym, z_xy


def imu_dt_mean(stamps) -> float:
    """Average IMU period over the valid (stamp > 0) samples (pipeline.py:526-535)."""
    v = np.sort(np.asarray(stamps)[np.asarray(stamps) > 0.0])
    return max(float((v[-1] - v[0]) / max(v.shape[0] - 1, 1)), 1e-12) if v.shape[0] >= 2 else 1e-12


class DropinNode:
    """K hypotheses stepped through the per-operator drop-ins, one scan at a time."""

    def __init__(self, beliefs: List[BeliefGaussianInfo], weights, bins, bin_map: BinMap, Q, pn_state, mn_state,
                 n_points_cap: int, tau: float = GC_TAU_SOFT_ASSIGN, weight_floor: Optional[float] = None, ctx=None):
        self.ctx = ctx or _abi.default_context()
        self.beliefs = list(beliefs)
        self.weights = np.asarray(weights, np.float64)
        self.bins = np.asarray(bins, np.float64)
        self.map = bin_map
        self.Q = np.asarray(Q, np.float64)
        self.pn, self.mn = pn_state, mn_state
        self.cap = int(n_points_cap)
        self.tau = float(tau)
        self.floor = 0.01 / len(beliefs) if weight_floor is None else float(weight_floor)
        self.origin = np.asarray(T_BASE_LIDAR[:3], np.float64)
        self.scan_count = 0
        self.combined = None

    def hypothesis(self, b_prev: BeliefGaussianInfo, scan, dev, io: IOGiven):
        """process_scan_single_hypothesis with the legacy bin path (pipeline.py:316-1591)."""
        ctx, o = self.ctx, self.origin
        bud, c_bud, _ = ops.point_budget_resample(dev["points"], dev["timestamps"], dev["weights"], None, None,
                                                  self.cap, ctx=ctx, device_out=True)
        bpred, c_pred, _ = ops.predict_diffusion(b_prev, self.Q, scan["dt_sec"], ctx=ctx)
        Sig_pred, _ = ops.spd_cholesky_inverse_lifted(bpred.L, ctx=ctx)
        sigma_warp = max(math.sqrt(Sig_pred[15, 15]), 0.01)
        st = scan["imu_stamps"]
        w_scan = ops.smooth_window_weights(st, scan["scan_start"], scan["scan_end"], sigma_warp, ctx=ctx)
        w_int = ops.smooth_window_weights(st, scan["t_last"], scan["t_scan"], sigma_warp, ctx=ctx)
        mu_inc = bpred.mean_increment(ctx=ctx)
        bg, ba = mu_inc[9:12], mu_inc[12:15]
        pose0 = b_prev.world_pose(ctx=ctx)
        pre = ops.preintegrate_imu_relative_pose_jax(st, scan["imu_gyro"], scan["imu_accel"], w_scan, pose0[3:6], bg,
                                                     ba, GC_GRAVITY_W, ctx=ctx)
        xi = _se3.se3_log(pre[0], ctx=ctx)
        ess_imu = float(pre[4])
        # measurement-noise IW statistics of the scan-to-scan window (pipeline.py:525-566)
        dt_imu = imu_dt_mean(st)
        wv = w_int * (st > 0.0)
        wnv = wv / (np.sum(wv) + GC_EPS_MASS)
        omega_avg = wnv @ (scan["imu_gyro"] - bg[None, :])
        # imu_gyro_meas_iw_suffstats_from_avg_rate_jax and imu_accel_meas_iw_suffstats_from_gravity_dir_jax
        # (measurement_noise_iw_jax.py:131-218) share the window: both from one launch
        dPsi_meas = np.zeros((3, 3, 3))
        dPsi_meas[0:2] = imu_meas_iw_suffstats_batch(scan["imu_gyro"], scan["imu_accel"], wv, bg, ba, omega_avg,
                                                     pose0[3:6], dt_imu, ctx=ctx)[0]
        # a4 -> a6 on the device-resident point arrays
        dsk, c_dsk, _ = ops.deskew_constant_twist(bud.points, bud.timestamps, bud.weights, scan["scan_start"],
                                                  scan["scan_end"], xi, ess_imu, GC_CHART_ID, b_prev.anchor_id,
                                                  ctx=ctx, device_out=True)
        dirs = ops.point_directions(dsk.points, o, ctx=ctx, device_out=True)
        sa, c_sa, _ = ops.bin_soft_assign(dirs, self.bins, self.tau, ctx=ctx, device_out=True)
        mm, c_mm, _ = ops.scan_bin_moment_match(dsk.points, None, dsk.weights, sa.responsibilities, None, o, ctx=ctx)
        m = self.map
        mf, c_mf, _ = ops.matrix_fisher_rotation_evidence(bpred, mm.s_dir, mm.S_dir_scatter, mm.N, m.S_dir,
                                                          m.S_dir_scatter, m.N_dir, ctx=ctx)
        tr, c_tr, _ = ops.planar_translation_evidence(bpred, mm.p_bar, mm.Sigma_p, mm.N, m.centroid, m.Sigma_c,
                                                      m.N_pos, m.S_dir_scatter, m.N_dir, mf.R_mf, ctx=ctx)
        # 22-D evidence, certificate aggregation, tempering (pipeline.py:1038-1117; matrix_fisher_evidence.py:729-756)
        L_raw, h_raw = io.L.copy(), io.h.copy()
        L_raw[0:3, 0:3] += tr.L_trans; h_raw[0:3] += tr.h_trans
        L_raw[3:6, 3:6] += mf.L_rot; h_raw[3:6] += mf.h_rot
        ic = io.cert
        retained = c_dsk.support.support_frac
        ess_ev = (ess_imu + c_sa.support.ess_total + c_mm.support.ess_total + 0.0 + 0.0) / 5.0
        ess_tot = (ess_ev + ic[0] + ic[1] + ic[2]) / 4.0
        exc = max(0.0, ic[6]) + max(0.0, ic[7])
        beta, _, _ = tempering_beta(L_raw, ess_tot, exc)
        L_ev, h_ev = beta * L_raw, beta * h_raw
        s_dt, s_ex = ops.compute_excitation_scales_jax(L_ev, bpred.L, ctx=ctx)
        Lps, hps = ops.apply_excitation_prior_scaling_jax(bpred.L, bpred.h, s_dt, s_ex, ctx=ctx)
        if GC_ALPHA_MIN != GC_ALPHA_MAX:
            raise NotImplementedError("the drop-in node runs at the reference constants α_min = α_max")
        alpha = GC_ALPHA_MIN
        prior = BeliefGaussianInfo(GC_CHART_ID, bpred.anchor_id, bpred.X_anchor, bpred.stamp_sec, bpred.z_lin, Lps,
                                   hps)
        post, c_fus, _ = ops.info_fusion_additive(prior, L_ev, h_ev, alpha, anchor_id=bpred.anchor_id, ctx=ctx)
        # total trigger magnitude of every certificate on the path (pipeline.py:1211)
        T = (c_bud.total_trigger_magnitude() + c_pred.total_trigger_magnitude() + ic[9] + 0.0
             + c_sa.total_trigger_magnitude() + c_mm.total_trigger_magnitude() + c_mf.total_trigger_magnitude()
             + c_tr.total_trigger_magnitude() + abs(1.0 - beta) + abs(s_dt) + abs(s_ex) + abs(1.0 - alpha)
             + c_fus.influence.psd_projection_delta + abs(1.0 - alpha))
        _, b_rec, _, _ = ops.pose_update_frobenius_recompose(post, T, ctx=ctx)
        dPsi_p, dnu_p = ops.process_noise_iw_suffstats_from_info_jax(Lps, hps, b_rec.L, b_rec.h, ctx=ctx)
        _, b_fin, _, _ = ops.anchor_drift_update(b_rec, ctx=ctx)
        return dict(belief=b_fin, dPsi_proc=dPsi_p, dnu_proc=dnu_p, dPsi_meas=dPsi_meas, T=T, beta=beta, xi=xi)

    def process_scan(self, scan, ios: List[IOGiven]):
        """One LiDAR scan for all K hypotheses (backend_node.py:2036-2119): the scan is uploaded once,
        every hypothesis runs the operator chain, then the barycenter and the IW applies."""
        ctx = self.ctx
        n = scan["points"].shape[0]
        dev = dict(points=_abi.DeviceArray.from_host(ctx, scan["points"]),
                   timestamps=_abi.DeviceArray.from_host(ctx, scan["timestamps"]),
                   weights=_abi.DeviceArray.from_host(ctx, scan["weights"]))
        assert dev["points"].shape == (n, 3)
        res = [self.hypothesis(b, scan, dev, io) for b, io in zip(self.beliefs, ios)]
        w = self.weights
        aP = sum(w[i] * r["dPsi_proc"] for i, r in enumerate(res))
        an = sum(w[i] * r["dnu_proc"] for i, r in enumerate(res))
        aM = sum(w[i] * r["dPsi_meas"] for i, r in enumerate(res))
        self.beliefs = [r["belief"] for r in res]
        K = len(self.beliefs)
        self.combined, _, _ = ops.hypothesis_barycenter_projection(self.beliefs, w, K, self.floor, ctx=ctx)
        wp = float(min(1, self.scan_count))
        self.pn, _ = ops.process_noise_iw_apply_suffstats_jax(self.pn, wp * aP, wp * an, ctx=ctx)
        self.mn, _ = ops.measurement_noise_apply_suffstats_jax(self.mn, aM, w.sum() * np.array([1.0, 1.0, 0.0]),
                                                               ctx=ctx)
        self.Q = ops.process_noise_state_to_Q_jax(self.pn, ctx=ctx)
        self.scan_count += 1
        return res
