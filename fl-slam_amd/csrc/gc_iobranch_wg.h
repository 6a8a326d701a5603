// gc_iobranch_wg.h — one hypothesis of the IMU/odom evidence branch (_compute_imu_odom_branch,
// backend/pipeline.py:595-776) as a 256-thread workgroup body. The batched pipeline runs these
// workgroups inside the fused bins launch (k_bins_io, gc_points.hip), beside the bin workgroups, so
// the branch needs no stream fork / join of its own. Device code of the factors: gc_iofactors.h.
#pragma once
#include <hip/hip_runtime.h>
#include "gc_pipe.h"
#include "gc_iofactors.h"
#include "gc_opsdev.h"

namespace gc {

constexpr int kIoN2 = kDZ * kDZ;
constexpr int kNFac = 9;  // odom, imu, gyro, preint, planar, vz, odom_vel, odom_wz, kinematic

// LDS (doubles): one union region U, first the preintegration scratch A, Bm (256 x 9 each), V1, V2
// (256 x 3) and the vMF weights, then (once those are dead) the factor L/h blocks (9 x 506); sort
// scratch 1024 | red 8 | misc 64 | extras 9 x 16. 7384 doubles = 59 KB, under the fused bins
// workgroup's 66.5 KB, so a merged launch keeps two bin workgroups per CU.
constexpr int kIoU = (256 * 24 > kNFac * (kIoN2 + kDZ)) ? 256 * 24 : kNFac * (kIoN2 + kDZ);
constexpr int kIoLdsDoubles = kIoU + 1024 + 8 + 64 + kNFac * kIofExtra;

// The predict's L_pred half (predict.py:43-98 after its first projection), for hypothesis hl, in the
// bins launch beside the bin tasks: the predict kernel certified Σ'_psd = Σ'_sym and formed the
// predicted moments without L_pred (gc_belief.hip, pred_mode 0); here L_pred = PSD((Σ'_sym + ε_l I)⁻¹),
// h_pred = L_pred μ and the predict certificate, by the routines and in the order of wg_predict's
// certified path (wg_psd_fast_lifted_chol's lifted factor, wg_chol_inverse, the projection of L'),
// so every value is the one the unsplit predict wrote. Only k_evidence reads them. pred_mode 1 (the
// predict ran the whole chain itself): nothing to do. LDS: kLpredLdsDoubles.
constexpr int kLpredLdsDoubles = 6 * kIoN2 + 4 * kDZ + 2 * kDZ + 8 + 8 + 4 * (kDZ + 2);
GC_DEV void pose_pred_lane(const PipeDev& P, int hl) {
  // pose_pred = X ⊞ μ_inc (for the IMU/odom branch, MF and planar; the predict kernel's bins need only
  // ξ_body): one lane, beside lpred_wg's loads and factorization (read after its barriers)
  double e[6], pp[6];
  se3_exp(P.mu_aux + (int64_t)hl * kMuAux + 22, e);
  se3_compose(P.X + (int64_t)hl * 6, e, pp);
  for (int k = 0; k < 6; ++k) P.pose_pred[(int64_t)hl * 6 + k] = pp[k];
}
GC_DEV void lpred_wg(const PipeDev& P, const ScanArgs& S, int hl, double* sm) {
  if (P.pred_mode[hl] != 0.0) {
    if (threadIdx.x == 192) pose_pred_lane(P, hl);
    __syncthreads();
    return;
  }
  constexpr int n = kDZ, N2 = kIoN2;
  double* W2 = sm;             // Σ', then L' raw
  double* Cl = W2 + N2;        // chol(Σ'_sym + ε_l I)
  double* Ws = Cl + N2;        // inverse scratch
  double* Lo = Ws + N2;        // Σ'_psd, then L_pred
  double* Sx = Lo + N2;        // 2 N2 + 4n (projection scratch)
  double* mu = Sx + 2 * N2 + 4 * n;
  double* ho = mu + n;
  double* red = ho + n;        // 8
  double* c2 = red + 8;        // 6 (+2)
  double* cb = c2 + 8;         // 4 x (kDZ + 2): lane_chol's broadcast rows (no static LDS in k_bins_io)
  const int t = threadIdx.x;
  const PredictPrefill pf = predict_prefill_load(P.Sig + (int64_t)hl * N2, P.Q, P.mu_fin + (int64_t)hl * n);
  predict_prefill_store(pf, S.dt, P.lambda_ou, W2, mu);
  __syncthreads();
  for (int idx = t; idx < N2; idx += kWG) {
    const int i = idx / n, j = idx % n;
    const double sym = 0.5 * (W2[i * n + j] + W2[j * n + i]);
    Lo[idx] = sym;
    Cl[idx] = sym + ((i == j) ? P.eps_lift : 0.0);
  }
  __syncthreads();
  const double trace_cov = wg_sum(t < n ? Lo[t * n + t] : 0.0, red);
  if (t == 192) pose_pred_lane(P, hl);  // wave 3, beside wave 0's factorization
  wg_chol<true>(Cl, n, cb);
  wg_chol_inverse(Cl, W2, Ws, n);  // L' raw
  wg_psd_project_fast<NoSideWork, true>(W2, Lo, P.eps_psd, n, Sx, red, c2, NoSideWork(), cb);
  wg_matvec(Lo, mu, ho, n);
  for (int i = t; i < N2; i += kWG) P.Lpred[(int64_t)hl * N2 + i] = Lo[i];
  if (t < n) P.hpred[(int64_t)hl * n + t] = ho[t];
  if (t == 0) {
    double* cert = P.pred_cert + (int64_t)hl * kPredCert;
    const double lift = 2.0 * P.eps_lift * n;
    const double psd = 0.0 + c2[0];  // the first projection's delta is 0 (certified)
    cert[0] = lift; cert[1] = psd; cert[2] = c2[2]; cert[3] = c2[3]; cert[4] = c2[4]; cert[5] = c2[5];
    cert[6] = trace_cov;
    cert[7] = lift + psd + fabs(1.0 - S.dt);
  }
  __syncthreads();
}

GC_DEV void io_branch_wg(const PipeDev& P, const ScanArgs& S, const double* __restrict__ odom, int hl, double* sm) {
  double* FL = sm;                          // factor k: L at FL + k*(N2+22), h after it (after the vMF)
  double* A = sm;                           // preint scratch (aliases FL: dead before FL is zeroed)
  double* Bm = A + 256 * 9;
  double* V1 = Bm + 256 * 9;
  double* V2 = V1 + 256 * 3;
  double* sc = sm + kIoU;                   // 1024
  double* red = sc + 1024;                  // 8
  double* misc = red + 8;                   // 64
  double* EX = misc + 64;                   // 9 x 16
  const int t = threadIdx.x;
  const double* aux = P.mu_aux + (int64_t)hl * kMuAux;  // [mu_prev 22, mu_inc 22, pose0 6]
  const double* mu_prev = aux;
  const double* mu_inc = aux + 22;
  const double* pose0 = aux + 44;
  const double* pose_pred = P.pose_pred + (int64_t)hl * 6;
  const double* io = P.imu_out + (int64_t)hl * kImuOut;  // [ess, sigma_warp, dt_imu, omega 3]
  const double sigma_warp = io[1], dt_imu = io[2];
  const int M = P.M;
  if (t == 0) {
    so3_exp(pose0 + 3, misc);  // R0 = Exp(rotvec0)
    // dt_int (compute_imu_integration_time, pipeline.py:262-313) computed below
  }
  // scan-to-scan window weights (unmasked: w_imu_int, pipeline.py:448-453)
  const int ia = 2 * t, ib = 2 * t + 1;
  const double ta = ia < M ? S.imu_t[ia] : 0.0, tb = ib < M ? S.imu_t[ib] : 0.0;
  const double wa = ia < M ? window_weight(ta, S.t_last, S.t_scan, sigma_warp) : 0.0;
  const double wb = ib < M ? window_weight(tb, S.t_last, S.t_scan, sigma_warp) : 0.0;
  // dt_int: Σ of the sorted in-window valid stamp intervals = max − min over them
  auto inwin = [&](double ts) { return ts > S.t_last - 1e-9 && ts <= S.t_scan + 1e-9 && ts > 0.0; };
  double cnt = 0.0, tmn = 1e308, tmx = -1e308;
  if (ia < M && inwin(ta)) { cnt += 1.0; tmn = fmin(tmn, ta); tmx = fmax(tmx, ta); }
  if (ib < M && inwin(tb)) { cnt += 1.0; tmn = fmin(tmn, tb); tmx = fmax(tmx, tb); }
  cnt = wg_sum(cnt, red);
  tmn = -wg_max(-tmn, red);
  tmx = wg_max(tmx, red);
  const double dt_int = cnt >= 2.0 ? fmax(0.0, fmin(tmx - tmn, S.t_scan - S.t_last)) : 0.0;
  __syncthreads();
  const double bg[3] = {mu_inc[9], mu_inc[10], mu_inc[11]};
  const double ba[3] = {mu_inc[12], mu_inc[13], mu_inc[14]};
  const double g[3] = {0.0, 0.0, -9.81 * P.gravity_scale};
  double* pre = misc + 16;  // kPreint = 25
  const ImuPair q = load_imu_pair(M, S.imu_t, S.imu_g, S.imu_a);
  wg_preintegrate(M, q, wa, wb, misc, bg, ba, g, A, Bm, V1, V2, pre);
  // time-resolved vMF gravity (imu_evidence.py:402-559): all threads; w = w_imu_int per slot
  {
    double* w = A;  // preint scratch is free again
    if (ia < M) w[ia] = wa;
    if (ib < M) w[ib] = wb;
    __syncthreads();
    double* F = FL + 1 * (kIoN2 + kDZ);
    double Lr[9], hr[3];
    wg_imu_vmf_tr(M, S.imu_a, S.imu_g, w, pose_pred + 3, ba, g, dt_imu, P.eps_psd, P.eps_mass, sc, red, Lr, hr,
                  EX + 1 * kIofExtra);
    __syncthreads();  // the preint scratch and the vMF weights are dead: the factor blocks take over U
    for (int i = t; i < kNFac * (kIoN2 + kDZ); i += kWG) FL[i] = 0.0;
    __syncthreads();
    if (t == 0)
      for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) F[(3 + i) * kDZ + 3 + j] = Lr[3 * i + j];
        F[kIoN2 + 3 + i] = hr[i];
      }
  }
  // Σ_g, Σ_a = measurement-IW modes (measurement_noise_iw_jax.py:38-56, backend_node.py:2021-2023)
  auto iw_mode = [&](int idx, double* out) {
    double Sg[9];
    const double den = P.nu_meas[idx] + 3.0 + 1.0;
    for (int k = 0; k < 9; ++k) Sg[k] = P.Psi_meas[9 * idx + k] / den;
    psd_project3_fast(Sg, P.eps_psd, out, nullptr);
  };
  const double* od_pose = odom;
  const double* od_cov = odom + 6;
  const double* tw = odom + 42;
  const double* twc = odom + 48;
  double twv[9], tww[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) { twv[3 * i + j] = twc[6 * i + j]; tww[3 * i + j] = twc[6 * (i + 3) + 3 + j]; }
  // one factor per lane of distinct waves (lanes 0, 64, 128, 192, then 1, 65, ...)
  const int lane = t & 63, wv = t >> 6;
  const int fac = (lane < 3) ? lane * 4 + wv : -1;  // 0..11
  if (fac >= 0) {
    double* F = nullptr;
    double* ex = nullptr;
    auto sel = [&](int k) { F = FL + k * (kIoN2 + kDZ); ex = EX + k * kIofExtra; };
    switch (fac) {
      case 0:
        sel(0);
        iof_odom_quadratic<false>(pose_pred, od_pose, od_cov, P.eps_psd, P.eps_lift, F, F + kIoN2, ex);
        break;
      case 1: {
        sel(2);
        double Sg[9], dR[9], drv[3];
        iw_mode(0, Sg);
        mat3_mul_tn(misc, pre, dR);  // R0ᵀ R_end
        so3_log(dR, drv);
        iof_gyro<false>(pose0 + 3, pose_pred + 3, drv, Sg, dt_int, P.eps_psd, P.eps_lift, P.eps_mass, F, F + kIoN2, ex);
        break;
      }
      case 2: {
        sel(3);
        double Sa[9], dp[3], dv[3];
        iw_mode(1, Sa);
        mat3_tvec(misc, pre + 9, dp);
        mat3_tvec(misc, pre + 12, dv);
        iof_preint<false>(pose0, pose0 + 3, mu_prev + 6, pose_pred, mu_inc + 6, dv, dp, Sa, dt_int, P.eps_psd, P.eps_lift,
                   P.eps_mass, F, F + kIoN2, ex);
        break;
      }
      case 3:
        sel(4);
        iof_scalar_prior(2, P.planar_z_ref - pose_pred[2], P.planar_z_sigma, F, F + kIoN2, ex);
        break;
      case 4:
        sel(5);
        iof_scalar_prior(8, -mu_inc[8], P.planar_vz_sigma, F, F + kIoN2, ex);
        ex[0] = mu_inc[8];
        break;
      case 5: {
        sel(6);
        double Rwb[9];
        so3_exp(pose_pred + 3, Rwb);
        iof_odom_velocity<false>(mu_inc + 6, Rwb, tw, twv, P.eps_psd, P.eps_lift, F, F + kIoN2, ex);
        break;
      }
      case 6:
        sel(7);
        iof_scalar_prior(5, tw[5] - io[5], sqrt(fmax(twc[35], 1e-12)), F, F + kIoN2, ex);
        break;
      case 7:
        sel(8);
        iof_kinematic<false>(pose0, pose_pred, tw, tw + 3, S.dt, twv, tww, P.eps_psd, P.eps_lift, F, F + kIoN2, ex);
        break;
      default:
        break;
    }
  }
  __syncthreads();
  // dependence scalings, sum in the reference's order (pipeline.py:728-750)
  const double* ex_im = EX + 1 * kIofExtra;
  const double* ex_kc = EX + 8 * kIofExtra;
  const double si = dependence_scale(fmax(ex_im[4], 0.0), P.eps_mass);
  const double mag = norm3(ex_kc) + norm3(ex_kc + 3);
  const double so = dependence_scale(mag, P.eps_mass);
  const double sc9[kNFac] = {so, si, si, 1.0, 1.0, 1.0, so, so, 1.0};
  double* Lout = P.io_L + (int64_t)hl * kIoN2;
  double* hout = P.io_h + (int64_t)hl * kDZ;
  for (int i = t; i < kIoN2 + kDZ; i += kWG) {
    double v = 0.0;
    for (int k = 0; k < kNFac; ++k) v = v + FL[k * (kIoN2 + kDZ) + i] * sc9[k];
    if (i < kIoN2) Lout[i] = v; else hout[i - kIoN2] = v;
  }
  if (t == 0) {
    const double* ex_od = EX;
    const double* ex_gy = EX + 2 * kIofExtra;
    const double* ex_pr = EX + 3 * kIofExtra;
    const double* ex_ov = EX + 6 * kIofExtra;
    // trigger magnitudes (certificates.py:439-455) of the 11 certs
    const double mer = ex_im[1] / (ex_im[2] + P.eps_mass);
    const double trig = ex_od[7] + (ex_im[8] + mer + fabs(1.0 - ex_im[3])) + fabs(1.0 - si) + ex_gy[4] + ex_pr[7] +
                        ex_ov[4] + ex_kc[7] + fabs(1.0 - so);
    double* c = P.io_cert + (int64_t)hl * kIoCert;
    c[0] = 0.0; c[1] = ex_im[1]; c[2] = 0.0;
    c[3] = 1.0; c[4] = ex_im[3]; c[5] = 1.0;
    c[6] = 0.0; c[7] = 0.0;
    c[8] = ex_od[6] + ex_im[7] + ex_gy[3];
    c[9] = trig;
    double* q = P.io_parts + (int64_t)hl * kIoParts;
    for (int k = 0; k < 6; ++k) q[k] = ex_od[k];
    for (int k = 0; k < 6; ++k) q[6 + k] = ex_im[k];  // kappa, ess_w, ess_raw, mean_rel, sigma, Rbar
    q[12] = si;
    for (int k = 0; k < 3; ++k) q[13 + k] = ex_gy[k];
    for (int k = 0; k < 6; ++k) q[16 + k] = ex_pr[k];
    q[22] = EX[4 * kIofExtra]; q[23] = EX[5 * kIofExtra];
    for (int k = 0; k < 3; ++k) q[24 + k] = ex_ov[k];
    q[27] = EX[7 * kIofExtra];
    for (int k = 0; k < 6; ++k) q[28 + k] = ex_kc[k];
    q[34] = so;
    q[35] = ex_od[6]; q[36] = ex_im[6]; q[37] = ex_gy[3]; q[38] = dt_int; q[39] = trig;
  }
}

}  // namespace gc
