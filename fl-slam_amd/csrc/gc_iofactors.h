// gc_iofactors.h — device code of the IMU/odom evidence branch,
// pipeline.py:595-776 and the 11 operators it calls. Shared by the batched pipeline
// (k_io_branch, gc_iobranch.hip) and the per-operator entries (gc_io_factor_batch,
// gc_imu_vmf_gravity_tr_batch).
//
//  odom_quadratic_evidence              backend/operators/odom_evidence.py:40-146
//  imu_vmf_gravity_evidence_time_resolved  imu_evidence.py:277-559 (+ kappa.py:172-232)
//  imu_dependence_inflation             imu_evidence.py:562-589
//  imu_gyro_rotation_evidence           imu_gyro_evidence.py:38-163
//  imu_preintegration_factor            imu_preintegration_factor.py:46-180
//  planar_z_prior / velocity_z_prior    planar_prior.py:55-195
//  odom_velocity_evidence               odom_twist_evidence.py:58-154
//  odom_yawrate_evidence                odom_twist_evidence.py:157-225
//  pose_twist_kinematic_consistency     odom_twist_evidence.py:251-397
//  odom_dependence_inflation            odom_twist_evidence.py:400-430
//
// Every factor writes its 22D contribution as sparse blocks into a caller-provided (L 22x22,
// h 22) pair (thread-local or LDS), plus a fixed-layout extras row. All f64.
#pragma once
#include "gc_math.h"
#include "gc_wgla.h"

namespace gc {

// ------------------------------------------------------------------ thread-local n <= 6 algebra
// Cyclic Jacobi eigen-decomposition of a symmetric n x n (row-major): w unsorted, V columns.
template <int N>
GC_DEV void eighN(const double* Ain, double* w, double* V) {
  double A[N * N];
  for (int i = 0; i < N * N; ++i) A[i] = Ain[i];
  for (int i = 0; i < N * N; ++i) V[i] = (i % (N + 1) == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 16; ++sweep) {
    double off = 0.0, dg = 0.0;
    for (int i = 0; i < N; ++i) {
      dg += A[i * N + i] * A[i * N + i];
      for (int j = i + 1; j < N; ++j) off += A[i * N + j] * A[i * N + j];
    }
    if (off <= 1e-36 * dg || off == 0.0) break;
    for (int p = 0; p < N - 1; ++p)
      for (int q = p + 1; q < N; ++q) {
        const double apq = A[p * N + q];
        if (apq == 0.0) continue;
        const double app = A[p * N + p], aqq = A[q * N + q];
        if (fabs(apq) <= 1e-18 * sqrt(fabs(app * aqq))) { A[p * N + q] = 0.0; A[q * N + p] = 0.0; continue; }
        const double th = (aqq - app) / (2.0 * apq);
        const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < N; ++k) {
          const double akp = A[k * N + p], akq = A[k * N + q];
          A[k * N + p] = c * akp - s * akq;
          A[k * N + q] = s * akp + c * akq;
        }
        for (int k = 0; k < N; ++k) {
          const double apk = A[p * N + k], aqk = A[q * N + k];
          A[p * N + k] = c * apk - s * aqk;
          A[q * N + k] = s * apk + c * aqk;
        }
        A[p * N + q] = 0.0; A[q * N + p] = 0.0;
        for (int k = 0; k < N; ++k) {
          const double vkp = V[k * N + p], vkq = V[k * N + q];
          V[k * N + p] = c * vkp - s * vkq;
          V[k * N + q] = s * vkp + c * vkq;
        }
      }
  }
  for (int i = 0; i < N; ++i) w[i] = A[i * N + i];
}

// domain_projection_psd_core (primitives.py:80-123) on n x n; cert = [proj, sym, min, max, cond, nnc]
template <int N>
GC_DEV void psd_projectN(const double* M, double eps, double* Mp, double* cert) {
  double S[N * N], w[N], V[N * N];
  double symd = 0.0;
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) {
      S[i * N + j] = 0.5 * (M[i * N + j] + M[j * N + i]);
      const double d = S[i * N + j] - M[i * N + j];
      symd += d * d;
    }
  eighN<N>(S, w, V);
  double proj = 0.0, mn = 1e308, mx = -1e308, nnc = 0.0;
  for (int k = 0; k < N; ++k) {
    w[k] = fmax(w[k], eps);
    mn = fmin(mn, w[k]);
    mx = fmax(mx, w[k]);
    nnc += (w[k] < 10.0 * eps) ? 1.0 : 0.0;
  }
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) {
      double v = 0.0;
      for (int k = 0; k < N; ++k) v += V[i * N + k] * w[k] * V[j * N + k];
      Mp[i * N + j] = v;
      const double d = v - S[i * N + j];
      proj += d * d;
    }
  if (cert) {
    cert[0] = sqrt(proj); cert[1] = sqrt(symd); cert[2] = mn; cert[3] = mx; cert[4] = mx / mn; cert[5] = nnc;
  }
}

// The certified shortcut of wg_psd_project_fast, thread-local: if Cholesky of (M_sym - eps I)
// succeeds every eigenvalue exceeds eps, the clamp is inactive and the projection is M_sym (the
// reference's V diag(λ) Vᵀ reconstructs it up to rounding). Otherwise the Jacobi projection runs.
// Used where only the projected matrix (not its cert) feeds the numbers.
template <int N>
GC_DEV void psd_fastN(const double* M, double eps, double* Mp) {
  double C[N * N];
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) {
      Mp[i * N + j] = 0.5 * (M[i * N + j] + M[j * N + i]);
      C[i * N + j] = Mp[i * N + j] - ((i == j) ? eps : 0.0);
    }
  bool ok = true;
  for (int j = 0; j < N && ok; ++j) {
    double d = C[j * N + j];
    for (int k = 0; k < j; ++k) d -= C[j * N + k] * C[j * N + k];
    if (!(d > 0.0)) { ok = false; break; }
    d = sqrt(d);
    C[j * N + j] = d;
    for (int i = j + 1; i < N; ++i) {
      double v = C[i * N + j];
      for (int k = 0; k < j; ++k) v -= C[i * N + k] * C[j * N + k];
      C[i * N + j] = v / d;
    }
  }
  if (!ok) psd_projectN<N>(M, eps, Mp, nullptr);
}

// PSD projection for a factor: the full (cert-producing) projection for the per-operator entries,
// the certified shortcut inside the pipeline (CERT = false: the cert eigen-statistics are not
// consumed there).
template <int N, bool CERT>
GC_DEV void psd_for(const double* M, double eps, double* Mp) {
  if constexpr (CERT) psd_projectN<N>(M, eps, Mp, nullptr);
  else psd_fastN<N>(M, eps, Mp);
}

// eigvalsh: (min, max, count < thr)
template <int N>
GC_DEV void eig_stats(const double* M, double thr, double* mn, double* mx, double* nbelow) {
  double w[N], V[N * N];
  eighN<N>(M, w, V);
  *mn = 1e308; *mx = -1e308; *nbelow = 0.0;
  for (int k = 0; k < N; ++k) {
    *mn = fmin(*mn, w[k]); *mx = fmax(*mx, w[k]);
    *nbelow += (w[k] < thr) ? 1.0 : 0.0;
  }
}

// spd_cholesky_inverse_lifted_core (primitives.py:169-192): (A + εI)^{-1}; returns lift = ε n.
template <int N>
GC_DEV double chol_inverse_liftedN(const double* A, double eps_lift, double* X) {
  double C[N * N];
  for (int i = 0; i < N * N; ++i) C[i] = A[i] + ((i % (N + 1) == 0) ? eps_lift : 0.0);
  for (int j = 0; j < N; ++j) {
    double d = C[j * N + j];
    for (int k = 0; k < j; ++k) d -= C[j * N + k] * C[j * N + k];
    d = sqrt(d);
    C[j * N + j] = d;
    for (int i = j + 1; i < N; ++i) {
      double v = C[i * N + j];
      for (int k = 0; k < j; ++k) v -= C[i * N + k] * C[j * N + k];
      C[i * N + j] = v / d;
    }
  }
  // Ci = C^{-1} (lower), X = Ciᵀ Ci
  double Ci[N * N];
  for (int c = 0; c < N; ++c)
    for (int i = 0; i < N; ++i) {
      if (i < c) { Ci[i * N + c] = 0.0; continue; }
      double v = (i == c) ? 1.0 : 0.0;
      for (int k = c; k < i; ++k) v -= C[i * N + k] * Ci[k * N + c];
      Ci[i * N + c] = v / C[i * N + i];
    }
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) {
      double v = 0.0;
      for (int k = (i > j ? i : j); k < N; ++k) v += Ci[k * N + i] * Ci[k * N + j];
      X[i * N + j] = v;
    }
  return eps_lift * N;
}

// a 3x3 block Lb (scaled by s) at (o, o) of L22 and Lb r (scaled) at o of h22
GC_DEV void put_block3(double* L22, double* h22, int o, const double* Lb, const double* r, double s) {
  for (int i = 0; i < 3; ++i) {
    double hv = 0.0;
    for (int j = 0; j < 3; ++j) {
      L22[(o + i) * kDZ + o + j] = s * Lb[3 * i + j];
      hv += (s * Lb[3 * i + j]) * r[j];
    }
    h22[o + i] = hv;
  }
}

GC_DEV double quad3(const double* r, const double* M) {
  double v[3];
  mat3_vec(M, r, v);
  return dot3(r, v);
}

// ------------------------------------------------------------------------------ factors
// Extras rows (GC_IOF_EXTRA = 16) — layouts in include/gcslam.h (GC_IOF_*).
constexpr int kIofExtra = 16;

// odom_quadratic_evidence: L/h pose block from the odometry pose observation.
// ex = [delta 6, nll, lift, eig_min, eig_max, cond, nnc]
template <bool CERT = true>
GC_DEV void iof_odom_quadratic(const double* pose_pred, const double* odom_pose, const double* cov6, double eps_psd,
                               double eps_lift, double* L22, double* h22, double* ex) {
  double inv[6], T[6], xi[6];
  {  // se3_relative(odom, pred) = pred^{-1} ∘ odom (se3_jax.py:442-459)
    double R[9], Rt[9], t[3];
    so3_exp(pose_pred + 3, R);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Rt[3 * i + j] = R[3 * j + i];
    mat3_vec(Rt, pose_pred, t);
    inv[0] = -t[0]; inv[1] = -t[1]; inv[2] = -t[2];
    so3_log(Rt, inv + 3);
    se3_compose(inv, odom_pose, T);
    se3_log(T, xi);
  }
  double Cp[36], Lp[36];
  psd_for<6, CERT>(cov6, eps_psd, Cp);
  const double lift = chol_inverse_liftedN<6>(Cp, eps_lift, Lp);
  double nll = 0.0;
  for (int i = 0; i < 6; ++i) {
    double hv = 0.0;
    for (int j = 0; j < 6; ++j) {
      L22[i * kDZ + j] = Lp[i * 6 + j];
      hv += Lp[i * 6 + j] * xi[j];
    }
    h22[i] = hv;
    nll += xi[i] * hv;
  }
  double mn = 0.0, mx = 0.0, nb = 0.0;
  if constexpr (CERT) {
    double Lpp[36];
    psd_projectN<6>(Lp, eps_psd, Lpp, nullptr);
    eig_stats<6>(Lpp, 1e-12, &mn, &mx, &nb);
  }
  for (int i = 0; i < 6; ++i) ex[i] = xi[i];
  ex[6] = 0.5 * nll; ex[7] = lift; ex[8] = mn; ex[9] = mx; ex[10] = mx / fmax(mn, 1e-18); ex[11] = nb;
}

// imu_gyro_rotation_evidence. ex = [r 3, nll, lift, eig_min, eig_max, nnc]
template <bool CERT = true>
GC_DEV void iof_gyro(const double* rv_start, const double* rv_end_pred, const double* drv, const double* Sg,
                     double dt_int, double eps_psd, double eps_lift, double eps_mass, double* L22, double* h22,
                     double* ex) {
  double Rs[9], Rd[9], Re[9], Rp[9], Rdiff[9], r[3];
  so3_exp(rv_start, Rs);
  so3_exp(drv, Rd);
  mat3_mul(Rs, Rd, Re);
  so3_exp(rv_end_pred, Rp);
  mat3_mul_tn(Rp, Re, Rdiff);
  so3_log(Rdiff, r);
  const double dtp = fmax(dt_int, 0.0), dte = dtp + eps_mass, ms = dtp / dte;
  double S[9], Sp[9], Lr[9];
  for (int k = 0; k < 9; ++k) S[k] = Sg[k] * dte;
  psd_for<3, CERT>(S, eps_psd, Sp);
  const double lift = chol_inverse_liftedN<3>(Sp, eps_lift, Lr);
  put_block3(L22, h22, 3, Lr, r, ms);
  double mn = 0.0, mx = 0.0, nb = 0.0;
  if constexpr (CERT) {
    double Lpp[9];
    psd_project3_fast(Lr, eps_psd, Lpp, nullptr);
    eig_stats<3>(Lpp, eps_psd, &mn, &mx, &nb);
  }
  ex[0] = r[0]; ex[1] = r[1]; ex[2] = r[2];
  ex[3] = 0.5 * quad3(r, Lr); ex[4] = lift; ex[5] = mn; ex[6] = mx; ex[7] = nb;
}

// imu_preintegration_factor. ex = [r_vel 3, r_pos 3, nll, lift, eig_min, eig_max, cond, nnc]
template <bool CERT = true>
GC_DEV void iof_preint(const double* p_start, const double* rv_start, const double* v_start, const double* p_end,
                       const double* v_end, const double* dv, const double* dp, const double* Sa, double dt_int,
                       double eps_psd, double eps_lift, double eps_mass, double* L22, double* h22, double* ex) {
  double R[9], dvw[3], dpw[3], rv[3], rp[3];
  so3_exp(rv_start, R);
  mat3_vec(R, dv, dvw);
  mat3_vec(R, dp, dpw);
  for (int k = 0; k < 3; ++k) {
    rv[k] = (v_start[k] + dvw[k]) - v_end[k];
    rp[k] = (p_start[k] + v_start[k] * dt_int + dpw[k]) - p_end[k];
  }
  const double dtp = fmax(dt_int, 0.0), dte = dtp + eps_mass, ms = dtp / dte;
  double Sv[9], Sp[9], Svp[9], Spp[9], Lv[9], Lp[9];
  for (int k = 0; k < 9; ++k) { Sv[k] = Sa[k] * dte; Sp[k] = Sa[k] * (dte * dte * dte); }
  psd_for<3, CERT>(Sv, eps_psd, Svp);
  psd_for<3, CERT>(Sp, eps_psd, Spp);
  const double lv = chol_inverse_liftedN<3>(Svp, eps_lift, Lv);
  const double lp = chol_inverse_liftedN<3>(Spp, eps_lift, Lp);
  put_block3(L22, h22, 0, Lp, rp, ms);
  put_block3(L22, h22, 6, Lv, rv, ms);
  double mn1 = 0.0, mx1 = 0.0, nb1 = 0.0, mn2 = 0.0, mx2 = 0.0, nb2 = 0.0;
  if constexpr (CERT) {
    double A[9];
    psd_project3_fast(Lv, eps_psd, A, nullptr);
    eig_stats<3>(A, eps_psd, &mn1, &mx1, &nb1);
    psd_project3_fast(Lp, eps_psd, A, nullptr);
    eig_stats<3>(A, eps_psd, &mn2, &mx2, &nb2);
  }
  for (int k = 0; k < 3; ++k) { ex[k] = rv[k]; ex[3 + k] = rp[k]; }
  ex[6] = 0.5 * quad3(rv, Lv) + 0.5 * quad3(rp, Lp);
  ex[7] = lv + lp;
  const double mn = fmin(mn1, mn2), mx = fmax(mx1, mx2);
  ex[8] = mn; ex[9] = mx; ex[10] = mx / fmax(mn, 1e-18); ex[11] = nb1 + nb2;
}

// planar_z_prior / velocity_z_prior / odom_yawrate_evidence: one diagonal entry.
// ex = [residual (or v_z), nll]
GC_DEV void iof_scalar_prior(int idx, double r, double sigma, double* L22, double* h22, double* ex) {
  const double prec = 1.0 / (sigma * sigma);
  L22[idx * kDZ + idx] = prec;
  h22[idx] = prec * r;
  ex[0] = r; ex[1] = 0.5 * r * r * prec;
}

// odom_velocity_evidence. ex = [r 3, nll, lift, eig_min, eig_max, cond, nnc]
template <bool CERT = true>
GC_DEV void iof_odom_velocity(const double* v_pred_w, const double* Rwb, const double* v_odom, const double* Sv,
                              double eps_psd, double eps_lift, double* L22, double* h22, double* ex) {
  double vb[3], r[3], Sp[9], Lv[9];
  mat3_tvec(Rwb, v_pred_w, vb);
  for (int k = 0; k < 3; ++k) r[k] = v_odom[k] - vb[k];
  psd_for<3, CERT>(Sv, eps_psd, Sp);
  const double lift = chol_inverse_liftedN<3>(Sp, eps_lift, Lv);
  put_block3(L22, h22, 6, Lv, r, 1.0);
  double mn = 0.0, mx = 0.0, nb = 0.0;
  if constexpr (CERT) eig_stats<3>(Sp, 1e-12, &mn, &mx, &nb);
  ex[0] = r[0]; ex[1] = r[1]; ex[2] = r[2];
  ex[3] = 0.5 * quad3(r, Lv); ex[4] = lift; ex[5] = mn; ex[6] = mx; ex[7] = mx / fmax(mn, 1e-18); ex[8] = nb;
}

// pose_twist_kinematic_consistency. ex = [r_trans 3, r_rot 3, nll, lift, eig_min, eig_max, cond]
template <bool CERT = true>
GC_DEV void iof_kinematic(const double* pose_prev, const double* pose_curr, const double* v_body, const double* w_body,
                          double dt, const double* Sv, const double* Sw, double eps_psd, double eps_lift, double* L22,
                          double* h22, double* ex) {
  double Rp[9], Rc[9], Rrel[9], dp[3], dth[3], rt[3], rr[3];
  so3_exp(pose_prev + 3, Rp);
  so3_exp(pose_curr + 3, Rc);
  mat3_vec(Rp, v_body, dp);
  mat3_mul_tn(Rp, Rc, Rrel);
  so3_log(Rrel, dth);
  for (int k = 0; k < 3; ++k) {
    rt[k] = dp[k] * dt - (pose_curr[k] - pose_prev[k]);
    rr[k] = w_body[k] * dt - dth[k];
  }
  const double dt2 = dt * dt + eps_psd;
  double St[9], Sr[9], Stp[9], Srp[9], Lt[9], Lr[9];
  for (int k = 0; k < 9; ++k) { St[k] = dt2 * Sv[k]; Sr[k] = dt2 * Sw[k]; }
  psd_for<3, CERT>(St, eps_psd, Stp);
  psd_for<3, CERT>(Sr, eps_psd, Srp);
  const double lt = chol_inverse_liftedN<3>(Stp, eps_lift, Lt);
  const double lr = chol_inverse_liftedN<3>(Srp, eps_lift, Lr);
  put_block3(L22, h22, 0, Lt, rt, 1.0);
  put_block3(L22, h22, 3, Lr, rr, 1.0);
  double mn1 = 0.0, mx1 = 0.0, nb1 = 0.0, mn2 = 0.0, mx2 = 0.0, nb2 = 0.0;
  if constexpr (CERT) {
    eig_stats<3>(Stp, 0.0, &mn1, &mx1, &nb1);
    eig_stats<3>(Srp, 0.0, &mn2, &mx2, &nb2);
  }
  for (int k = 0; k < 3; ++k) { ex[k] = rt[k]; ex[3 + k] = rr[k]; }
  ex[6] = 0.5 * quad3(rt, Lt) + 0.5 * quad3(rr, Lr);
  ex[7] = lt + lr;
  const double mn = fmin(mn1, mn2), mx = fmax(mx1, mx2);
  ex[8] = mn; ex[9] = mx; ex[10] = mx / fmax(mn, 1e-18);
}

// imu_dependence_inflation / odom_dependence_inflation: 1 / (1 + m² + ε_mass)
GC_DEV double dependence_scale(double m, double eps_mass) { return 1.0 / (1.0 + m * m + eps_mass); }

// ------------------------------------------------------------ time-resolved vMF gravity (WG)
// imu_vmf_gravity_evidence_time_resolved over M <= 512 IMU slots, all 256 threads of the
// workgroup (two slots per thread). Medians of the transport errors (jnp.median: mean of the
// two middle order statistics of the 512) by stable rank counting in LDS. sc: >= 2*512 doubles.
// Thread 0 writes L (3x3 rotation block) into Lrot9, h into hrot3 and
// ex = [kappa, ess_w, ess_raw, mean_rel, sigma, Rbar, nll, nll_per_ess, psd_delta, eig_min,
//       eig_max, cond, nnc, xbar 3].
GC_DEV double wg_median_512(double* v, int M, double* red) {
  // jnp.median: bitonic sort of the M values padded with +inf to 512 (256 threads, one
  // compare-exchange each per stage), then the mean of the two middle order statistics (M even)
  // or the middle one. Order statistics do not depend on how ties are broken. v: 512 doubles.
  const int t = threadIdx.x;
  for (int i = t; i < 512; i += kWG)
    if (i >= M) v[i] = __builtin_inf();
  __syncthreads();
  for (int k = 2; k <= 512; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int i = 2 * j * (t / j) + (t % j), q = i + j;
      const bool up = (i & k) == 0;
      const double a = v[i], b = v[q];
      if ((a > b) == up) { v[i] = b; v[q] = a; }
      __syncthreads();
    }
  const double r = (M % 2 == 0) ? 0.5 * (v[M / 2 - 1] + v[M / 2]) : v[M / 2];
  __syncthreads();
  (void)red;
  return r;
}

GC_DEV void wg_imu_vmf_tr(int M, const double* accel, const double* gyro, const double* w, const double* rotvec,
                          const double* ba, const double* g, double dt, double eps_psd, double eps_mass, double* sc,
                          double* red, double* Lrot9, double* hrot3, double* ex) {
  const int t = threadIdx.x;
  double* e = sc;        // M transport errors
  double* dev = sc + 512;  // |e - median|
  double ev[2] = {0.0, 0.0};
  for (int s = 0; s < 2; ++s) {
    const int i = 2 * t + s;
    if (i >= M) continue;
    auto ac = [&](int j, int k) { return accel[3 * j + k] - ba[k]; };
    double df[3], f[3], om[3], cr[3];
    for (int k = 0; k < 3; ++k) {
      if (i == 0) df[k] = (ac(1, k) - ac(0, k)) / (dt + eps_mass);
      else if (i == M - 1) df[k] = (ac(M - 1, k) - ac(M - 2, k)) / (dt + eps_mass);
      else df[k] = (ac(i + 1, k) - ac(i - 1, k)) / (2 * dt + eps_mass);
      f[k] = ac(i, k);
      om[k] = gyro[3 * i + k];
    }
    cross3(om, f, cr);
    const double x0 = df[0] + cr[0], x1 = df[1] + cr[1], x2 = df[2] + cr[2];
    ev[s] = sqrt(x0 * x0 + x1 * x1 + x2 * x2);
    e[i] = ev[s];
  }
  __syncthreads();
  const double med = wg_median_512(e, M, red);  // sorts e in place; ev keeps this thread's values
  for (int s = 0; s < 2; ++s) {
    const int i = 2 * t + s;
    if (i < M) dev[i] = fabs(ev[s] - med);
  }
  __syncthreads();
  const double sigma = wg_median_512(dev, M, red) / 0.6745 + eps_mass;
  double rel_s = 0.0, wr_s = 0.0, w_s = 0.0, S[3] = {0.0, 0.0, 0.0};
  for (int s = 0; s < 2; ++s) {
    const int i = 2 * t + s;
    if (i >= M) continue;
    const double q = ev[s] / sigma;
    const double rel = exp(-0.5 * (q * q));
    const double wr = w[i] * rel;
    const double a0 = accel[3 * i] - ba[0], a1 = accel[3 * i + 1] - ba[1], a2 = accel[3 * i + 2] - ba[2];
    const double n = sqrt(a0 * a0 + a1 * a1 + a2 * a2) + eps_mass;
    S[0] += wr * (a0 / n); S[1] += wr * (a1 / n); S[2] += wr * (a2 / n);
    rel_s += rel; wr_s += wr; w_s += w[i];
  }
  double sums[6] = {wr_s, w_s, rel_s, S[0], S[1], S[2]};
  wg_sum_n<6>(sums, sc);  // e / dev no longer needed
  const double ess_w = sums[0], ess_raw = sums[1], mrel = sums[2] / (double)M;
  S[0] = sums[3]; S[1] = sums[4]; S[2] = sums[5];
  if (t == 0) {
    const double Sn = norm3(S);
    const double xb[3] = {S[0] / (Sn + eps_mass), S[1] / (Sn + eps_mass), S[2] / (Sn + eps_mass)};
    const double Rbar = Sn / (ess_w + eps_mass);
    const double kappa = kappa_blend(Rbar, 1e-6, 3.0, 0.8, 0.03);
    double R0[9], mg[3], mu0[3];
    so3_exp(rotvec, R0);
    const double gn = norm3(g) + eps_mass;
    for (int k = 0; k < 3; ++k) mg[k] = -(g[k] / gn);
    mat3_tvec(R0, mg, mu0);
    const double xdm = dot3(xb, mu0);
    double c[3];
    cross3(mu0, xb, c);
    double Hm[9], Hs[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        Hm[3 * i + j] = kappa * (((i == j) ? xdm : 0.0) - 0.5 * (xb[i] * mu0[j] + mu0[i] * xb[j]));
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Hs[3 * i + j] = 0.5 * (Hm[3 * i + j] + Hm[3 * j + i]);
    double cert[6];
    psd_project3(Hs, eps_psd, Lrot9, cert);
    for (int k = 0; k < 3; ++k) hrot3[k] = kappa * c[k];  // h = -g_rot, g_rot = -κ μ0 × x̄
    const double nll = -kappa * dot3(mu0, xb);
    ex[0] = kappa; ex[1] = ess_w; ex[2] = ess_raw; ex[3] = mrel; ex[4] = sigma; ex[5] = Rbar;
    ex[6] = nll; ex[7] = nll / (ess_w + eps_mass); ex[8] = cert[0]; ex[9] = cert[2]; ex[10] = cert[3];
    ex[11] = cert[4]; ex[12] = cert[5]; ex[13] = xb[0]; ex[14] = xb[1]; ex[15] = xb[2];
  }
  __syncthreads();
}

}  // namespace gc
