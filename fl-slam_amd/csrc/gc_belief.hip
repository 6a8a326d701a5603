// gc_belief.hip — batched-small per-hypothesis kernels of the GC-SLAM v2 scan pipeline.
// One 256-thread workgroup per hypothesis; 22x22 information-form algebra in LDS.
//
//  a2  PredictDiffusion            backend/operators/predict.py:43-98
//  a3  IMU windows + preintegration backend/operators/imu_preintegration.py:19-147,
//                                   pipeline.py:436-566 (scan window, ξ_body, meas-IW stats)
//  a7  MatrixFisherRotation         archive/legacy_operators/matrix_fisher_evidence.py:155-394
//  a8  PlanarTranslationEvidence    matrix_fisher_evidence.py:413-671, 22D embed :729-756
//  a9  evidence sum, tempering β, excitation scaling   pipeline.py:1038-1148, excitation.py
//  a10 FusionScaleFromCertificates  fusion.py:46-142 (+ pose-6 conditioning pipeline.py:1157-1177)
//  a11 InfoFusionAdditive           fusion.py:150-230
//  a12 PoseUpdateFrobeniusRecompose recompose.py:50-205
//  a13 PoseCovInflationPushforward  build-defined (source deleted, CHANGELOG.md:1246) — unpinned
//  a14 AnchorDriftUpdate            anchor_drift.py:93-191
//  a15 IW suffstats/apply, Q        inverse_wishart_jax.py:35-185, measurement_noise_iw_jax.py
//  a16 HypothesisBarycenter         hypothesis.py:51-236 (fixed-order partial sums + final)
#include <hip/hip_runtime.h>
#include "gc_internal.h"
#include "gc_pipe.h"
#include "gc_wgla.h"
#include "gc_opsdev.h"
#include "gc_budget.h"

namespace gc {

constexpr int N2 = kDZ * kDZ;


// ------------------------------------------------------------------ small shared helpers
// X ∘ Exp(δ[0:6]) (belief.py:408-425), thread-local.
GC_DEV void compose_exp(const double* X, const double* d6, double* out) {
  double e[6];
  se3_exp(d6, e);
  se3_compose(X, e, out);
}

// Lower-triangular solve of one column: y = C^{-1} e_j; returns Σ_k y_k² (= (A^{-1})_jj).
GC_DEV double inv_diag_from_chol(const double* C, int n, int j) {
  double y[kDZ];
  double s = 0.0;
  for (int i = 0; i < n; ++i) {
    double v = (i == j) ? 1.0 : 0.0;
    if (i >= j)
      for (int k = j; k < i; ++k) v -= C[i * n + k] * y[k];
    y[i] = (i >= j) ? v / C[i * n + i] : 0.0;
    s += y[i] * y[i];
  }
  return s;
}

// ========================================================================= a2 + a3
// Per hypothesis: predict (OU diffusion, 2 PSD projections), predicted moments, IMU soft
// windows, parallel-scan preintegration (prefix products of the 512 Exp(ω dt) factors),
// ξ_body = se3_log(Δpose), and the gyro/accel measurement-noise IW statistics.
// a4's per-point time window (deskew_constant_twist.py:61-68) depends on the point only, not on the
// hypothesis: the selected points' w x window once per scan, read by every hypothesis's bins task
// (k_bins_io) in place of the raw weight (the budget's mass scale is applied there). Points j = first
// kWG + t, stepping by step workgroups.
GC_DEV double window_point(const ScanArgs& S, int64_t j, int64_t n_sel, double w, double tr) {
  const double denom = fmax(S.t1 - S.t0, 1e-12);
  return j < n_sel ? w * window_weight(tr, S.t0, S.t1, 0.1 * denom) : 0.0;
}
GC_DEV void window_points(const PipeDev& P, const ScanArgs& S, int64_t first, int64_t step) {
  const int64_t stride = budget_stride(S.n_in, P.n_cap), n_sel = (S.n_in + stride - 1) / stride;
  for (int64_t j = first * kWG + threadIdx.x; j < P.n_cap; j += step * kWG)
    P.w_win[j] = j < n_sel ? window_point(S, j, n_sel, S.w_raw[j * stride], S.t_raw[j * stride]) : 0.0;
}

template <int OCC>
GC_DEV void predict_imu_body(const PipeDev& P, const ScanArgs& S) {
  extern __shared__ double sm[];
  double* Lp = sm;
  double* W1 = Lp + N2;
  double* W2 = W1 + N2;
  double* W3 = W2 + N2;
  double* W4 = W3 + N2;
  double* Sx = W4 + N2;                 // 2 N2 + 4*22
  double* vec = Sx + 2 * N2 + 4 * kDZ;  // 6 x 22
  double* red = vec + 6 * kDZ;          // 8
  double* c1 = red + 8;                 // 6
  double* c2 = c1 + 6;                  // 6
  double* misc = c2 + 6;                // 64
  double* A = misc + 64;                // 256 x 9
  double* Bm = A + 256 * 9;             // 256 x 9
  double* V1 = Bm + 256 * 9;            // 256 x 3
  double* V2 = V1 + 256 * 3;            // 256 x 3
  const int h = blockIdx.x;
  const int t = threadIdx.x;
  const int n = kDZ;
  if (h >= P.Hl) {
    // kBudgetBlocks extra workgroups when they fit beside the hypotheses (launch_predict_imu): the a1
    // budget statistics (point_budget.py:60-113; they only read the staged weights) and the window of
    // the points. The last workgroup to arrive (agent-scope acq_rel ticket) sums the partials in
    // block order, the same fixed order as k_budget_final, and re-arms the ticket. The first re-arms
    // k_bins_io's task counter for this scan's bins launch (next on the stream).
    const int b = h - P.Hl;
    if (b == 0 && t == 0) P.task_ctr[0] = 0u;
    const int64_t stride = budget_stride(S.n_in, P.n_cap);
    budget_partial_block(S.w_raw, S.n_in, stride, b, P.budget_part, sm);
    window_points(P, S, b, kBudgetBlocks);
    if (t == 0) {
      const unsigned prev =
          __hip_atomic_fetch_add(P.budget_ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == kBudgetBlocks - 1) {
        budget_final_values(P.budget_part, S.n_in, P.n_cap, stride, P.budget);
        __hip_atomic_store(P.budget_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  // otherwise the hypothesis workgroups take the window's points themselves: at one occupancy the
  // first kWinPre of this thread's points are loaded here, beside the belief, and written at the end
  const bool win_extra = (int)gridDim.x > P.Hl, win_here = !win_extra;
  if (win_here && h == 0 && t == 0) P.task_ctr[0] = 0u;
  // without the budget workgroups the scalars were formed at staging (S.budget): copied for the
  // kernels after this one (the slot may be restaged once the bins are done, before evidence reads them)
  if (!win_extra && h == 0 && t < 8) P.budget[t] = S.budget[t];
  constexpr int kWinPre = OCC == 1 ? 2 : 0;
  const int64_t w_stride = budget_stride(S.n_in, P.n_cap), w_sel = (S.n_in + w_stride - 1) / w_stride;
  double pw[kWinPre > 0 ? kWinPre : 1], pt[kWinPre > 0 ? kWinPre : 1];
#pragma unroll
  for (int k = 0; k < kWinPre; ++k) {
    const int64_t j = ((int64_t)h + (int64_t)k * P.Hl) * kWG + t;
    const bool in = win_here && j < w_sel;
    pw[k] = in ? S.w_raw[j * w_stride] : 0.0;
    pt[k] = in ? S.t_raw[j * w_stride] : 0.0;
  }
  double* hprev = vec;
  double* mu_prev = vec + kDZ;
  double* hpred = vec + 2 * kDZ;
  double* mu_inc = vec + 3 * kDZ;
  double* xrow1 = vec + 4 * kDZ;  // the lift iterations' broadcast rows (waves 1 and 2)
  double* xrow2 = vec + 5 * kDZ;
  const double ef = exp(-2.0 * P.lambda_ou * S.dt);
  const double dc = (1.0 - ef) / (2.0 * P.lambda_ou + kF64Eps);

  GC_PHASE(P, 0);
  // this thread's IMU slots, loaded beside the belief (one exposed latency for both) and parked in
  // the preintegration scratch (Bm..V2, 15 doubles per thread, not live before the IMU section)
  if (S.sig_cached) {
    // the cached Σ / μ of the previous scan's evidence (L and h are not read): Σ' = e^{-2λdt}Σ + dc Q
    // formed here in W3, its loads in flight with the IMU slots'
    const PredictPrefill pf = predict_prefill_load(P.Sig + (int64_t)h * N2, P.Q, P.mu_fin + (int64_t)h * n);
    imu_pair_store(load_imu_pair(P.M, S.imu_t, S.imu_g, S.imu_a), Bm + 15 * t);
    predict_prefill_store(pf, S.dt, P.lambda_ou, W3, mu_prev);
    __syncthreads();
  } else {
    imu_pair_store(load_imu_pair(P.M, S.imu_t, S.imu_g, S.imu_a), Bm + 15 * t);
    for (int i = t; i < N2; i += kWG) Lp[i] = P.L[(int64_t)h * N2 + i];
    if (t < n) hprev[t] = P.h[(int64_t)h * n + t];
    __syncthreads();
    // μ = (L + εI)⁻¹ h and Σ = (L + εI)⁻¹ by the evidence kernel's routines (so the operands are those
    // a cached scan would read, bit for bit), stored for the bins launch's L_pred workgroup
    wg_solve_lifted(Lp, hprev, mu_prev, P.eps_lift, n, W1);  // W1 = chol(L + εI)
    wg_chol_inverse(W1, W3, W2, n);                          // W3 = Σ
    for (int i = t; i < N2; i += kWG) {
      P.Sig[(int64_t)h * N2 + i] = W3[i];
      W3[i] = ef * W3[i] + dc * P.Q[i];
    }
    if (t < n) P.mu_fin[(int64_t)h * n + t] = mu_prev[t];
    __syncthreads();
  }
  GC_PHASE(P, 1);
  // --- a2 predict (predict.py:43-98) split at its first projection. L_pred = PSD((Σ'_psd + ε_l I)⁻¹)
  // and h_pred = L_pred μ are only read after the bins (evidence); the bins need ξ_body, i.e. the
  // predicted moments μ_inc = (L_pred + ε_l I)⁻¹ h_pred and σ_warp² = (L_pred + ε_l I)⁻¹[15,15]
  // (pipeline.py:436-453). With Σ'_psd = Σ'_sym certified (Cholesky of Σ'_sym − ε_psd I on wave 0, as
  // the full chain's first projection), (L_pred + ε_l I)⁻¹ L_pred = (I + ε_l(Σ'_sym + ε_l I))⁻¹ =: K⁻¹
  // (L_pred's own projection clamp is inactive whenever the lift iteration's bound holds: its
  // eigenvalues are >= 1/(‖Σ'‖ + ε_l) > 4 ε_l >> ε_psd), so μ_inc = K⁻¹ μ and σ_warp² = (K⁻¹(Σ'_sym +
  // ε_l I))[15,15], each a well-conditioned solve (wave_lift_iterate, waves 1 and 2) instead of the
  // chain Cholesky → inverse → projection → Cholesky → solve of the ill-conditioned L_pred (cond ~1e13
  // at the bench: the two routes agree to ~1e-16, oracle check in tests). L_pred / h_pred / the cert
  // are then formed by lpred_wg in the bins launch beside the bin tasks (pred_mode 0). Wave 3: pose0
  // = world pose of belief_prev and R0 = Exp(its rotation vector). If the certificate or the
  // iteration's bound fails, the whole factorised chain runs here instead (pred_mode 1).
  for (int idx = t; idx < N2; idx += kWG) {
    const int i = idx / n, j = idx % n;
    Sx[idx] = 0.5 * (W3[i * n + j] + W3[j * n + i]) - ((i == j) ? P.eps_psd : 0.0);
  }
  __syncthreads();
  if (t < 64) {
    const bool okc = wave0_chol<kDZ, true>(Sx, n);
    if (t == 0) red[4] = okc ? 0.0 : 1.0;
    if (t == 0) GC_STAMP(P.io_parts, 26);
  } else if (t < 128) {
    const int lane = t - 64;
    double x = 0.0;
    const bool ok = wave_lift_iterate<kDZ>(W3, lane < n ? mu_prev[lane] : 0.0, P.eps_lift, xrow1, n, x);
    if (lane < n) mu_inc[lane] = x;
    if (lane == 0) red[5] = ok ? 0.0 : 1.0;
    if (lane == 0) GC_STAMP(P.io_parts, 27);
  } else if (t < 192) {
    const int lane = t - 128;
    const double c = lane < n ? 0.5 * (W3[lane * n + 15] + W3[15 * n + lane]) + (lane == 15 ? P.eps_lift : 0.0) : 0.0;
    double x = 0.0;
    const bool ok = wave_lift_iterate<kDZ>(W3, c, P.eps_lift, xrow2, n, x);
    if (lane == 15) misc[6] = fmax(sqrt(x), 0.01);  // sigma_warp
    if (lane == 0) red[6] = ok ? 0.0 : 1.0;
    if (lane == 0) GC_STAMP(P.io_parts, 28);
  } else {
    if (t == 192) {
      // pose0 = world pose of belief_prev = X ⊞ μ: with the cached posterior, the previous scan's
      // k_combine_local already formed exactly this (compose_exp2 of the same X and μ_fin, the same
      // routine) as the tape's world pose in P.diag[0:6]
      if (S.sig_cached) {
        for (int k = 0; k < 6; ++k) misc[k] = P.diag[(int64_t)h * kHypDiag + k];
      } else {
        compose_exp(P.X + (int64_t)h * 6, mu_prev, misc);
      }
      for (int k = 0; k < 6; ++k) P.mu_aux[(int64_t)h * kMuAux + 44 + k] = misc[k];
      double R0[9];
      so3_exp(misc + 3, R0);
      for (int k = 0; k < 9; ++k) misc[16 + k] = R0[k];
      GC_STAMP(P.io_parts, 29);
    }
    // dt_imu (pipeline.py:526-535) from the parked IMU stamps on wave 3 after lane 192's pose0 (the
    // lift waves 1-2 and the certificate on wave 0 are longer): count, min and max over the valid
    // (stamp > 0) samples, exact in any order; lane l takes the slots of threads l + 64 k
    const int lane = t - 192;
    double cnt = 0.0, tmn = 1e308, tmx = -1e308;
    for (int k = 0; k < 4; ++k) {
      const int tt = lane + 64 * k;
      const double sa = Bm[15 * tt], sb = Bm[15 * tt + 1];
      if (2 * tt < P.M && sa > 0.0) { cnt += 1.0; tmn = fmin(tmn, sa); tmx = fmax(tmx, sa); }
      if (2 * tt + 1 < P.M && sb > 0.0) { cnt += 1.0; tmn = fmin(tmn, sb); tmx = fmax(tmx, sb); }
    }
    cnt = wave_sum(cnt);
    tmn = wave_min(tmn);
    tmx = wave_max(tmx);
    if (lane == 0) misc[7] = fmax(cnt >= 2.0 ? (tmx - tmn) / fmax(cnt - 1.0, 1.0) : 0.0, 1e-12);
  }
  __syncthreads();
  const bool fast = red[4] == 0.0 && red[5] == 0.0 && red[6] == 0.0 && P.predict_route == 0;
  __syncthreads();
  GC_PHASE(P, 2);
  if (!fast) {
    // the factorised route (predict.py:43-98 as restated in wg_predict): L_pred -> W1, h_pred, and
    // chol(L_pred + ε_l I) -> W4 for the predicted moments; Σ' is in W3 (Sig_cached = W2 form)
    wg_predict(Lp, hprev, P.Q, S.dt, P.eps_psd, P.eps_lift, P.lambda_ou, W1, hpred, mu_prev,
               P.pred_cert + (int64_t)h * kPredCert, W2, W3, W4, Sx, red, c1, c2, false, W3, nullptr, W4,
               NoSideWork(), P.io_parts);
    for (int i = t; i < N2; i += kWG) P.Lpred[(int64_t)h * N2 + i] = W1[i];
    if (t < n) P.hpred[(int64_t)h * n + t] = hpred[t];
    if (t < 64) {
      wave0_chol_solve<kDZ>(W4, hpred, mu_inc, n);
    } else if (t == 64) {
      const double s1515 = inv_diag_from_chol(W4, n, 15);
      misc[6] = fmax(sqrt(s1515), 0.01);  // sigma_warp
    }
    __syncthreads();
  }
  if (t == 0) P.pred_mode[h] = fast ? 0.0 : 1.0;
  if (t < n) P.mu_aux[(int64_t)h * kMuAux + t] = mu_prev[t];
  GC_PHASE(P, 3);
  GC_PHASE(P, 4);
  if (t < n) P.mu_aux[(int64_t)h * kMuAux + 22 + t] = mu_inc[t];
  // ------------------------------------------------------------------ IMU (a3)
  const ImuPair q = imu_pair_load(Bm + 15 * t);  // own slots: no barrier needed
  const double sigma_warp = misc[6];
  const double bg[3] = {mu_inc[9], mu_inc[10], mu_inc[11]};
  const double ba[3] = {mu_inc[12], mu_inc[13], mu_inc[14]};
  const int M = P.M;
  // dt_imu over valid (stamp > 0) samples (pipeline.py:526-535), reduced on wave 2 in the first phase
  const double dt_imu = misc[7];
  // two samples per thread: a = 2t, b = 2t+1
  const int ia = 2 * t, ib = 2 * t + 1;
  const double ta = q.ta, tb = q.tb;
  const double wa = ia < M ? window_weight(ta, S.t0, S.t1, sigma_warp) : 0.0;
  const double wb = ib < M ? window_weight(tb, S.t0, S.t1, sigma_warp) : 0.0;
  const double* R0 = misc + 16;
  double* pre = misc + 32;  // kPreint
  const double kG[3] = {0.0, 0.0, -9.81 * P.gravity_scale};  // GC_GRAVITY_W · imu_gravity_scale
  const double *ga = q.ga, *gb = q.gb, *aa = q.aa, *ab = q.ab;
  // --- scan-to-scan window: omega_avg and measurement-noise IW statistics
  //     (pipeline.py:537-566, measurement_noise_iw_jax.py:130-218); their five sums reduced beside the
  //     preintegration's p_end (one wg_sum_n, each element in wg_sum's order)
  auto wint = [&](int i, double ti) {
    return (i < M) ? window_weight(ti, S.t_last, S.t_scan, sigma_warp) * (ti > 0.0 ? 1.0 : 0.0) : 0.0;
  };
  const double wia = wint(ia, q.ta), wib = wint(ib, q.tb);
  double om[5] = {wia + wib, 0.0, 0.0, 0.0, wa + wb};
  for (int k = 0; k < 3; ++k) om[1 + k] = wia * (ga[k] - bg[k]) + wib * (gb[k] - bg[k]);
  GC_PHASE(P, 5);
  wg_preintegrate<true, 5>(M, q, wa, wb, R0, bg, ba, kG, A, Bm, V1, V2, pre, P.io_parts, om);
  GC_PHASE(P, 6);
  const double ess_scan = om[4];
  const double wsum = om[0] + P.eps_mass;
  for (int k = 0; k < 3; ++k) om[k] = om[1 + k] / wsum;
  double rr[12];
  {
    const double f0 = -(R0[0] * kG[0] + R0[3] * kG[1] + R0[6] * kG[2]);
    const double f1 = -(R0[1] * kG[0] + R0[4] * kG[1] + R0[7] * kG[2]);
    const double f2 = -(R0[2] * kG[0] + R0[5] * kG[1] + R0[8] * kG[2]);
    const double fp[3] = {f0, f1, f2};
    double rga[3], rgb[3], raa[3], rab[3];
    for (int k = 0; k < 3; ++k) {
      rga[k] = (ga[k] - bg[k]) - om[k]; rgb[k] = (gb[k] - bg[k]) - om[k];
      raa[k] = (aa[k] - ba[k]) - fp[k]; rab[k] = (ab[k] - ba[k]) - fp[k];
    }
    int q = 0;
    for (int i = 0; i < 3; ++i)
      for (int j = i; j < 3; ++j, ++q) {
        rr[q] = (wia / wsum) * rga[i] * rga[j] + (wib / wsum) * rgb[i] * rgb[j];
        rr[6 + q] = (wia / wsum) * raa[i] * raa[j] + (wib / wsum) * rab[i] * rab[j];
      }
  }
  GC_PHASE(P, 7);
  wg_sum_n<12>(rr, A);
  GC_PHASE(P, 8);
  if (t == 64) {  // ξ_body = se3_log(R0ᵀ Δpose) on wave 1 beside thread 0's IW statistics
    double dR[9], dpose[6], xi[6];
    mat3_mul_tn(R0, pre, dR);
    mat3_tvec(R0, pre + 9, dpose);
    so3_log(dR, dpose + 3);
    se3_log(dpose, xi);
    for (int k = 0; k < 6; ++k) P.xi[(int64_t)h * 6 + k] = xi[k];
  }
  if (t == 0) {
    double* out = P.dPsiM + (int64_t)h * 27;
    for (int blk = 0; blk < 2; ++blk) {
      const double* r = rr + 6 * blk;
      const double M3[9] = {r[0], r[1], r[2], r[1], r[3], r[4], r[2], r[4], r[5]};
      double Pp[9];
      psd_project3_fast(M3, P.eps_psd, Pp, nullptr);
      for (int k = 0; k < 9; ++k) out[9 * blk + k] = Pp[k] * dt_imu;
    }
    for (int k = 0; k < 9; ++k) out[18 + k] = 0.0;
    double* io = P.imu_out + (int64_t)h * kImuOut;
    io[0] = ess_scan; io[1] = sigma_warp; io[2] = dt_imu;
    io[3] = om[0]; io[4] = om[1]; io[5] = om[2]; io[6] = 0.0; io[7] = 0.0;
  }
  if (win_here) {
#pragma unroll
    for (int k = 0; k < kWinPre; ++k) {
      const int64_t j = ((int64_t)h + (int64_t)k * P.Hl) * kWG + t;
      if (j < P.n_cap) P.w_win[j] = window_point(S, j, w_sel, pw[k], pt[k]);
    }
    window_points(P, S, (int64_t)h + (int64_t)kWinPre * P.Hl, P.Hl);  // the rest, if any
  }
}

// Two register budgets of the same kernel: OCC = 1 (the body's natural ~294 VGPRs, no spill) while
// the hypotheses fit one workgroup per CU; OCC = 2 (256 VGPRs, ~150 B of spill) when they do not
// (C5's 1024). With the a1 budget formed at staging, H = 256 runs at OCC = 1 (its predict had been
// OCC = 2 beside 64 budget workgroups, 320 on 256 CUs: 46 -> ~41 us).
template <int OCC>
__global__ void __launch_bounds__(256, OCC) k_predict_imu(PipeDev P, ScanArgs S) {
  predict_imu_body<OCC>(P, S);
}

static size_t lds_predict() {
  return sizeof(double) * (5 * N2 + 2 * N2 + 4 * kDZ + 6 * kDZ + 8 + 12 + 64 + 256 * 24);
}

bool predict_budget_inline(const PipeDev& P) { return P.Hl + kBudgetBlocks <= P.cus; }

hipError_t launch_predict_imu(const PipeDev& P, const ScanArgs& S, hipStream_t st) {
  // P.Hl hypothesis workgroups + kBudgetBlocks budget / window workgroups when they all fit one round
  // (they then run beside the hypotheses for free); otherwise the budget scalars were formed when the
  // slot was staged (S.budget, predict_budget_inline) and the hypotheses' workgroups form the window
  const bool extra = predict_budget_inline(P);
  if (!extra && !S.budget) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)(P.Hl + (extra ? kBudgetBlocks : 0));
  const int cus = P.cus;
  if ((int)grid > cus) {
    if (hipError_t e = ensure_dyn_lds((const void*)k_predict_imu<2>, lds_predict())) return e;
    hipLaunchKernelGGL(k_predict_imu<2>, dim3(grid), dim3(256), lds_predict(), st, P, S);
  } else {
    if (hipError_t e = ensure_dyn_lds((const void*)k_predict_imu<1>, lds_predict())) return e;
    hipLaunchKernelGGL(k_predict_imu<1>, dim3(grid), dim3(256), lds_predict(), st, P, S);
  }
  return hipGetLastError();
}

}  // namespace gc
