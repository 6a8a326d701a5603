// gc_opsdev.h — device building blocks of the per-hypothesis operators, shared by the batched
// scan pipeline kernels (gc_belief.hip, gc_evidence.hip) and the per-operator batched entries
// (gc_ops.hip), so both paths run the same arithmetic.
//
//  thread-level: Matrix-Fisher / planar per-bin rows and finalisation (a7, a8), Frobenius
//  recompose (a12), anchor drift ρ (a14), pose-covariance pushforward of one bin (a13).
//  workgroup-level: lifted mean/world pose of a belief, OU predict (a2), process-noise IW
//  block statistics (a15).
#pragma once
#include "gc_math.h"
#include "gc_wgla.h"

namespace gc {

constexpr int kNN = kDZ * kDZ;

// ------------------------------------------------------------------------------------ a7
// Output record of matrix_fisher_rotation_evidence (matrix_fisher_evidence.py:155-394).
constexpr int kMF = 32;  // [R_mf 9, L_rot 9, h_rot 3, delta 3, svd 3, N_eff, nll/ess, psd Δ, trig, nll]
// Per-bin cross-covariance row (thread b): r = w_b u_map u_scanᵀ (9) and w_b (1), with
// w_b = √(N_s N_m + ε) · R̄_s R̄_m (matrix_fisher_evidence.py:180-205).
GC_DEV void mf_bin_row(double sN, const double* s_dir, double mN, const double* m_dir, double eps, double* r) {
  const double wb = sqrt(sN * mN + eps);
  const double sn = sqrt(s_dir[0] * s_dir[0] + s_dir[1] * s_dir[1] + s_dir[2] * s_dir[2]);
  const double mn = sqrt(m_dir[0] * m_dir[0] + m_dir[1] * m_dir[1] + m_dir[2] * m_dir[2]);
  double us[3], um[3];
  for (int k = 0; k < 3; ++k) { us[k] = s_dir[k] / (sn + eps); um[k] = m_dir[k] / (mn + eps); }
  const double conf = (sn * (1.0 / (sN + eps))) * (mn * (1.0 / (mN + eps)));
  const double wf = wb * conf;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r[3 * i + j] = wf * um[i] * us[j];
  r[9] = wf;
}
// SVD, det-sign fix, R_mf = U Vᵀ, L = V diag(s1+s2, s0+s2, s0+s1) Vᵀ, δ = log(R_predᵀ R_mf),
// PSD(L), h = L δ (matrix_fisher_evidence.py:206-262).
// The two halves of mf_finalize, so the planar rows (which need only R_mf) can start while the
// information half runs on another wave: mf_rotation writes R_mf to out[0:9], the singular values to
// out[24:27] and V to Vout (9); mf_information reads them and writes the rest of the record.
GC_DEV void mf_rotation(const double* acc, double* out, double* Vout) {
  double U[9], s3[3], V[9];
  svd3(acc, U, s3, V);
  double UVt[9];
  mat3_mul_nt(U, V, UVt);
  const double dsg = det3(UVt);
  const double sgn = (dsg > 0.0) ? 1.0 : ((dsg < 0.0) ? -1.0 : 0.0);
  for (int k = 0; k < 3; ++k) U[3 * k + 2] *= sgn;
  double Rmf[9];
  mat3_mul_nt(U, V, Rmf);
  for (int k = 0; k < 9; ++k) { out[k] = Rmf[k]; Vout[k] = V[k]; }
  for (int k = 0; k < 3; ++k) out[24 + k] = s3[k];
}
GC_DEV void mf_information(const double* acc, const double* Rp, const double* Vin, double eps, double eps_psd,
                           double* out) {
  double s3[3], V[9], Rmf[9];
  for (int k = 0; k < 9; ++k) { V[k] = Vin[k]; Rmf[k] = out[k]; }
  for (int k = 0; k < 3; ++k) s3[k] = out[24 + k];
  const double ld[3] = {s3[1] + s3[2], s3[0] + s3[2], s3[0] + s3[1]};
  double Lr[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      Lr[3 * i + j] = V[3 * i] * ld[0] * V[3 * j] + V[3 * i + 1] * ld[1] * V[3 * j + 1] +
                      V[3 * i + 2] * ld[2] * V[3 * j + 2];
  double Rerr[9], dl[3], Lrot[9], cc[6];
  mat3_mul_tn(Rp, Rmf, Rerr);
  so3_log(Rerr, dl);
  psd_project3_fast(Lr, eps_psd, Lrot, cc);
  double hr[3];
  mat3_vec(Lrot, dl, hr);
  const double Neff = acc[9];
  const double nll = 0.5 * (dl[0] * hr[0] + dl[1] * hr[1] + dl[2] * hr[2]);
  for (int k = 0; k < 9; ++k) out[9 + k] = Lrot[k];
  for (int k = 0; k < 3; ++k) { out[18 + k] = hr[k]; out[21 + k] = dl[k]; }
  out[27] = Neff;
  out[28] = nll / (Neff + eps);
  out[29] = cc[0];
  out[30] = cc[0] + eps / (Neff + eps);  // trigger: psd Δ + mass-ε ratio
  out[31] = nll;
}
GC_DEV void mf_finalize(const double* acc, const double* Rp, double eps, double eps_psd, double* out) {
  double U[9], s3[3], V[9];
  svd3(acc, U, s3, V);
  double UVt[9];
  mat3_mul_nt(U, V, UVt);
  const double dsg = det3(UVt);
  const double sgn = (dsg > 0.0) ? 1.0 : ((dsg < 0.0) ? -1.0 : 0.0);
  for (int k = 0; k < 3; ++k) U[3 * k + 2] *= sgn;
  double Rmf[9];
  mat3_mul_nt(U, V, Rmf);
  const double ld[3] = {s3[1] + s3[2], s3[0] + s3[2], s3[0] + s3[1]};
  double Lr[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      Lr[3 * i + j] = V[3 * i] * ld[0] * V[3 * j] + V[3 * i + 1] * ld[1] * V[3 * j + 1] +
                      V[3 * i + 2] * ld[2] * V[3 * j + 2];
  double Rerr[9], dl[3], Lrot[9], cc[6];
  mat3_mul_tn(Rp, Rmf, Rerr);
  so3_log(Rerr, dl);
  psd_project3_fast(Lr, eps_psd, Lrot, cc);
  double hr[3];
  mat3_vec(Lrot, dl, hr);
  const double Neff = acc[9];
  const double nll = 0.5 * (dl[0] * hr[0] + dl[1] * hr[1] + dl[2] * hr[2]);
  for (int k = 0; k < 9; ++k) { out[k] = Rmf[k]; out[9 + k] = Lrot[k]; }
  for (int k = 0; k < 3; ++k) { out[18 + k] = hr[k]; out[21 + k] = dl[k]; out[24 + k] = s3[k]; }
  out[27] = Neff;
  out[28] = nll / (Neff + eps);
  out[29] = cc[0];
  out[30] = cc[0] + eps / (Neff + eps);  // trigger: psd Δ + mass-ε ratio
  out[31] = nll;
}

// ------------------------------------------------------------------------------------ a8
// Output record of planar_translation_evidence (matrix_fisher_evidence.py:413-671).
constexpr int kPT = 26;  // [t_wls 3, L_t 9, h_t 3, delta 3, z_scale, N_eff, nll/ess, psd Δ, trig, xy, z, nll]
// Per-bin WLS row (thread b): W_b = √(N_s N_pos + ε) (Σ_map + R Σ_p Rᵀ + εI)⁻¹ (9), W_b t_b (3),
// √(·) (1), with t_b = c_map − R p̄.
GC_DEV void planar_bin_row(const double* R, double sN, const double* s_pbar, const double* s_Sig, double mNpos,
                           const double* m_c, const double* m_Sig, double eps, double* r) {
  double RS[9], RSR[9], Sc[9], Si[9], rp[3], tb[3];
  mat3_mul(R, s_Sig, RS);
  mat3_mul_nt(RS, R, RSR);
  for (int k = 0; k < 9; ++k) Sc[k] = m_Sig[k] + RSR[k] + ((k % 4 == 0) ? eps : 0.0);
  inv3(Sc, Si);
  const double wb = sqrt(sN * mNpos + eps);
  mat3_vec(R, s_pbar, rp);
  for (int k = 0; k < 3; ++k) tb[k] = m_c[k] - rp[k];
  for (int k = 0; k < 9; ++k) r[k] = wb * Si[k];
  double hb[3];
  mat3_vec(r, tb, hb);
  r[9] = hb[0]; r[10] = hb[1]; r[11] = hb[2];
  r[12] = wb;
}
// t_wls = (L + εI)⁻¹ h; L ⊙ m mᵀ with m = [1, 1, z_scale]; δ = t_wls − t_pred; PSD; h = L δ.
GC_DEV void planar_finalize(const double* acc, double zsc, const double* tp, double eps, double eps_psd,
                            double* out) {
  double Lr[9];
  for (int k = 0; k < 9; ++k) Lr[k] = acc[k] + ((k % 4 == 0) ? eps : 0.0);
  double tw[3];
  solve3(Lr, acc + 9, tw);
  const double msk[3] = {1.0, 1.0, zsc};
  double Lm[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Lm[3 * i + j] = acc[3 * i + j] * msk[i] * msk[j];
  const double dl[3] = {tw[0] - tp[0], tw[1] - tp[1], tw[2] - tp[2]};
  double Lt[9], cc[6], ht[3];
  psd_project3_fast(Lm, eps_psd, Lt, cc);
  mat3_vec(Lt, dl, ht);
  const double Neff = acc[12];
  const double nll = 0.5 * (dl[0] * ht[0] + dl[1] * ht[1] + dl[2] * ht[2]);
  for (int k = 0; k < 3; ++k) { out[k] = tw[k]; out[12 + k] = ht[k]; out[15 + k] = dl[k]; }
  for (int k = 0; k < 9; ++k) out[3 + k] = Lt[k];
  out[18] = zsc;
  out[19] = Neff;
  out[20] = nll / (Neff + eps);
  out[21] = cc[0];
  out[22] = cc[0] + eps / (Neff + eps);
  out[23] = 0.5 * (Lt[0] + Lt[4]);
  out[24] = Lt[8];
  out[25] = nll;
}
// Vertical observability of the map: λ3/λ1 of Σ_b S_dir_scatter / (Σ_b N_dir + ε)
// (matrix_fisher_evidence.py:572-589), from the summed scatter (9) and N_dir total.
GC_DEV double planar_z_scale(const double* Ssum, double Ntot, double eps) {
  double T[9];
  for (int k = 0; k < 9; ++k) T[k] = Ssum[k] / (Ntot + eps);
  double ev[3];
  eigvalsh3_desc(T, ev);
  return fmax(ev[2], 0.0) / fmax(ev[0], eps);
}

// ------------------------------------------------------------------------------------ a12
// Frobenius recompose given δz = (L + εI)⁻¹h (recompose.py:50-205): s = T/(T + c_frob),
// δ' = δ + s·½[z_lin, δ] (BCH3 on the pose slice), X_new = X ∘ Exp(δ'). Writes X_new (6),
// δ' (6) and the bch term (6); returns s.
GC_DEV double recompose_pose_R(const double* X, const double* RX, const double* zl, const double* dz, double T,
                               double c_frob, double* X_new, double* dpc, double* bch) {
  const double s = T / (T + c_frob);
  double c1[3], c2[3], c3[3];
  cross3(zl + 3, dz, c1);
  cross3(zl, dz + 3, c2);
  cross3(zl + 3, dz + 3, c3);
  for (int k = 0; k < 3; ++k) {
    bch[k] = 0.5 * (c1[k] + c2[k]);
    bch[3 + k] = 0.5 * c3[k];
    dpc[k] = dz[k] + s * bch[k];
    dpc[3 + k] = dz[3 + k] + s * bch[3 + k];
  }
  double e[6], Re[9];
  se3_exp(dpc, e);
  so3_exp(e + 3, Re);
  se3_compose_R(X, RX, e, Re, X_new);
  return s;
}
// with RX = so3_exp(X rot) formed here (recompose_pose_R takes it formed elsewhere: the same bits)
GC_DEV double recompose_pose(const double* X, const double* zl, const double* dz, double T, double c_frob,
                             double* X_new, double* dpc, double* bch) {
  double RX[9];
  so3_exp(X + 3, RX);
  return recompose_pose_R(X, RX, zl, dz, T, c_frob, X_new, dpc, bch);
}

// ------------------------------------------------------------------------------------ a14
// ρ = clip(max(‖δt‖/0.5, ‖δθ‖/0.2), 0, 1) (anchor_drift.py:64-91); also returns the drifts.
GC_DEV double drift_rho(const double* mu, double* drift_m, double* drift_r) {
  const double dm = sqrt(mu[0] * mu[0] + mu[1] * mu[1] + mu[2] * mu[2]);
  const double dr = sqrt(mu[3] * mu[3] + mu[4] * mu[4] + mu[5] * mu[5]);
  if (drift_m) *drift_m = dm;
  if (drift_r) *drift_r = dr;
  return clampd(fmax(dm / 0.5, dr / 0.2), 0.0, 1.0);
}

// ------------------------------------------------------------------------------------ a13
// Push one scan bin into the world frame (build-defined PoseCovInflationPushforward):
// s_dir → R s, S → R S Rᵀ, N_dir = N_pos = N, sum_p = N p_w, sum_ppT = N (Σ_w + p_w p_wᵀ) with
// Σ_w = R Σ_p Rᵀ + J Σ_pose Jᵀ, J = [R | −R[p̄]×], p_w = R p̄ + t. Σ_pose: 6x6 (row stride ld).
// With Σ_pose = [[A, B], [Bᵀ, C]] and K = [p̄]× (Kᵀ = −K), J Σ_pose Jᵀ = R (A + BK + (BK)ᵀ − KCK) Rᵀ:
// the inflation is added in the body frame and rotated once with Σ_p (the same Σ_w as the oracle's
// J Σ Jᵀ up to rounding, a third of its products).
// s: bin stats record (GC_BIN_STATS layout); o: map record (kMapRec).
GC_DEV void pushforward_bin(const double* s, const double* R, const double* tt, const double* Sp, int ld,
                            double* o) {
  const double N = s[0];
  double v3[3], M3[9], M4[9];
  mat3_vec(R, s + 1, v3);
  for (int k = 0; k < 3; ++k) o[k] = v3[k];
  mat3_mul(R, s + 4, M3);
  mat3_mul_nt(M3, R, M4);
  for (int k = 0; k < 9; ++k) o[3 + k] = M4[k];
  o[12] = N; o[13] = N;
  double pw[3];
  mat3_vec(R, s + 13, pw);
  for (int k = 0; k < 3; ++k) pw[k] += tt[k];
  const double* pb = s + 13;
  const double K[9] = {0.0, -pb[2], pb[1], pb[2], 0.0, -pb[0], -pb[1], pb[0], 0.0};
  double A[9], Bm[9], C[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      A[3 * i + j] = Sp[i * ld + j];
      Bm[3 * i + j] = Sp[i * ld + 3 + j];
      C[3 * i + j] = Sp[(3 + i) * ld + 3 + j];
    }
  double BK[9], CK[9], KCK[9], Mb[9];
  mat3_mul(Bm, K, BK);
  mat3_mul(C, K, CK);
  mat3_mul(K, CK, KCK);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      Mb[3 * i + j] = s[16 + 3 * i + j] + ((A[3 * i + j] + (BK[3 * i + j] + BK[3 * j + i])) - KCK[3 * i + j]);
  mat3_mul(R, Mb, M3);
  mat3_mul_nt(M3, R, M4);
  for (int k = 0; k < 3; ++k) o[14 + k] = N * pw[k];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) o[17 + 3 * i + j] = N * (M4[3 * i + j] + pw[i] * pw[j]);
}

// ------------------------------------------------------------------------------------ a15
constexpr int kIwBlockStart[7] = {0, 3, 6, 9, 12, 15, 16};
constexpr int kIwBlockDim[7] = {3, 3, 3, 3, 3, 1, 6};
// Process-noise IW statistics entry idx of (7, 6, 6) (inverse_wishart_jax.py:71-123):
// dΨ_b = (r rᵀ + Σ_post)[block b] with r = μ_post − μ_pred, zero outside the d_b x d_b block.
GC_DEV double iw_proc_stat(int idx, const double* mupo, const double* mups, const double* Spost) {
  const int b = idx / 36, i = (idx % 36) / 6, j = idx % 6;
  const int d = kIwBlockDim[b], s0 = kIwBlockStart[b];
  if (i >= d || j >= d) return 0.0;
  const double r_i = mupo[s0 + i] - mups[s0 + i], r_j = mupo[s0 + j] - mups[s0 + j];
  return r_i * r_j + Spost[(s0 + i) * kDZ + (s0 + j)];
}

// ------------------------------------------------------------------------------------ a2
constexpr int kPredCertLen = 8;  // [lift, psd Δ, eig_min, eig_max, cond, nnc, trace Σ', trigger]
// predict_diffusion core (predict.py:43-98), one workgroup: μ = (L+εI)⁻¹h, Σ = (L+εI)⁻¹,
// Σ' = e^{-2λdt}Σ + (1−e^{-2λdt})/(2λ) Q, PSD, L' = (Σ'+εI)⁻¹, PSD, h' = L' μ.
// Lp (in, n x n, LDS) and hprev (in) are preserved; outputs Lout/hout/mu (LDS), cert (thread 0).
// Scratch: W1..W3 (n x n each), Sx (2 n² + 4 n), red (>= 8), c1/c2 (6 each).
// full_cert: exact eigen certificate (per-operator entry); otherwise the Cholesky-certified
// fast projection (pipeline: only the projection delta is consumed, eigen fields NaN).
// Llift (batched pipeline, fast path): also returns chol(L_pred + ε_lift I) there (n x n; may alias
// W3), factored beside L_pred's certificate, with side() on wave 3 meanwhile (mu is final by then).
// The Sig_cached form of wg_predict's first step in two halves, so the caller can put the global loads
// of Σ, Q and μ in flight beside its own (one exposed latency): predict_prefill_load() then, after the
// caller's loads, predict_prefill_store() writes W2 and μ (a barrier must follow before wg_predict is
// called with Sig_cached = W2).
struct PredictPrefill {
  double s[2], q[2], m;
};
GC_DEV PredictPrefill predict_prefill_load(const double* Sig, const double* Q, const double* mu_cached) {
  const int t = threadIdx.x;
  PredictPrefill f;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int i = t + r * kWG;
    f.s[r] = i < kNN ? Sig[i] : 0.0;
    f.q[r] = i < kNN ? Q[i] : 0.0;
  }
  f.m = t < kDZ ? mu_cached[t] : 0.0;
  return f;
}
GC_DEV void predict_prefill_store(const PredictPrefill& f, double dt, double lambda_ou, double* W2, double* mu) {
  const int t = threadIdx.x;
  const double ef = exp(-2.0 * lambda_ou * dt);
  const double dc = (1.0 - ef) / (2.0 * lambda_ou + kF64Eps);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int i = t + r * kWG;
    if (i < kNN) W2[i] = ef * f.s[r] + dc * f.q[r];
  }
  if (t < kDZ) mu[t] = f.m;
}

template <typename Side = NoSideWork>
GC_DEV void wg_predict(const double* Lp, const double* hprev, const double* Q, double dt, double eps_psd,
                       double eps_lift, double lambda_ou, double* Lout, double* hout, double* mu, double* cert,
                       double* W1, double* W2, double* W3, double* Sx, double* red, double* c1, double* c2,
                       bool full_cert = false, const double* Sig_cached = nullptr,
                       const double* mu_cached = nullptr, double* Llift = nullptr, const Side& side = Side(),
                       double* sink = nullptr) {
  const int t = threadIdx.x, n = kDZ;
  (void)sink;
  const double ef = exp(-2.0 * lambda_ou * dt);
  const double dc = (1.0 - ef) / (2.0 * lambda_ou + kF64Eps);
  if (Sig_cached == W2) {
    // the caller has already formed W2 = e^{-2λdt} Σ + dc Q and μ (predict_prefill) and synchronised
  } else if (Sig_cached) {
    // The batched pipeline's evidence kernel already factorised this very (L + εI) with the same
    // routines (Σ_post and μ_fin of the previous scan): bit-identical, so reuse them; Σ and Q
    // arrive in one round trip
    for (int i = t; i < kNN; i += kWG) W2[i] = ef * Sig_cached[i] + dc * Q[i];
    if (t < n) mu[t] = mu_cached[t];
    __syncthreads();
  } else {
    wg_solve_lifted(Lp, hprev, mu, eps_lift, n, W1);  // W1 = chol(L + εI)
    wg_chol_inverse(W1, W2, W3, n);                    // W2 = Σ
    for (int i = t; i < kNN; i += kWG) W2[i] = ef * W2[i] + dc * Q[i];
    __syncthreads();
  }
  if (full_cert) {
    wg_psd_project(W2, W3, eps_psd, n, Sx, red, c1);  // Σ'_psd -> W3
  } else {
    // Σ'_psd -> W3, certified on wave 0 while wave 1 factors Σ'_psd + εI into W1 (wg_inverse_lifted's
    // factorization)
    GC_MARK(sink, 26);
    wg_psd_fast_lifted_chol(W2, W3, eps_psd, eps_lift, n, Sx, W1, red, c1);
  }
  GC_MARK(sink, 27);
  double trl = (t < n) ? W3[t * n + t] : 0.0;
  const double trace_cov = wg_sum(trl, red);
  if (full_cert) {
    wg_inverse_lifted(W3, W2, eps_lift, n, W1, Lout);  // L' raw -> W2 (Lout as work)
    wg_psd_project(W2, Lout, eps_psd, n, Sx, red, c2);
  } else {
    wg_chol_inverse(W1, W2, Lout, n);  // L' raw -> W2 (Lout as work)
    GC_MARK(sink, 28);
    if (Llift) wg_psd_fast_lifted_chol(W2, Lout, eps_psd, eps_lift, n, Sx, Llift, red, c2, side);
    else wg_psd_project_fast(W2, Lout, eps_psd, n, Sx, red, c2);
  }
  GC_MARK(sink, 29);
  wg_matvec(Lout, mu, hout, n);
  if (t == 0 && cert) {
    const double lift = 2.0 * eps_lift * n;
    cert[0] = lift; cert[1] = c1[0] + c2[0]; cert[2] = c2[2]; cert[3] = c2[3]; cert[4] = c2[4]; cert[5] = c2[5];
    cert[6] = trace_cov;
    cert[7] = lift + (c1[0] + c2[0]) + fabs(1.0 - dt);  // trigger; dt_scale = dt (predict.py:185-189)
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------ a3
// Weighted IMU preintegration (imu_preintegration.py:46-147) over M <= 512 samples, two per
// thread (a = 2t, b = 2t+1): rotation by an inclusive wave-shuffle + cross-wave scan of the 3x3 factors
// Exp((ω−b_g) w dt), velocity by a prefix sum, position by the closed-form sum
// p = Σ v_i de_i + ½ a_i de_i². wa/wb are the two samples' weights, R0 the start rotation.
// Thread 0 writes out[kPreint] = [R_end 9, p_end 3, v_end 3, Σde, Σa_body de 3,
// Σa_world_nog de 3, Σa_world de 3]. Scratch A, Bm: 256 x 9; V1, V2: 256 x 3.
constexpr int kPreint = 25;
// A thread's two IMU slots a = 2t, b = 2t+1 (and the stamp of 2t+2), zero past M. Loaded once; the
// batched predict issues the loads at kernel entry so their latency hides behind the 22x22 algebra.
struct ImuPair {
  double ta, tb, tn;
  double ga[3], gb[3], aa[3], ab[3];
};
GC_DEV ImuPair load_imu_pair(int M, const double* stamps, const double* gyro, const double* accel) {
  const int ia = 2 * threadIdx.x, ib = ia + 1;
  ImuPair q;
  q.ta = ia < M ? stamps[ia] : 0.0;
  q.tb = ib < M ? stamps[ib] : 0.0;
  q.tn = ib + 1 < M ? stamps[ib + 1] : 0.0;
  for (int k = 0; k < 3; ++k) {
    q.ga[k] = ia < M ? gyro[3 * ia + k] : 0.0;
    q.aa[k] = ia < M ? accel[3 * ia + k] : 0.0;
    q.gb[k] = ib < M ? gyro[3 * ib + k] : 0.0;
    q.ab[k] = ib < M ? accel[3 * ib + k] : 0.0;
  }
  return q;
}
// Park / restore an ImuPair in 15 doubles of LDS (per thread), so it need not stay in registers.
GC_DEV void imu_pair_store(const ImuPair& q, double* d) {
  d[0] = q.ta; d[1] = q.tb; d[2] = q.tn;
  for (int k = 0; k < 3; ++k) { d[3 + k] = q.ga[k]; d[6 + k] = q.gb[k]; d[9 + k] = q.aa[k]; d[12 + k] = q.ab[k]; }
}
GC_DEV ImuPair imu_pair_load(const double* d) {
  ImuPair q;
  q.ta = d[0]; q.tb = d[1]; q.tn = d[2];
  for (int k = 0; k < 3; ++k) { q.ga[k] = d[3 + k]; q.gb[k] = d[6 + k]; q.aa[k] = d[9 + k]; q.ab[k] = d[12 + k]; }
  return q;
}
// ENDS: only R_end and p_end are formed (out[0:12]; the batched predict's ξ_body needs nothing else),
// with NX further per-thread values (extra, replaced by their workgroup sums) reduced beside p_end in
// the same wg_sum_n (the same order per element as their own reduction would give).
template <bool ENDS = false, int NX = 0>
GC_DEV void wg_preintegrate(int M, const ImuPair& q, double wa, double wb, const double* R0, const double* bg,
                            const double* ba, const double* g, double* A, double* Bm, double* V1, double* V2,
                            double* out, double* sink = nullptr, double* extra = nullptr) {
  const int t = threadIdx.x;
  (void)sink;
  const int ia = 2 * t, ib = 2 * t + 1;
  const double ta = q.ta, tb = q.tb;
  // dt_i = max(t_{i+1} - t_i, 0), last slot 0 (imu_preintegration.py:84-85)
  const double dta = (ib < M) ? fmax(tb - ta, 0.0) : 0.0;
  const double dtb = ib < M ? ((ib + 1 < M) ? fmax(q.tn - tb, 0.0) : 0.0) : 0.0;
  const double dea = (ia < M ? wa : 0.0) * dta, deb = (ib < M ? wb : 0.0) * dtb;
  const double *ga = q.ga, *gb = q.gb, *aa = q.aa, *ab = q.ab;
  double dRa[9], dRb[9], Pl[9];
  {
    double wv[3] = {(ga[0] - bg[0]) * dea, (ga[1] - bg[1]) * dea, (ga[2] - bg[2]) * dea};
    so3_exp(wv, dRa);
    double wv2[3] = {(gb[0] - bg[0]) * deb, (gb[1] - bg[1]) * deb, (gb[2] - bg[2]) * deb};
    so3_exp(wv2, dRb);
    mat3_mul(dRa, dRb, Pl);
  }
  GC_MARK(sink, 40);
  // inclusive scan of 3x3 products X_t = Pl_0 ... Pl_t: six DPP levels inside each wave (scan_dpp_f64:
  // lanes without a source take the identity, I X = X exactly), then the wave totals (left to right)
  // applied on the left; result rows in A for the reads below
  double* src = A;
  {
    const int lane = t & 63, w = t >> 6;
    (void)lane;
    double X[9];
    for (int k = 0; k < 9; ++k) X[k] = Pl[k];
    const auto level = [&](auto shift) {
      double Y[9], Z[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) Y[k] = shift(X[k], (k % 4 == 0) ? 1.0 : 0.0);
      mat3_mul(Y, X, Z);
#pragma unroll
      for (int k = 0; k < 9; ++k) X[k] = Z[k];
    };
    level([](double v, double o) { return scan_dpp_f64<0x111>(v, o); });
    level([](double v, double o) { return scan_dpp_f64<0x112>(v, o); });
    level([](double v, double o) { return scan_dpp_f64<0x114>(v, o); });
    level([](double v, double o) { return scan_dpp_f64<0x118>(v, o); });
    level([](double v, double o) { return scan_dpp_f64<0x142, 0xA>(v, o); });
    level([](double v, double o) { return scan_dpp_f64<0x143, 0xC>(v, o); });
    if (lane == 63)
      for (int k = 0; k < 9; ++k) Bm[w * 9 + k] = X[k];
    __syncthreads();
    if (w > 0) {
      double W[9], Z[9];
      for (int k = 0; k < 9; ++k) W[k] = Bm[k];
      for (int v = 1; v < w; ++v) {
        mat3_mul(W, Bm + v * 9, Z);
        for (int k = 0; k < 9; ++k) W[k] = Z[k];
      }
      mat3_mul(W, X, Z);
      for (int k = 0; k < 9; ++k) X[k] = Z[k];
    }
    for (int k = 0; k < 9; ++k) A[t * 9 + k] = X[k];
    __syncthreads();
  }
  GC_MARK(sink, 41);
  double Ea[9], Rb[9];
  if (t == 0) {
    for (int k = 0; k < 9; ++k) Ea[k] = R0[k];
  } else {
    mat3_mul(R0, src + (t - 1) * 9, Ea);
  }
  mat3_mul(Ea, dRa, Rb);
  double nga[3], ngb[3], awa[3], awb[3];
  const double aba[3] = {aa[0] - ba[0], aa[1] - ba[1], aa[2] - ba[2]};
  const double abb[3] = {ab[0] - ba[0], ab[1] - ba[1], ab[2] - ba[2]};
  mat3_vec(Ea, aba, nga);
  mat3_vec(Rb, abb, ngb);
  for (int k = 0; k < 3; ++k) { awa[k] = nga[k] + g[k]; awb[k] = ngb[k] + g[k]; }
  // prefix sum of velocity increments (inclusive rows in V1; the reads below take row t-1):
  // shuffle levels inside each wave, then the preceding waves' totals
  double* vs = V1;
  {
    const int lane = t & 63, w = t >> 6;
    double v[3];
    for (int k = 0; k < 3; ++k) v[k] = awa[k] * dea + awb[k] * deb;
    (void)lane;
#pragma unroll
    for (int k = 0; k < 3; ++k) {  // the same six DPP levels (identity 0.0)
      v[k] = scan_dpp_f64<0x111>(v[k], 0.0) + v[k];
      v[k] = scan_dpp_f64<0x112>(v[k], 0.0) + v[k];
      v[k] = scan_dpp_f64<0x114>(v[k], 0.0) + v[k];
      v[k] = scan_dpp_f64<0x118>(v[k], 0.0) + v[k];
      v[k] = scan_dpp_f64<0x142, 0xA>(v[k], 0.0) + v[k];
      v[k] = scan_dpp_f64<0x143, 0xC>(v[k], 0.0) + v[k];
    }
    if (lane == 63)
      for (int k = 0; k < 3; ++k) V2[w * 3 + k] = v[k];
    __syncthreads();
    for (int u = 0; u < w; ++u)
      for (int k = 0; k < 3; ++k) v[k] = V2[u * 3 + k] + v[k];
    for (int k = 0; k < 3; ++k) V1[t * 3 + k] = v[k];
    __syncthreads();
  }
  GC_MARK(sink, 42);
  double pc[3];
  for (int k = 0; k < 3; ++k) {
    const double va = (t > 0) ? vs[(t - 1) * 3 + k] : 0.0;
    const double vb = va + awa[k] * dea;
    pc[k] = va * dea + 0.5 * awa[k] * (dea * dea) + vb * deb + 0.5 * awb[k] * (deb * deb);
  }
  if constexpr (ENDS) {
    double s[3 + NX];
    for (int k = 0; k < 3; ++k) s[k] = pc[k];
    for (int i = 0; i < NX; ++i) s[3 + i] = extra[i];
    GC_MARK(sink, 43);
    wg_sum_n<3 + NX>(s, Bm);
    for (int i = 0; i < NX; ++i) extra[i] = s[3 + i];
    if (t == 0) {
      mat3_mul(R0, src + (kWG - 1) * 9, out);  // R_end
      for (int k = 0; k < 3; ++k) out[9 + k] = s[k];  // p_end (world)
    }
    __syncthreads();
    return;
  }
  double sums[13];
  for (int k = 0; k < 3; ++k) {
    sums[k] = pc[k];
    sums[3 + k] = aba[k] * dea + abb[k] * deb;
    sums[6 + k] = nga[k] * dea + ngb[k] * deb;
    sums[9 + k] = awa[k] * dea + awb[k] * deb;
  }
  sums[12] = dea + deb;
  GC_MARK(sink, 43);
  wg_sum_n<13>(sums, Bm);  // 13 sums in wg_sum's order with two barriers (Bm: free again)
  if (t == 0) {
    mat3_mul(R0, src + (kWG - 1) * 9, out);  // R_end
    for (int k = 0; k < 3; ++k) {
      out[9 + k] = sums[k];                  // p_end (world)
      out[12 + k] = vs[(kWG - 1) * 3 + k];   // v_end (world)
      out[16 + k] = sums[3 + k];
      out[19 + k] = sums[6 + k];
      out[22 + k] = sums[9 + k];
    }
    out[15] = sums[12];
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------ a15
constexpr double kIwRhoProc[7] = {0.99, 0.995, 0.95, 0.999, 0.999, 0.9999, 0.9999};  // constants.py:265-281
constexpr double kIwRhoMeas[3] = {0.995, 0.995, 0.99};

// ν projection: ν_min + softplus(ν − ν_min), then soft cap at ν_max (inverse_wishart_jax.py:160-170).
GC_DEV double nu_project(double nu_raw, double dim, double nu_max) {
  const double nmin = dim + 1.0 + 0.5;
  const double nf = nmin + softplus(nu_raw - nmin);
  return nu_max - softplus(nu_max - nf);
}

// Process-noise IW apply (inverse_wishart_jax.py:126-185), one workgroup:
// Ψ_b' = PSD((ρ_b Ψ_b + w dΨ_b) ⊙ mask_b), ν_b' = proj(ρ_b ν_b + w dν_b).
// Outputs may alias the inputs (all reads precede the writes). cert (thread 0) =
// [Σ_b psd Δ_b, Σ_b |ν_b' − ν_b,raw|]. Scratch: Qs 216, blk 36, blkp 36, Sx 2*36+24, red 16,
// c6 8, tab 32.
// den_b of process_noise_state_to_Q_jax (inverse_wishart_jax.py:35-68): softplus⁺(ν_b − d_b − 1)
GC_DEV double iw_q_den(double nu_b, int b) { return softplus(50.0 * (nu_b - kIwBlockDim[b] - 1.0)) / 50.0 + 1e-12; }

// WITH_Q: the apply followed by process_noise_state_to_Q_jax of the updated state (wg_iw_Q's result,
// bit for bit) with Q's blocks formed from the apply's own results instead of a second pass over the
// state: each 3x3 / 1x1 block's thread projects Ψ'_b / den_b right after forming Ψ'_b, and the 6x6
// block's Cholesky certificate of Ψ'_6 / den_6 − εI runs on wave 2 beside the apply's own certificate
// (wg_psd_project_fast's side slot). That speculation holds when the apply's 6x6 projection takes its
// shortcut (then Ψ'_6 = sym(M_6) exactly); otherwise, or if its own Cholesky fails, the 6x6 block is
// projected after the apply as wg_iw_Q does. Q_out: global 22x22; Qp: NN doubles of LDS; X: 2 x 36 + 8.
template <bool WITH_Q = false>
GC_DEV void wg_iw_proc_apply(const double* nu, const double* Psi, const double* dPsi, const double* dnu, double w,
                             double eps_psd, double nu_max, double* nu_out, double* Psi_out, double* cert,
                             double* Qs, double* blk, double* blkp, double* Sx, double* red, double* c6,
                             double* tab, double* raw_out = nullptr, double* Q_out = nullptr, double* Qp = nullptr,
                             double* X = nullptr) {
  const int t = threadIdx.x;
  if constexpr (WITH_Q) {
    for (int idx = t; idx < kNN; idx += kWG) Qp[idx] = 0.0;
    __syncthreads();
  }
  double nn_t = 0.0;
  if (t < 7) {
    const double nr = kIwRhoProc[t] * nu[t] + w * dnu[t];
    const double nn = nu_project(nr, kIwBlockDim[t], nu_max);
    tab[16 + t] = fabs(nn - nr);
    tab[24 + t] = nn;
    nn_t = nn;
  }
  if (t < 6) {
    // 3x3 blocks (t < 5) and the 1x1 block (t = 5) in registers. The reference projects each masked
    // block padded to 6x6, [A, 0; 0, 0] -> [PSD(A), 0; 0, εI], so P = PSD(leading 3x3) or
    // diag(max(a, ε), ε, ε), and the projection delta picks up (6 - d) ε²; written out entry by
    // entry (no run-time indexed array)
    const double rho = kIwRhoProc[t];
    const double* Ps = Psi + t * 36;
    const double* dP = dPsi + t * 36;
    double Pp[9], d2;
    if (t == 5) {
      const double a = rho * Ps[0] + w * dP[0], pv = fmax(a, eps_psd);
      for (int k = 0; k < 9; ++k) Pp[k] = (k == 0) ? pv : ((k % 4 == 0) ? eps_psd : 0.0);
      d2 = 5.0 * eps_psd * eps_psd + (pv - a) * (pv - a);
      if (raw_out)
        for (int k = 0; k < 36; ++k) raw_out[t * 36 + k] = k == 0 ? a : 0.0;
    } else {
      double A[9], c[6];
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) A[3 * i + j] = rho * Ps[6 * i + j] + w * dP[6 * i + j];
      psd_project3_fast(A, eps_psd, Pp, c);
      d2 = 3.0 * eps_psd * eps_psd + c[0] * c[0];
      if (raw_out)  // the masked block, padded to 6x6 (the reference's projection operand)
        for (int k = 0; k < 36; ++k) raw_out[t * 36 + k] = (k / 6 < 3 && k % 6 < 3) ? A[3 * (k / 6) + k % 6] : 0.0;
    }
    tab[8 + t] = sqrt(d2);
    for (int k = 0; k < 36; ++k) {
      const int i = k / 6, j = k % 6;
      Qs[t * 36 + k] = (i < 3 && j < 3) ? Pp[3 * i + j] : ((i == j) ? eps_psd : 0.0);
    }
    if constexpr (WITH_Q) {  // Q's block t from Ψ'_t in registers (wg_iw_Q's arithmetic)
      const int s0 = kIwBlockStart[t];
      const double dn = iw_q_den(nn_t, t);
      if (kIwBlockDim[t] == 1) {
        Qp[s0 * kDZ + s0] = fmax(Pp[0] / dn, eps_psd);
      } else {
        double A2[9], P2[9];
        for (int k = 0; k < 9; ++k) A2[k] = Pp[k] / dn;
        psd_project3_fast(A2, eps_psd, P2, nullptr);
        for (int i = 0; i < 3; ++i)
          for (int j = 0; j < 3; ++j) Qp[(s0 + i) * kDZ + (s0 + j)] = P2[3 * i + j];
      }
    }
  }
  if (t < 36) {
    blk[t] = kIwRhoProc[6] * Psi[6 * 36 + t] + w * dPsi[6 * 36 + t];
    if (raw_out) raw_out[6 * 36 + t] = blk[t];
  }
  __syncthreads();
  if constexpr (WITH_Q) {
    const double d6 = iw_q_den(tab[24 + 6], 6);
    // wave 2: X = sym(M_6) / den_6 (= Ψ'_6 / den_6 under the shortcut) and the Cholesky of X − εI formed as
    // wg_psd_project_fast forms it (X is exactly symmetric, so its symmetrisation is X itself)
    const auto spec = [&]() {
      const int l = threadIdx.x & 63;
      if (l < 36) {
        const int i = l / 6, j = l % 6;
        X[l] = (0.5 * (blk[6 * i + j] + blk[6 * j + i])) / d6;
      }
      wave_lds_sync();
      if (l < 36) {
        const int i = l / 6, j = l % 6;
        X[36 + l] = 0.5 * (X[6 * i + j] + X[6 * j + i]) - ((i == j) ? eps_psd : 0.0);
      }
      wave_lds_sync();
      const bool ok = wave0_chol<8, true>(X + 36, 6);
      if (l == 0) X[72] = ok ? 0.0 : 1.0;
    };
    wg_psd_project_fast(blk, blkp, eps_psd, 6, Sx, red, c6, spec);
    const bool shortcut = c6[2] != c6[2];  // the apply's projection is sym(M_6) (eigen fields not computed)
    const bool q_ok = shortcut && X[72] == 0.0;
    __syncthreads();
    if (q_ok) {
      if (t < 36) Qp[(16 + t / 6) * kDZ + 16 + t % 6] = X[t];
    } else {  // wg_iw_Q's 6x6 form on the apply's result
      if (t < 36) X[t] = blkp[t] / d6;
      __syncthreads();
      wg_psd_project_fast(X, X + 36, eps_psd, 6, Sx, red, nullptr);
      if (t < 36) Qp[(16 + t / 6) * kDZ + 16 + t % 6] = X[36 + t];
    }
    __syncthreads();
    for (int idx = t; idx < kNN; idx += kWG) Q_out[idx] = Qp[idx];
  } else {
    wg_psd_project_fast(blk, blkp, eps_psd, 6, Sx, red, c6);
  }
  for (int k = t; k < 6 * 36; k += kWG) Psi_out[k] = Qs[k];
  if (t < 36) Psi_out[6 * 36 + t] = blkp[t];
  if (t < 7) nu_out[t] = tab[24 + t];
  __syncthreads();
  if (t == 0 && cert) {
    double pd = c6[0], na = 0.0;
    for (int b = 0; b < 6; ++b) pd += tab[8 + b];
    for (int b = 0; b < 7; ++b) na += tab[16 + b];
    cert[0] = pd;
    cert[1] = na;
  }
  __syncthreads();
}

// Measurement-noise IW apply (measurement_noise_iw_jax.py:59-100), threads 0..2 (one block each):
// Ψ' = PSD(sym(ρ Ψ + dΨ)), ν' = proj(ρ ν + dν). tab: 6 doubles; cert (thread 0) = [Σ psd Δ, Σ |Δν|].
GC_DEV void wg_iw_meas_apply(const double* nu, const double* Psi, const double* dPsi, const double* dnu,
                             double eps_psd, double nu_max, double* nu_out, double* Psi_out, double* cert,
                             double* tab, double* raw_out = nullptr) {
  const int t = threadIdx.x;
  if (t < 3) {
    double Mr[9], Mp[9], cc[6], Ms[9];
    for (int k = 0; k < 9; ++k) Mr[k] = kIwRhoMeas[t] * Psi[t * 9 + k] + dPsi[t * 9 + k];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Ms[3 * i + j] = 0.5 * (Mr[3 * i + j] + Mr[3 * j + i]);
    psd_project3_fast(Ms, eps_psd, Mp, cc);
    if (raw_out)
      for (int k = 0; k < 9; ++k) raw_out[t * 9 + k] = Ms[k];
    const double nr = kIwRhoMeas[t] * nu[t] + dnu[t];
    const double nn = nu_project(nr, 3.0, nu_max);
    tab[t] = cc[0];
    tab[3 + t] = fabs(nn - nr);
    for (int k = 0; k < 9; ++k) Psi_out[t * 9 + k] = Mp[k];
    nu_out[t] = nn;
  }
  __syncthreads();
  if (t == 0 && cert) {
    cert[0] = tab[0] + tab[1] + tab[2];
    cert[1] = tab[3] + tab[4] + tab[5];
  }
  __syncthreads();
}

// process_noise_state_to_Q_jax (inverse_wishart_jax.py:35-68). Q is block diagonal (the masked
// 6x6 patches overwrite each other's zero padding), so its PSD projection is the direct sum of
// the active blocks' projections: 3x3 blocks in registers, the 6x6 extrinsic block on the WG.
// Q_out: global 22x22. Scratch: Qs (72), Qp (n²), Sx (2*36+24), red (16).
GC_DEV void wg_iw_Q(const double* nu, const double* Psi, double eps_psd, double* Q_out, double* Qs, double* Qp,
                    double* Sx, double* red) {
  const int t = threadIdx.x, n = kDZ;
  for (int idx = t; idx < kNN; idx += kWG) Qp[idx] = 0.0;
  __syncthreads();
  auto den = [&](int b) { return iw_q_den(nu[b], b); };
  if (t < 6) {
    const int b = t, d = kIwBlockDim[b], s0 = kIwBlockStart[b];
    const double dn = den(b);
    if (d == 1) {
      Qp[s0 * n + s0] = fmax(Psi[b * 36] / dn, eps_psd);
    } else {
      double A[9], Pp[9];
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) A[3 * i + j] = Psi[b * 36 + 6 * i + j] / dn;
      psd_project3_fast(A, eps_psd, Pp, nullptr);
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Qp[(s0 + i) * n + (s0 + j)] = Pp[3 * i + j];
    }
  }
  const double d6 = den(6);
  for (int idx = t; idx < 36; idx += kWG) Qs[idx] = Psi[6 * 36 + idx] / d6;
  __syncthreads();
  double* Q6 = Qs + 36;
  wg_psd_project_fast(Qs, Q6, eps_psd, 6, Sx, red, nullptr);
  for (int idx = t; idx < 36; idx += kWG) Qp[(16 + idx / 6) * n + (16 + idx % 6)] = Q6[idx];
  __syncthreads();
  for (int idx = t; idx < kNN; idx += kWG) Q_out[idx] = Qp[idx];
  __syncthreads();
}

}  // namespace gc
