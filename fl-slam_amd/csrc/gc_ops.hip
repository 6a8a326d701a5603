// gc_ops.hip — per-operator batched entries (include/gcslam.h "Per-operator entries"):
// each reference operator of the hot path as one launch over H independent items (one
// 256-thread workgroup per hypothesis, 22x22 algebra in LDS), running the same device code as
// the batched scan pipeline (gc_opsdev.h). The Python operator mirror (gcslam.ops) calls these
// with H = 1 for the reference's per-hypothesis call sites.
//
//  a2  predict_diffusion                  backend/operators/predict.py:43-214
//  a3  smooth_window_weights, preintegrate_imu_relative_pose_jax   imu_preintegration.py:19-147
//  a7  matrix_fisher_rotation_evidence    archive/legacy_operators/matrix_fisher_evidence.py:83-394
//  a8  planar_translation_evidence        matrix_fisher_evidence.py:413-671
//  a9  compute/apply_excitation_prior_scaling   backend/operators/excitation.py:14-64
//  a10 fusion_scale_from_certificates     backend/operators/fusion.py:46-142
//  a11 info_fusion_additive               backend/operators/fusion.py:150-230
//  a12 pose_update_frobenius_recompose    backend/operators/recompose.py:50-205
//  a14 anchor_drift_update                backend/operators/anchor_drift.py:93-191
//  a15 process/measurement-noise IW       inverse_wishart_jax.py:35-185, measurement_noise_iw_jax.py:59-218
//  a16 hypothesis_barycenter_projection   backend/operators/hypothesis.py:51-236
//  a17 BeliefGaussianInfo.mean_increment / world pose   common/belief.py:373-425
#include <hip/hip_runtime.h>
#include "gc_internal.h"
#include "gc_opsdev.h"
#include "gc_cond.h"

namespace gc {

namespace {

constexpr int N = kDZ;
constexpr double kGravity[3] = {0.0, 0.0, -9.81};

// Bump allocator over the dynamic LDS block.
struct Arena {
  double* p;
  GC_DEV double* take(int n) {
    double* r = p;
    p += n;
    return r;
  }
};

GC_DEV void load_mat(double* dst, const double* src) {
  for (int i = threadIdx.x; i < kNN; i += kWG) dst[i] = src[i];
}
GC_DEV void load_vec(double* dst, const double* src, int n) {
  if ((int)threadIdx.x < n) dst[threadIdx.x] = src[threadIdx.x];
}

// ------------------------------------------------------------------ a17 mean + world pose
__global__ void __launch_bounds__(256) k_op_world_pose(const double* X, const double* L, const double* h,
                                                       double eps_lift, double* pose, double* mean) {
  extern __shared__ double sm[];
  Arena a{sm};
  double* Ls = a.take(kNN);
  double* C = a.take(kNN);
  double* hs = a.take(N);
  double* mu = a.take(N);
  const int k = blockIdx.x, t = threadIdx.x;
  load_mat(Ls, L + (int64_t)k * kNN);
  load_vec(hs, h + (int64_t)k * N, N);
  __syncthreads();
  wg_solve_lifted(Ls, hs, mu, eps_lift, N, C);
  if (mean && t < N) mean[(int64_t)k * N + t] = mu[t];
  if (t == 0 && pose) {
    double e[6];
    se3_exp(mu, e);
    se3_compose(X + (int64_t)k * 6, e, pose + (int64_t)k * 6);
  }
}

// ------------------------------------------------------------------ a17 lifted inverse
// spd_cholesky_inverse_lifted_core (primitives.py:169-192): (L + ε I)⁻¹ by the Cholesky factor and
// C⁻ᵀ C⁻¹ (the pipeline's routines: wg_inverse_lifted), n <= 22, one workgroup per matrix
__global__ void __launch_bounds__(256) k_op_inverse_lifted(int n, const double* L, double eps_lift, double* out) {
  extern __shared__ double sm[];
  double* Ls = sm;
  double* W = Ls + n * n;
  double* W2 = W + n * n;
  const int k = blockIdx.x, t = threadIdx.x;
  for (int i = t; i < n * n; i += kWG) Ls[i] = L[(int64_t)k * n * n + i];
  __syncthreads();
  double* Linv = W2 + n * n;
  wg_inverse_lifted(Ls, Linv, eps_lift, n, W, W2);
  for (int i = t; i < n * n; i += kWG) out[(int64_t)k * n * n + i] = Linv[i];
}

// --------------------------------------------------------------------------------- a2
__global__ void __launch_bounds__(256) k_op_predict(const double* L, const double* h, const double* Q, double dt,
                                                    double eps_psd, double eps_lift, double lambda_ou,
                                                    double* L_out, double* h_out, double* cert) {
  extern __shared__ double sm[];
  Arena a{sm};
  double* Lp = a.take(kNN);
  double* Lo = a.take(kNN);
  double* W1 = a.take(kNN);
  double* W2 = a.take(kNN);
  double* W3 = a.take(kNN);
  double* Sx = a.take(2 * kNN + 4 * N);
  double* hp = a.take(N);
  double* ho = a.take(N);
  double* mu = a.take(N);
  double* red = a.take(16);
  double* c1 = a.take(8);
  double* c2 = a.take(8);
  const int k = blockIdx.x, t = threadIdx.x;
  load_mat(Lp, L + (int64_t)k * kNN);
  load_vec(hp, h + (int64_t)k * N, N);
  __syncthreads();
  // the pipeline's Cholesky-certified projections, then the reference's ConditioningCert of L_pred
  // (predict.py:183-188) by Sturm counts when the second clamp is inactive (gc_cond.h)
  double* ck = cert + (int64_t)k * kPredCertLen;
  wg_predict(Lp, hp, Q, dt, eps_psd, eps_lift, lambda_ou, Lo, ho, mu, ck, W1, W2, W3, Sx, red, c1, c2);
  if (c2[2] != c2[2]) {  // NaN: the shortcut was taken (wg_predict ends with a barrier)
    if (t < 64) wave_conditioning<kDZ>(Lo, eps_psd, Sx, c2 + 2);
    __syncthreads();
    if (t == 0)
      for (int q = 2; q < 6; ++q) ck[q] = c2[q];
  }
  for (int i = t; i < kNN; i += kWG) L_out[(int64_t)k * kNN + i] = Lo[i];
  if (t < N) h_out[(int64_t)k * N + t] = ho[t];
}

// --------------------------------------------------------------------------------- a3
__global__ void k_op_window_weights(int M, const double* stamps, double t0, double t1, double sigma, double* w) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < M) w[i] = window_weight(stamps[i], t0, t1, sigma);
}

constexpr int kPreintOut = 32;
// out: [delta_pose 6, delta_R 9, p_body 3, v_body 3, ess, a_body_mean 3, a_world_nog_mean 3,
//       a_world_mean 3, dt_eff_sum]
__global__ void __launch_bounds__(256) k_op_preintegrate(int M, const double* stamps, const double* gyro,
                                                         const double* accel, const double* w, int64_t w_stride,
                                                         const double* rotvec0, const double* bg, const double* ba,
                                                         double g0, double g1, double g2, double* out) {
  extern __shared__ double sm[];
  Arena a{sm};
  double* A = a.take(256 * 9);
  double* Bm = a.take(256 * 9);
  double* V1 = a.take(256 * 3);
  double* V2 = a.take(256 * 3);
  double* red = a.take(16);
  double* pre = a.take(kPreint);
  double* R0 = a.take(9);
  const int k = blockIdx.x, t = threadIdx.x;
  const double* wk = w + (int64_t)k * w_stride;
  if (t == 0) so3_exp(rotvec0 + 3 * k, R0);
  __syncthreads();
  const int ia = 2 * t, ib = 2 * t + 1;
  const double wa = ia < M ? wk[ia] : 0.0, wb = ib < M ? wk[ib] : 0.0;
  const double g[3] = {g0, g1, g2};
  const ImuPair q = load_imu_pair(M, stamps, gyro, accel);
  wg_preintegrate(M, q, wa, wb, R0, bg + 3 * k, ba + 3 * k, g, A, Bm, V1, V2, pre);
  double ess_l = 0.0;
  for (int i = t; i < M; i += kWG) ess_l += wk[i];
  const double ess = wg_sum(ess_l, red);
  if (t == 0) {
    double* o = out + (int64_t)k * kPreintOut;
    double dR[9], pb[3], vb[3];
    mat3_mul_tn(R0, pre, dR);
    mat3_tvec(R0, pre + 9, pb);
    mat3_tvec(R0, pre + 12, vb);
    for (int q = 0; q < 3; ++q) o[q] = pb[q];
    so3_log(dR, o + 3);
    for (int q = 0; q < 9; ++q) o[6 + q] = dR[q];
    for (int q = 0; q < 3; ++q) { o[15 + q] = pb[q]; o[18 + q] = vb[q]; }
    o[21] = ess;
    const double den = fmax(pre[15], 1e-12);
    for (int q = 0; q < 3; ++q) {
      o[22 + q] = pre[16 + q] / den;
      o[25 + q] = pre[19 + q] / den;
      o[28 + q] = pre[22 + q] / den;
    }
    o[31] = pre[15];
  }
}

// IMU measurement-noise IW statistics (measurement_noise_iw_jax.py:130-218), per hypothesis:
// r = (ω_i − b_g) − ω̄ (gyro) and r = (a_i − b_a) − f_pred, f_pred = −R0ᵀ g (accel);
// dΨ = PSD(sym(Σ w̃_i r rᵀ)) · max(dt_imu, 1e-12), w̃ = w / (Σw + ε). out (H, 18) = [gyro 9, accel 9].
__global__ void __launch_bounds__(256) k_op_imu_meas_stats(int M, const double* gyro, const double* accel,
                                                           const double* w, const double* bg, const double* ba,
                                                           const double* omega, const double* rotvec0, double dt_imu,
                                                           double eps_mass, double eps_psd, double* out) {
  __shared__ double red[16];
  __shared__ double fp[3];
  const int k = blockIdx.x, t = threadIdx.x;
  if (t == 0) {
    double R0[9];
    so3_exp(rotvec0 + 3 * k, R0);
    for (int i = 0; i < 3; ++i)
      fp[i] = -(R0[i] * kGravity[0] + R0[3 + i] * kGravity[1] + R0[6 + i] * kGravity[2]);
  }
  __syncthreads();
  double sw = 0.0;
  for (int i = t; i < M; i += kWG) sw += w[i];
  const double wsum = wg_sum(sw, red) + eps_mass;
  double rr[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = t; i < M; i += kWG) {
    const double wn = w[i] / wsum;
    double rg[3], ra[3];
    for (int q = 0; q < 3; ++q) {
      rg[q] = (gyro[3 * i + q] - bg[3 * k + q]) - omega[3 * k + q];
      ra[q] = (accel[3 * i + q] - ba[3 * k + q]) - fp[q];
    }
    int q = 0;
    for (int a = 0; a < 3; ++a)
      for (int b = a; b < 3; ++b, ++q) {
        rr[q] += wn * rg[a] * rg[b];
        rr[6 + q] += wn * ra[a] * ra[b];
      }
  }
  for (int q = 0; q < 12; ++q) rr[q] = wg_sum(rr[q], red);
  if (t == 0) {
    for (int blk = 0; blk < 2; ++blk) {
      const double* r = rr + 6 * blk;
      const double M3[9] = {r[0], r[1], r[2], r[1], r[3], r[4], r[2], r[4], r[5]};
      double Pp[9];
      psd_project3(M3, eps_psd, Pp, nullptr);
      for (int q = 0; q < 9; ++q) out[(int64_t)k * 18 + 9 * blk + q] = Pp[q] * fmax(dt_imu, 1e-12);
    }
  }
}

// --------------------------------------------------------------------------------- a7
constexpr int kScatter = 17;  // [eigenvalues 3 (desc), eigenvectors 9 (columns), lin, plan, sph, aniso, eff_rank]
constexpr int kMFOut = kMF + 2 * kScatter;
// compute_scatter_metrics (matrix_fisher_evidence.py:83-147) of Σ_b S_b / (Σ_b N_b + ε).
GC_DEV void scatter_metrics(const double* Ssum, double Ntot, double eps, double* o) {
  double T[9], w[3], V[9];
  for (int q = 0; q < 9; ++q) T[q] = Ssum[q] * (1.0 / (Ntot + eps));
  eigh3(T, w, V);
  int idx[3] = {0, 1, 2};  // descending order
  for (int i = 0; i < 3; ++i)
    for (int j = i + 1; j < 3; ++j)
      if (w[idx[j]] > w[idx[i]]) { const int tmp = idx[i]; idx[i] = idx[j]; idx[j] = tmp; }
  double lam[3];
  for (int i = 0; i < 3; ++i) {
    lam[i] = fmax(w[idx[i]], 0.0);
    o[i] = lam[i];
    for (int r = 0; r < 3; ++r) o[3 + 3 * r + i] = V[3 * r + idx[i]];
  }
  const double il = 1.0 / (lam[0] + eps);
  const double tot = lam[0] + lam[1] + lam[2] + eps;
  double ent = 0.0;
  for (int i = 0; i < 3; ++i) {
    const double p = lam[i] / tot;
    ent -= p * log(p + eps);
  }
  o[12] = (lam[0] - lam[1]) * il;
  o[13] = (lam[1] - lam[2]) * il;
  o[14] = lam[2] * il;
  o[15] = 1.0 - lam[2] * il;
  o[16] = exp(ent);
}

__global__ void __launch_bounds__(256) k_op_matrix_fisher(int B, const double* pose, const double* s_dir,
                                                          const double* s_N, const double* s_S, const double* m_dir,
                                                          const double* m_N, const double* m_S, double eps_psd,
                                                          double eps, double* out) {
  __shared__ double tab[64 * 10];
  __shared__ double acc[32];
  const int k = blockIdx.x, t = threadIdx.x;
  const int64_t kb = (int64_t)k * B;
  if (t < B) mf_bin_row(s_N[kb + t], s_dir + 3 * (kb + t), m_N[t], m_dir + 3 * t, eps, tab + t * 10);
  __syncthreads();
  if (t < 10) {
    double s = 0.0;
    for (int b = 0; b < B; ++b) s += tab[b * 10 + t];
    acc[t] = s;
  }
  // summed scatter matrices and masses for the metrics (fixed bin order)
  if (t >= 32 && t < 32 + 10) {
    const int q = t - 32;
    double ss = 0.0, sm = 0.0;
    for (int b = 0; b < B; ++b) {
      ss += (q < 9) ? (s_S ? s_S[9 * (kb + b) + q] : 0.0) : s_N[kb + b];
      sm += (q < 9) ? (m_S ? m_S[9 * b + q] : 0.0) : m_N[b];
    }
    acc[12 + q] = ss;
    acc[22 + q] = sm;
  }
  __syncthreads();
  double* o = out + (int64_t)k * kMFOut;
  if (t == 0) {
    double Rp[9];
    so3_exp(pose + 6 * k + 3, Rp);
    mf_finalize(acc, Rp, eps, eps_psd, o);
  } else if (t == 1) {
    scatter_metrics(acc + 22, acc[31], eps, o + kMF);              // map
  } else if (t == 2) {
    scatter_metrics(acc + 12, acc[21], eps, o + kMF + kScatter);   // scan
  }
}

// --------------------------------------------------------------------------------- a8
__global__ void __launch_bounds__(256) k_op_planar(int B, const double* pose, const double* R_hat,
                                                   const double* s_pbar, const double* s_Sig, const double* s_N,
                                                   const double* m_c, const double* m_Sig, const double* m_Npos,
                                                   const double* m_S, const double* m_Nd, double eps_psd,
                                                   double eps, double* out) {
  __shared__ double tab[64 * 13];
  __shared__ double acc[16];
  __shared__ double zs[12];
  const int k = blockIdx.x, t = threadIdx.x;
  const int64_t kb = (int64_t)k * B;
  if (t < B)
    planar_bin_row(R_hat + 9 * k, s_N[kb + t], s_pbar + 3 * (kb + t), s_Sig + 9 * (kb + t), m_Npos[t], m_c + 3 * t,
                   m_Sig + 9 * t, eps, tab + t * 13);
  if (t >= 64 && t < 64 + 10) {
    const int q = t - 64;
    double s = 0.0;
    for (int b = 0; b < B; ++b) s += (q < 9) ? m_S[9 * b + q] : m_Nd[b];
    zs[q] = s;
  }
  __syncthreads();
  if (t < 13) {
    double s = 0.0;
    for (int b = 0; b < B; ++b) s += tab[b * 13 + t];
    acc[t] = s;
  }
  __syncthreads();
  if (t == 0) {
    const double zsc = planar_z_scale(zs, zs[9], eps);
    planar_finalize(acc, zsc, pose + 6 * k, eps, eps_psd, out + (int64_t)k * kPT);
  }
}

// --------------------------------------------------------------------------------- a9
// s_dt = e_dt/(e_dt + π_dt + ε), s_ex likewise on the extrinsic trace; the prior's rows/cols 15
// and 16..21 scale by (1 − s). s_out (H, 2); with L_ev == NULL it is an input (apply only).
__global__ void __launch_bounds__(256) k_op_excitation(const double* L_ev, const double* L_prior,
                                                       const double* h_prior, double eps, double* s_out,
                                                       double* L_out, double* h_out) {
  __shared__ double s2[2];
  const int k = blockIdx.x, t = threadIdx.x;
  const double* Lp = L_prior + (int64_t)k * kNN;
  if (t == 0 && !L_ev) {  // apply-only: the scales come in through s_out
    s2[0] = s_out[2 * k];
    s2[1] = s_out[2 * k + 1];
  } else if (t == 0) {
    const double* Le = L_ev + (int64_t)k * kNN;
    double eex = 0.0, pex = 0.0;
    for (int q = 16; q < 22; ++q) { eex += Le[q * N + q]; pex += Lp[q * N + q]; }
    const double edt = Le[15 * N + 15], pdt = Lp[15 * N + 15];
    s2[0] = edt / (edt + pdt + eps);
    s2[1] = eex / (eex + pex + eps);
    s_out[2 * k] = s2[0];
    s_out[2 * k + 1] = s2[1];
  }
  __syncthreads();
  auto f = [&](int i) { return i == 15 ? 1.0 - s2[0] : (i >= 16 ? 1.0 - s2[1] : 1.0); };
  for (int idx = t; idx < kNN; idx += kWG) {
    const int i = idx / N, j = idx % N;
    double v = Lp[idx];
    if (i >= 15) v = f(i) * v;
    if (j >= 15) v = f(j) * v;
    L_out[(int64_t)k * kNN + idx] = v;
  }
  if (t < N) h_out[(int64_t)k * N + t] = f(t) * h_prior[(int64_t)k * N + t];
}

// -------------------------------------------------------------------------------- a10
// rows (H, 8) = [cond, ess_total, support_frac, excitation_total, dt_asymmetry, z_to_xy_ratio,
// power_beta, nll_per_ess]; out (H, 4) = [alpha, excitation_total, ess_to_excitation, cond_to_support].
__global__ void k_op_fusion_scale(int H, const double* rows, double amin, double amax, double c0, double eps_mass,
                                  double* out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= H) return;
  const double* r = rows + 8 * k;
  const double cond = r[0], ess = r[1], sf = r[2], exc = r[3], dta = r[4], zxy = r[5], pb = r[6], nll = r[7];
  double q = sqrt((c0 / (cond + c0)) * (ess / (ess + 1.0)));
  q *= exp(-nll) * clampd(dta, 0.0, 1.0);
  q *= clampd(zxy / (zxy + 1.0), 0.0, 1.0) * clampd(exc / (exc + 1.0), 0.0, 1.0);
  q *= clampd(pb, 0.0, 1.0);
  double* o = out + 4 * k;
  o[0] = clampd(amin + (amax - amin) * q, amin, amax);
  o[1] = exc;
  o[2] = ess / (exc + eps_mass);
  o[3] = cond / (sf + eps_mass);
}

// -------------------------------------------------------------------------------- a11
__global__ void __launch_bounds__(256) k_op_info_fusion(const double* L_pred, const double* h_pred,
                                                        const double* L_ev, const double* h_ev, const double* alpha,
                                                        double eps_psd, double* L_out, double* h_out, double* cert) {
  extern __shared__ double sm[];
  Arena a{sm};
  double* W = a.take(kNN);
  double* Lo = a.take(kNN);
  double* Sx = a.take(2 * kNN + 4 * N);
  double* red = a.take(16);
  double* c6 = a.take(8);
  const int k = blockIdx.x, t = threadIdx.x;
  const double al = alpha[k];
  for (int i = t; i < kNN; i += kWG) W[i] = L_pred[(int64_t)k * kNN + i] + al * L_ev[(int64_t)k * kNN + i];
  __syncthreads();
  wg_psd_project_certified(W, Lo, eps_psd, Sx, red, c6);
  for (int i = t; i < kNN; i += kWG) L_out[(int64_t)k * kNN + i] = Lo[i];
  if (t < N) h_out[(int64_t)k * N + t] = h_pred[(int64_t)k * N + t] + al * h_ev[(int64_t)k * N + t];
  if (t < 6) cert[6 * k + t] = c6[t];
}

// -------------------------------------------------------------------------- a12 / a14
// mode 0: recompose (res 19 = [δ' 6, X_new 6, s, bch 6]); mode 1: anchor drift (res 3 = [ρ, drift_m, drift_r]).
__global__ void __launch_bounds__(256) k_op_recompose_drift(int mode, const double* X, const double* z, const double* L,
                                                            const double* h, const double* T, double c_frob,
                                                            double eps_lift, double* X_out, double* z_out,
                                                            double* h_out, double* res) {
  extern __shared__ double sm[];
  Arena a{sm};
  double* Ls = a.take(kNN);
  double* C = a.take(kNN);
  double* hs = a.take(N);
  double* zs = a.take(N);
  double* dz = a.take(N);
  double* sh = a.take(N);
  double* zo = a.take(N);
  double* sc = a.take(32);
  const int k = blockIdx.x, t = threadIdx.x;
  load_mat(Ls, L + (int64_t)k * kNN);
  load_vec(hs, h + (int64_t)k * N, N);
  load_vec(zs, z + (int64_t)k * N, N);
  __syncthreads();
  wg_solve_lifted(Ls, hs, dz, eps_lift, N, C);
  if (t == 0) {
    if (mode == 0) {
      double bch[6];
      sc[12] = recompose_pose(X + 6 * k, zs, dz, T[k], c_frob, sc, sc + 6, bch);  // X_new, δ'
      double* r = res + 19 * k;
      for (int q = 0; q < 6; ++q) { r[q] = sc[6 + q]; r[6 + q] = sc[q]; r[13 + q] = bch[q]; }
      r[12] = sc[12];
    } else {
      double dm, dr;
      const double rho = drift_rho(dz, &dm, &dr);
      double d6[6], e[6];
      for (int q = 0; q < 6; ++q) d6[q] = rho * dz[q];
      se3_exp(d6, e);
      se3_compose(X + 6 * k, e, sc);
      sc[12] = rho;
      res[3 * k] = rho; res[3 * k + 1] = dm; res[3 * k + 2] = dr;
    }
  }
  __syncthreads();
  if (t < N) {
    if (mode == 0) {
      sh[t] = (t < 6) ? sc[6 + t] : 0.0;  // shift = δ' on the pose slice
      zo[t] = zs[t] - sh[t];
    } else {
      sh[t] = 0.0;
      zo[t] = (1.0 - sc[12]) * dz[t];
    }
  }
  __syncthreads();
  if (t < N) {
    double v = 0.0;
    if (mode == 0) {
      v = hs[t];
      for (int q = 0; q < 6; ++q) v -= Ls[t * N + q] * sh[q];
    } else {
      for (int q = 0; q < N; ++q) v += Ls[t * N + q] * zo[q];
    }
    h_out[(int64_t)k * N + t] = v;
    z_out[(int64_t)k * N + t] = zo[t];
  }
  if (t < 6) X_out[6 * k + t] = sc[t];
}

// -------------------------------------------------------------------------------- a15
__global__ void __launch_bounds__(256) k_op_iw_proc_stats(const double* L_pred, const double* h_pred,
                                                          const double* L_post, const double* h_post, double eps_lift,
                                                          double* dPsi, double* dnu) {
  extern __shared__ double sm[];
  Arena a{sm};
  double* Lq = a.take(kNN);
  double* Lp = a.take(kNN);
  double* C1 = a.take(kNN);
  double* C2 = a.take(kNN);
  double* Sp = a.take(kNN);
  double* W = a.take(kNN);
  double* hq = a.take(N);
  double* hp = a.take(N);
  double* mq = a.take(N);
  double* mp = a.take(N);
  const int k = blockIdx.x, t = threadIdx.x;
  load_mat(Lq, L_pred + (int64_t)k * kNN);
  load_mat(Lp, L_post + (int64_t)k * kNN);
  load_vec(hq, h_pred + (int64_t)k * N, N);
  load_vec(hp, h_post + (int64_t)k * N, N);
  __syncthreads();
  wg_solve_lifted(Lq, hq, mq, eps_lift, N, C1);
  wg_solve_lifted(Lp, hp, mp, eps_lift, N, C2);
  wg_chol_inverse(C2, Sp, W, N);
  for (int idx = t; idx < 7 * 36; idx += kWG) dPsi[(int64_t)k * 252 + idx] = iw_proc_stat(idx, mp, mq, Sp);
  if (t < 7) dnu[7 * k + t] = 1.0;
}

__global__ void __launch_bounds__(256) k_op_iw_proc_apply(const double* nu, const double* Psi, const double* dPsi,
                                                          const double* dnu, double eps_psd, double nu_max,
                                                          double* nu_out, double* Psi_out, double* cert) {
  __shared__ double Qs[216], blk[36], blkp[36], Sx[2 * 36 + 24], red[16], c6[8], tab[32];
  wg_iw_proc_apply(nu, Psi, dPsi, dnu, 1.0, eps_psd, nu_max, nu_out, Psi_out, cert, Qs, blk, blkp, Sx, red, c6, tab);
}

__global__ void __launch_bounds__(256) k_op_iw_meas_apply(const double* nu, const double* Psi, const double* dPsi,
                                                          const double* dnu, double eps_psd, double nu_max,
                                                          double* nu_out, double* Psi_out, double* cert) {
  __shared__ double tab[8];
  wg_iw_meas_apply(nu, Psi, dPsi, dnu, eps_psd, nu_max, nu_out, Psi_out, cert, tab);
}

__global__ void __launch_bounds__(256) k_op_iw_Q(const double* nu, const double* Psi, double eps_psd, double* Q) {
  extern __shared__ double sm[];
  Arena a{sm};
  double* Qs = a.take(72);
  double* Qp = a.take(kNN);
  double* Sx = a.take(2 * 36 + 24);
  double* red = a.take(16);
  wg_iw_Q(nu, Psi, eps_psd, Q, Qs, Qp, Sx, red);
}

// -------------------------------------------------------------------------------- a16
// Stage 1 (grid H): μ_j = (L_j + εI)⁻¹ h_j.
__global__ void __launch_bounds__(256) k_op_means(const double* L, const double* h, double eps_lift, double* mus) {
  extern __shared__ double sm[];
  Arena a{sm};
  double* Ls = a.take(kNN);
  double* C = a.take(kNN);
  double* hs = a.take(N);
  double* mu = a.take(N);
  const int k = blockIdx.x;
  load_mat(Ls, L + (int64_t)k * kNN);
  load_vec(hs, h + (int64_t)k * N, N);
  __syncthreads();
  wg_solve_lifted(Ls, hs, mu, eps_lift, N, C);
  if ((int)threadIdx.x < N) mus[(int64_t)k * N + threadIdx.x] = mu[threadIdx.x];
}
// Stage 2 (one workgroup): floored, renormalised weights; L = PSD(Σ w L_j), h, z_lin; spread;
// cert (16) = [floor_adjustment, spread, ess, support_frac, mass_eps, psd cert 6, pad].
__global__ void __launch_bounds__(256) k_op_barycenter(int H, const double* L, const double* h, const double* z,
                                                       const double* mus, const double* w, double floor, double eps_psd,
                                                       double* L_out, double* h_out, double* z_out, double* cert) {
  extern __shared__ double sm[];
  Arena a{sm};
  double* Lr = a.take(kNN);
  double* Lo = a.take(kNN);
  double* Sx = a.take(2 * kNN + 4 * N);
  double* red = a.take(16);
  double* c6 = a.take(8);
  double* mom = a.take(N);
  const int t = threadIdx.x;
  double lw = 0.0;
  for (int k = t; k < H; k += kWG) lw += fmax(w[k], floor);
  const double wsum = wg_sum(lw, red);
  for (int i = t; i < kNN; i += kWG) {
    double s = 0.0;
    for (int k = 0; k < H; ++k) s += (fmax(w[k], floor) / wsum) * L[(int64_t)k * kNN + i];
    Lr[i] = s;
  }
  if (t < N) {
    double sh = 0.0, sz = 0.0, sm_ = 0.0;
    for (int k = 0; k < H; ++k) {
      const double wn = fmax(w[k], floor) / wsum;
      sh += wn * h[(int64_t)k * N + t];
      sz += wn * z[(int64_t)k * N + t];
      sm_ += wn * mus[(int64_t)k * N + t];
    }
    h_out[t] = sh;
    z_out[t] = sz;
    mom[t] = sm_;
  }
  __syncthreads();
  wg_psd_project_certified(Lr, Lo, eps_psd, Sx, red, c6);
  for (int i = t; i < kNN; i += kWG) L_out[i] = Lo[i];
  double sp = 0.0, l2 = 0.0, lc = 0.0, la = 0.0;
  for (int k = t; k < H; k += kWG) {
    const double wf = fmax(w[k], floor), wn = wf / wsum;
    double d2 = 0.0;
    for (int i = 0; i < N; ++i) {
      const double d = mus[(int64_t)k * N + i] - mom[i];
      d2 += d * d;
    }
    sp += wn * d2;
    l2 += wn * wn;
    lc += (wn > floor) ? 1.0 : 0.0;
    la += fabs(wf - w[k]);
  }
  const double spread = wg_sum(sp, red), s2 = wg_sum(l2, red), cnt = wg_sum(lc, red), adj = wg_sum(la, red);
  if (t == 0) {
    cert[0] = adj; cert[1] = spread; cert[2] = 1.0 / s2; cert[3] = cnt / H; cert[4] = adj / H;
    for (int q = 0; q < 6; ++q) cert[5 + q] = c6[q];
    for (int q = 11; q < 16; ++q) cert[q] = 0.0;
  }
}

size_t lds_bytes(int doubles) { return sizeof(double) * (size_t)doubles; }
hipError_t allow_lds(const void* fn, size_t bytes) {
  return bytes > 65536 ? ensure_dyn_lds(fn, bytes) : hipSuccess;
}

}  // namespace
}  // namespace gc

using namespace gc;

#define GC_OP_CTX(ctx) GC_CHECK_ARG(nullptr, (ctx) != nullptr, "ctx is NULL")

extern "C" {

int32_t gc_belief_world_pose_batch(gc_ctx* ctx, int32_t H, const double* d_X, const double* d_L, const double* d_h,
                                   double eps_lift, double* d_pose_out, double* d_mean_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, H > 0 && d_X && d_L && d_h && (d_pose_out || d_mean_out), "bad arguments");
  const size_t sh = lds_bytes(2 * kNN + 2 * kDZ);
  hipLaunchKernelGGL(k_op_world_pose, dim3(H), dim3(256), sh, ctx->stream, d_X, d_L, d_h, eps_lift, d_pose_out,
                     d_mean_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_spd_inverse_lifted_batch(gc_ctx* ctx, int32_t H, int32_t n, const double* d_L, double eps_lift,
                                    double* d_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, H > 0 && n >= 1 && n <= kDZ && d_L && d_out, "bad arguments (n in [1, 22])");
  hipLaunchKernelGGL(k_op_inverse_lifted, dim3(H), dim3(256), lds_bytes(4 * n * n), ctx->stream, n, d_L, eps_lift,
                     d_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_predict_diffusion_batch(gc_ctx* ctx, int32_t H, const double* d_L, const double* d_h, const double* d_Q,
                                   double dt_sec, double eps_psd, double eps_lift, double lambda_ou, double* d_L_out,
                                   double* d_h_out, double* d_cert_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, H > 0 && d_L && d_h && d_Q && d_L_out && d_h_out && d_cert_out, "bad arguments");
  GC_CHECK_ARG(ctx, lambda_ou >= 0.0, "lambda_ou must be >= 0");
  const size_t sh = lds_bytes(5 * kNN + 2 * kNN + 4 * kDZ + 3 * kDZ + 32);
  GC_HIP(ctx, allow_lds((const void*)k_op_predict, sh));
  hipLaunchKernelGGL(k_op_predict, dim3(H), dim3(256), sh, ctx->stream, d_L, d_h, d_Q, dt_sec, eps_psd, eps_lift,
                     lambda_ou, d_L_out, d_h_out, d_cert_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_smooth_window_weights(gc_ctx* ctx, int32_t M, const double* d_stamps, double t0, double t1, double sigma,
                                 double* d_w_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, M >= 0 && d_stamps && d_w_out, "bad arguments");
  if (M == 0) return GC_OK;
  hipLaunchKernelGGL(k_op_window_weights, dim3((M + 255) / 256), dim3(256), 0, ctx->stream, M, d_stamps, t0, t1, sigma,
                     d_w_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_preintegrate_imu_batch(gc_ctx* ctx, int32_t H, int32_t M, const double* d_stamps, const double* d_gyro,
                                  const double* d_accel, const double* d_weights, int64_t weights_stride,
                                  const double* d_rotvec0, const double* d_gyro_bias, const double* d_accel_bias,
                                  const double* h_gravity3, double* d_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, H > 0 && M >= 1 && M <= 512, "need H > 0 and 1 <= M <= 512");
  GC_CHECK_ARG(ctx, d_stamps && d_gyro && d_accel && d_weights && d_rotvec0 && d_gyro_bias && d_accel_bias && d_out,
               "NULL buffer");
  GC_CHECK_ARG(ctx, weights_stride == 0 || weights_stride >= M, "weights_stride must be 0 or >= M");
  const double g0 = h_gravity3 ? h_gravity3[0] : kGravity[0], g1 = h_gravity3 ? h_gravity3[1] : kGravity[1],
               g2 = h_gravity3 ? h_gravity3[2] : kGravity[2];
  const size_t sh = lds_bytes(256 * 24 + 16 + kPreint + 9);
  GC_HIP(ctx, allow_lds((const void*)k_op_preintegrate, sh));
  hipLaunchKernelGGL(k_op_preintegrate, dim3(H), dim3(256), sh, ctx->stream, M, d_stamps, d_gyro, d_accel, d_weights,
                     weights_stride, d_rotvec0, d_gyro_bias, d_accel_bias, g0, g1, g2, d_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_imu_meas_iw_suffstats_batch(gc_ctx* ctx, int32_t H, int32_t M, const double* d_gyro, const double* d_accel,
                                       const double* d_weights, const double* d_gyro_bias, const double* d_accel_bias,
                                       const double* d_omega_avg, const double* d_rotvec0, double dt_imu,
                                       double eps_mass, double eps_psd, double* d_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, H > 0 && M >= 1, "need H > 0 and M >= 1");
  GC_CHECK_ARG(ctx, d_gyro && d_accel && d_weights && d_gyro_bias && d_accel_bias && d_omega_avg && d_rotvec0 && d_out,
               "NULL buffer");
  hipLaunchKernelGGL(k_op_imu_meas_stats, dim3(H), dim3(256), 0, ctx->stream, M, d_gyro, d_accel, d_weights,
                     d_gyro_bias, d_accel_bias, d_omega_avg, d_rotvec0, dt_imu, eps_mass, eps_psd, d_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_matrix_fisher_batch(gc_ctx* ctx, int32_t H, int32_t B, const double* d_pose_pred, const double* d_scan_s_dir,
                               const double* d_scan_N, const double* d_scan_S_dir_scatter, const double* d_map_S_dir,
                               const double* d_map_N_dir, const double* d_map_S_dir_scatter, double eps_psd,
                               double eps_mass, double* d_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, H > 0 && B >= 1 && B <= 64, "need H > 0 and 1 <= B <= 64");
  GC_CHECK_ARG(ctx, d_pose_pred && d_scan_s_dir && d_scan_N && d_map_S_dir && d_map_N_dir && d_out, "NULL buffer");
  hipLaunchKernelGGL(k_op_matrix_fisher, dim3(H), dim3(256), 0, ctx->stream, B, d_pose_pred, d_scan_s_dir, d_scan_N,
                     d_scan_S_dir_scatter, d_map_S_dir, d_map_N_dir, d_map_S_dir_scatter, eps_psd, eps_mass, d_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_planar_translation_batch(gc_ctx* ctx, int32_t H, int32_t B, const double* d_pose_pred, const double* d_R_hat,
                                    const double* d_scan_p_bar, const double* d_scan_Sigma_p, const double* d_scan_N,
                                    const double* d_map_centroid, const double* d_map_Sigma_c,
                                    const double* d_map_N_pos, const double* d_map_S_dir_scatter,
                                    const double* d_map_N_dir, double eps_psd, double eps_mass, double* d_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, H > 0 && B >= 1 && B <= 64, "need H > 0 and 1 <= B <= 64");
  GC_CHECK_ARG(ctx, d_pose_pred && d_R_hat && d_scan_p_bar && d_scan_Sigma_p && d_scan_N && d_map_centroid &&
                        d_map_Sigma_c && d_map_N_pos && d_map_S_dir_scatter && d_map_N_dir && d_out,
               "NULL buffer");
  hipLaunchKernelGGL(k_op_planar, dim3(H), dim3(256), 0, ctx->stream, B, d_pose_pred, d_R_hat, d_scan_p_bar,
                     d_scan_Sigma_p, d_scan_N, d_map_centroid, d_map_Sigma_c, d_map_N_pos, d_map_S_dir_scatter,
                     d_map_N_dir, eps_psd, eps_mass, d_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_excitation_scaling_batch(gc_ctx* ctx, int32_t H, const double* d_L_ev, const double* d_L_prior,
                                    const double* d_h_prior, double eps, double* d_s_out, double* d_L_out,
                                    double* d_h_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, H > 0 && d_L_prior && d_h_prior && d_s_out && d_L_out && d_h_out, "bad arguments");
  hipLaunchKernelGGL(k_op_excitation, dim3(H), dim3(256), 0, ctx->stream, d_L_ev, d_L_prior, d_h_prior, eps, d_s_out,
                     d_L_out, d_h_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_fusion_scale_batch(gc_ctx* ctx, int32_t H, const double* d_rows, double alpha_min, double alpha_max,
                              double c0_cond, double eps_mass, double* d_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, H > 0 && d_rows && d_out, "bad arguments");
  GC_CHECK_ARG(ctx, alpha_min <= alpha_max, "alpha_min must be <= alpha_max");
  hipLaunchKernelGGL(k_op_fusion_scale, dim3((H + 63) / 64), dim3(64), 0, ctx->stream, H, d_rows, alpha_min, alpha_max,
                     c0_cond, eps_mass, d_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_info_fusion_additive_batch(gc_ctx* ctx, int32_t H, const double* d_L_pred, const double* d_h_pred,
                                      const double* d_L_ev, const double* d_h_ev, const double* d_alpha,
                                      double eps_psd, double* d_L_out, double* d_h_out, double* d_cert_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, H > 0 && d_L_pred && d_h_pred && d_L_ev && d_h_ev && d_alpha && d_L_out && d_h_out && d_cert_out,
               "bad arguments");
  const size_t sh = lds_bytes(4 * kNN + 4 * kDZ + 24);
  hipLaunchKernelGGL(k_op_info_fusion, dim3(H), dim3(256), sh, ctx->stream, d_L_pred, d_h_pred, d_L_ev, d_h_ev,
                     d_alpha, eps_psd, d_L_out, d_h_out, d_cert_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

static int32_t recompose_drift(gc_ctx* ctx, int mode, int32_t H, const double* d_X, const double* d_z,
                               const double* d_L, const double* d_h, const double* d_T, double c_frob, double eps_lift,
                               double* d_X_out, double* d_z_out, double* d_h_out, double* d_res) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, H > 0 && d_X && d_z && d_L && d_h && d_X_out && d_z_out && d_h_out && d_res, "bad arguments");
  GC_CHECK_ARG(ctx, mode == 1 || d_T, "T is NULL");
  const size_t sh = lds_bytes(2 * kNN + 5 * kDZ + 32);
  hipLaunchKernelGGL(k_op_recompose_drift, dim3(H), dim3(256), sh, ctx->stream, mode, d_X, d_z, d_L, d_h, d_T, c_frob,
                     eps_lift, d_X_out, d_z_out, d_h_out, d_res);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_recompose_batch(gc_ctx* ctx, int32_t H, const double* d_X, const double* d_z, const double* d_L,
                           const double* d_h, const double* d_T, double c_frob, double eps_lift, double* d_X_out,
                           double* d_z_out, double* d_h_out, double* d_res_out) {
  return recompose_drift(ctx, 0, H, d_X, d_z, d_L, d_h, d_T, c_frob, eps_lift, d_X_out, d_z_out, d_h_out, d_res_out);
}

int32_t gc_anchor_drift_batch(gc_ctx* ctx, int32_t H, const double* d_X, const double* d_z, const double* d_L,
                              const double* d_h, double eps_lift, double* d_X_out, double* d_z_out, double* d_h_out,
                              double* d_res_out) {
  return recompose_drift(ctx, 1, H, d_X, d_z, d_L, d_h, nullptr, 0.0, eps_lift, d_X_out, d_z_out, d_h_out, d_res_out);
}

int32_t gc_iw_process_suffstats_batch(gc_ctx* ctx, int32_t H, const double* d_L_pred, const double* d_h_pred,
                                      const double* d_L_post, const double* d_h_post, double eps_lift,
                                      double* d_dPsi_out, double* d_dnu_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, H > 0 && d_L_pred && d_h_pred && d_L_post && d_h_post && d_dPsi_out && d_dnu_out, "bad arguments");
  const size_t sh = lds_bytes(6 * kNN + 4 * kDZ);
  GC_HIP(ctx, allow_lds((const void*)k_op_iw_proc_stats, sh));
  hipLaunchKernelGGL(k_op_iw_proc_stats, dim3(H), dim3(256), sh, ctx->stream, d_L_pred, d_h_pred, d_L_post, d_h_post,
                     eps_lift, d_dPsi_out, d_dnu_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_iw_process_apply(gc_ctx* ctx, const double* d_nu, const double* d_Psi, const double* d_dPsi,
                            const double* d_dnu, double eps_psd, double nu_max, double* d_nu_out, double* d_Psi_out,
                            double* d_cert_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, d_nu && d_Psi && d_dPsi && d_dnu && d_nu_out && d_Psi_out && d_cert_out, "NULL buffer");
  hipLaunchKernelGGL(k_op_iw_proc_apply, dim3(1), dim3(256), 0, ctx->stream, d_nu, d_Psi, d_dPsi, d_dnu, eps_psd, nu_max,
                     d_nu_out, d_Psi_out, d_cert_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_iw_process_Q(gc_ctx* ctx, const double* d_nu, const double* d_Psi, double eps_psd, double* d_Q_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, d_nu && d_Psi && d_Q_out, "NULL buffer");
  hipLaunchKernelGGL(k_op_iw_Q, dim3(1), dim3(256), lds_bytes(72 + kNN + 96 + 16), ctx->stream, d_nu, d_Psi, eps_psd,
                     d_Q_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_iw_meas_apply(gc_ctx* ctx, const double* d_nu, const double* d_Psi, const double* d_dPsi,
                         const double* d_dnu, double eps_psd, double nu_max, double* d_nu_out, double* d_Psi_out,
                         double* d_cert_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, d_nu && d_Psi && d_dPsi && d_dnu && d_nu_out && d_Psi_out && d_cert_out, "NULL buffer");
  hipLaunchKernelGGL(k_op_iw_meas_apply, dim3(1), dim3(256), 0, ctx->stream, d_nu, d_Psi, d_dPsi, d_dnu, eps_psd, nu_max,
                     d_nu_out, d_Psi_out, d_cert_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_hypothesis_barycenter(gc_ctx* ctx, int32_t H, const double* d_L, const double* d_h, const double* d_z,
                                 const double* d_weights, double weight_floor, double eps_psd, double eps_lift,
                                 double* d_L_out, double* d_h_out, double* d_z_out, double* d_cert_out) {
  GC_OP_CTX(ctx);
  GC_CHECK_ARG(ctx, H > 0 && d_L && d_h && d_z && d_weights && d_L_out && d_h_out && d_z_out && d_cert_out,
               "bad arguments");
  void* scr;
  if (int rc = gc::scratch(ctx, sizeof(double) * (size_t)H * kDZ, &scr)) return rc;
  hipLaunchKernelGGL(k_op_means, dim3(H), dim3(256), lds_bytes(2 * kNN + 2 * kDZ), ctx->stream, d_L, d_h, eps_lift,
                     (double*)scr);
  GC_LAUNCH_CHECK(ctx);
  const size_t sh = lds_bytes(4 * kNN + 5 * kDZ + 24);
  hipLaunchKernelGGL(k_op_barycenter, dim3(1), dim3(256), sh, ctx->stream, H, d_L, d_h, d_z, (const double*)scr,
                     d_weights, weight_floor, eps_psd, d_L_out, d_h_out, d_z_out, d_cert_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

}  // extern "C"
