// gc_evidence.hip — per-hypothesis evidence, fusion and recompose (a7-a14), the IW process
// statistics (a15), and the per-scan combine (a16) + IW apply + map update, as batched
// one-workgroup-per-hypothesis kernels. See gc_belief.hip for the reference map.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include "gc_internal.h"
#include "gc_pipe.h"
#include "gc_wgla.h"
#include "gc_opsdev.h"
#include "gc_binfin.h"

namespace gc {

constexpr int NN = kDZ * kDZ;

GC_DEV void compose_exp2(const double* X, const double* d6, double* out) {
  double e[6];
  se3_exp(d6, e);
  se3_compose(X, e, out);
}

// Sum a per-bin table [B][W] (W <= 16) over bins into out[W] on wave 0: lane (q, c) = (lane / 16,
// lane % 16) sums column c over bins q, q + 4, ... in ascending order, then the four quarters are
// combined as (q0 + q1) + (q2 + q3) by two xor-shuffles (a fixed order: deterministic).
GC_DEV void sum_bins(const double* tab, int B, int W, double* out) {
  const int t = threadIdx.x;
  if (t < 64) {
    const int c = t & 15, q = t >> 4;
    double s = 0.0;
    if (c < W)
      for (int b = q; b < B; b += 4) s += tab[b * W + c];
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (t < W) out[t] = s;
  }
  __syncthreads();
}

// ==================================================================== a7 .. a15 per hypothesis
// cond6 = λ_max / λ_min of the pose-6 block, both floored at ε_psd (non-finite -> ε_psd); writes
// eigmin_pose6 to *eigmin
GC_DEV double pose6_cond(double lmin, double lmax, double eps_psd, double* eigmin) {
  const double mn = fmax(isfinite(lmin) ? lmin : eps_psd, eps_psd);
  const double mx = fmax(isfinite(lmax) ? lmax : eps_psd, eps_psd);
  *eigmin = mn;
  return mx / mn;
}

template <bool FOLD>
GC_DEV void evidence_body(const PipeDev& P, const ScanArgs& S) {
  extern __shared__ double sm[];
  double* Lpr = sm;          // L_pred
  double* Lev = Lpr + NN;    // L_raw -> L_ev
  double* Lps = Lev + NN;    // excitation-scaled prior
  double* Lpo = Lps + NN;    // L_post
  double* Wc = Lpo + NN;     // chol(L_post + εI)
  double* W2 = Wc + NN;      // scratch / Σ_post
  double* W3 = W2 + NN;      // scratch
  double* Sx = W3 + NN;      // 2NN + 4*22
  double* vec = Sx + 2 * NN + 4 * kDZ;  // 10 x 22
  double* red = vec + 10 * kDZ;         // 8
  double* tab = red + 8;                // 64 x 16 per-bin table (kEvidenceTabDoubles)
  double* acc = tab + kEvidenceTabDoubles;  // 32
  double* sc = acc + 32;                // 128 scalars
  double* c6 = sc + 128;                // 6
  double* mf = c6 + 6;                  // kMF  Matrix-Fisher record
  double* pt = mf + kMF;                // kPT  planar record
  const int hl = blockIdx.x;
  const int t = threadIdx.x;
  const int n = kDZ, B = P.B;
  double* hev = vec;
  double* hps = vec + kDZ;
  double* hpo = vec + 2 * kDZ;
  double* dz = vec + 3 * kDZ;
  double* mupo = vec + 5 * kDZ;
  double* mups = vec + 6 * kDZ;
  double* hfin = vec + 7 * kDZ;
  double* zl = vec + 8 * kDZ;
  double* mufin = vec + 9 * kDZ;
  const double eps = P.eps_mass;

  for (int i = t; i < NN; i += kWG) {
    Lpr[i] = P.Lpred[(int64_t)hl * NN + i];
    Lev[i] = P.io_L[(int64_t)hl * NN + i];
  }
  if (t < n) {
    hev[t] = P.io_h[(int64_t)hl * n + t];
    zl[t] = P.z[(int64_t)hl * n + t];
  }
  const double* st = P.stats + (int64_t)hl * B * 38;
  if constexpr (FOLD) {
    // the a6 finalize of this hypothesis folded in (scan_bins_pipeline, BinsFold): its chunk records
    // summed in chunk order (the split kernel's sums, bit for bit) into the per-bin table's space
    // (B * NF_BASE + REC_EXTRA doubles: the host folds only when fold_record_fits(B)), then one lane
    // per bin; the split kernel's ticket is published here (the bins have completed)
    if (hl == 0 && t == 0 && S.done_word)
      __hip_atomic_store(S.done_word, S.ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const int RL = B * NF_BASE + REC_EXTRA;
    // 11 chunks per batch: the 21-22 chunk records of C5 / H = 256 in two L2 round trips (8: three;
    // the same order and bits, 1.1897 -> 1.1890 ms at H = 256, tools/r4_ab_slots.sh)
    finalize_reduce<4, 11>(S.fin_part + (int64_t)hl * S.fin_chunks * RL, RL, B * NF_BASE + 1, S.fin_chunks, tab);
    __syncthreads();
    if (t < B) {
      double* ax = P.binaux + ((int64_t)hl * B + t) * 2;
      finalize_bin(tab + t * NF_BASE, NF_BASE, P.eps_psd, eps, P.stats + ((int64_t)hl * B + t) * GC_BIN_STATS, ax,
                   ax + 1);
    } else if (t == 64) {
      const double* ex = tab + B * NF_BASE;
      double* c = P.bincert + (int64_t)hl * GC_BIN_CERT;
      c[4] = ex[0] / (ex[3] + eps);
      c[5] = ex[1];
      c[6] = ex[2];
    }
    __syncthreads();  // the stats, aux and cert rows written above are read below (workgroup scope)
  }
  // a6 certificate of the bins (binning.py:285-324): the cross-bin reductions of the split finalize's
  // per-bin terms, on wave 0 in k_bins_finalize's wave_sum order (lane b = bin b, B <= 64); thread 0
  // reads them back below (its own writes)
  if (t < 64) {
    double Nl = 0.0, N2l = 0.0, psdl = 0.0, epsl = 0.0, sfl = 0.0;
    if (t < B) {
      const double N = st[t * 38];
      const double* ax = P.binaux + ((int64_t)hl * B + t) * 2;
      Nl = N; N2l = N * N; psdl = ax[0]; epsl = ax[1]; sfl = N / (N + eps);
    }
    const double Nt = wave_sum(Nl), N2 = wave_sum(N2l), psd = wave_sum(psdl), mer = wave_max(epsl),
                 sf = wave_sum(sfl);
    if (t == 0) {
      double* c = P.bincert + (int64_t)hl * 8;
      c[0] = Nt * Nt / (N2 + eps);
      c[1] = sf / (double)B;
      c[2] = psd;
      c[3] = mer;
      c[7] = psd + mer;
    }
  }
  GC_PHASE(P, 10);
  // ---------------------------------------------- a7 MatrixFisher: per-bin cross-covariance
  if (t < B) {
    const double* s = st + t * 38;
    const double* m = P.map + t * kMapRec;
    mf_bin_row(s[0], s + 1, m[12], m, eps, tab + t * 10);
  } else if (t == 64) {  // R_pred on wave 1 beside the per-bin rows (B <= 64)
    so3_exp(P.pose_pred + (int64_t)hl * 6 + 3, sc + 100);
  }
  __syncthreads();
  GC_PHASE(P, 30);
  sum_bins(tab, B, 10, acc);
  GC_PHASE(P, 31);
  // R_mf first; the rest of the MF record (information, δ, PSD, h) on wave 1 beside the planar rows,
  // which need only R_mf (mf_rotation / mf_information: the same operations as mf_finalize; evidence
  // 43.5 -> 39.4 us at H = 32, tools/r4_trace2.sh)
  if (t == 0) mf_rotation(acc, mf, sc + 116);
  __syncthreads();
  GC_PHASE(P, 11);
  // ---------------------------------------------- a8 planar translation WLS (R_hat = R_mf)
  if (t < B) {
    const double* s = st + t * 38;
    const double* m = P.map + t * kMapRec;
    const double* md = P.map_der + t * kMapDer;
    planar_bin_row(mf, s[0], s + 13, s + 16, m[13], md + 4, md + 7, eps, tab + t * 13);
  } else if (t == 64) {
    mf_information(acc, sc + 100, sc + 116, eps, P.eps_psd, mf);
  } else if (t == 128) {  // log R_mf for the tape on wave 2 beside the planar rows (B <= 64)
    so3_log(mf, sc + 110);
  }
  __syncthreads();
  GC_PHASE(P, 32);
  sum_bins(tab, B, 13, acc);
  GC_PHASE(P, 33);
  if (t == 0) planar_finalize(acc, P.map_misc[0], P.pose_pred + (int64_t)hl * 6, eps, P.eps_psd, pt);
  __syncthreads();
  GC_PHASE(P, 12);
  // ---------------------------------------------- a9 evidence sum: L_raw = L_io + L_lidar
  if (t < 9) {
    const int i = t / 3, j = t % 3;
    Lev[i * n + j] += pt[3 + t];                  // translation block [0:3, 0:3]
    Lev[(3 + i) * n + (3 + j)] += mf[9 + t];      // rotation block [3:6, 3:6]
    // the two 3x3 information matrices before their PSD projections, for the projection certificates
    // (gc_certs.hip): L_rot = V diag(s1+s2, s0+s2, s0+s1) Vᵀ as mf_information forms it, L_trans =
    // the summed WLS information masked by the z-scale as planar_finalize forms it
    const double* V = sc + 116;
    const double* s3 = mf + 24;
    const double msk[3] = {1.0, 1.0, P.map_misc[0]};
    double* raw = P.praw + (int64_t)hl * 18;
    raw[t] = V[3 * i] * (s3[1] + s3[2]) * V[3 * j] + V[3 * i + 1] * (s3[0] + s3[2]) * V[3 * j + 1] +
             V[3 * i + 2] * (s3[0] + s3[1]) * V[3 * j + 2];
    raw[9 + t] = acc[t] * msk[i] * msk[j];
  }
  if (t < 3) { hev[t] += pt[12 + t]; hev[3 + t] += mf[18 + t]; }
  __syncthreads();
  if (t == 0) {
    // aggregate_certificates([deskew, assign, moments, MF, planar]) then [ev, odom, imu, gyro]
    const double* bc = P.bincert + (int64_t)hl * 8;
    const double* io = P.io_cert + (int64_t)hl * kIoCert;
    const double* im = P.imu_out + (int64_t)hl * kImuOut;
    const double retained = bc[6] / (P.budget[4] + eps);
    const double ess_ev = (im[0] + exp(bc[4]) + bc[0] + 0.0 + 0.0) / 5.0;
    const double sf_ev = (retained + bc[5] + bc[1] + 1.0 + 1.0) / 5.0;
    const double ess_tot = (ess_ev + io[0] + io[1] + io[2]) / 4.0;
    const double sf_tot = (sf_ev + io[3] + io[4] + io[5]) / 4.0;
    const double exc = fmax(0.0, io[6]) + fmax(0.0, io[7]);
    const double nll = mf[28] + pt[20] + io[8];
    // tempering β from raw-evidence sentinels (pipeline.py:1070-1111)
    double dp = 0.0, dp2 = 0.0, dv = 0.0, dv2 = 0.0;
    for (int k = 0; k < 6; ++k) { dp += Lev[15 * n + k] * Lev[15 * n + k]; dp2 += Lev[k * n + 15] * Lev[k * n + 15]; }
    for (int k = 6; k < 9; ++k) { dv += Lev[15 * n + k] * Lev[15 * n + k]; dv2 += Lev[k * n + 15] * Lev[k * n + 15]; }
    const double dpose = sqrt(dp) + sqrt(dp2), dvel = sqrt(dv) + sqrt(dv2);
    const double dt_asym = clampd(fabs(dvel - dpose) / (dvel + dpose + eps), 0.0, 1.0);
    const double zxy = fabs(Lev[2 * n + 2]) / (0.5 * (fabs(Lev[0]) + fabs(Lev[n + 1])) + eps);
    const double e2x = ess_tot / (exc + eps);
    const double s_all = clampd(dt_asym * (zxy / (zxy + P.power_beta_z_c)) * (1.0 / (1.0 + e2x / P.power_beta_exc_c)), 0.0, 1.0);
    const double beta = clampd(P.power_beta_min + (1.0 - P.power_beta_min) * s_all, P.power_beta_min, 1.0);
    sc[50] = beta; sc[51] = dt_asym; sc[52] = zxy; sc[53] = ess_tot; sc[54] = sf_tot; sc[55] = exc; sc[56] = nll;
  }
  __syncthreads();
  const double beta = sc[50];
  for (int i = t; i < NN; i += kWG) Lev[i] *= beta;
  if (t < n) hev[t] *= beta;
  __syncthreads();
  // excitation scales (excitation.py:14-64) and the scaled prior
  if (t == 0) {
    double eex = 0.0, pex = 0.0;
    for (int k = 16; k < 22; ++k) { eex += Lev[k * n + k]; pex += Lpr[k * n + k]; }
    const double edt = Lev[15 * n + 15], pdt = Lpr[15 * n + 15];
    sc[57] = edt / (edt + pdt + 1e-12);
    sc[58] = eex / (eex + pex + 1e-12);
  }
  __syncthreads();
  const double s_dt = sc[57], s_ex = sc[58];
  auto afac = [&](int i) { return i == 15 ? 1.0 - s_dt : (i >= 16 ? 1.0 - s_ex : 1.0); };
  for (int idx = t; idx < NN; idx += kWG) {
    const int i = idx / n, j = idx % n;
    double v = Lpr[idx];
    if (i == 15 || i >= 16) v = afac(i) * v;
    if (j == 15 || j >= 16) v = afac(j) * v;
    Lps[idx] = v;
  }
  if (t < n) hps[t] = afac(t) * P.hpred[(int64_t)hl * n + t];
  __syncthreads();
  GC_PHASE(P, 13);
  // a10: pose-6 conditioning of L_ev and the fusion scale α
  const bool alpha_fixed = P.alpha_min == P.alpha_max;
  {
    double* P6 = W3;
    for (int idx = t; idx < 36; idx += kWG) {
      const int i = idx / 6, j = idx % 6;
      double v = 0.5 * (Lev[i * n + j] + Lev[j * n + i]);
      P6[idx] = isfinite(v) ? v : 0.0;
      P.lpose[(int64_t)hl * 36 + idx] = Lev[i * n + j];  // L_evidence[pose, pose] for the tape
    }
    __syncthreads();
    if (!alpha_fixed) {
      double lmin = 0.0, lmax = 0.0;
      if (t < 64) wave_extreme_eigvals<6>(P6, lmin, lmax);  // only λ_min / λ_max are consumed
      if (t == 0) {
        const double cond6 = pose6_cond(lmin, lmax, P.eps_psd, P.diag + (int64_t)hl * kHypDiag + 39);
        const double ess_ev = sc[53], exc = sc[55];
        double q = sqrt((P.c0_cond / (cond6 + P.c0_cond)) * (ess_ev / (ess_ev + 1.0)));
        q *= exp(-sc[56]) * clampd(sc[51], 0.0, 1.0);
        q *= clampd(sc[52] / (sc[52] + 1.0), 0.0, 1.0) * clampd(exc / (exc + 1.0), 0.0, 1.0);
        q *= clampd(sc[50], 0.0, 1.0);
        sc[59] = clampd(P.alpha_min + (P.alpha_max - P.alpha_min) * q, P.alpha_min, P.alpha_max);
        sc[60] = cond6;
      }
    } else if (t == 0) {
      // α_min = α_max (the reference constants): clamp(α_min + 0·q, α_min, α_min) is α_min for any
      // q, so the fusion goes ahead and the pose-6 conditioning (diagnostics only) runs on wave 2
      // beside the fusion's Cholesky
      sc[59] = P.alpha_min;
    }
    __syncthreads();
  }
  const double alpha = sc[59];
  GC_PHASE(P, 14);
  // a11 InfoFusionAdditive
  for (int i = t; i < NN; i += kWG) W2[i] = Lps[i] + alpha * Lev[i];
  if (t < n) hpo[t] = hps[t] + alpha * hev[t];
  __syncthreads();
  {
    // the pose-6 conditioning of L_ev (P6 = W3) for the tape when α did not need it, beside the factorization
    const auto cond_side = [&]() {
      if (!alpha_fixed) return;
      double lmin = 0.0, lmax = 0.0;
      wave_extreme_eigvals<6>(W3, lmin, lmax);
      if ((t & 63) == 0) sc[60] = pose6_cond(lmin, lmax, P.eps_psd, P.diag + (int64_t)hl * kHypDiag + 39);
    };
    // The fusion's PSD projection (fusion.py:150-230) certified from the factorization the recompose
    // needs anyway: L_post = L_sym, Wc = chol(L_sym + ε_l I) on wave 0 (wave 1: the symmetry deviation,
    // wave 3: cond_side); then δz = (L_post + ε_l I)⁻¹ h_post on wave 0 beside the first phase of
    // Σ_post = Wc⁻ᵀ Wc⁻¹ on wave 1, whose trace bounds the spectrum: λ_min(L_sym) >= 1 / tr Σ_post − ε_l.
    // Above 4 ε_psd the clamp is inactive and the projection is L_sym, as the Cholesky of
    // L_sym − ε_psd I certified before (one 22x22 factorization fewer on the chain); otherwise the
    // projection runs (wg_psd_fast_lifted_chol) and the two solves are repeated on its result.
    for (int idx = t; idx < NN; idx += kWG) {
      const int i = idx / n, j = idx % n;
      const double sym = 0.5 * (W2[i * n + j] + W2[j * n + i]);
      Lpo[idx] = sym;
      Wc[idx] = sym + ((i == j) ? P.eps_lift : 0.0);
    }
    __syncthreads();
    if (t < 64) {
      (void)wave0_chol<kDZ, false>(Wc, n);
      if (t == 0) GC_STAMP(P.io_parts, 9);
    } else if (t < 128) {
      double symloc = 0.0;
      for (int idx = t - 64; idx < NN; idx += 64) {
        const int i = idx / n, j = idx % n;
        const double d = 0.5 * (W2[i * n + j] + W2[j * n + i]) - W2[idx];
        symloc += d * d;
      }
      symloc = wave_sum(symloc);
      if (t == 64) red[5] = symloc;
    } else if (t >= 192) {
      cond_side();
    } else if (t == 128) {
      so3_exp(P.X + (int64_t)hl * 6 + 3, sc + 24);  // R_X for the recompose (recompose_pose_R)
    }
    __syncthreads();
    // δz on wave 0 and the forward substitution of Σ_post (its first phase; Sx is free) with its trace on
    // wave 1
    const auto solve_and_phase1 = [&]() {
      if (t < 64) {
        wave0_chol_solve<kDZ>(Wc, hpo, dz, n);
        if (t == 0) GC_STAMP(P.io_parts, 38);
      } else if (t < 128) {
        chol_inverse_phase1_lane(Wc, Sx, n, t - 64);
        double tr = 0.0;
        if (t - 64 < n)
          for (int k = 0; k < n; ++k) tr += Sx[(t - 64) * n + k] * Sx[(t - 64) * n + k];
        tr = wave_sum(tr);
        if (t == 64) red[6] = tr;
        if (t == 64) GC_STAMP(P.io_parts, 39);
      }
      __syncthreads();
    };
    solve_and_phase1();
    const double bound = 1.0 / red[6] - P.eps_lift;
    if (bound >= 4.0 * P.eps_psd) {
      if (t == 0) {
        const double nan = __builtin_nan("");
        c6[0] = 0.0; c6[1] = sqrt(red[5]); c6[2] = nan; c6[3] = nan; c6[4] = nan; c6[5] = nan;
      }
    } else {
      wg_psd_fast_lifted_chol(W2, Lpo, P.eps_psd, P.eps_lift, n, Sx, Wc, red, c6);
      solve_and_phase1();
    }
    __syncthreads();
  }
  GC_PHASE(P, 15);
  // a12 recompose: T from every operator's trigger magnitude (pipeline.py:1211), then δ' and X_new on
  // thread 0, beside the second phase of Σ_post -> W2 (also the next scan's predict Σ, P.Sig) on waves 1-3
  if (t == 0) {
    const double* bc = P.bincert + (int64_t)hl * 8;
    const double trig_budget = 1e-12 / (P.budget[0] + 1e-12);
    double T = trig_budget + P.pred_cert[(int64_t)hl * kPredCert + 7] + P.io_cert[(int64_t)hl * kIoCert + 9];
    T += 0.0 + bc[7] + mf[30] + pt[22];                // deskew, assign (exact), moments, MF, planar
    T += fabs(1.0 - sc[50]);                           // PowerTempering
    T += fabs(1.0 - (1.0 - s_dt)) + fabs(1.0 - (1.0 - s_ex));  // ExcitationPriorScaling
    T += fabs(1.0 - alpha);                            // FusionScale
    T += c6[0] + fabs(1.0 - alpha);                    // InfoFusionAdditive
    sc[61] = T;
    sc[62] = c6[0];
    double bch[6];
    sc[63] = recompose_pose_R(P.X + (int64_t)hl * 6, sc + 24, zl, dz, sc[61], P.c_frob, sc + 64, sc + 70, bch);  // X_new, δ'
    GC_STAMP(P.io_parts, 51);
  } else if (t >= 64) {
    chol_inverse_phase2_part(W2, Sx, n, t - 64, kWG - 64);
    if (t == 64) GC_STAMP(P.io_parts, 52);
  }
  __syncthreads();
  // μ_post = (L_post + ε_l I)⁻¹ h_rec with h_rec = h_post − L_post[:, 0:6] δ' (recompose.py:173-181):
  // (L + ε_l I)⁻¹ L = I − ε_l Σ_post, so μ_post = δz − δ' + ε_l Σ_post[:, 0:6] δ' — a 22 x 6 product with
  // the Σ_post just formed instead of a third triangular solve with the ill-conditioned factor
  if (t < n) {
    const double sh = (t < 6) ? sc[70 + t] : 0.0;
    double c = 0.0;
    for (int k = 0; k < 6; ++k) c += W2[t * n + k] * sc[70 + k];
    mupo[t] = (dz[t] - sh) + P.eps_lift * c;
    zl[t] = zl[t] - sh;
  }
  GC_PHASE(P, 16);
  // a15 process-noise IW statistics (inverse_wishart_jax.py:71-123)
  if (s_dt == 0.0 && s_ex == 0.0) {
    // no dt / extrinsic excitation: every afac is 1.0, so Lps and hps are L_pred and h_pred bit for
    // bit and μ_pred = (L_pred + εI)⁻¹ h_pred is predict's μ_inc (the predict kernel's predicted moments)
    if (t < n) mups[t] = P.mu_aux[(int64_t)hl * kMuAux + 22 + t];
    __syncthreads();
  } else {
    __syncthreads();
    for (int i = t; i < NN; i += kWG) W3[i] = Lps[i] + ((i / n == i % n) ? P.eps_lift : 0.0);
    __syncthreads();
    wg_chol(W3, n);
    wg_chol_solve(W3, hps, mups, n);
  }
  GC_PHASE(P, 17);
  // a14 anchor drift (anchor_drift.py:93-191) and, for hypothesis 0 only, the a13 map increment
  // (backend_node.py:2081-2083, build-defined pushforward), beside the a15 process-noise statistics
  // (inverse_wishart_jax.py:71-123) and Σ_post's store. Every SE(3) map of the two compositions with
  // X_new, Exp(μ) and Exp(ρ μ) (compose_exp2: se3_exp, both rotations' so3_exp, the product's so3_log)
  // is split over waves, each piece the same routine on the same operands (bit-identical):
  //   step 1: ρ (wave 0), se3_exp(μ_post) (wave 1, hypothesis 0), so3_exp(μ_post rot) (wave 2,
  //           hypothesis 0), R_Xnew = so3_exp(X_new rot) (wave 3);
  //   step 2: h_fin, μ_fin (wave 0); z_t = X_new ∘ Exp(μ_post), R = Exp(z_t rot), the pushforward
  //           (wave 1, hypothesis 0); X_fin = X_new ∘ Exp(ρ μ_post) (wave 2, lane 128); the statistics
  //           and Σ_post's store on the rest of waves 2-3.
  // Neither step writes what the other waves read.
  double* e_zt = sc;        // 6
  double* R_ezt = sc + 6;   // 9
  double* R_xn = sc + 15;   // 9
  if (t == 0) {
    sc[98] = drift_rho(mupo, nullptr, nullptr);
  } else if (t == 64 && P.h_begin + hl == 0) {
    se3_exp(mupo, e_zt);
  } else if (t == 128 && P.h_begin + hl == 0) {
    so3_exp(mupo + 3, R_ezt);
  } else if (t == 192) {
    so3_exp(sc + 64 + 3, R_xn);
  }
  __syncthreads();
  if (t < 64) {
    const double rho = sc[98];
    if (t == 0) GC_STAMP(P.io_parts, 36);
    if (t < n) zl[t] = (1.0 - rho) * mupo[t];
    wave_lds_sync();
    if (t < n) {  // h_fin = L_post z (wg_matvec's row order)
      double v = 0.0;
      for (int k = 0; k < n; ++k) v += Lpo[t * n + k] * zl[k];
      hfin[t] = v;
    }
    wave_lds_sync();
    wave0_chol_solve<kDZ>(Wc, hfin, mufin, n);
    if (t == 0) GC_STAMP(P.io_parts, 37);
  } else if (t < 128) {
    if (P.h_begin + hl == 0) {
      if (t == 64) {
        double zt[6], R[9];
        se3_compose_R(sc + 64, R_xn, e_zt, R_ezt, zt);
        so3_exp(zt + 3, R);
        for (int k = 0; k < 9; ++k) sc[80 + k] = R[k];
        sc[89] = zt[0]; sc[90] = zt[1]; sc[91] = 0.0;  // planar map: t[2] = 0 (CHANGELOG.md:575-578)
        for (int k = 0; k < 6; ++k) P.h0rec[k] = zt[k];
        GC_STAMP(P.io_parts, 34);
      }
      // hypothesis 0's pose covariance and deskew twist for the in-scan PrimitiveMap update
      if (t - 64 < 36) P.h0rec[6 + (t - 64)] = W2[((t - 64) / 6) * n + (t - 64) % 6];
      else if (t - 64 < 42) P.h0rec[42 + (t - 100)] = P.xi[(int64_t)hl * 6 + (t - 100)];
      wave_lds_sync();
      for (int b = t - 64; b < B; b += 64) pushforward_bin(st + b * 38, sc + 80, sc + 89, W2, n, P.map_inc + b * kMapRec);
      if (t == 64) GC_STAMP(P.io_parts, 35);
    }
  } else {
    if (t == 128) {  // X_fin = X_new ∘ Exp(ρ μ_post) (compose_exp2's pieces)
      const double rho = sc[98];
      double d6[6], e[6], Re[9];
      for (int k = 0; k < 6; ++k) d6[k] = rho * mupo[k];
      se3_exp(d6, e);
      so3_exp(e + 3, Re);
      se3_compose_R(sc + 64, R_xn, e, Re, sc + 92);
    }
    for (int i = t - 128; i < NN; i += kWG - 128) P.Sig[(int64_t)hl * NN + i] = W2[i];
    for (int idx = t - 128; idx < 7 * 36; idx += kWG - 128)
      P.dPsiP[(int64_t)hl * 252 + idx] = iw_proc_stat(idx, mupo, mups, W2);
  }
  __syncthreads();
  const double rho = sc[98];
  GC_PHASE(P, 18);
  GC_PHASE(P, 19);
  // write the final belief and per-hypothesis outputs
  for (int i = t; i < NN; i += kWG) P.L[(int64_t)hl * NN + i] = Lpo[i];
  if (t < n) {
    P.z[(int64_t)hl * n + t] = zl[t];
    P.h[(int64_t)hl * n + t] = hfin[t];
    P.mu_fin[(int64_t)hl * n + t] = mufin[t];
  }
  if (t == 0) {
    for (int k = 0; k < 6; ++k) P.X[(int64_t)hl * 6 + k] = sc[92 + k];
    P.stamp[hl] += S.dt;
    double* dg = P.diag + (int64_t)hl * kHypDiag;  // [0, 6): the world pose, k_combine_local
    dg[6] = sc[61]; dg[7] = sc[50]; dg[8] = alpha; dg[9] = s_dt; dg[10] = s_ex; dg[11] = rho;
    dg[12] = sc[63]; dg[13] = sc[60]; dg[14] = sc[53]; dg[15] = sc[51]; dg[16] = sc[52]; dg[17] = sc[56];
    dg[18] = mf[30]; dg[19] = pt[22]; dg[20] = sc[62];
    for (int k = 0; k < 3; ++k) dg[21 + k] = pt[k];       // t_wls
    for (int k = 0; k < 3; ++k) dg[24 + k] = sc[110 + k];  // log R_mf
    for (int k = 0; k < 3; ++k) dg[27 + k] = mf[24 + k];  // MF singular values
    for (int k = 0; k < 6; ++k) dg[30 + k] = P.xi[(int64_t)hl * 6 + k];
    double mu2 = 0.0;
    for (int k = 0; k < n; ++k) mu2 += mufin[k] * mufin[k];
    dg[36] = sc[54]; dg[37] = sc[55]; dg[38] = mu2;  // |μ|² for the combine's spread; [39] eigmin_pose6
  }
}

// one or two workgroups per CU, as k_predict_imu (gc_belief.hip): two only when H_l exceeds the CUs;
// FOLD: the a6 finalize at the start (its own instantiation: compiled into the kernel without it,
// the shard sizes that keep the split finalize ran 0.7 % slower)
template <int OCC, bool FOLD>
__global__ void __launch_bounds__(256, OCC) k_evidence(PipeDev P, ScanArgs S) {
  evidence_body<FOLD>(P, S);
}

// ==================================================================== a16 partial sums (local)
// grid: ceil(P_len / 64) blocks x 256 threads; block covers 64 record entries, its 4 waves sum
// interleaved hypothesis subsets, combined in fixed order (deterministic).
// The workgroups past the record's are one thread per hypothesis: the tape's world pose
// X_fin ⊞ μ_fin (a single-lane chain of SE(3) maps, ~3 µs) off k_evidence's critical tail.
__global__ void __launch_bounds__(256) k_combine_local(PipeDev P) {
  // 16 record entries per workgroup x 16 hypothesis groups (hypotheses g, g+16, ...): at H = 256 a
  // thread's 16 hypotheses are one batch of loads in flight; the 16 group partials are then
  // summed in a fixed tree
  __shared__ double part[16][16];
  __shared__ double red[8];
  const int nrec = (partial_len(P.B) + 15) / 16;
  if ((int)blockIdx.x >= nrec) {
    const int h = ((int)blockIdx.x - nrec) * kWG + (int)threadIdx.x;
    if (h < P.Hl) {
      double pose[6];
      compose_exp2(P.X + (int64_t)h * 6, P.mu_fin + (int64_t)h * kDZ, pose);
      for (int k = 0; k < 6; ++k) P.diag[(int64_t)h * kHypDiag + k] = pose[k];
    }
    return;
  }
  const int t = threadIdx.x, lane = t & 15, g = t >> 4;
  const int n = kDZ, Hl = P.Hl;
  const int e = blockIdx.x * 16 + lane;
  const int PLn = partial_len(P.B);
  // this lane's record entry as (source row, stride, weight kind), resolved once; the hypothesis
  // loop is then branch-free (clamped rows, 0/1 masks) with 16 independent loads in flight
  const double* W = P.weights + P.h_begin;
  const double* src = W;
  int64_t stride = 0;
  double use_src = 0.0, use_norm = 0.0, live = 1.0;  // value = w * (use_src ? src : 1)
  if (e < kPH) { src = P.L + e; stride = NN; use_src = 1.0; use_norm = 1.0; }
  else if (e < kPZ) { src = P.h + (e - kPH); stride = n; use_src = 1.0; use_norm = 1.0; }
  else if (e < kPMU) { src = P.z + (e - kPZ); stride = n; use_src = 1.0; use_norm = 1.0; }
  else if (e < kPMU2) { src = P.mu_fin + (e - kPMU); stride = n; use_src = 1.0; use_norm = 1.0; }
  else if (e == kPMU2) { src = P.diag + 38; stride = kHypDiag; use_src = 1.0; use_norm = 1.0; }  // |μ|², k_evidence
  else if (e < kPDNUP) { src = P.dPsiP + (e - kPDPSIP); stride = 252; use_src = 1.0; }
  else if (e < kPDPSIM) { }  // dν_proc: w
  else if (e < kPDNUM) { src = P.dPsiM + (e - kPDPSIM); stride = 27; use_src = 1.0; }
  else if (e < kPDNUM + 2) { }  // dν_meas gyro/accel: w
  else live = 0.0;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  double v[16], wr[16], m[16];
  const auto load_batch = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = k0 + 16 * j;
      const int kc = k < Hl ? k : Hl - 1;
      m[j] = k < Hl ? live : 0.0;
      wr[j] = W[kc];
      v[j] = src[(int64_t)kc * stride];
    }
  };
  // the first batch of values is in flight while the weight sum is formed (it needs neither)
  load_batch(g);
  // floored / renormalised weights over ALL hypotheses (hypothesis.py:77-82), replicated
  double loc = 0.0;
  for (int k = t; k < P.H; k += kWG) loc += fmax(P.weights[k], P.weight_floor);
  const double wsum = wg_sum(loc, red);
  const double inv_wsum = 1.0 / wsum;
  for (int k0 = g; k0 < Hl; k0 += 256) {
    if (k0 != g) load_batch(k0);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const double wk = use_norm != 0.0 ? fmax(wr[j], P.weight_floor) * inv_wsum : wr[j];
      acc[j & 3] += m[j] * wk * (use_src != 0.0 ? v[j] : 1.0);
    }
  }
  part[g][lane] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (g == 0 && e < PLn) {
    double q[4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
      q[a] = (part[4 * a][lane] + part[4 * a + 1][lane]) + (part[4 * a + 2][lane] + part[4 * a + 3][lane]);
    double r = (q[0] + q[1]) + (q[2] + q[3]);
    if (e >= kPX0 && e < kPX0 + 6) r = (P.h_begin == 0) ? P.X[e - kPX0] : 0.0;
    else if (e == kPSTAMP0) r = (P.h_begin == 0) ? P.stamp[0] : 0.0;
    else if (e >= rec_h0(P.B)) r = (P.h_begin == 0) ? P.h0rec[e - rec_h0(P.B)] : 0.0;
    else if (e >= kPMAP) r = (P.h_begin == 0) ? P.map_inc[e - kPMAP] : 0.0;
    P.send[e] = r;
  }
}

// Map-derived statistics for the evidence of the next scan (bin_atlas.py:166-207) and the
// self-adaptive planar z-scale (matrix_fisher_evidence.py:572-589).
GC_DEV void map_derive_wg(const PipeDev& P, double* red, double* tab) {
  const int t = threadIdx.x, B = P.B;
  const double eps = P.eps_mass;
  if (t < B) {
    const double* m = P.map + t * kMapRec;
    double* d = P.map_der + t * kMapDer;
    const double nr = sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
    for (int k = 0; k < 3; ++k) d[k] = m[k] / (nr + eps);
    const double invd = 1.0 / (m[12] + eps + kF64Eps);
    d[3] = kappa_blend(nr * invd, 1e-6, 3.0, 0.8, 0.03);
    const double invp = 1.0 / (m[13] + eps + kF64Eps);
    double c[3], Sr[9], Sp[9];
    for (int k = 0; k < 3; ++k) c[k] = m[14 + k] * invp;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Sr[3 * i + j] = m[17 + 3 * i + j] * invp - c[i] * c[j];
    psd_project3_fast(Sr, P.eps_psd, Sp, nullptr);
    for (int k = 0; k < 3; ++k) d[4 + k] = c[k];
    for (int k = 0; k < 9; ++k) d[7 + k] = Sp[k];
    d[16] = 0.0;
    double* r = tab + t * 10;
    for (int k = 0; k < 9; ++k) r[k] = m[3 + k];
    r[9] = m[12];
  }
  __syncthreads();
  sum_bins(tab, B, 10, red);
  if (t == 0) {
    double Tm[9], lam[3];
    const double Nt = red[9] + eps;
    for (int k = 0; k < 9; ++k) Tm[k] = red[k] / Nt;
    eigvalsh3_desc(Tm, lam);
    P.map_misc[0] = fmax(lam[2], 0.0) / fmax(lam[0], eps);
    P.map_misc[1] = red[9];
  }
  __syncthreads();
}

__global__ void __launch_bounds__(256) k_map_derive(PipeDev P) {
  __shared__ double red[16];
  __shared__ double tab[64 * 10];
  map_derive_wg(P, red, tab);
}

GC_DEV void iw_Q_wg(const PipeDev& P, double* Qs, double* Qp, double* Sx, double* red) {
  wg_iw_Q(P.nu_proc, P.Psi_proc, P.eps_psd, P.Q, Qs, Qp, Sx, red);
}

__global__ void __launch_bounds__(256) k_iw_Q(PipeDev P) {
  extern __shared__ double sm[];
  iw_Q_wg(P, sm, sm + NN, sm + 2 * NN, sm + 4 * NN + 4 * kDZ);
}

// ================================================= a16 combine + a15 IW apply + map update
__global__ void __launch_bounds__(256) k_combine_final(PipeDev P, ScanArgs S) {
  extern __shared__ double sm[];
  double* Lr = sm;
  double* Lc = Lr + NN;
  double* Sx = Lc + NN;  // 2NN + 88
  double* red = Sx + 2 * NN + 4 * kDZ;
  double* c6 = red + 16;
  double* blk = c6 + 8;   // 36
  double* blkp = blk + 36;
  double* tab = blkp + 36;  // 64 x 10
  double* Qs = tab + 640;   // NN
  double* Qp = Qs + NN;     // NN
  const int t = threadIdx.x, n = kDZ;
  const int PLn = partial_len(P.B);
  if (blockIdx.x == 1) {
    GC_PHASE_WG(P, 44, 1);
    // ---- map update on a second workgroup, beside the IW / Q chain of workgroup 0 (nothing there
    // reads the map): γ·map + increments of hypothesis 0 (bin_atlas.py:137-163, :232-257), the
    // increments reduced in the same rank order as workgroup 0's record (0.0 + Σ_g, so the value
    // is the same whether or not workgroup 0 has already rewritten an aliased single-rank record)
    for (int e = t; e < P.B * kMapRec; e += kWG) {
      double s = 0.0;
      for (int g = 0; g < P.G; ++g) s += P.gather[(int64_t)g * PLn + kPMAP + e];
      P.map[e] = P.forgetting * P.map[e] + s;
    }
    __syncthreads();
    map_derive_wg(P, red, tab);
    GC_PHASE_WG(P, 45, 1);
    return;
  }
  if (blockIdx.x == 3) {
    GC_PHASE_WG(P, 46, 3);
    // ---- the measurement-noise IW apply (measurement_noise_iw_jax.py:59-100) on a fourth
    // workgroup, beside the process-noise apply and Q rebuild of workgroup 2 (neither reads what
    // the other writes; nothing on this stream reads the measurement IW state before the next
    // scan's bins launch): its record entries reduced in the same rank order, 0.0 + Σ_g
    double* Ri = Lc;  // record entries [kPDPSIM, kPX0)
    for (int e = kPDPSIM + t; e < kPX0; e += kWG) {
      double s = 0.0;
      for (int g = 0; g < P.G; ++g) s += P.gather[(int64_t)g * PLn + e];
      Ri[e - kPDPSIM] = s;
    }
    // the LiDAR block as this scan saw it (the in-scan map update's Σ_lidar: the reference builds the
    // scan's measurement covariances from the IW state before the scan's own apply)
    if (t < 10) P.smap_snap[kSnapIW + t] = t == 0 ? P.nu_meas[2] : P.Psi_meas[18 + t - 1];
    __syncthreads();
    wg_iw_meas_apply(P.nu_meas, P.Psi_meas, Ri, Ri + (kPDNUM - kPDPSIM), P.eps_psd, P.nu_max, P.nu_meas, P.Psi_meas,
                     P.iw_cert + 2, tab, P.iwraw + 7 * 36);
    GC_PHASE_WG(P, 47, 3);
    return;
  }
  if (blockIdx.x == 2) {
    GC_PHASE_WG(P, 48, 2);
    // ---- the process-noise IW apply and the Q rebuild on a third workgroup, beside workgroup 0's barycenter:
    // they read only the records' IW statistics (reduced here in the same rank order as workgroup
    // 0's record, 0.0 + Σ_g) and the IW state, and nothing of theirs is read there
    double* Ri = Lc;  // record entries [kPDPSIP, kPX0)
    for (int e = kPDPSIP + t; e < kPX0; e += kWG) {
      double s = 0.0;
      for (int g = 0; g < P.G; ++g) s += P.gather[(int64_t)g * PLn + e];
      Ri[e - kPDPSIP] = s;
    }
    __syncthreads();
    GC_PHASE_WG(P, 22, 2);
    // process-noise IW apply (inverse_wishart_jax.py:126-185), weight min(1, scan_count), and Q of the
    // updated state (:35-68) formed beside it from the apply's own blocks (wg_iw_proc_apply<true>)
    wg_iw_proc_apply<true>(P.nu_proc, P.Psi_proc, Ri, Ri + (kPDNUP - kPDPSIP), S.w_process, P.eps_psd, P.nu_max,
                           P.nu_proc, P.Psi_proc, P.iw_cert, Qs, blk, blkp, Sx, red, c6, tab, P.iwraw, P.Q, Qp, Lr);
    GC_PHASE_WG(P, 23, 2);
    GC_PHASE_WG(P, 24, 2);
    GC_PHASE_WG(P, 25, 2);
    return;
  }
  GC_PHASE(P, 20);
  // fixed rank-order reduction of the gathered partial records
  for (int e = t; e < PLn; e += kWG) {
    double s = 0.0;
    for (int g = 0; g < P.G; ++g) s += P.gather[(int64_t)g * PLn + e];
    P.send[e] = s;  // reuse send as the reduced record
    if (e >= rec_h0(P.B)) P.smap_snap[e - rec_h0(P.B)] = s;
  }
  if (t < 8) P.smap_snap[kSnapBudget + t] = P.budget[t];
  __syncthreads();
  const double* R = P.send;
  for (int i = t; i < NN; i += kWG) Lr[i] = R[kPL + i];
  __syncthreads();
  wg_psd_project_fast(Lr, Lc, P.eps_psd, n, Sx, red, c6);
  GC_PHASE(P, 21);
  double* cb = P.comb;
  for (int i = t; i < NN; i += kWG) cb[i] = Lc[i];
  if (t < n) { cb[NN + t] = R[kPH + t]; cb[NN + n + t] = R[kPZ + t]; }
  if (t < 6) cb[NN + 2 * n + t] = R[kPX0 + t];
  // weight-only certificate terms (hypothesis.py:183-205), replicated on every rank
  double l2 = 0.0, lc = 0.0, la = 0.0, lw = 0.0;
  for (int k = t; k < P.H; k += kWG) lw += fmax(P.weights[k], P.weight_floor);
  const double wsum = wg_sum(lw, red);
  for (int k = t; k < P.H; k += kWG) {
    const double wf = fmax(P.weights[k], P.weight_floor), wn = wf / wsum;
    l2 += wn * wn; lc += (wn > P.weight_floor) ? 1.0 : 0.0; la += fabs(wf - P.weights[k]);
  }
  double s3[3] = {l2, lc, la};
  wg_sum_n<3>(s3, tab);  // wg_sum's order, two barriers (tab: free until the IW apply)
  const double s2 = s3[0], scnt = s3[1], sadj = s3[2];
  if (t == 0) {
    double* cc = cb + NN + 2 * n + 6;
    cc[0] = R[kPSTAMP0];
    cc[1] = c6[0]; cc[2] = c6[2]; cc[3] = c6[3]; cc[4] = c6[4]; cc[5] = c6[5];
    cc[6] = 1.0 / s2; cc[7] = scnt / P.H; cc[8] = sadj / P.H; cc[9] = sadj;
    double mm = 0.0;
    for (int i = 0; i < n; ++i) mm += R[kPMU + i] * R[kPMU + i];
    cc[10] = R[kPMU2] - mm;  // spread proxy Σ w‖μ_j‖² − ‖Σ w μ_j‖²
  }
  GC_PHASE(P, 49);
}

// ------------------------------------------------------------------------------ launchers
static size_t lds_evidence() { return sizeof(double) * (7 * NN + 2 * NN + 4 * kDZ + 10 * kDZ + 8 + 64 * 16 + 32 + 128 + 6 + kMF + kPT); }
static size_t lds_final() { return sizeof(double) * (2 * NN + 2 * NN + 4 * kDZ + 16 + 8 + 72 + 640 + 2 * NN); }

}  // namespace gc

namespace gc {
static hipError_t allow_big_lds(const void* fn, size_t bytes) {
  return bytes > 65536 ? ensure_dyn_lds(fn, bytes) : hipSuccess;
}
hipError_t launch_evidence(const PipeDev& P, const ScanArgs& S, hipStream_t st) {
  const bool two = P.Hl > P.cus, fold = S.fin_part != nullptr;
#define GC_EVL(OCC, FOLD)                                                                        \
  do {                                                                                           \
    if (hipError_t e = allow_big_lds((const void*)k_evidence<OCC, FOLD>, lds_evidence())) return e; \
    hipLaunchKernelGGL((k_evidence<OCC, FOLD>), dim3(P.Hl), dim3(256), lds_evidence(), st, P, S);   \
  } while (0)
  if (two) {
    if (fold) GC_EVL(2, true);
    else GC_EVL(2, false);
  } else {
    if (fold) GC_EVL(1, true);
    else GC_EVL(1, false);
  }
#undef GC_EVL
  return hipGetLastError();
}
hipError_t launch_combine_local(const PipeDev& P, hipStream_t st) {
  const int nrec = (partial_len(P.B) + 15) / 16, npose = (P.Hl + kWG - 1) / kWG;
  hipLaunchKernelGGL(k_combine_local, dim3(nrec + npose), dim3(256), 0, st, P);
  return hipGetLastError();
}
hipError_t launch_combine_final(const PipeDev& P, const ScanArgs& S, hipStream_t st, hipEvent_t done) {
  if (hipError_t e = allow_big_lds((const void*)k_combine_final, lds_final())) return e;
  // workgroup 0: record reduction, barycenter, certificates; 1: map update + derive; 2: process IW
  // apply, Q; 3: measurement IW apply
  if (done) hipExtLaunchKernelGGL(k_combine_final, dim3(4), dim3(256), lds_final(), st, nullptr, done, 0, P, S);
  else hipLaunchKernelGGL(k_combine_final, dim3(4), dim3(256), lds_final(), st, P, S);
  return hipGetLastError();
}
hipError_t launch_map_derive(const PipeDev& P, hipStream_t st) {
  hipLaunchKernelGGL(k_map_derive, dim3(1), dim3(256), 0, st, P);
  return hipGetLastError();
}
hipError_t launch_iw_Q(const PipeDev& P, hipStream_t st) {
  hipLaunchKernelGGL(k_iw_Q, dim3(1), dim3(256), sizeof(double) * (4 * NN + 4 * kDZ + 16), st, P);
  return hipGetLastError();
}
}  // namespace gc
