// gc_certs.hip — in-scan ConditioningCerts of the per-hypothesis 22x22 PSD projections.
//
// The reference emits a ConditioningCert [eig_min, eig_max, cond, near_null_count] of the clamped
// spectrum on every predict (predict.py:183-188: L_pred) and fusion (fusion.py:150-230: L_post) call.
// The batched scan certifies both projections by Cholesky and skips their eigen-decompositions; with
// in-scan certificates on (gc_pipeline_set_inscan_certs) this launch, right after the evidence kernel,
// produces the reference's certificate fields for every hypothesis inside the scan:
//   one wave per (hypothesis, matrix): Householder tridiagonalisation of M_sym with one row per lane
//   (v and w broadcast through a wave-private LDS row), then lanes 0-31 / 32-63 multisect for λ_min /
//   λ_max with Sturm counts (the inertia of T − σI, as LAPACK dstebz; 33 sections per round, 11
//   rounds: 2^-55 of the Gershgorin width, the absolute accuracy of eigh), and one more count at
//   σ = 10 ε for the near-null count (eigenvalues below 10 ε, clamped or not).
//   eig_min = max(λ_min, ε), eig_max = max(λ_max, ε), cond = eig_max / eig_min.
#include <hip/hip_runtime.h>
#include "gc_internal.h"
#include "gc_pipe.h"
#include "gc_wgla.h"
#include "gc_opsdev.h"
#include "gc_cond.h"

namespace gc {
namespace {

constexpr int kCertWaves = 4;  // (hypothesis, matrix) items per 256-thread workgroup

// grid ceil(2 Hl / 4): wave w of workgroup b takes item 4 b + w = 2 h + m (m = 0: L_pred, 1: L_post)
__global__ void __launch_bounds__(256) k_hyp_certs(PipeDev P) {
  __shared__ double buf[kCertWaves][3 * kDZ + 8];
  const int wv = threadIdx.x >> 6;
  const int item = blockIdx.x * kCertWaves + wv;
  if (item >= 2 * P.Hl) return;
  const int h = item >> 1, m = item & 1;
  const double* M = (m == 0 ? P.Lpred : P.L) + (int64_t)h * kDZ * kDZ;
  wave_conditioning<kDZ>(M, P.eps_psd, buf[wv], P.hcond + ((int64_t)h * 2 + m) * 4);
}

// ------------------------------------------------------------------ full projection certificates
// The reference's cert_vec [projection_delta, sym_delta, eig_min, eig_max, cond, near_null_count] of
// every remaining PSD projection of a scan (domain_projection_psd_core, primitives.py:80-123), from
// the unprojected operands by a full eigen-decomposition (the scan itself certifies these projections
// by Cholesky and keeps only their deltas):
//   per hypothesis, one thread per 3x3 (psd_project3: cyclic Jacobi): the B bins' Σ_p re-formed from
//   the bin row's raw sums exactly as finalize_bin forms it (binning.py:175-187), then the MF L_rot and
//   planar L_trans that k_evidence stored unprojected (P.praw);
//   per scan, one workgroup each (wg_psd_project: parallel Jacobi): the barycenter L (the reduced
//   record in P.send, hypothesis.py:99), the 7 process-IW blocks padded to 6x6 (P.iwraw,
//   k_combine_final) and Q assembled from the updated IW state (inverse_wishart_jax.py:35-68); the 3
//   measurement blocks (3x3) by psd_project3 on one lane.
constexpr int kScanCertLds = 2 * kDZ * kDZ + 2 * kDZ * kDZ + 4 * kDZ + 8 + 8;

GC_DEV void bin_sigma_raw(const double* o, double eps_mass, double* Sr) {
  // finalize_bin's Σ_raw (gc_binfin.h) from its stats row: N = o[0], Σ p = o[26:29], Σ p pᵀ = o[29:38]
  const double invN = 1.0 / (o[0] + eps_mass + kF64Eps);
  const double pb[3] = {o[26] * invN, o[27] * invN, o[28] * invN};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Sr[3 * i + j] = o[29 + 3 * i + j] * invN - pb[i] * pb[j];
}

__global__ void __launch_bounds__(256) k_proj_certs(PipeDev P) {
  const int B = P.B, per = B + 2;
  const int nh = (P.Hl * per + kWG - 1) / kWG;
  if ((int)blockIdx.x < nh) {
    const int item = blockIdx.x * kWG + threadIdx.x;
    if (item >= P.Hl * per) return;
    const int h = item / per, k = item % per;
    double A[9], Mp[9], c[6];
    if (k < B) {
      bin_sigma_raw(P.stats + ((int64_t)h * B + k) * GC_BIN_STATS, P.eps_mass, A);
    } else {
      const double* r = P.praw + (int64_t)h * 18 + (k - B) * 9;
      for (int q = 0; q < 9; ++q) A[q] = r[q];
    }
    psd_project3(A, P.eps_psd, Mp, c);
    for (int q = 0; q < 6; ++q) P.pcert[(int64_t)item * 6 + q] = c[q];
    return;
  }
  __shared__ double sm[kScanCertLds];
  const int s = (int)blockIdx.x - nh, t = threadIdx.x, n22 = kDZ;
  double* M = sm;
  double* Mp = M + kDZ * kDZ;
  double* scr = Mp + kDZ * kDZ;
  double* red = scr + 2 * kDZ * kDZ + 4 * kDZ;
  double* c6 = red + 8;
  int n;
  if (s == GC_PCERT_BARY) {
    n = n22;
    for (int i = t; i < kDZ * kDZ; i += kWG) M[i] = P.send[kPL + i];
  } else if (s < GC_PCERT_MEAS0) {
    n = 6;
    for (int i = t; i < 36; i += kWG) M[i] = P.iwraw[(s - GC_PCERT_PROC0) * 36 + i];
  } else if (s < GC_PCERT_Q) {
    // a 3x3 block: psd_project3 on one lane (the per-operator entries route d <= 3 there as well)
    if (t == 0) {
      double A[9], Ap[9], c[6];
      for (int i = 0; i < 9; ++i) A[i] = P.iwraw[7 * 36 + (s - GC_PCERT_MEAS0) * 9 + i];
      psd_project3(A, P.eps_psd, Ap, c);
      for (int q = 0; q < 6; ++q) P.pcert[((int64_t)P.Hl * per + s) * 6 + q] = c[q];
    }
    return;
  } else {
    // Q = ⊕ Ψ_b / den_b over the masked blocks (block diagonal; wg_iw_Q's den)
    n = n22;
    for (int i = t; i < kDZ * kDZ; i += kWG) {
      const int r = i / kDZ, q = i % kDZ;
      double v = 0.0;
      for (int b = 0; b < 7; ++b) {
        const int s0 = kIwBlockStart[b], d = kIwBlockDim[b];
        if (r >= s0 && r < s0 + d && q >= s0 && q < s0 + d) {
          const double den = softplus(50.0 * (P.nu_proc[b] - d - 1.0)) / 50.0 + 1e-12;
          v = P.Psi_proc[b * 36 + 6 * (r - s0) + (q - s0)] / den;
        }
      }
      M[i] = v;
    }
  }
  __syncthreads();
  double* out = P.pcert + ((int64_t)P.Hl * per + s) * 6;
  if (n == kDZ) {
    // the 22x22 barycenter and Q: the extremes and the near-null count by the tridiagonal Sturm
    // multisection (wave 0, as k_hyp_certs) beside the symmetry deviation (wave 1); when no eigenvalue
    // lies below eps_psd the clamp moves nothing and the projection delta is 0 (the reference's is the
    // rounding of V diag(λ) Vᵀ), otherwise the full Jacobi projection below
    int* below = reinterpret_cast<int*>(red + 6);
    if (t < 64) {
      wave_conditioning<kDZ>(M, P.eps_psd, scr, c6 + 2, below);
    } else if (t < 128) {
      double sl = 0.0;
      for (int idx = t - 64; idx < kDZ * kDZ; idx += 64) {
        const int i = idx / kDZ, j = idx % kDZ;
        const double dd = 0.5 * (M[i * kDZ + j] + M[j * kDZ + i]) - M[idx];
        sl += dd * dd;
      }
      sl = wave_sum(sl);
      if (t == 64) c6[1] = sqrt(sl);
    }
    __syncthreads();
    if (*below == 0) {
      if (t == 0) {
        out[0] = 0.0; out[1] = c6[1];
        for (int q = 2; q < 6; ++q) out[q] = c6[q];
      }
      return;
    }
    __syncthreads();
  }
  wg_psd_project(M, Mp, P.eps_psd, n, scr, red, c6);
  if (t < 6) out[t] = c6[t];
}

}  // namespace

hipError_t launch_hyp_certs(const PipeDev& P, hipStream_t st) {
  hipLaunchKernelGGL(k_hyp_certs, dim3((unsigned)((2 * P.Hl + kCertWaves - 1) / kCertWaves)), dim3(256), 0, st, P);
  return hipGetLastError();
}

hipError_t launch_proj_certs(const PipeDev& P, hipStream_t st) {
  const int nh = (P.Hl * (P.B + 2) + kWG - 1) / kWG;
  hipLaunchKernelGGL(k_proj_certs, dim3((unsigned)(nh + kScanCerts)), dim3(256), 0, st, P);
  return hipGetLastError();
}

}  // namespace gc
