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

namespace gc {
namespace {

constexpr int kCertWaves = 4;  // (hypothesis, matrix) items per 256-thread workgroup

// Sturm count: eigenvalues of the tridiagonal (d, e) below sig (LAPACK dstebz's pivmin guard)
template <int N>
GC_DEV int sturm_count(const double* d, const double* e2, double sig, double pivmin) {
  int cnt = 0;
  double q = d[0] - sig;
  if (fabs(q) < pivmin) q = -pivmin;
  cnt += q < 0.0;
#pragma unroll
  for (int i = 1; i < N; ++i) {
    q = (d[i] - sig) - e2[i - 1] / q;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
  }
  return cnt;
}

// One wave: the ConditioningCert of the symmetrised N x N row-major M (global) into out4.
// buf: 3 N + 8 doubles of wave-private LDS.
template <int N>
GC_DEV void wave_conditioning(const double* __restrict__ M, double eps, double* buf, double* out4,
                              int* below_eps = nullptr) {
  const int lane = threadIdx.x & 63;
  const bool row = lane < N;
  double a[N];  // row `lane` of the symmetrised matrix (zeros on idle lanes)
#pragma unroll
  for (int j = 0; j < N; ++j) a[j] = row ? 0.5 * (M[lane * N + j] + M[j * N + lane]) : 0.0;
  double* vb = buf;       // the step's Householder vector v, then w, broadcast
  double* wb = buf + N;
  double* db = buf + 2 * N;
  double e[N];
#pragma unroll
  for (int k = 0; k < N - 2; ++k) {
    // column k below the diagonal: A[i][k] on lane i (symmetric: its row's entry k)
    const double xk = a[k];
    const double ss = wave_sum(lane >= k + 2 && row ? xk * xk : 0.0);
    const double x0 = readlane_f64(xk, k + 1);
    const double sigma = sqrt(fma(x0, x0, ss));
    if (ss == 0.0) {  // already tridiagonal in this column (wave-uniform)
      e[k] = x0;
      continue;
    }
    const double alpha = x0 >= 0.0 ? -sigma : sigma;
    const double beta = 1.0 / (sigma * (sigma + fabs(x0)));  // 2 / vᵀv
    const double vl = lane > k + 1 && row ? xk : (lane == k + 1 ? x0 - alpha : 0.0);
    if (lane < N) vb[lane] = vl;
    wave_lds_sync();
    double acc = 0.0;  // (A v)_lane over j > k
#pragma unroll
    for (int j = k + 1; j < N; ++j) acc = fma(a[j], vb[j], acc);
    const double pl = lane > k && row ? beta * acc : 0.0;
    const double pv = wave_sum(pl * vl);
    const double K = 0.5 * beta * pv;
    const double wl = fma(-K, vl, pl);
    if (lane < N) wb[lane] = wl;
    wave_lds_sync();
    if (lane > k && row) {
#pragma unroll
      for (int j = k + 1; j < N; ++j) a[j] = a[j] - (vl * wb[j] + wl * vb[j]);
    }
    wave_lds_sync();  // the next step rewrites vb / wb
    e[k] = alpha;
  }
  // T: d on the diagonal (lane i's a[i]), e[N-2] = A[N-1][N-2]
  double dself = 0.0;
#pragma unroll
  for (int j = 0; j < N; ++j) dself = lane == j ? a[j] : dself;
  if (lane < N) db[lane] = dself;
  const double last = readlane_f64(a[N - 2], N - 1);
  wave_lds_sync();
  double d[N], e2[N];
#pragma unroll
  for (int i = 0; i < N; ++i) d[i] = db[i];
  e[N - 2] = last;
  e[N - 1] = 0.0;
  double lo = d[0] - fabs(e[0]), hi = d[0] + fabs(e[0]), emax2 = 0.0;
#pragma unroll
  for (int i = 1; i < N; ++i) {
    const double r = fabs(e[i - 1]) + fabs(e[i]);
    lo = fmin(lo, d[i] - r);
    hi = fmax(hi, d[i] + r);
    emax2 = fmax(emax2, e[i - 1] * e[i - 1]);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) e2[i] = e[i] * e[i];
  const double pivmin = 2.2250738585072014e-308 * fmax(1.0, emax2);
  const int half = lane >> 5, l = lane & 31;
  double lo_b = lo, hi_b = hi;  // this half's bracket: λ_min (half 0) or λ_max (half 1)
  const int target = half == 0 ? 1 : N;
  for (int round = 0; round < 11; ++round) {
    const double step = (hi_b - lo_b) * (1.0 / 33.0);
    const double sig = fma((double)(l + 1), step, lo_b);
    const int cnt = sturm_count<N>(d, e2, sig, pivmin);
    const uint64_t m = __builtin_amdgcn_ballot_w64(cnt >= target);
    const uint32_t mh = (uint32_t)(half == 0 ? m : (m >> 32));
    const int f = mh ? __builtin_ctz(mh) : 32;
    const double na = f == 0 ? lo_b : fma((double)f, step, lo_b);
    const double nb = f == 32 ? hi_b : fma((double)(f + 1), step, lo_b);
    lo_b = na;
    hi_b = nb;
  }
  const double mid = 0.5 * (lo_b + hi_b);
  const double lmin = readlane_f64(mid, 0), lmax = readlane_f64(mid, 32);
  const int nnc = sturm_count<N>(d, e2, 10.0 * eps, pivmin);  // every lane the same
  if (below_eps && lane == 0) *below_eps = sturm_count<N>(d, e2, eps, pivmin);  // eigenvalues the clamp moves
  if (lane == 0) {
    const double mn = fmax(lmin, eps), mx = fmax(lmax, eps);
    out4[0] = mn;
    out4[1] = mx;
    out4[2] = mx / mn;
    out4[3] = (double)nnc;
  }
}

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
