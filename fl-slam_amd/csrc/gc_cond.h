// gc_cond.h — the reference's ConditioningCert fields of a symmetric 22 x 22 (or smaller) matrix on
// one wave, without an eigen-decomposition (shared by the in-scan certificates, gc_certs.hip, and the
// single-hypothesis operator entries, gc_ops.hip):
//   Householder tridiagonalisation of M_sym with one row per lane (v and w broadcast through a
//   wave-private LDS row), then lanes 0-31 / 32-63 multisect for λ_min / λ_max with Sturm counts (the
//   inertia of T − σI, as LAPACK dstebz; 33 sections per round, 11 rounds: 2^-55 of the Gershgorin
//   width, the absolute accuracy of eigh), and one more count at σ = 10 ε for the near-null count.
//   eig_min = max(λ_min, ε), eig_max = max(λ_max, ε), cond = eig_max / eig_min
//   (domain_projection_psd_core, primitives.py:80-123).
#pragma once
#include <hip/hip_runtime.h>
#include "gc_wgla.h"

namespace gc {

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

// domain_projection_psd_core of a 22 x 22 LDS matrix with every cert field (primitives.py:80-123) and
// no Jacobi sweep when the clamp is inactive: the Cholesky-certified shortcut (wg_psd_project_fast:
// projection = M_sym, projection_delta 0), then the eigen fields of M_sym by wave_conditioning on
// wave 0; an active clamp runs the full Jacobi projection, which fills every field itself. cert6 must
// be in LDS (all threads read its eig_min slot); scratch: 2 n² + 4 n doubles (also the wave's buffer).
GC_DEV void wg_psd_project_certified(const double* M, double* Mp, double eps, double* scratch, double* red,
                                     double* cert6) {
  wg_psd_project_fast(M, Mp, eps, kDZ, scratch, red, cert6);
  __syncthreads();
  const bool shortcut = cert6[2] != cert6[2];  // NaN: the eigen fields were not computed
  __syncthreads();
  if (shortcut) {
    if (threadIdx.x < 64) wave_conditioning<kDZ>(Mp, eps, scratch, cert6 + 2);
    __syncthreads();
  }
}

}  // namespace gc
