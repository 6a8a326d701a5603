// gc_wgla.h — workgroup-cooperative f64 dense linear algebra on LDS-resident matrices
// (n <= 22), for the batched-small kernels (one 256-thread workgroup per hypothesis).
//
// Restates fl_slam_poc/common/primitives.py: domain_projection_psd_core (:80-123),
// spd_cholesky_solve_lifted_core (:141-166), spd_cholesky_inverse_lifted_core (:169-192).
// The symmetric eigensolver is a parallel cyclic Jacobi (round-robin pairing, n/2 disjoint
// rotations per round applied as 2x2 tile updates, so each tile is owned by one thread and
// a round needs two barriers). Eigenvalues agree with LAPACK's eigh to ~1e-15 relative; the
// clamped reconstruction V max(λ, ε) Vᵀ is basis-independent, so PSD outputs match.
//
// Every function must be called by all 256 threads of the workgroup (uniform control flow).
#pragma once
#include "gc_math.h"

namespace gc {

constexpr int kWG = 256;
constexpr int kDZ = 22;

// dev instrumentation (gc_pipe.h GC_PHASE) inside device helpers: sink = P.io_parts (or nullptr)
#ifdef GC_PHASE_TIMING
#define GC_MARK(sink, i)                                                                        \
  do {                                                                                          \
    __syncthreads();                                                                            \
    if ((sink) && blockIdx.x == 0 && threadIdx.x == 0) (sink)[i] = (double)__builtin_readcyclecounter(); \
  } while (0)
// one thread's own stamp, no barrier (workgroup 0)
#define GC_STAMP(sink, i)                                                               \
  do {                                                                                  \
    if ((sink) && blockIdx.x == 0) (sink)[i] = (double)__builtin_readcyclecounter();    \
  } while (0)
#else
#define GC_MARK(sink, i) \
  do {                   \
  } while (0)
#define GC_STAMP(sink, i) \
  do {                    \
  } while (0)
#endif

GC_DEV int tid() { return threadIdx.x; }

GC_DEV double readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// Wave reductions (every lane active): within each 16-lane row a DPP butterfly (quad_perm
// [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror: each step pairs a lane with a partner holding a
// disjoint partial, so the row ends with one bit-identical total), then the four row totals by
// v_readlane as ((r0 + r1) + (r2 + r3)): VALU and SALU only, where the xor butterfly of
// __shfl_xor was six dependent ds_bpermute round trips through the LDS pipe. The result is wave-
// uniform; the order is fixed (deterministic).
template <int CTRL>
GC_DEV double wdpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
// DPP lane shift of a wave prefix scan: lane l takes lane l - k of its 16-lane row (row_shr:k, CTRL =
// 0x110 + k), or the last lane of the row before (row_bcast:15, CTRL 0x142, ROW_MASK 0xA: rows 1 and 3)
// or of row 1 (row_bcast:31, CTRL 0x143, ROW_MASK 0xC: rows 2 and 3); lanes without a source keep
// `old` (the scan's identity). Six steps (1, 2, 4, 8 in rows, then the two broadcasts) give an inclusive
// scan over the wave with VALU moves only (the __shfl_up form: six ds_bpermute round trips per value).
template <int CTRL, int ROW_MASK = 0xF>
GC_DEV double scan_dpp_f64(double v, double old) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), CTRL, ROW_MASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), CTRL, ROW_MASK, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <typename Op>
GC_DEV double wave_reduce(double v, const Op& op) {
  v = op(v, wdpp_f64<0xB1>(v));   // quad_perm [1,0,3,2]
  v = op(v, wdpp_f64<0x4E>(v));   // quad_perm [2,3,0,1]
  v = op(v, wdpp_f64<0x141>(v));  // row_half_mirror
  v = op(v, wdpp_f64<0x140>(v));  // row_mirror
  return op(op(readlane_f64(v, 0), readlane_f64(v, 16)), op(readlane_f64(v, 32), readlane_f64(v, 48)));
}
GC_DEV double wave_sum(double v) {
  return wave_reduce(v, [](double a, double b) { return a + b; });
}
GC_DEV double wave_max(double v) {
  return wave_reduce(v, [](double a, double b) { return fmax(a, b); });
}
GC_DEV double wave_min(double v) {
  return wave_reduce(v, [](double a, double b) { return fmin(a, b); });
}
// Deterministic workgroup sum (fixed wave tree + fixed wave order). red: >= 4 doubles of LDS.
GC_DEV double wg_sum(double v, double* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return r;
}
GC_DEV double wg_max(double v, double* red) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  __syncthreads();
  return r;
}

// Workgroup sum of s (wg_sum's order) and maxima of m1, m2 with three barriers instead of nine.
// scratch: 12 doubles of LDS not otherwise live.
GC_DEV void wg_sum_max2(double& s, double& m1, double& m2, double* scratch) {
  s = wave_sum(s);
  m1 = wave_max(m1);
  m2 = wave_max(m2);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    const int w = threadIdx.x >> 6;
    scratch[w] = s; scratch[4 + w] = m1; scratch[8 + w] = m2;
  }
  __syncthreads();
  s = (scratch[0] + scratch[1]) + (scratch[2] + scratch[3]);
  m1 = fmax(fmax(scratch[4], scratch[5]), fmax(scratch[6], scratch[7]));
  m2 = fmax(fmax(scratch[8], scratch[9]), fmax(scratch[10], scratch[11]));
  __syncthreads();
}

// N workgroup sums with two barriers instead of 3N (fixed shuffle tree + fixed wave order, as
// wg_sum). scratch: 4N doubles of LDS not otherwise live. Results replace v on every thread.
template <int N>
GC_DEV void wg_sum_n(double (&v)[N], double* scratch) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = wave_sum(v[i]);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int i = 0; i < N; ++i) scratch[(threadIdx.x >> 6) * N + i] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = (scratch[i] + scratch[N + i]) + (scratch[2 * N + i] + scratch[3 * N + i]);
  __syncthreads();
}

GC_DEV void wg_copy(double* dst, const double* src, int count) {
  for (int i = threadIdx.x; i < count; i += kWG) dst[i] = src[i];
  __syncthreads();
}

// ---- register-resident factorizations (n <= 22). Wave 0 holds one matrix row per lane (row i
// in lane i, rows >= n padded with the identity, which leaves the leading block's factors
// unchanged); column broadcasts are v_readlane (compile-time lane, loops fully unrolled). No LDS
// traffic or workgroup barriers inside the factorization: ~5x shorter latency than the
// LDS/barrier-per-column form on the 22x22 information matrices of the per-hypothesis kernels.
//
// Right-looking Cholesky of the lane rows a (lower triangle significant). CHECKED: a pivot <= 0
// (or NaN) clears ok and is replaced by 1 so the rest stays finite (wg_chol_checked semantics).
// The pivot scale is one v_rsq_f64 + a Goldschmidt step (d = √p and 1/d to ~1 ulp) instead of a
// correctly rounded sqrt and a per-lane division. Column k is broadcast as: L[k+1][k] by
// readlane (it feeds the next pivot), L[k+2..][k] through a 22-double LDS row of the calling wave
// (one ds_write per lane, then same-address broadcast reads, no readlane hazard NOPs). One wave, in
// program order, so the LDS row needs no barrier.
// DYN: the broadcast rows live in the caller's dynamic LDS (dyn, 4 x (NM + 2) doubles) instead of a
// static block, for kernels whose dynamic LDS must start at address 0 (k_bins_io's lpred_wg)
template <int NM, bool CHECKED, bool DYN = false>
GC_DEV void lane_chol(double (&a)[NM], int lane, bool& ok, double* dyn = nullptr) {
  // one broadcast row per wave: two waves may factor two matrices at once
  double* colbuf;
  if constexpr (DYN) {
    colbuf = dyn + (threadIdx.x >> 6) * (NM + 2);
  } else {
    __shared__ __attribute__((aligned(16))) double colbufs[4][NM + 2];
    colbuf = colbufs[threadIdx.x >> 6];
  }
#pragma unroll
  for (int k = 0; k < NM; ++k) {
    double piv = readlane_f64(a[k], k);
    if constexpr (CHECKED) {
      if (!(piv > 0.0)) { ok = false; piv = 1.0; }
    }
    const double y = __builtin_amdgcn_rsq(piv);
    double g = piv * y, h = 0.5 * y;
    const double r = fma(-g, h, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    const double inv = h + h;
    a[k] = lane == k ? g : (lane > k ? a[k] * inv : a[k]);
    if (k + 1 < NM) {
      if (k + 2 < NM) colbuf[lane < NM ? lane : NM + 1] = a[k];
      a[k + 1] -= a[k] * (lane == k + 1 ? a[k] : readlane_f64(a[k], k + 1));  // next pivot: no readlane
#pragma unroll
      for (int j = k + 2; j < NM; ++j) a[j] -= a[k] * colbuf[j];
    }
  }
}

template <int NM>
GC_DEV void lane_load_rows(const double* A, int n, int lane, double (&a)[NM]) {
#pragma unroll
  for (int j = 0; j < NM; ++j)
    a[j] = (lane < n && j < n) ? (j <= lane ? A[lane * n + j] : 0.0) : (lane == j ? 1.0 : 0.0);
}

template <int NM>
GC_DEV void lane_store_lower(double* A, int n, int lane, const double (&a)[NM]) {
  if (lane < n) {
#pragma unroll
    for (int j = 0; j < NM; ++j)
      if (j < n) A[lane * n + j] = j <= lane ? a[j] : 0.0;
  }
}

// wave-0 factorization padded to NM = 8 (the 6x6 / 3x3 blocks of IW, Q, pose-6) or kDZ = 22:
// the padded identity costs full columns, so small blocks take the short form
template <int NM, bool CHECKED, bool DYN = false>
GC_DEV bool wave0_chol(double* A, int n, double* dyn = nullptr) {
  const int lane = threadIdx.x & 63;  // any single wave (wave 0, or wave 1 beside a wave-0 factorization)
  double a[NM];
  lane_load_rows<NM>(A, n, lane, a);
  bool ok = true;
  lane_chol<NM, CHECKED, DYN>(a, lane, ok, dyn);
  lane_store_lower<NM>(A, n, lane, a);
  return ok;
}

// In-place lower Cholesky of the n x n (row-major) A; upper triangle zeroed.
template <bool DYN = false>
GC_DEV void wg_chol(double* A, int n, double* dyn = nullptr) {
  if (threadIdx.x < 64) {
    if (n <= 8) (void)wave0_chol<8, false, DYN>(A, n, dyn);
    else (void)wave0_chol<kDZ, false, DYN>(A, n, dyn);
  }
  __syncthreads();
}

// In-place lower Cholesky that reports failure (a pivot <= 0 or NaN): returns true on success
// on every thread. flag: one LDS double.
GC_DEV bool wg_chol_checked(double* A, int n, double* flag) {
  if (threadIdx.x < 64) {
    const bool ok = n <= 8 ? wave0_chol<8, true>(A, n) : wave0_chol<kDZ, true>(A, n);
    if (threadIdx.x == 0) flag[0] = ok ? 0.0 : 1.0;
  }
  __syncthreads();
  const bool ok = flag[0] == 0.0;
  __syncthreads();
  return ok;
}

// x = (C Cᵀ)^{-1} b for lower-triangular C (result visible to all on return). Wave 0, lane i holds
// row i and column i of C: forward substitution broadcasts y_j, backward x_j, one readlane each.
template <int NM>
GC_DEV void wave0_chol_solve(const double* C, const double* b, double* x, int n) {
  const int lane = threadIdx.x & 63;  // any single wave (callers: wave 0, or wave 1 beside wave-0 work)
  const bool live = lane < n;
  double c[NM], ct[NM];
#pragma unroll
  for (int j = 0; j < NM; ++j) {
    const bool in = live && j < n;
    c[j] = in ? (j <= lane ? C[lane * n + j] : 0.0) : (lane == j ? 1.0 : 0.0);
    ct[j] = in ? (j >= lane ? C[j * n + lane] : 0.0) : (lane == j ? 1.0 : 0.0);
  }
  const double idiag = 1.0 / (live ? C[lane * n + lane] : 1.0);  // off the dependency chain
  double r = live ? b[lane] : 0.0, y = 0.0;
#pragma unroll
  for (int j = 0; j < NM; ++j) {  // y_j = (b_j - Σ_{k<j} C_jk y_k) / C_jj
    const double yj = readlane_f64(r * idiag, j);
    if (lane == j) y = yj;
    r -= c[j] * yj;
  }
  r = y;
  double xv = 0.0;
#pragma unroll
  for (int j = NM - 1; j >= 0; --j) {  // x_j = (y_j - Σ_{k>j} C_kj x_k) / C_jj
    const double xj = readlane_f64(r * idiag, j);
    if (lane == j) xv = xj;
    r -= ct[j] * xj;
  }
  if (live) x[lane] = xv;
}
GC_DEV void wg_chol_solve(const double* C, const double* b, double* x, int n) {
  if (threadIdx.x < 64) {
    if (n <= 8) wave0_chol_solve<8>(C, b, x, n);
    else wave0_chol_solve<kDZ>(C, b, x, n);
  }
  __syncthreads();
}

// Ainv = C^{-ᵀ} C^{-1} (primitives.py:186-191: L_chol_inv.T @ L_chol_inv). scratch: n*n.
// Phase 1 (wave 0): lane j forward-substitutes column j of W = C^{-1} in registers, C read by
// same-address LDS broadcast, the row sums split over 4 accumulators (short dependency chain); the
// 1/C_ii are divided once, lane i's, and broadcast by readlane (the same correctly rounded
// quotients as a division per lane and row, 6.0k -> 4.0k cycles for 22x22,
// profiles/r03/chol_latency_micro.txt); W is stored transposed (scratch row j = column j).
// j must be the calling lane's index within its wave (lanes j >= n only contribute their 1/C_jj
// slot, unread). Phase 2 (all 4
// waves): thread (g = t/32, j = t%32) forms Ainv[i][j] = Σ_k W[k][i] W[k][j] for i ≡ g (mod 8),
// its column j of W in registers and column i broadcast; k ascends over the full range (the
// entries below the triangles are exact zeros), the order of the reference's product.
GC_DEV void chol_inverse_phase1_lane(const double* C, double* scratch, int n, int j) {
  const int lane = threadIdx.x & 63;
  const double rdiag = 1.0 / (lane < n ? C[lane * n + lane] : 1.0);
  if (j < n) {
    double col[kDZ];
#pragma unroll
    for (int i = 0; i < kDZ; ++i) {
      col[i] = 0.0;
      if (i < n) {
        const double* Ci = C + i * n;
        double s[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < i; ++k) s[k & 3] = fma(Ci[k], col[k], s[k & 3]);
        const double v = ((i == j) ? 1.0 : 0.0) - ((s[0] + s[1]) + (s[2] + s[3]));
        col[i] = i >= j ? v * readlane_f64(rdiag, i) : 0.0;
      }
    }
#pragma unroll
    for (int k = 0; k < kDZ; ++k)
      if (k < n) scratch[j * n + k] = col[k];
  }
}
GC_DEV void chol_inverse_phase1(const double* C, double* scratch, int n) {
  chol_inverse_phase1_lane(C, scratch, n, threadIdx.x);
}
// phase 2 on threads tid in [0, nthr) (a multiple of 32): the same products, rows i = g (mod nthr/32)
GC_DEV void chol_inverse_phase2_part(double* Ainv, const double* scratch, int n, int tid, int nthr) {
  const int j = tid & 31, g = tid >> 5;
  if (j < n) {
    double wj[kDZ];
#pragma unroll
    for (int k = 0; k < kDZ; ++k) wj[k] = k < n ? scratch[j * n + k] : 0.0;
    for (int i = g; i < n; i += nthr / 32) {
      const double* wi = scratch + i * n;
      double v = 0.0;
#pragma unroll
      for (int k = 0; k < kDZ; ++k)
        if (k < n) v = fma(wi[k], wj[k], v);
      Ainv[i * n + j] = v;
    }
  }
}
GC_DEV void chol_inverse_phase2(double* Ainv, const double* scratch, int n) {
  chol_inverse_phase2_part(Ainv, scratch, n, threadIdx.x, kWG);
}
GC_DEV void wg_chol_inverse(const double* C, double* Ainv, double* scratch, int n) {
  chol_inverse_phase1(C, scratch, n);
  __syncthreads();
  chol_inverse_phase2(Ainv, scratch, n);
  __syncthreads();
}
// wg_chol_inverse(C) and, on wave 1 while wave 0 forward-substitutes, x = (C Cᵀ)⁻¹ b
// (wave0_chol_solve): the two results are exactly those of the separate calls.
GC_DEV void wg_chol_inverse_and_solve(const double* C, double* Ainv, double* scratch, int n, const double* b,
                                      double* x) {
  if (threadIdx.x < 64) chol_inverse_phase1(C, scratch, n);
  else if (threadIdx.x < 128) {
    if (n <= 8) wave0_chol_solve<8>(C, b, x, n);
    else wave0_chol_solve<kDZ>(C, b, x, n);
  }
  __syncthreads();
  chol_inverse_phase2(Ainv, scratch, n);
  __syncthreads();
}

// Lifted solve / inverse (primitives.py:141-192). work: n*n scratch, work2: n*n scratch.
GC_DEV void wg_solve_lifted(const double* L, const double* b, double* x, double eps_lift, int n,
                            double* work) {
  for (int idx = threadIdx.x; idx < n * n; idx += kWG)
    work[idx] = L[idx] + ((idx / n == idx % n) ? eps_lift : 0.0);
  __syncthreads();
  wg_chol(work, n);
  wg_chol_solve(work, b, x, n);
}
GC_DEV void wg_inverse_lifted(const double* L, double* Linv, double eps_lift, int n, double* work,
                              double* work2) {
  for (int idx = threadIdx.x; idx < n * n; idx += kWG)
    work[idx] = L[idx] + ((idx / n == idx % n) ? eps_lift : 0.0);
  __syncthreads();
  wg_chol(work, n);
  wg_chol_inverse(work, Linv, work2, n);
}

// Round-robin (circle method) pair k of round r for even n: p < q.
GC_DEV void rr_pair(int n, int r, int k, int* p, int* q) {
  const int m = n - 1;
  int a, b;
  if (k == 0) {
    a = m;
    b = r % m;
  } else {
    a = (r + k) % m;
    b = (r - k + m) % m;
  }
  *p = a < b ? a : b;
  *q = a < b ? b : a;
}

// Parallel cyclic Jacobi on the symmetric n x n (n even, <= 22) A (destroyed). If V != nullptr
// it accumulates eigenvectors (columns). w receives the (unsorted) eigenvalues.
// cs: 2*(n/2) doubles + n/2 ints worth of LDS (pass >= 3*n doubles), red: 4 doubles.
GC_DEV void wg_jacobi_eigh(double* A, double* V, double* w, int n, double* cs, double* red) {
  const int half = n / 2;
  const int tiles = half * half;
  int* pq = reinterpret_cast<int*>(cs + 2 * half);
  if (V)
    for (int idx = threadIdx.x; idx < n * n; idx += kWG) V[idx] = (idx / n == idx % n) ? 1.0 : 0.0;
  // diagonal norm for the relative convergence test
  double dloc = 0.0;
  for (int i = threadIdx.x; i < n; i += kWG) dloc += A[i * n + i] * A[i * n + i];
  double offloc = 0.0;
  for (int idx = threadIdx.x; idx < n * n; idx += kWG)
    if (idx / n != idx % n) offloc += A[idx] * A[idx];
  const double fro2 = wg_sum(dloc + offloc, red);
  double off = wg_sum(offloc, red);
  // stop once the off-diagonal mass is at rounding level (||offdiag||_F <= 1e-15 ||A||_F)
  for (int sweep = 0; sweep < 20 && off > 1e-30 * fro2 && off > 1e-300; ++sweep) {
    for (int r = 0; r < n - 1; ++r) {
      if ((int)threadIdx.x < half) {
        int p, q;
        rr_pair(n, r, threadIdx.x, &p, &q);
        const double apq = A[p * n + q], app = A[p * n + p], aqq = A[q * n + q];
        double c = 1.0, s = 0.0;
        if (apq != 0.0 && fabs(apq) > 1e-300 && fabs(apq) > 1e-18 * sqrt(fabs(app * aqq))) {
          const double th = (aqq - app) / (2.0 * apq);
          const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
          c = 1.0 / sqrt(t * t + 1.0);
          s = t * c;
        }
        cs[2 * threadIdx.x] = c;
        cs[2 * threadIdx.x + 1] = s;
        pq[2 * threadIdx.x] = p;
        pq[2 * threadIdx.x + 1] = q;
      }
      __syncthreads();
      // A tiles: B' = G_Iᵀ B G_J
      for (int t = threadIdx.x; t < tiles; t += kWG) {
        const int I = t / half, J = t % half;
        const int pi = pq[2 * I], qi = pq[2 * I + 1], pj = pq[2 * J], qj = pq[2 * J + 1];
        const double ci = cs[2 * I], si = cs[2 * I + 1], cj = cs[2 * J], sj = cs[2 * J + 1];
        const double b00 = A[pi * n + pj], b01 = A[pi * n + qj], b10 = A[qi * n + pj], b11 = A[qi * n + qj];
        // B G_J : columns
        const double c00 = cj * b00 - sj * b01, c01 = sj * b00 + cj * b01;
        const double c10 = cj * b10 - sj * b11, c11 = sj * b10 + cj * b11;
        // G_Iᵀ (B G_J) : rows
        double n00 = ci * c00 - si * c10, n01 = ci * c01 - si * c11;
        double n10 = si * c00 + ci * c10, n11 = si * c01 + ci * c11;
        if (I == J) { n01 = 0.0; n10 = 0.0; }
        A[pi * n + pj] = n00; A[pi * n + qj] = n01; A[qi * n + pj] = n10; A[qi * n + qj] = n11;
      }
      if (V) {
        const int items = n * half;
        for (int t = (int)threadIdx.x - tiles; t < items; t += kWG) {
          if (t < 0) continue;
          const int i = t / half, k = t % half;
          const int p = pq[2 * k], q = pq[2 * k + 1];
          const double c = cs[2 * k], s = cs[2 * k + 1];
          const double vp = V[i * n + p], vq = V[i * n + q];
          V[i * n + p] = c * vp - s * vq;
          V[i * n + q] = s * vp + c * vq;
        }
      }
      __syncthreads();
    }
    offloc = 0.0;
    for (int idx = threadIdx.x; idx < n * n; idx += kWG)
      if (idx / n != idx % n) offloc += A[idx] * A[idx];
    off = wg_sum(offloc, red);
  }
  for (int i = threadIdx.x; i < n; i += kWG) w[i] = A[i * n + i];
  __syncthreads();
}

// domain_projection_psd_core (primitives.py:80-123) on an n x n LDS matrix (n even <= 22).
// M (input, preserved) -> Mp. cert6 (LDS or registers, written by all) =
// [projection_delta, sym_delta, eig_min, eig_max, cond, near_null_count].
// scratch: 2*n*n + 4*n doubles.
GC_DEV void wg_psd_project(const double* M, double* Mp, double eps, int n, double* scratch,
                           double* red, double* cert6) {
  double* S = scratch;             // symmetrised, then Jacobi workspace
  double* V = scratch + n * n;     // eigenvectors
  double* w = scratch + 2 * n * n; // eigenvalues (clamped)
  double* cs = w + n;              // 3n
  double symloc = 0.0;
  for (int idx = threadIdx.x; idx < n * n; idx += kWG) {
    const int i = idx / n, j = idx % n;
    const double s = 0.5 * (M[i * n + j] + M[j * n + i]);
    const double d = s - M[idx];
    symloc += d * d;
    Mp[idx] = s;  // keep M_sym in Mp for the delta
    S[idx] = s;
  }
  const double symd = wg_sum(symloc, red);
  wg_jacobi_eigh(S, V, w, n, cs, red);
  double mnl = 1e308, mxl = -1e308, nnl = 0.0;
  if ((int)threadIdx.x < n) {
    const double wc = fmax(w[threadIdx.x], eps);
    w[threadIdx.x] = wc;
    mnl = wc; mxl = wc; nnl = (wc < 10.0 * eps) ? 1.0 : 0.0;
  }
  const double mn = -wg_max(-mnl, red);
  const double mx = wg_max(mxl, red);
  const double nn = wg_sum(nnl, red);
  double projloc = 0.0;
  for (int idx = threadIdx.x; idx < n * n; idx += kWG) {
    const int i = idx / n, j = idx % n;
    double v = 0.0;
    for (int k = 0; k < n; ++k) v += V[i * n + k] * w[k] * V[j * n + k];
    const double d = v - Mp[idx];
    projloc += d * d;
    S[idx] = v;
  }
  const double proj = wg_sum(projloc, red);
  for (int idx = threadIdx.x; idx < n * n; idx += kWG) Mp[idx] = S[idx];
  __syncthreads();
  if (cert6 && threadIdx.x == 0) {
    cert6[0] = sqrt(proj); cert6[1] = sqrt(symd); cert6[2] = mn; cert6[3] = mx;
    cert6[4] = mx / mn; cert6[5] = nn;
  }
  __syncthreads();
}

// domain_projection_psd_core with a certified shortcut, for the batched pipeline: if
// Cholesky of (M_sym - eps I) succeeds, every eigenvalue exceeds eps, the clamp is inactive and
// the projection is M_sym itself (the reference's V diag(λ) Vᵀ reconstructs M_sym up to
// rounding, ~1e-15 ||M||). projection_delta is then 0 and the eigen fields of cert6 are NaN
// (not computed). Otherwise the full Jacobi projection runs. scratch: 2n*n + 4n doubles.
struct NoSideWork {
  GC_DEV void operator()() const {}
};
// side(): optional wave-level work for wave 2, run beside the Cholesky (no barrier inside)
template <typename Side = NoSideWork, bool DYN = false>
GC_DEV void wg_psd_project_fast(const double* M, double* Mp, double eps, int n, double* scratch,
                                double* red, double* cert6, const Side& side = Side(), double* dyn = nullptr) {
  for (int idx = threadIdx.x; idx < n * n; idx += kWG) {
    const int i = idx / n, j = idx % n;
    scratch[idx] = 0.5 * (M[i * n + j] + M[j * n + i]) - ((i == j) ? eps : 0.0);
  }
  __syncthreads();
  // Cholesky on wave 0; the symmetry deviation (cert field 1) on wave 1 meanwhile
  if (threadIdx.x < 64) {
    const bool okc = n <= 8 ? wave0_chol<8, true, DYN>(scratch, n, dyn) : wave0_chol<kDZ, true, DYN>(scratch, n, dyn);
    if (threadIdx.x == 0) red[4] = okc ? 0.0 : 1.0;
  } else if (threadIdx.x < 128) {
    double symloc = 0.0;
    for (int idx = threadIdx.x - 64; idx < n * n; idx += 64) {
      const int i = idx / n, j = idx % n;
      const double d = 0.5 * (M[i * n + j] + M[j * n + i]) - M[idx];
      symloc += d * d;
    }
    symloc = wave_sum(symloc);
    if (threadIdx.x == 64) red[5] = symloc;
  } else if (threadIdx.x < 192) {
    side();
  }
  __syncthreads();
  const bool spd = red[4] == 0.0;
  const double symd = red[5];
  __syncthreads();
  if (spd) {
    for (int idx = threadIdx.x; idx < n * n; idx += kWG) {
      const int i = idx / n, j = idx % n;
      Mp[idx] = 0.5 * (M[i * n + j] + M[j * n + i]);
    }
    if (cert6 && threadIdx.x == 0) {
      const double nan = __builtin_nan("");
      cert6[0] = 0.0; cert6[1] = sqrt(symd); cert6[2] = nan; cert6[3] = nan; cert6[4] = nan; cert6[5] = nan;
    }
    __syncthreads();
    return;
  }
  wg_psd_project(M, Mp, eps, n, scratch, red, cert6);
}

// wg_psd_project_fast of M and the lifted factorization of its result, the two Cholesky
// factorizations at once: wave 0 certifies M_sym − εI (as wg_psd_project_fast), wave 1 factors
// M_sym + ε_lift I into Cl, which is chol(Mp + ε_lift I) whenever the certificate holds (Mp =
// M_sym then, the same values the separate calls would factor: bit-identical), wave 2 the symmetry
// deviation, wave 3 side(). If the certificate fails, the Jacobi projection runs and Cl is
// refactored from Mp. On return Mp is the projection and Cl its lifted factor (lower, upper zeroed).
// scratch: 2n*n + 4n doubles; Cl: n*n.
template <typename Side = NoSideWork>
GC_DEV void wg_psd_fast_lifted_chol(const double* M, double* Mp, double eps, double eps_lift, int n, double* scratch,
                                    double* Cl, double* red, double* cert6, const Side& side = Side()) {
  for (int idx = threadIdx.x; idx < n * n; idx += kWG) {
    const int i = idx / n, j = idx % n;
    const double sym = 0.5 * (M[i * n + j] + M[j * n + i]);
    scratch[idx] = sym - ((i == j) ? eps : 0.0);
    Cl[idx] = sym + ((i == j) ? eps_lift : 0.0);
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const bool okc = n <= 8 ? wave0_chol<8, true>(scratch, n) : wave0_chol<kDZ, true>(scratch, n);
    if (threadIdx.x == 0) red[4] = okc ? 0.0 : 1.0;
  } else if (threadIdx.x < 128) {
    if (n <= 8) (void)wave0_chol<8, false>(Cl, n);
    else (void)wave0_chol<kDZ, false>(Cl, n);
  } else if (threadIdx.x < 192) {
    double symloc = 0.0;
    for (int idx = threadIdx.x - 128; idx < n * n; idx += 64) {
      const int i = idx / n, j = idx % n;
      const double d = 0.5 * (M[i * n + j] + M[j * n + i]) - M[idx];
      symloc += d * d;
    }
    symloc = wave_sum(symloc);
    if (threadIdx.x == 128) red[5] = symloc;
  } else {
    side();
  }
  __syncthreads();
  const bool spd = red[4] == 0.0;
  const double symd = red[5];
  __syncthreads();
  if (spd) {
    for (int idx = threadIdx.x; idx < n * n; idx += kWG) {
      const int i = idx / n, j = idx % n;
      Mp[idx] = 0.5 * (M[i * n + j] + M[j * n + i]);
    }
    if (cert6 && threadIdx.x == 0) {
      const double nan = __builtin_nan("");
      cert6[0] = 0.0; cert6[1] = sqrt(symd); cert6[2] = nan; cert6[3] = nan; cert6[4] = nan; cert6[5] = nan;
    }
    __syncthreads();
    return;
  }
  wg_psd_project(M, Mp, eps, n, scratch, red, cert6);
  for (int idx = threadIdx.x; idx < n * n; idx += kWG) Cl[idx] = Mp[idx] + ((idx / n == idx % n) ? eps_lift : 0.0);
  __syncthreads();
  wg_chol(Cl, n);
}

GC_DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// x = (I + B)⁻¹ b with B = ε (S_sym + ε I), S an n x n LDS matrix (row-major, symmetrised here), on one
// wave: lane i < n owns row i of B and b_i (b_lane), and returns x_i. This is (L' + εI)⁻¹ L' applied
// in the predict when L' = (S + εI)⁻¹ (a lifted inverse): (L' + εI)⁻¹ L' = (I + ε(S + εI))⁻¹, whose
// matrix is within ‖B‖ of the identity, so a Richardson iteration x ← b − B x (from x = b) converges
// by a factor ‖B‖∞ per step and its rounding is that of one well-conditioned product; the step count
// is the one that takes ‖B‖∞^k below 2^-56 (uniform over the wave). Returns false (x = b) when
// ‖B‖∞ > 1/4: the caller then takes the factorised route. xrow: an n-double LDS row of this wave.
template <int NM>
GC_DEV bool wave_lift_iterate(const double* S, double b_lane, double eps, double* xrow, int n, double& x_out) {
  const int lane = threadIdx.x & 63;
  const bool live = lane < n;
  double br[NM];
  double rs = 0.0;
#pragma unroll
  for (int j = 0; j < NM; ++j) {
    const bool in = live && j < n;
    br[j] = in ? eps * (0.5 * (S[lane * n + j] + S[j * n + lane]) + (j == lane ? eps : 0.0)) : 0.0;
    rs += fabs(br[j]);
  }
  const double r = wave_max(rs);
  const double bi = live ? b_lane : 0.0;
  x_out = bi;
  if (!(r <= 0.25)) return false;
  const int iters = r > 0.0 ? (int)ceil(38.816242111356935 / -log(r)) : 1;  // 56 ln 2 / -ln r
  double xi = bi;
  for (int it = 0; it < iters; ++it) {
    if (live) xrow[lane] = xi;
    wave_lds_sync();
    double s[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int j = 0; j < NM; ++j)
      if (j < n) s[j & 3] = fma(br[j], xrow[j], s[j & 3]);
    wave_lds_sync();  // every lane's reads of the row are done before the next step rewrites it
    xi = bi - ((s[0] + s[1]) + (s[2] + s[3]));
  }
  x_out = xi;
  return true;
}

// The parallel cyclic Jacobi of wg_jacobi_eigh (eigenvalues only) on wave 0 for n <= 16: the
// same round-robin rotations and convergence test, with wave barriers and shuffle sums in place of
// workgroup barriers (a 6x6 needs ~40 rounds; the workgroup form pays two barriers per round).
GC_DEV void wave_jacobi_eigvals(double* A, double* w, int n, double* cs) {
  const int lane = threadIdx.x;  // caller: threadIdx.x < 64
  const int half = n / 2, tiles = half * half;
  int* pq = reinterpret_cast<int*>(cs + 2 * half);
  double dloc = 0.0, offloc = 0.0;
  for (int i = lane; i < n; i += 64) dloc += A[i * n + i] * A[i * n + i];
  for (int idx = lane; idx < n * n; idx += 64)
    if (idx / n != idx % n) offloc += A[idx] * A[idx];
  const double fro2 = wave_sum(dloc + offloc);
  double off = wave_sum(offloc);
  for (int sweep = 0; sweep < 20 && off > 1e-30 * fro2 && off > 1e-300; ++sweep) {
    for (int r = 0; r < n - 1; ++r) {
      if (lane < half) {
        int p, q;
        rr_pair(n, r, lane, &p, &q);
        const double apq = A[p * n + q], app = A[p * n + p], aqq = A[q * n + q];
        double c = 1.0, s = 0.0;
        if (apq != 0.0 && fabs(apq) > 1e-300 && fabs(apq) > 1e-18 * sqrt(fabs(app * aqq))) {
          const double th = (aqq - app) / (2.0 * apq);
          const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
          c = 1.0 / sqrt(t * t + 1.0);
          s = t * c;
        }
        cs[2 * lane] = c;
        cs[2 * lane + 1] = s;
        pq[2 * lane] = p;
        pq[2 * lane + 1] = q;
      }
      wave_lds_sync();
      for (int t = lane; t < tiles; t += 64) {
        const int I = t / half, J = t % half;
        const int pi = pq[2 * I], qi = pq[2 * I + 1], pj = pq[2 * J], qj = pq[2 * J + 1];
        const double ci = cs[2 * I], si = cs[2 * I + 1], cj = cs[2 * J], sj = cs[2 * J + 1];
        const double b00 = A[pi * n + pj], b01 = A[pi * n + qj], b10 = A[qi * n + pj], b11 = A[qi * n + qj];
        const double c00 = cj * b00 - sj * b01, c01 = sj * b00 + cj * b01;
        const double c10 = cj * b10 - sj * b11, c11 = sj * b10 + cj * b11;
        double n00 = ci * c00 - si * c10, n01 = ci * c01 - si * c11;
        double n10 = si * c00 + ci * c10, n11 = si * c01 + ci * c11;
        if (I == J) { n01 = 0.0; n10 = 0.0; }
        A[pi * n + pj] = n00; A[pi * n + qj] = n01; A[qi * n + pj] = n10; A[qi * n + qj] = n11;
      }
      wave_lds_sync();
    }
    offloc = 0.0;
    for (int idx = lane; idx < n * n; idx += 64)
      if (idx / n != idx % n) offloc += A[idx] * A[idx];
    off = wave_sum(offloc);
  }
  for (int i = lane; i < n; i += 64) w[i] = A[i * n + i];
}

// eigvalsh (ascending not required) of the symmetrised n x n M -> w. scratch: n*n + 3n.
GC_DEV void wg_eigvalsh(const double* M, double* w, int n, double* scratch, double* red) {
  double* S = scratch;
  double* cs = scratch + n * n;
  for (int idx = threadIdx.x; idx < n * n; idx += kWG) {
    const int i = idx / n, j = idx % n;
    S[idx] = 0.5 * (M[i * n + j] + M[j * n + i]);
  }
  __syncthreads();
  if (n <= 16) {
    if (threadIdx.x < 64) wave_jacobi_eigvals(S, w, n, cs);
    __syncthreads();
    return;
  }
  wg_jacobi_eigh(S, nullptr, w, n, cs, red);
}

// Extreme eigenvalues of a symmetric N x N (N <= 8) in LDS, wave 0 only (no workgroup barrier):
// every lane runs the same Householder tridiagonalisation in registers (the Lanczos/LAPACK
// reduction, so no broadcast is needed afterwards), then lanes 0-31 multisect for λ_min and lanes
// 32-63 for λ_max with Sturm counts (the inertia of T − σI, as LAPACK dstebz): 33 sections per
// round, 11 rounds take the Gershgorin interval to 2^-55 of its width (absolute accuracy ~u‖A‖,
// that of eigh). Replaces the full Jacobi sweep where only the conditioning is consumed.
template <int N>
GC_DEV void wave_extreme_eigvals(const double* S, double& lmin, double& lmax) {
  double A[N][N];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) A[i][j] = S[i * N + j];
  double d[N], e[N];
#pragma unroll
  for (int k = 0; k < N - 2; ++k) {
    double ss = 0.0;
#pragma unroll
    for (int i = k + 2; i < N; ++i) ss = fma(A[i][k], A[i][k], ss);
    const double x0 = A[k + 1][k];
    const double sigma = sqrt(fma(x0, x0, ss));
    if (ss == 0.0) {  // already tridiagonal in this column
      e[k] = x0;
      continue;
    }
    const double alpha = x0 >= 0.0 ? -sigma : sigma;
    double v[N];
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = i > k + 1 ? A[i][k] : 0.0;
    v[k + 1] = x0 - alpha;
    const double beta = 1.0 / (sigma * (sigma + fabs(x0)));  // 2 / vᵀv
    double p[N];
#pragma unroll
    for (int i = k + 1; i < N; ++i) {
      double acc = 0.0;
#pragma unroll
      for (int j = k + 1; j < N; ++j) acc = fma(A[i][j], v[j], acc);
      p[i] = beta * acc;
    }
    double pv = 0.0;
#pragma unroll
    for (int i = k + 1; i < N; ++i) pv = fma(p[i], v[i], pv);
    const double K = 0.5 * beta * pv;
#pragma unroll
    for (int i = k + 1; i < N; ++i) p[i] = fma(-K, v[i], p[i]);  // w
#pragma unroll
    for (int i = k + 1; i < N; ++i)
#pragma unroll
      for (int j = k + 1; j < N; ++j) A[i][j] = A[i][j] - (v[i] * p[j] + p[i] * v[j]);
    e[k] = alpha;
  }
  e[N - 2] = A[N - 1][N - 2];
  e[N - 1] = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) d[i] = A[i][i];
  double lo = d[0] - fabs(e[0]), hi = d[0] + fabs(e[0]), emax2 = 0.0;
#pragma unroll
  for (int i = 1; i < N; ++i) {
    const double r = fabs(e[i - 1]) + fabs(e[i]);
    lo = fmin(lo, d[i] - r);
    hi = fmax(hi, d[i] + r);
    emax2 = fmax(emax2, e[i - 1] * e[i - 1]);
  }
  const double pivmin = 2.2250738585072014e-308 * fmax(1.0, emax2);
  const int lane = threadIdx.x & 63, half = lane >> 5, l = lane & 31;
  double a = lo, b = hi;  // this half's bracket: λ_min (half 0) or λ_max (half 1)
  const int target = half == 0 ? 1 : N;  // first σ with count(σ) >= target lies above the eigenvalue
  for (int round = 0; round < 11; ++round) {
    const double step = (b - a) * (1.0 / 33.0);
    const double sig = fma((double)(l + 1), step, a);
    int cnt = 0;
    double q = d[0] - sig;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
#pragma unroll
    for (int i = 1; i < N; ++i) {
      q = (d[i] - sig) - e[i - 1] * e[i - 1] / q;
      if (fabs(q) < pivmin) q = -pivmin;
      cnt += q < 0.0;
    }
    const uint64_t m = __builtin_amdgcn_ballot_w64(cnt >= target);
    const uint32_t mh = (uint32_t)(half == 0 ? m : (m >> 32));
    const int f = mh ? __builtin_ctz(mh) : 32;  // first section point above the eigenvalue
    const double na = f == 0 ? a : fma((double)f, step, a);
    const double nb = f == 32 ? b : fma((double)(f + 1), step, a);
    a = na;
    b = nb;
  }
  const double mid = 0.5 * (a + b);
  lmin = readlane_f64(mid, 0);
  lmax = readlane_f64(mid, 32);
}

// y = A x (n x n, LDS), threads < n
GC_DEV void wg_matvec(const double* A, const double* x, double* y, int n) {
  if ((int)threadIdx.x < n) {
    double v = 0.0;
    for (int k = 0; k < n; ++k) v += A[threadIdx.x * n + k] * x[k];
    y[threadIdx.x] = v;
  }
  __syncthreads();
}

}  // namespace gc
