// gc_math.h — register-resident f64 math for the GC-SLAM v2 kernels (gfx950).
//
// Lie maps restate fl_slam_poc/common/geometry/se3_jax.py (so3_exp :259-301, so3_log :304-366,
// se3_V :137-174, _se3_V_inv :177-217, se3_exp :473-504, se3_log :220-256, se3_compose
// :420-438); kappa restates backend/operators/kappa.py:130-169; the 3x3 symmetric eigen / SVD
// replace jnp.linalg.eigh / svd on 3x3 blocks (matrix_fisher_evidence.py:199-233,
// binning.py:183-189). Everything is branch-uniform per lane and allocation-free.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define GC_DEV __device__ __forceinline__

namespace gc {

constexpr double kSmallAngle = 1e-7;
constexpr double kNearPi = 1e-7;
constexpr double kPi = 3.141592653589793238462643383279502884;
constexpr double kF64Eps = 2.220446049250313e-16;

GC_DEV double clampd(double x, double lo, double hi) { return fmin(fmax(x, lo), hi); }

// jax.nn.sigmoid, evaluated without overflow.
GC_DEV double sigmoid(double x) {
  if (x >= 0.0) return 1.0 / (1.0 + exp(-x));
  double e = exp(x);
  return e / (1.0 + e);
}

// smooth_window_weights (imu_preintegration.py:19-43)
GC_DEV double window_weight(double t, double t0, double t1, double sigma) {
  const double sig = fmax(sigma, 1e-6);
  const double wr = sigmoid((t - t0) / sig) * sigmoid((t1 - t) / sig);
  return wr * (1.0 - 1e-12) + 1e-12;
}

// jax.nn.softplus = log1p(exp(-|x|)) + max(x, 0)
GC_DEV double softplus(double x) { return log1p(exp(-fabs(x))) + fmax(x, 0.0); }

// ---------------------------------------------------------------- 3-vectors / 3x3 (row-major)
GC_DEV void mat3_mul(const double* A, const double* B, double* C) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}
GC_DEV void mat3_mul_tn(const double* A, const double* B, double* C) {  // Aᵀ B
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      C[3 * i + j] = A[i] * B[j] + A[3 + i] * B[3 + j] + A[6 + i] * B[6 + j];
}
GC_DEV void mat3_mul_nt(const double* A, const double* B, double* C) {  // A Bᵀ
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      C[3 * i + j] = A[3 * i] * B[3 * j] + A[3 * i + 1] * B[3 * j + 1] + A[3 * i + 2] * B[3 * j + 2];
}
GC_DEV void mat3_vec(const double* A, const double* x, double* y) {
  for (int i = 0; i < 3; ++i) y[i] = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
}
GC_DEV void mat3_tvec(const double* A, const double* x, double* y) {  // Aᵀ x
  for (int i = 0; i < 3; ++i) y[i] = A[i] * x[0] + A[3 + i] * x[1] + A[6 + i] * x[2];
}
GC_DEV void cross3(const double* a, const double* b, double* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}
GC_DEV double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
GC_DEV double norm3(const double* a) { return sqrt(dot3(a, a)); }
GC_DEV double det3(const double* A) {
  return A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) +
         A[2] * (A[3] * A[7] - A[4] * A[6]);
}

// I + a K + b K², K = [w]×  (the Rodrigues / V form shared by so3_exp and se3_V)
GC_DEV void rodrigues_form(const double* w, double a, double b, double* R) {
  const double x = w[0], y = w[1], z = w[2];
  const double xx = x * x, yy = y * y, zz = z * z;
  // K² = w wᵀ - |w|² I
  R[0] = 1.0 + b * (-(yy + zz));
  R[4] = 1.0 + b * (-(xx + zz));
  R[8] = 1.0 + b * (-(xx + yy));
  R[1] = -a * z + b * (x * y);
  R[3] = a * z + b * (x * y);
  R[2] = a * y + b * (x * z);
  R[6] = -a * y + b * (x * z);
  R[5] = -a * x + b * (y * z);
  R[7] = a * x + b * (y * z);
}

// se3_jax.py:259-301
GC_DEV void so3_exp(const double* w, double* R) {
  const double ts = dot3(w, w);
  const double th = sqrt(ts);
  double a, b;
  if (th < kSmallAngle) {
    a = 1.0;
    b = 0.5;
  } else {
    double s, c;
    sincos(th, &s, &c);
    const double sts = (ts < kSmallAngle * kSmallAngle) ? 1.0 : ts;
    a = s / th;
    b = (1.0 - c) / sts;
  }
  rodrigues_form(w, a, b, R);
}

// B=(1-cos)/θ², C=(θ-sin)/θ³ with the θ<1e-7 Taylor branch (se3_jax.py:137-174)
GC_DEV void se3_BC(double ts, double* B, double* C) {
  const double th = sqrt(ts);
  if (th < kSmallAngle) {
    *B = 0.5 - ts / 24.0;
    *C = 1.0 / 6.0 - ts / 120.0;
  } else {
    double s, c;
    sincos(th, &s, &c);
    const double sts = (ts < kSmallAngle * kSmallAngle) ? 1.0 : ts;
    *B = (1.0 - c) / sts;
    *C = (th - s) / (sts * th);
  }
}

// se3_jax.py:137-175
GC_DEV void se3_V(const double* phi, double* V) {
  double B, C;
  se3_BC(dot3(phi, phi), &B, &C);
  rodrigues_form(phi, B, C, V);
}

// se3_jax.py:473-504 : out = [V(φ)ρ, φ]
GC_DEV void se3_exp(const double* xi, double* out) {
  const double* phi = xi + 3;
  double B, C, V[9];
  se3_BC(dot3(phi, phi), &B, &C);
  rodrigues_form(phi, B, C, V);
  mat3_vec(V, xi, out);
  out[3] = phi[0];
  out[4] = phi[1];
  out[5] = phi[2];
}

// se3_jax.py:304-366 (incl. the softmax-mixed near-π axis)
GC_DEV void so3_log(const double* R, double* w) {
  const double c = clampd(0.5 * ((R[0] + R[4] + R[8]) - 1.0), -1.0, 1.0);
  const double th = acos(c);
  const double v0 = 0.5 * (R[7] - R[5]), v1 = 0.5 * (R[2] - R[6]), v2 = 0.5 * (R[3] - R[1]);
  if (th < kSmallAngle) {
    w[0] = v0; w[1] = v1; w[2] = v2;
    return;
  }
  if (fabs(th - kPi) < kNearPi) {
    const double z0 = 50.0 * (R[0] + 1.0), z1 = 50.0 * (R[4] + 1.0), z2 = 50.0 * (R[8] + 1.0);
    const double zm = fmax(z0, fmax(z1, z2));
    double e0 = exp(z0 - zm), e1 = exp(z1 - zm), e2 = exp(z2 - zm);
    const double es = e0 + e1 + e2;
    e0 /= es; e1 /= es; e2 /= es;
    double ax[3];
    for (int i = 0; i < 3; ++i)
      ax[i] = e0 * (R[3 * i] + (i == 0)) + e1 * (R[3 * i + 1] + (i == 1)) + e2 * (R[3 * i + 2] + (i == 2));
    double n = norm3(ax);
    n = (n < kSmallAngle) ? 1.0 : n;
    for (int i = 0; i < 3; ++i) w[i] = ax[i] / n * th;
    return;
  }
  double s = sin(th);
  s = (fabs(s) < kSmallAngle) ? 1.0 : s;
  const double k = th / (2.0 * s);
  w[0] = k * (2.0 * v0); w[1] = k * (2.0 * v1); w[2] = k * (2.0 * v2);
}

// se3_jax.py:177-217
GC_DEV void se3_V_inv(const double* phi, double* Vi) {
  const double ts = dot3(phi, phi);
  const double th = sqrt(ts);
  double D;
  if (th < kSmallAngle) {
    D = 1.0 / 12.0 + ts / 720.0;
  } else {
    double s, c;
    sincos(th, &s, &c);
    const double sts = (ts < kSmallAngle * kSmallAngle) ? 1.0 : ts;
    D = 1.0 / sts - (1.0 + c) / (2.0 * th * s + 1e-12);
  }
  rodrigues_form(phi, -0.5, D, Vi);
}

// se3_jax.py:220-256
GC_DEV void se3_log(const double* T, double* xi) {
  double R[9], phi[3], Vi[9];
  so3_exp(T + 3, R);
  so3_log(R, phi);
  se3_V_inv(phi, Vi);
  mat3_vec(Vi, T, xi);
  xi[3] = phi[0]; xi[4] = phi[1]; xi[5] = phi[2];
}

// se3_jax.py:420-438
// se3_compose given Ra = so3_exp(a rot) and Rb = so3_exp(b rot) (formed elsewhere, e.g. on other waves)
GC_DEV void se3_compose_R(const double* a, const double* Ra, const double* b, const double* Rb, double* out) {
  double Rab[9], t[3];
  mat3_vec(Ra, b, t);
  mat3_mul(Ra, Rb, Rab);
  double o[6];
  o[0] = a[0] + t[0]; o[1] = a[1] + t[1]; o[2] = a[2] + t[2];
  so3_log(Rab, o + 3);
  for (int i = 0; i < 6; ++i) out[i] = o[i];
}
GC_DEV void se3_compose(const double* a, const double* b, double* out) {
  double Ra[9], Rb[9];
  so3_exp(a + 3, Ra);
  so3_exp(b + 3, Rb);
  se3_compose_R(a, Ra, b, Rb, out);
}

// se3_jax.py:442-453 : [-Rᵀ t, log(Rᵀ)]
GC_DEV void se3_inverse(const double* a, double* out) {
  double R[9], Rt[9], o[6];
  so3_exp(a + 3, R);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Rt[3 * i + j] = R[3 * j + i];
  mat3_vec(Rt, a, o);
  o[0] = -o[0]; o[1] = -o[1]; o[2] = -o[2];
  so3_log(Rt, o + 3);
  for (int i = 0; i < 6; ++i) out[i] = o[i];
}

// kappa.py:130-169
GC_DEV double kappa_blend(double R, double eps_r, double d, double r0, double tau) {
  const double Rc = clampd(R, 0.0, 1.0 - eps_r);
  const double R2 = Rc * Rc;
  const double k_low = (Rc * (d - R2)) / (1.0 - R2 + eps_r);
  const double k_high = -log(fmax(1.0 - R2, eps_r));
  const double s = sigmoid((Rc - r0) / fmax(tau, 1e-6));
  return (1.0 - s) * k_low + s * k_high;
}

// ------------------------------------------------------- symmetric 3x3 eigen (cyclic Jacobi)
// A (row-major, symmetrised by caller) -> w[3] unsorted, V columns = eigenvectors.
GC_DEV void jacobi_rot3(double* A, double* V, int p, int q) {
  const double apq = A[3 * p + q];
  const double app = A[3 * p + p], aqq = A[3 * q + q];
  if (apq == 0.0 || fabs(apq) <= 1e-300) return;
  if (fabs(apq) <= 1e-18 * sqrt(fabs(app * aqq))) {
    A[3 * p + q] = 0.0; A[3 * q + p] = 0.0;
    return;
  }
  const double th = (aqq - app) / (2.0 * apq);
  const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
  const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
  for (int k = 0; k < 3; ++k) {  // columns: A G
    const double akp = A[3 * k + p], akq = A[3 * k + q];
    A[3 * k + p] = c * akp - s * akq;
    A[3 * k + q] = s * akp + c * akq;
  }
  for (int k = 0; k < 3; ++k) {  // rows: Gᵀ A
    const double apk = A[3 * p + k], aqk = A[3 * q + k];
    A[3 * p + k] = c * apk - s * aqk;
    A[3 * q + k] = s * apk + c * aqk;
  }
  A[3 * p + q] = 0.0; A[3 * q + p] = 0.0;
  for (int k = 0; k < 3; ++k) {
    const double vkp = V[3 * k + p], vkq = V[3 * k + q];
    V[3 * k + p] = c * vkp - s * vkq;
    V[3 * k + q] = s * vkp + c * vkq;
  }
}

GC_DEV void eigh3(const double* Ain, double* w, double* V) {
  double A[9];
  for (int i = 0; i < 9; ++i) A[i] = Ain[i];
  for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 12; ++sweep) {
    const double off = A[1] * A[1] + A[2] * A[2] + A[5] * A[5];
    const double dg = A[0] * A[0] + A[4] * A[4] + A[8] * A[8];
    if (off <= 1e-36 * dg || off == 0.0) break;
    jacobi_rot3(A, V, 0, 1);
    jacobi_rot3(A, V, 0, 2);
    jacobi_rot3(A, V, 1, 2);
  }
  w[0] = A[0]; w[1] = A[4]; w[2] = A[8];
}

// domain_projection_psd_core on a 3x3 (primitives.py:80-123). cert = [proj, sym, min, max, cond, nnc]
GC_DEV void psd_project3(const double* M, double eps, double* Mp, double* cert) {
  double S[9];
  double symd = 0.0;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      S[3 * i + j] = 0.5 * (M[3 * i + j] + M[3 * j + i]);
      const double d = S[3 * i + j] - M[3 * i + j];
      symd += d * d;
    }
  double w[3], V[9];
  eigh3(S, w, V);
  double proj = 0.0, mn = 1e308, mx = -1e308, nnc = 0.0;
  for (int k = 0; k < 3; ++k) {
    w[k] = fmax(w[k], eps);
    mn = fmin(mn, w[k]);
    mx = fmax(mx, w[k]);
    nnc += (w[k] < 10.0 * eps) ? 1.0 : 0.0;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      const double v = V[3 * i] * w[0] * V[3 * j] + V[3 * i + 1] * w[1] * V[3 * j + 1] +
                       V[3 * i + 2] * w[2] * V[3 * j + 2];
      Mp[3 * i + j] = v;
      const double d = v - S[3 * i + j];
      proj += d * d;
    }
  if (cert) {
    cert[0] = sqrt(proj); cert[1] = sqrt(symd); cert[2] = mn; cert[3] = mx; cert[4] = mx / mn; cert[5] = nnc;
  }
}

// psd_project3 with the certified shortcut of wg_psd_project_fast: if the Cholesky of
// S_sym - eps I succeeds, every eigenvalue exceeds eps, the clamp is inactive and the projection is
// S_sym (the reference's V diag(λ) Vᵀ reconstructs it up to rounding); projection delta 0 and the
// eigen fields of cert NaN. Otherwise the Jacobi form.
GC_DEV void psd_project3_fast(const double* M, double eps, double* Mp, double* cert) {
  double S[9], symd = 0.0;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      S[3 * i + j] = 0.5 * (M[3 * i + j] + M[3 * j + i]);
      const double d = S[3 * i + j] - M[3 * i + j];
      symd += d * d;
    }
  const double a00 = S[0] - eps;
  const double l10 = S[3] / sqrt(fmax(a00, 1e-300)), l20 = S[6] / sqrt(fmax(a00, 1e-300));
  const double a11 = S[4] - eps - l10 * l10;
  const double l21 = (S[7] - l20 * l10) / sqrt(fmax(a11, 1e-300));
  const double a22 = S[8] - eps - l20 * l20 - l21 * l21;
  if (a00 > 0.0 && a11 > 0.0 && a22 > 0.0) {
    for (int k = 0; k < 9; ++k) Mp[k] = S[k];
    if (cert) {
      const double nan = __builtin_nan("");
      cert[0] = 0.0; cert[1] = sqrt(symd); cert[2] = nan; cert[3] = nan; cert[4] = nan; cert[5] = nan;
    }
    return;
  }
  psd_project3(M, eps, Mp, cert);
}

// Sorted (descending) eigenvalues of a symmetric 3x3.
GC_DEV void eigvalsh3_desc(const double* M, double* lam) {
  double V[9], w[3];
  eigh3(M, w, V);
  double a = w[0], b = w[1], c = w[2], t;
  if (a < b) { t = a; a = b; b = t; }
  if (b < c) { t = b; b = c; c = t; }
  if (a < b) { t = a; a = b; b = t; }
  lam[0] = a; lam[1] = b; lam[2] = c;
}

// ------------------------------------------------------------- 3x3 SVD (one-sided Jacobi)
// H = U diag(s) Vᵀ, s descending (LAPACK gesdd convention). Degenerate columns of U are
// completed to an orthonormal, right-handed-agnostic basis (H = 0 gives U = V = I).
// Registers only: one-sided Jacobi sweeps with the rotation from one square root
// and one division (t = 2γ·sgn(β−α) / (|β−α| + √((β−α)² + 4γ²)), the classical tan of the
// smaller angle), the column sort as a compare-exchange network of selects and the degenerate-column
// completion unrolled (no dynamically indexed arrays, so nothing spills to scratch memory).
// Columns count as orthogonal once |γ| <= ε √(αβ) (ε = 2.2e-16, tol2 = ε²: the rounding floor of γ;
// a 1e-17 threshold sits below it and rotates on noise to the 16-sweep cap: 12.8 sweeps on average
// against 3.3 for the same s, U Vᵀ and V to 1e-15, tools/probe/probe_mf.hip).
GC_DEV void svd3(const double* Hin, double* U, double* s, double* V, double tol2 = 4.9e-32, int* nsweep = nullptr) {
  double a[9], v[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) { a[i] = Hin[i]; v[i] = (i % 4 == 0) ? 1.0 : 0.0; }
  for (int sweep = 0; sweep < 16; ++sweep) {
    bool rot = false;
#pragma unroll
    for (int pq = 0; pq < 3; ++pq) {
      const int p = (pq == 2) ? 1 : 0, q = (pq == 0) ? 1 : 2;
      const double al = a[p] * a[p] + a[3 + p] * a[3 + p] + a[6 + p] * a[6 + p];
      const double be = a[q] * a[q] + a[3 + q] * a[3 + q] + a[6 + q] * a[6 + q];
      const double ga = a[p] * a[q] + a[3 + p] * a[3 + q] + a[6 + p] * a[6 + q];
      if (ga == 0.0 || ga * ga <= tol2 * (al * be)) continue;
      rot = true;
      const double d = be - al;
      const double t = (d >= 0.0 ? 2.0 * ga : -2.0 * ga) / (fabs(d) + sqrt(d * d + 4.0 * ga * ga));
      const double c = 1.0 / sqrt(1.0 + t * t), sn = c * t;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double ap = a[3 * k + p], aq = a[3 * k + q];
        a[3 * k + p] = c * ap - sn * aq;
        a[3 * k + q] = sn * ap + c * aq;
        const double vp = v[3 * k + p], vq = v[3 * k + q];
        v[3 * k + p] = c * vp - sn * vq;
        v[3 * k + q] = sn * vp + c * vq;
      }
    }
    if (nsweep) *nsweep = sweep + 1;
    if (!rot) break;
  }
  double sv[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) sv[j] = sqrt(a[j] * a[j] + a[3 + j] * a[3 + j] + a[6 + j] * a[6 + j]);
  // descending, stable: exchange (0,1), (1,2), (0,1) when strictly smaller
  const auto cx = [&](int i, int j) {
    const bool sw = sv[i] < sv[j];
    const double x = sv[i], y = sv[j];
    sv[i] = sw ? y : x; sv[j] = sw ? x : y;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double ai = a[3 * k + i], aj = a[3 * k + j], vi = v[3 * k + i], vj = v[3 * k + j];
      a[3 * k + i] = sw ? aj : ai; a[3 * k + j] = sw ? ai : aj;
      v[3 * k + i] = sw ? vj : vi; v[3 * k + j] = sw ? vi : vj;
    }
  };
  cx(0, 1); cx(1, 2); cx(0, 1);
  const double tol = 1e-14 * fmax(sv[0], 1e-300);
  double u[9];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    s[j] = sv[j];
    if (sv[j] > tol && sv[j] > 0.0) {
      const double inv = 1.0 / sv[j];
#pragma unroll
      for (int k = 0; k < 3; ++k) u[3 * k + j] = a[3 * k + j] * inv;
    } else {
      // the unit axis least aligned with the previous columns, Gram-Schmidt'ed against them
      double best = -1.0, e0 = 0.0, e1 = 0.0, e2 = 0.0;
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) {
        double e[3] = {ax == 0 ? 1.0 : 0.0, ax == 1 ? 1.0 : 0.0, ax == 2 ? 1.0 : 0.0};
#pragma unroll
        for (int pj = 0; pj < j; ++pj) {
          const double dd = u[3 * ax + pj];
#pragma unroll
          for (int k = 0; k < 3; ++k) e[k] -= dd * u[3 * k + pj];
        }
        const double nn = norm3(e);
        const bool take = nn > best + 1e-12;
        best = take ? nn : best;
        e0 = take ? e[0] : e0; e1 = take ? e[1] : e1; e2 = take ? e[2] : e2;
      }
      const double inv = 1.0 / best;
      u[j] = e0 * inv; u[3 + j] = e1 * inv; u[6 + j] = e2 * inv;
    }
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) { U[i] = u[i]; V[i] = v[i]; }
}

// LU with partial pivoting 3x3 inverse (jnp.linalg.inv semantics). Unrolled, the row exchanges as
// selects: nothing is indexed at run time, so the arrays stay in registers.
GC_DEV void inv3(const double* Ain, double* X) {
  double A[9], Xl[9];
  int piv[3] = {0, 1, 2};
#pragma unroll
  for (int i = 0; i < 9; ++i) A[i] = Ain[i];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    int p = k;
    double m = fabs(A[3 * k + k]);
#pragma unroll
    for (int i = k + 1; i < 3; ++i) {
      const bool g = fabs(A[3 * i + k]) > m;
      m = g ? fabs(A[3 * i + k]) : m;
      p = g ? i : p;
    }
#pragma unroll
    for (int i = k + 1; i < 3; ++i) {
      const bool sw = p == i;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const double a = A[3 * k + j], b = A[3 * i + j];
        A[3 * k + j] = sw ? b : a;
        A[3 * i + j] = sw ? a : b;
      }
      const int pa = piv[k], pb = piv[i];
      piv[k] = sw ? pb : pa;
      piv[i] = sw ? pa : pb;
    }
#pragma unroll
    for (int i = k + 1; i < 3; ++i) {
      A[3 * i + k] /= A[3 * k + k];
#pragma unroll
      for (int j = k + 1; j < 3; ++j) A[3 * i + j] -= A[3 * i + k] * A[3 * k + j];
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double y[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      double v = (piv[i] == c) ? 1.0 : 0.0;
#pragma unroll
      for (int j = 0; j < i; ++j) v -= A[3 * i + j] * y[j];
      y[i] = v;
    }
#pragma unroll
    for (int i = 2; i >= 0; --i) {
      double v = y[i];
#pragma unroll
      for (int j = i + 1; j < 3; ++j) v -= A[3 * i + j] * Xl[3 * j + c];
      Xl[3 * i + c] = v / A[3 * i + i];
    }
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) X[i] = Xl[i];
}

// Solve A x = b (3x3, partial pivoting) — jnp.linalg.solve semantics.
GC_DEV void solve3(const double* A, const double* b, double* x) {
  double Ai[9];
  inv3(A, Ai);
  mat3_vec(Ai, b, x);
}

// p0 = Exp(α ξ)^{-1} p  (deskew_constant_twist.py:50-58: se3_exp then so3_exp of the rotvec)
GC_DEV void deskew_point(const double* p, double alpha, const double* xi, double* out) {
  const double rho[3] = {alpha * xi[0], alpha * xi[1], alpha * xi[2]};
  const double phi[3] = {alpha * xi[3], alpha * xi[4], alpha * xi[5]};
  const double ts = dot3(phi, phi);
  const double th = sqrt(ts);
  double Bv, Cv, a, b;
  if (th < kSmallAngle) {
    Bv = 0.5 - ts / 24.0;
    Cv = 1.0 / 6.0 - ts / 120.0;
    a = 1.0;
    b = 0.5;
  } else {
    double s, c;
    sincos(th, &s, &c);
    const double sts = (ts < kSmallAngle * kSmallAngle) ? 1.0 : ts;
    Bv = (1.0 - c) / sts;
    Cv = (th - s) / (sts * th);
    a = s / th;
    b = Bv;
  }
  double V[9], R[9], t[3], q[3];
  rodrigues_form(phi, Bv, Cv, V);
  mat3_vec(V, rho, t);
  rodrigues_form(phi, a, b, R);
  q[0] = p[0] - t[0]; q[1] = p[1] - t[1]; q[2] = p[2] - t[2];
  mat3_tvec(R, q, out);
}

// unit ray direction from the LiDAR origin (pipeline.py:589-593)
GC_DEV void direction(const double* p, const double* o, double eps, double* d) {
  const double r0 = p[0] - o[0], r1 = p[1] - o[1], r2 = p[2] - o[2];
  const double den = sqrt(r0 * r0 + r1 * r1 + r2 * r2) + eps;
  d[0] = r0 / den; d[1] = r1 / den; d[2] = r2 / den;
}

}  // namespace gc
