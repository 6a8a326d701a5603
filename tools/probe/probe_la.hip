// Dev probe (not product): latency (cycles) of the workgroup linear-algebra primitives on one
// 256-thread workgroup with a 22x22 SPD matrix in LDS (gc_wgla.h).
#include "../../fl-slam_amd/csrc/gc_wgla.h"
#include <cstdio>
#include <cmath>

using namespace gc;

__global__ void __launch_bounds__(256) k_la(const double* Ain, long long* out) {
  __shared__ double A[484], C[484], X[484], W[484], W2[2 * 484 + 88], b[22], x[22], red[8], c6[6];
  const int t = threadIdx.x, n = 22;
  auto load = [&] {
    for (int i = t; i < 484; i += 256) A[i] = Ain[i];
    if (t < 22) b[t] = 1.0 + t;
    __syncthreads();
  };
  load();
  long long c0, c1;
  int slot = 0;
#define TIMEIT(EXPR)                                              \
  for (int rep = 0; rep < 3; ++rep) {                             \
    for (int i = t; i < 484; i += 256) C[i] = A[i];               \
    __syncthreads();                                              \
    __builtin_amdgcn_sched_barrier(0);                            \
    c0 = clock64();                                               \
    __builtin_amdgcn_sched_barrier(0);                            \
    EXPR;                                                         \
    __syncthreads();                                              \
    __builtin_amdgcn_sched_barrier(0);                            \
    c1 = clock64();                                               \
    __builtin_amdgcn_sched_barrier(0);                            \
    if (t == 0 && rep == 2) out[slot] = c1 - c0;                  \
  }                                                               \
  ++slot;
  TIMEIT(wg_chol(C, n))
  TIMEIT(wg_chol_checked(C, n, red))
  wg_chol(A, n);  // A <- chol(A) for the solve / inverse timings
  for (int i = t; i < 484; i += 256) X[i] = A[i];
  __syncthreads();
  TIMEIT(wg_chol_solve(C, b, x, n))
  TIMEIT(wg_chol_inverse(C, X, W, n))
  for (int i = t; i < 484; i += 256) A[i] = Ain[i];
  __syncthreads();
  TIMEIT(wg_psd_project_fast(C, X, 1e-12, n, W2, red, c6))
  TIMEIT(wg_matvec(C, b, x, n))
  TIMEIT(wg_sum((double)t, red))
  TIMEIT(wg_psd_project(C, X, 1e-12, n, W2, red, c6))
}

__global__ void __launch_bounds__(256) k_check(const double* Ain, double* out) {
  __shared__ double C[484], X[484], W[484], b[22], x[22];
  const int t = threadIdx.x, n = 22;
  for (int i = t; i < 484; i += 256) C[i] = Ain[i];
  if (t < 22) b[t] = 1.0 + t;
  __syncthreads();
  gc::wg_chol(C, n);
  gc::wg_chol_solve(C, b, x, n);
  gc::wg_chol_inverse(C, X, W, n);
  for (int i = t; i < 484; i += 256) { out[i] = C[i]; out[484 + i] = X[i]; }
  if (t < 22) out[968 + t] = x[t];
}

int main() {
  double h[484];
  for (int i = 0; i < 22; ++i)
    for (int j = 0; j < 22; ++j) h[i * 22 + j] = (i == j ? 30.0 : 0.0) + 1.0 / (1.0 + i + j);
  double* d; long long* o; long long ho[16] = {0};
  hipMalloc(&d, sizeof(h)); hipMalloc(&o, sizeof(ho));
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_la, dim3(1), dim3(256), 0, 0, d, o);
  hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost);
  const char* names[] = {"wg_chol", "wg_chol_checked", "wg_chol_solve", "wg_chol_inverse", "wg_psd_project_fast",
                         "wg_matvec", "wg_sum", "wg_psd_project (Jacobi)"};
  for (int i = 0; i < 8; ++i) printf("%-26s %8lld cycles\n", names[i], ho[i]);
  double* dc; hipMalloc(&dc, 990 * 8);
  hipLaunchKernelGGL(k_check, dim3(1), dim3(256), 0, 0, d, dc);
  static double hc[990];
  hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
  double e1 = 0, e2 = 0, e3 = 0;
  for (int i = 0; i < 22; ++i) {
    double r = -(1.0 + i);
    for (int j = 0; j < 22; ++j) {
      double s = 0, q = 0;
      for (int k = 0; k < 22; ++k) { s += hc[i * 22 + k] * hc[j * 22 + k]; q += h[i * 22 + k] * hc[484 + k * 22 + j]; }
      e1 = fmax(e1, fabs(s - h[i * 22 + j]));
      e2 = fmax(e2, fabs(q - (i == j)));
      r += h[i * 22 + j] * hc[968 + j];
    }
    e3 = fmax(e3, fabs(r));
  }
  printf("residuals: |CC^T-A| %.3e  |A Ainv - I| %.3e  |A x - b| %.3e\n", e1, e2, e3);
  return 0;
}
