// Dev microbenchmark (build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I fl-slam_amd/csrc -I include
// tools/probe/lift_lat.hip -o tools/probe/lift_lat): single-workgroup latency (s_memtime cycles) of the
// predict's lift iteration (wave_lift_iterate, gc_wgla.h: x = (I + ε(S + εI))⁻¹ b on one wave) against
// the spectrum scale of S (r = ε ||S||∞ sets the iteration count), its set-up alone, and the 22x22 wave
// Cholesky beside it, one workgroup on an otherwise idle GPU.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "gc_wgla.h"
using namespace gc;
constexpr int N2 = kDZ * kDZ;

__global__ void __launch_bounds__(256) klift(const double* A, double eps, double* out) {
  __shared__ double S[N2], xrow[kDZ], C[N2];
  const int t = threadIdx.x;
  for (int i = t; i < N2; i += 256) { S[i] = A[i]; C[i] = A[i]; }
  __syncthreads();
  long c0 = __builtin_readcyclecounter();
  double x = 0.0;
  bool ok = false;
  if (t < 64) ok = wave_lift_iterate<kDZ>(S, t < kDZ ? 1.0 + 0.01 * t : 0.0, eps, xrow, kDZ, x);
  __syncthreads();
  long c1 = __builtin_readcyclecounter();
  if (t < 64) (void)wave0_chol<kDZ, true>(C, kDZ);
  __syncthreads();
  long c2 = __builtin_readcyclecounter();
  // the set-up alone: the rows of B, their absolute row sums and the wave maximum, the step count
  double rs = 0.0;
  if (t < 64) {
    const int lane = t;
    for (int j = 0; j < kDZ; ++j)
      if (lane < kDZ) rs += fabs(eps * (0.5 * (S[lane * kDZ + j] + S[j * kDZ + lane]) + (j == lane ? eps : 0.0)));
    rs = wave_max(rs);
  }
  __syncthreads();
  long c3 = __builtin_readcyclecounter();
  if (t == 0) {
    out[0] = (double)(c1 - c0);
    out[1] = (double)(c2 - c1);
    out[2] = (double)(c3 - c2);
    out[3] = ok ? 1.0 : 0.0;
    out[4] = x;
    out[5] = rs;
  }
}

int main() {
  double *dA, *dO;
  (void)hipMalloc(&dA, N2 * 8);
  (void)hipMalloc(&dO, 64);
  for (double scale : {1e3, 1e5, 1e6, 1e7, 1e8}) {
    std::vector<double> A(N2);
    for (int i = 0; i < kDZ; ++i)
      for (int j = 0; j < kDZ; ++j) A[i * kDZ + j] = (i == j ? scale : 0.01 * scale / (1 + std::abs(i - j)));
    (void)hipMemcpy(dA, A.data(), N2 * 8, hipMemcpyHostToDevice);
    double o[6];
    for (int it = 0; it < 5; ++it) {
      hipLaunchKernelGGL(klift, dim3(1), dim3(256), 0, 0, dA, 1e-9, dO);
      (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(o, dO, sizeof(o), hipMemcpyDeviceToHost);
    const double r = o[5], iters = r > 0 ? std::ceil(38.816242111356935 / -std::log(r)) : 1;
    printf("scale %8.0e  r %.3e  iterations %3.0f  lift %7.0f cycles  set-up %6.0f  wave chol 22 %7.0f  ok %d\n", scale,
           r, iters, o[0], o[2], o[1], (int)o[3]);
  }
  return 0;
}
