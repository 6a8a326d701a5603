// Dev probe (GPU box): single-lane latency (s_memtime cycles per call, chained over 64 calls) of the
// Lie maps on the per-hypothesis kernels' serial paths (sincos, so3_exp, so3_log, se3_exp, the
// compose X ∘ Exp(δ)) and of the wave reductions (wave_sum: DPP + readlane).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -Ifl-slam_amd/csrc tools/probe/probe_lie.hip -o tools/probe/probe_lie
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "gc_math.h"
#include "gc_wgla.h"

using namespace gc;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);   \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

// a result's completion before the next stamp: its low word read into an SGPR
#define DONE(x)                                                                  \
  do {                                                                           \
    int s_;                                                                      \
    asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(s_) : "v"(__double2loint(x))); \
    sink += s_;                                                                  \
  } while (0)

#ifndef REPS
#define REPS 64
#endif
constexpr int kReps = REPS;
__global__ void k_lie(const double* in, double* cyc, int* out) {
  int sink = 0;
  const int lane = threadIdx.x;
  double x[6];
  for (int k = 0; k < 6; ++k) x[k] = in[k];
  double c[8];
  double v = x[3];
  // 0: sincos
  DONE(v);
  double t0 = (double)__builtin_readcyclecounter();
  if (lane == 0)
    for (int r = 0; r < kReps; ++r) { double s, co; sincos(v, &s, &co); v = s + co * 1e-3; }
  DONE(v);
  double t1 = (double)__builtin_readcyclecounter();
  c[0] = (t1 - t0) / kReps;
  // 1: so3_exp
  double w[3] = {x[3], x[4], x[5]}, R[9];
  t0 = (double)__builtin_readcyclecounter();
  if (lane == 0)
    for (int r = 0; r < kReps; ++r) { so3_exp(w, R); w[0] = R[1] * 0.5; w[1] = R[2] * 0.5; w[2] = R[5] * 0.5; }
  DONE(w[0]);
  t1 = (double)__builtin_readcyclecounter();
  c[1] = (t1 - t0) / kReps;
  // 2: so3_log
  so3_exp(x + 3, R);
  t0 = (double)__builtin_readcyclecounter();
  if (lane == 0)
    for (int r = 0; r < kReps; ++r) { so3_log(R, w); R[1] += w[0] * 1e-9; R[3] -= w[0] * 1e-9; }
  DONE(w[0]);
  t1 = (double)__builtin_readcyclecounter();
  c[2] = (t1 - t0) / kReps;
  // 3: se3_exp
  double e[6];
  t0 = (double)__builtin_readcyclecounter();
  if (lane == 0)
    for (int r = 0; r < kReps; ++r) { se3_exp(x, e); x[3] = e[0] * 0.1; x[4] = e[4]; }
  DONE(x[3]);
  t1 = (double)__builtin_readcyclecounter();
  c[3] = (t1 - t0) / kReps;
  // 4: compose X ∘ Exp(δ)
  double X[6] = {1.0, 2.0, 0.0, 0.1, -0.2, 0.3}, o[6];
  t0 = (double)__builtin_readcyclecounter();
  if (lane == 0)
    for (int r = 0; r < kReps; ++r) {
      double ee[6];
      se3_exp(x, ee);
      se3_compose(X, ee, o);
      x[3] = o[3] * 1e-3; x[0] = o[0] * 1e-3;
    }
  DONE(x[3]);
  t1 = (double)__builtin_readcyclecounter();
  c[4] = (t1 - t0) / kReps;
  // 5: acos
  v = x[4] * 0.1;
  t0 = (double)__builtin_readcyclecounter();
  if (lane == 0)
    for (int r = 0; r < kReps; ++r) v = acos(v) * 0.3;
  DONE(v);
  t1 = (double)__builtin_readcyclecounter();
  c[5] = (t1 - t0) / kReps;
  // 6: wave_sum (all lanes)
  double q = in[lane % 6];
  t0 = (double)__builtin_readcyclecounter();
  for (int r = 0; r < kReps; ++r) q = wave_sum(q) * 1e-3 + (double)lane;
  DONE(q);
  t1 = (double)__builtin_readcyclecounter();
  c[6] = (t1 - t0) / kReps;
  // 7: sqrt + division chain
  v = x[5] + 2.0;
  t0 = (double)__builtin_readcyclecounter();
  if (lane == 0)
    for (int r = 0; r < kReps; ++r) v = 1.0 / sqrt(v) + 1.5;
  DONE(v);
  t1 = (double)__builtin_readcyclecounter();
  c[7] = (t1 - t0) / kReps;
  if (lane == 0) {
    for (int k = 0; k < 8; ++k) cyc[blockIdx.x * 8 + k] = c[k];
    out[blockIdx.x] = sink + (int)(o[0] + v + q);
  }
}

int main() {
  const int G = 16;
  double h[6] = {0.3, -0.2, 0.1, 0.4, -0.3, 0.2};
  double *din, *dc;
  int* dout;
  CK(hipMalloc(&din, sizeof(h)));
  CK(hipMalloc(&dc, 8 * G * sizeof(double)));
  CK(hipMalloc(&dout, G * sizeof(int)));
  CK(hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice));
  // pass 0 right after load (instruction cache cold), pass 1 warm; per-call cycles over kReps calls
  // (the cold pass amortises its misses over the kReps calls, so it bounds them from below)
  double c[2][8 * G];
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(k_lie, dim3(G), dim3(64), 0, 0, din, dc, dout);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(c[pass], dc, sizeof(c[pass]), hipMemcpyDeviceToHost));
  }
  const char* nm[8] = {"sincos", "so3_exp", "so3_log", "se3_exp", "se3_exp+compose", "acos", "wave_sum", "1/sqrt"};
  std::printf("%-18s %10s %10s\n", "", "cold", "warm");
  for (int k = 0; k < 8; ++k) {
    double m[2] = {0, 0};
    for (int p = 0; p < 2; ++p)
      for (int g = 0; g < G; ++g) m[p] += c[p][8 * g + k] / G;
    std::printf("%-18s %10.0f %10.0f cycles/call\n", nm[k], m[0], m[1]);
  }
  return 0;
}
