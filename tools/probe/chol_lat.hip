// Dev microbenchmark (build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I fl-slam_amd/csrc -I include
// tools/probe/chol_lat.hip -o tools/probe/chol_lat): single-workgroup latency (s_memtime cycles and s_memrealtime ticks) of the
// 22x22 wave Cholesky, the Cholesky inverse and the fused PSD-certify + lifted factorization of
// the per-hypothesis chain kernels (gc_wgla.h), one workgroup on an otherwise idle GPU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "gc_wgla.h"
using namespace gc;
constexpr int N2 = kDZ * kDZ;
__global__ void __launch_bounds__(256) kbench(const double* A, double* out, double* res) {
  __shared__ double M[N2], S[N2], C[N2], W[N2], X[2 * N2 + 4 * kDZ], red[16], c1[8];
  const int t = threadIdx.x;
  for (int i = t; i < N2; i += 256) M[i] = A[i];
  __syncthreads();
  long c[8], r[8];
  int k = 0;
  auto mark = [&]() { __syncthreads(); c[k] = __builtin_readcyclecounter(); r[k] = wall_clock64(); ++k; };
  mark();
  for (int i = t; i < N2; i += 256) S[i] = M[i];
  mark();  // 1: copy
  if (t < 64) wave0_chol<kDZ, true>(S, kDZ);
  mark();  // 2: one wave Cholesky
  wg_chol_inverse(S, C, W, kDZ);
  mark();  // 3: chol inverse
  wg_psd_fast_lifted_chol(M, W, 1e-12, 1e-10, kDZ, X, S, red, c1);
  mark();  // 4: psd fast + lifted chol
  if (t < 64) chol_inverse_phase1(S, W, kDZ);
  mark();  // 5: inverse phase 1 only
  chol_inverse_phase2(C, W, kDZ);
  mark();  // 6: inverse phase 2 only
  if (t == 0)
    for (int i = 1; i < k; ++i) { out[2 * i] = (double)(c[i] - c[i - 1]); out[2 * i + 1] = (double)(r[i] - r[i - 1]); }
  for (int i = t; i < N2; i += 256) res[i] = C[i];
}

template <int NM, int VAR>
__device__ void lane_chol_v(double (&a)[NM], int lane, bool& ok) {
  __shared__ __attribute__((aligned(16))) double colbufs[4][NM + 2];
  double* colbuf = colbufs[threadIdx.x >> 6];
#pragma unroll
  for (int k = 0; k < NM; ++k) {
    double piv = readlane_f64(a[k], k);
    if (!(piv > 0.0)) { ok = false; piv = 1.0; }
    const double y = __builtin_amdgcn_rsq(piv);
    double g = piv * y, h = 0.5 * y;
    const double r = fma(-g, h, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    const double inv = h + h;
    if (VAR & 8) a[k] = lane == k ? g : a[k] * inv;  // rows above k hold unread values either way
    else a[k] = lane == k ? g : (lane > k ? a[k] * inv : a[k]);
    if (k + 1 < NM) {
      if (k + 2 < NM) colbuf[lane < NM ? lane : NM + 1] = a[k];
      if (VAR & 1) a[k + 1] -= a[k] * readlane_f64(a[k], k + 1);
      else a[k + 1] -= a[k] * (lane == k + 1 ? a[k] : readlane_f64(a[k], k + 1));
#pragma unroll
      for (int j = k + 2; j < NM; ++j) a[j] -= a[k] * colbuf[j];
      if (VAR & 2) {
#pragma unroll
        for (int j = k + 1; j < NM; ++j) asm volatile("" : "+v"(a[j]));
      }
      if (VAR & 4) asm volatile("" : "+v"(a[k + 1]));
    }
  }
}
template <int VAR>
__device__ bool wave0_chol_v(double* A, int n) {
  const int lane = threadIdx.x & 63;
  double a[kDZ];
  lane_load_rows<kDZ>(A, n, lane, a);
  bool ok = true;
  lane_chol_v<kDZ, VAR>(a, lane, ok);
  lane_store_lower<kDZ>(A, n, lane, a);
  return ok;
}
template <int VAR>
__global__ void __launch_bounds__(256) kvar(const double* A, double* out, double* res) {
  __shared__ double S[N2];
  const int t = threadIdx.x;
  for (int i = t; i < N2; i += 256) S[i] = A[i];
  __syncthreads();
  long c0 = __builtin_readcyclecounter();
  if (t < 64) {
    if (VAR < 0) wave0_chol<kDZ, true>(S, kDZ);
    else wave0_chol_v<VAR < 0 ? 0 : VAR>(S, kDZ);
  }
  __syncthreads();
  long c1 = __builtin_readcyclecounter();
  if (t == 0) out[0] = (double)(c1 - c0);
  for (int i = t; i < N2; i += 256) res[i] = S[i];
}
template <int VAR>
void runvar(const double* dA, double* dO, double* dR, const std::vector<double>& ref, const char* nm) {
  for (int it = 0; it < 5; ++it) { hipLaunchKernelGGL(kvar<VAR>, dim3(1), dim3(256), 0, 0, dA, dO, dR); (void)hipDeviceSynchronize(); }
  double o; std::vector<double> r(N2);
  (void)hipMemcpy(&o, dO, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(r.data(), dR, N2 * 8, hipMemcpyDeviceToHost);
  int diff = 0;
  for (int i = 0; i < N2; ++i) diff += (r[i] != ref[i]);
  printf("chol variant %-28s %8.0f cycles, %d entries differ from the product\n", nm, o, diff);
}

// chol_inverse_phase1_lane with the 22 reciprocals 1/C_ii formed once (lane i) and broadcast by
// readlane, instead of every lane dividing by every pivot (the same correctly rounded quotients)
__device__ void phase1_rcp(const double* C, double* scratch, int n, int j) {
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
        const double inv = readlane_f64(rdiag, i);
        col[i] = i >= j ? v * inv : 0.0;
      }
    }
#pragma unroll
    for (int k = 0; k < kDZ; ++k)
      if (k < n) scratch[j * n + k] = col[k];
  }
}
template <int VAR>
__global__ void __launch_bounds__(256) kinv(const double* A, double* out, double* res) {
  __shared__ double S[N2], W[N2];
  const int t = threadIdx.x;
  for (int i = t; i < N2; i += 256) S[i] = A[i];
  __syncthreads();
  if (t < 64) wave0_chol<kDZ, true>(S, kDZ);
  __syncthreads();
  long c0 = __builtin_readcyclecounter();
  if (t < 64) {
    if (VAR == 0) chol_inverse_phase1_lane(S, W, kDZ, t);
    else phase1_rcp(S, W, kDZ, t);
  }
  __syncthreads();
  long c1 = __builtin_readcyclecounter();
  if (t == 0) out[0] = (double)(c1 - c0);
  for (int i = t; i < N2; i += 256) res[i] = W[i];
}
template <int VAR>
void runinv(const double* dA, double* dO, double* dR, std::vector<double>& ref, const char* nm, bool set) {
  for (int it = 0; it < 5; ++it) { hipLaunchKernelGGL(kinv<VAR>, dim3(1), dim3(256), 0, 0, dA, dO, dR); (void)hipDeviceSynchronize(); }
  double o; std::vector<double> r(N2);
  (void)hipMemcpy(&o, dO, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(r.data(), dR, N2 * 8, hipMemcpyDeviceToHost);
  if (set) ref = r;
  int diff = 0;
  for (int i = 0; i < N2; ++i) diff += (r[i] != ref[i]);
  printf("inverse phase1 %-26s %8.0f cycles, %d entries differ from the product\n", nm, o, diff);
}
int main() {
  std::vector<double> A(N2);
  // SPD: B Bᵀ + 22 I
  std::vector<double> B(N2);
  unsigned s = 1;
  for (auto& b : B) { s = s * 1664525u + 1013904223u; b = (s >> 8) * (1.0 / 16777216.0) - 0.5; }
  for (int i = 0; i < kDZ; ++i)
    for (int j = 0; j < kDZ; ++j) {
      double v = i == j ? kDZ : 0.0;
      for (int q = 0; q < kDZ; ++q) v += B[i * kDZ + q] * B[j * kDZ + q];
      A[i * kDZ + j] = v;
    }
  double *dA, *dO, *dR;
  hipMalloc(&dA, N2 * 8); hipMalloc(&dO, 64 * 8); hipMalloc(&dR, N2 * 8);
  hipMemcpy(dA, A.data(), N2 * 8, hipMemcpyHostToDevice);
  const char* nm[] = {"", "copy", "wave chol 22", "wg_chol_inverse", "psd_fast_lifted_chol", "inverse phase1", "inverse phase2"};
  for (int it = 0; it < 5; ++it) {
    hipLaunchKernelGGL(kbench, dim3(1), dim3(256), 0, 0, dA, dO, dR);
    hipDeviceSynchronize();
  }
  double o[64];
  hipMemcpy(o, dO, sizeof o, hipMemcpyDeviceToHost);
  for (int i = 1; i < 7; ++i) printf("%-24s %8.0f cycles %6.0f ticks(100MHz) = %6.2f us\n", nm[i], o[2 * i], o[2 * i + 1], o[2 * i + 1] / 100.0);
  std::vector<double> ref(N2);
  runvar<-1>(dA, dO, dR, ref, "product (wave0_chol)");
  (void)hipMemcpy(ref.data(), dR, N2 * 8, hipMemcpyDeviceToHost);
  runvar<-1>(dA, dO, dR, ref, "product again");
  runvar<0>(dA, dO, dR, ref, "copy of product");
  runvar<1>(dA, dO, dR, ref, "always readlane");
  runvar<2>(dA, dO, dR, ref, "eager updates (pin all)");
  runvar<3>(dA, dO, dR, ref, "readlane + pin all");
  runvar<4>(dA, dO, dR, ref, "pin next pivot");
  runvar<5>(dA, dO, dR, ref, "readlane + pin next");
  runvar<8>(dA, dO, dR, ref, "scale every row");
  runvar<0>(dA, dO, dR, ref, "copy of product");
  runvar<8>(dA, dO, dR, ref, "scale every row");
  runvar<9>(dA, dO, dR, ref, "scale every row + readlane");
  runinv<0>(dA, dO, dR, ref, "product", true);
  runinv<1>(dA, dO, dR, ref, "reciprocals by readlane", false);
  runinv<0>(dA, dO, dR, ref, "product", false);
  runinv<1>(dA, dO, dR, ref, "reciprocals by readlane", false);
  return 0;
}
