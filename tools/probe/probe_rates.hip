// Dev probe (not product): f64 MFMA / VALU issue rates on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) k_mfma(double* out, int iters, double a, double b) {
  v4d acc[4] = {};
  double x = a + threadIdx.x, y = b;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[k], 0, 0, 0);
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
}
__global__ void __launch_bounds__(256) k_mfma8(double* out, int iters, double a, double b) {
  v4d acc[8] = {};
  double x = a + threadIdx.x, y = b;
  for (int i = 0; i < iters / 2; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[k], 0, 0, 0);
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3] + acc[4][0] + acc[7][1];
}
// waves 0,2 MFMA; waves 1,3 VALU (same per-wave work as k_mfma / k_fma)
__global__ void __launch_bounds__(256) k_split(double* out, int iters, double a, double b) {
  const int wv = threadIdx.x >> 6;
  double r = 0;
  if (wv & 1) {
    double acc[8];
    for (int k = 0; k < 8; ++k) acc[k] = a + k + threadIdx.x;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = fma(acc[k], b, a);
    }
    for (int k = 0; k < 8; ++k) r += acc[k];
  } else {
    v4d acc[4] = {};
    double x = a + threadIdx.x, y = b;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[k], 0, 0, 0);
    }
    r = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
  }
  out[blockIdx.x * 256 + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_fma(double* out, int iters, double a, double b) {
  double acc[8];
  for (int k = 0; k < 8; ++k) acc[k] = a + k + threadIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = fma(acc[k], b, a);
  }
  double s = 0; for (int k = 0; k < 8; ++k) s += acc[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_mix(double* out, int iters, double a, double b) {
  v4d acc[4] = {};
  double f[8];
  for (int k = 0; k < 8; ++k) f[k] = a + k + threadIdx.x;
  double x = a + threadIdx.x, y = b;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[k], 0, 0, 0);
      f[2 * k] = fma(f[2 * k], b, a); f[2 * k + 1] = fma(f[2 * k + 1], b, a);
      f[2 * k] = fma(f[2 * k], b, a); f[2 * k + 1] = fma(f[2 * k + 1], b, a);
      f[2 * k] = fma(f[2 * k], b, a); f[2 * k + 1] = fma(f[2 * k + 1], b, a);
      f[2 * k] = fma(f[2 * k], b, a); f[2 * k + 1] = fma(f[2 * k + 1], b, a);
    }
  }
  double s = 0; for (int k = 0; k < 8; ++k) s += f[k];
  out[blockIdx.x * 256 + threadIdx.x] = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3] + s;
}
int main() {
  double* out; hipMalloc(&out, sizeof(double) * 256 * 4096);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 4096, grid = 2048;
  float ms;
  hipLaunchKernelGGL(k_mfma, dim3(grid), dim3(256), 0, 0, out, iters, 1.0, 0.5);
  hipEventRecord(e0); hipLaunchKernelGGL(k_mfma, dim3(grid), dim3(256), 0, 0, out, iters, 1.0, 0.5); hipEventRecord(e1);
  hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  double n_mfma = (double)grid * 4 * iters * 4;
  printf("mfma f64 16x16x4: %.3f ms, %.2f TFLOP/s, %.1f cycles/MFMA/SIMD at 2.4GHz\n", ms, n_mfma * 2048 / (ms * 1e-3) / 1e12,
         ms * 1e-3 * 2.4e9 * 1024 / n_mfma);
  hipLaunchKernelGGL(k_fma, dim3(grid), dim3(256), 0, 0, out, iters, 1.0, 0.5);
  hipEventRecord(e0); hipLaunchKernelGGL(k_fma, dim3(grid), dim3(256), 0, 0, out, iters, 1.0, 0.5); hipEventRecord(e1);
  hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  double n_fma = (double)grid * 4 * iters * 8;
  printf("valu f64 fma: %.3f ms, %.2f TFLOP/s, %.2f cycles/wave-instr/SIMD\n", ms, n_fma * 64 * 2 / (ms * 1e-3) / 1e12,
         ms * 1e-3 * 2.4e9 * 1024 / n_fma);
  hipLaunchKernelGGL(k_mix, dim3(grid), dim3(256), 0, 0, out, iters, 1.0, 0.5);
  hipEventRecord(e0); hipLaunchKernelGGL(k_mix, dim3(grid), dim3(256), 0, 0, out, iters, 1.0, 0.5); hipEventRecord(e1);
  hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("mix (4 mfma + 32 fma per iter, in-wave): %.3f ms\n", ms);
  hipEventRecord(e0); hipLaunchKernelGGL(k_mfma8, dim3(grid), dim3(256), 0, 0, out, iters, 1.0, 0.5); hipEventRecord(e1);
  hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("mfma 8 accumulators: %.3f ms (same MFMA count)\n", ms);
  hipEventRecord(e0); hipLaunchKernelGGL(k_split, dim3(grid), dim3(256), 0, 0, out, iters, 1.0, 0.5); hipEventRecord(e1);
  hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("split waves (half mfma-only of k_mfma, half fma-only of k_fma): %.3f ms; serial would be %.3f\n", ms, 0.0);
  return 0;
}
