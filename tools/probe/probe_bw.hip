// Dev probe (not product): achievable HBM rates on one MI355X for the contract kernels' access
// mix: pure streaming writes (BinSoftAssign's responsibility rows), pure streaming reads
// (ScanBinMomentMatch), and a copy. 6.4 GB per pass (the responsibility matrix of one scan).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) k_write(d2* __restrict__ out, long n2, double v) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256) out[i] = d2{v, v + 1.0};
}
__global__ void __launch_bounds__(256) k_write_nt(d2* __restrict__ out, long n2, double v) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256)
    __builtin_nontemporal_store(d2{v, v + 1.0}, out + i);
}
__global__ void __launch_bounds__(256) k_read(const d2* __restrict__ in, long n2, double* out) {
  double s = 0.0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256) {
    const d2 x = in[i];
    s += x[0] + x[1];
  }
  if (s == 12345.0) out[0] = s;
}
__global__ void __launch_bounds__(256) k_copy(const d2* __restrict__ in, d2* __restrict__ out, long n2) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256) out[i] = in[i];
}

int main() {
  const long bytes = 6400L << 20;
  const long n2 = bytes / 16;
  d2 *a, *b;
  double* o;
  if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&o, 64)) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms;
  for (int grid : {1024, 4096, 16384}) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, a, n2, 1.0);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep) printf("grid %5d write    %.2f TB/s\n", grid, bytes / (ms * 1e-3) / 1e12);
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k_write_nt, dim3(grid), dim3(256), 0, 0, b, n2, 1.0);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep) printf("grid %5d write_nt %.2f TB/s\n", grid, bytes / (ms * 1e-3) / 1e12);
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, n2, o);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep) printf("grid %5d read     %.2f TB/s\n", grid, bytes / (ms * 1e-3) / 1e12);
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, a, b, n2);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep) printf("grid %5d copy     %.2f TB/s (r+w)\n", grid, 2.0 * bytes / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
