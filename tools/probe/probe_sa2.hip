// Dev probe (not product): where do the extra HBM reads of the soft-assign contract kernel come
// from? Store-pattern kernels of the same 6.4 GB responsibility output (H=256 x 65,536 x 48 f64),
// plain and non-temporal, timed with events; run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
// passes to read their traffic. Build (CPU container):
//   hipcc -O3 --offload-arch=gfx950 -I include tools/probe/probe_sa2.hip -o tools/probe/probe_sa2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef double dvec2 __attribute__((ext_vector_type(2)));
constexpr int B = 48;

// contiguous 16 B / lane grid-stride stream (the write ceiling)
template <bool NT>
__global__ void __launch_bounds__(256) k_lin(double* out, int64_t n2, double v) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
    const dvec2 x = dvec2{v, v + 1.0};
    if (NT) __builtin_nontemporal_store(x, reinterpret_cast<dvec2*>(out) + i);
    else reinterpret_cast<dvec2*>(out)[i] = x;
  }
}
// the shipped pattern: per wave 64 rows; per block of 16 bins, 8 instructions of 8 rows x 128 B
template <bool NT>
__global__ void __launch_bounds__(256) k_rows8(double* R, int64_t n, int iters, double v) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, h = blockIdx.y;
  double* Rh = R + (int64_t)h * n * B;
  const int64_t chunk0 = (int64_t)blockIdx.x * iters * 256;
  for (int it = 0; it < iters; ++it) {
    const int64_t wbase = chunk0 + (int64_t)it * 256 + wv * 64;
    if (wbase >= n) break;
    for (int blk = 0; blk < 3; ++blk) {
      const int i0 = lane >> 3, q = lane & 7;
      double* rowp = Rh + (wbase + i0) * B + 16 * blk + 2 * q;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const dvec2 x = dvec2{v, v};
        if (NT) __builtin_nontemporal_store(x, reinterpret_cast<dvec2*>(rowp + 8 * m * B));
        else *reinterpret_cast<dvec2*>(rowp + 8 * m * B) = x;
      }
    }
  }
}
// a wave's 64 rows are one contiguous 24 KB span: 24 instructions of 1 KB contiguous
template <bool NT>
__global__ void __launch_bounds__(256) k_span(double* R, int64_t n, int iters, double v) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, h = blockIdx.y;
  double* Rh = R + (int64_t)h * n * B;
  const int64_t chunk0 = (int64_t)blockIdx.x * iters * 256;
  for (int it = 0; it < iters; ++it) {
    const int64_t wbase = chunk0 + (int64_t)it * 256 + wv * 64;
    if (wbase >= n) break;
    dvec2* sp = reinterpret_cast<dvec2*>(Rh + wbase * B);
#pragma unroll
    for (int m = 0; m < 24; ++m) {
      const dvec2 x = dvec2{v, v};
      if (NT) __builtin_nontemporal_store(x, sp + 64 * m + lane);
      else sp[64 * m + lane] = x;
    }
  }
}
// 8 B / lane: 16 lanes x 8 B = one 128-B row segment, 4 rows per instruction (a 16-lane point group)
template <bool NT>
__global__ void __launch_bounds__(256) k_rows4(double* R, int64_t n, int iters, double v) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, h = blockIdx.y, g = lane >> 4, bl = lane & 15;
  double* Rh = R + (int64_t)h * n * B;
  const int64_t chunk0 = (int64_t)blockIdx.x * iters * 256;
  for (int it = 0; it < iters; ++it) {
    const int64_t wbase = chunk0 + (int64_t)it * 256 + wv * 64;
    if (wbase >= n) break;
    for (int s = 0; s < 16; ++s) {
      double* row = Rh + (wbase + 4 * s + g) * B + bl;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (NT) __builtin_nontemporal_store(v, row + 16 * j);
        else row[16 * j] = v;
      }
    }
  }
}

int main() {
  const int H = 256;
  const int64_t n = 65536;
  double* resp;
  hipMalloc(&resp, sizeof(double) * H * n * B);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double bytes = (double)H * n * B * 8;
  auto timeit = [&](const char* name, auto fn) {
    fn();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) fn();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    printf("%-22s %8.3f ms  %7.0f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  const int64_t n2 = (int64_t)H * n * B / 2;
  timeit("lin", [&] { hipLaunchKernelGGL(k_lin<false>, dim3(16384), dim3(256), 0, 0, resp, n2, 1.0); });
  timeit("lin_nt", [&] { hipLaunchKernelGGL(k_lin<true>, dim3(16384), dim3(256), 0, 0, resp, n2, 1.0); });
  timeit("rows8", [&] { hipLaunchKernelGGL(k_rows8<false>, dim3(64, H), dim3(256), 0, 0, resp, n, 4, 1.0); });
  timeit("rows8_nt", [&] { hipLaunchKernelGGL(k_rows8<true>, dim3(64, H), dim3(256), 0, 0, resp, n, 4, 1.0); });
  timeit("span", [&] { hipLaunchKernelGGL(k_span<false>, dim3(64, H), dim3(256), 0, 0, resp, n, 4, 1.0); });
  timeit("span_nt", [&] { hipLaunchKernelGGL(k_span<true>, dim3(64, H), dim3(256), 0, 0, resp, n, 4, 1.0); });
  timeit("rows4", [&] { hipLaunchKernelGGL(k_rows4<false>, dim3(64, H), dim3(256), 0, 0, resp, n, 4, 1.0); });
  timeit("rows4_nt", [&] { hipLaunchKernelGGL(k_rows4<true>, dim3(64, H), dim3(256), 0, 0, resp, n, 4, 1.0); });
  printf("%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
