// Dev probe (not product): write-bandwidth ceilings for the soft-assign output pattern vs the
// product kernel. Build: hipcc -O3 --offload-arch=gfx950 -I include tools/probe/probe_sa.hip
//   fl-slam_amd/gcslam/libgcslam.so -o tools/probe/probe_sa
#include "../../fl-slam_amd/csrc/gc_points.hip"
#include <cstdio>
#include <vector>

typedef double dvec2 __attribute__((ext_vector_type(2)));
// contiguous 16 B / lane stream
__global__ void __launch_bounds__(256) k_store_lin(double* out, int64_t n2, double v) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256)
    reinterpret_cast<dvec2*>(out)[i] = dvec2{v, v + 1.0};
}
// the soft-assign store pattern: per wave 64 rows x 384 B, 3 blocks x 8 pieces per lane
__global__ void __launch_bounds__(256) k_store_sa(double* R, int64_t n, int iters, double v) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, h = blockIdx.y;
  double* Rh = R + (int64_t)h * n * 48;
  const int64_t chunk0 = (int64_t)blockIdx.x * iters * 256;
  for (int it = 0; it < iters; ++it) {
    const int64_t wbase = chunk0 + (int64_t)it * 256 + wv * 64;
    if (wbase >= n) break;
    for (int blk = 0; blk < 3; ++blk) {
      const int i0 = lane >> 3, q = lane & 7;
      double* rowp = Rh + (wbase + i0) * 48 + 16 * blk + 2 * q;
#pragma unroll
      for (int m = 0; m < 8; ++m) *reinterpret_cast<dvec2*>(rowp + 8 * m * 48) = dvec2{v, v};
    }
  }
}

int main() {
  const int H = 256; const int64_t n = 65536; const int B = 48;
  double *dirs, *resp, *part, *bins; int32_t* idx;
  hipMalloc(&dirs, sizeof(double) * H * n * 3);
  hipMalloc(&resp, sizeof(double) * H * n * B);
  hipMalloc(&part, sizeof(double) * 2 * 64 * H);
  hipMalloc(&idx, sizeof(int32_t) * H * n);
  hipMalloc(&bins, sizeof(double) * 3 * B);
  std::vector<double> hb(3 * B), hd(3 * n);
  for (int b = 0; b < B; ++b) {
    double z = 1.0 - (2.0 * b + 1.0) / B, r = sqrt(1 - z * z), ph = b * 2.399963229728653;
    hb[3 * b] = r * cos(ph); hb[3 * b + 1] = r * sin(ph); hb[3 * b + 2] = z;
  }
  for (int64_t i = 0; i < n; ++i) {
    double z = 1.0 - (2.0 * i + 1.0) / n, r = sqrt(1 - z * z), ph = i * 0.7;
    hd[3 * i] = r * cos(ph); hd[3 * i + 1] = r * sin(ph); hd[3 * i + 2] = z;
  }
  hipMemcpy(bins, hb.data(), sizeof(double) * 3 * B, hipMemcpyHostToDevice);
  for (int h = 0; h < H; ++h) hipMemcpy(dirs + (int64_t)h * n * 3, hd.data(), sizeof(double) * 3 * n, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const double bytes = (double)H * n * B * 8;
  auto timeit = [&](const char* name, auto fn) {
    fn(); hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) fn();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
    printf("%-28s %8.3f ms  %7.0f GB/s (resp bytes)\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  timeit("store_lin grid 4096", [&] { hipLaunchKernelGGL(k_store_lin, dim3(4096), dim3(256), 0, 0, resp, (int64_t)H * n * B / 2, 1.0); });
  timeit("store_lin grid 16384", [&] { hipLaunchKernelGGL(k_store_lin, dim3(16384), dim3(256), 0, 0, resp, (int64_t)H * n * B / 2, 1.0); });
  timeit("store_sa pattern", [&] { hipLaunchKernelGGL(k_store_sa, dim3(64, H), dim3(256), 0, 0, resp, n, 4, 1.0); });
  timeit("k_soft_assign<3,true>", [&] { hipLaunchKernelGGL((gc::k_soft_assign<3, true>), dim3(64, H), dim3(256), 0, 0, n, B, 4, dirs, bins, 10.0, resp, idx, part); });
  timeit("k_soft_assign<3,true> noidx", [&] { hipLaunchKernelGGL((gc::k_soft_assign<3, true>), dim3(64, H), dim3(256), 0, 0, n, B, 4, dirs, bins, 10.0, resp, (int32_t*)nullptr, part); });
  return 0;
}
