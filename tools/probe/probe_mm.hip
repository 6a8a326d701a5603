// Dev probe (not product): moment-match contract kernel vs a pure read stream of the same bytes.
// Build with -DPROBE_NOMFMA to replace every f64 MFMA by a 4-wide VALU FMA (same operands).
#ifdef PROBE_NOMFMA
#define __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, x, y, z) ((c) + (a) * (b))
#endif
#include "../../fl-slam_amd/csrc/gc_points.hip"
#include <cstdio>
#include <vector>

typedef double dvec2 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256) k_read(const dvec2* __restrict__ a, int64_t n2, double* out) {
  dvec2 s = {0, 0};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) s += a[i];
  if (s.x == 12345.678) out[0] = s.y;
}

__global__ void k_fill(double* a, int64_t n, uint64_t seed, double lo, double hi) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27;
    a[i] = lo + (hi - lo) * (double)(x >> 11) * 0x1.0p-53;
  }
}

int main(int argc, char** argv) {
  const bool rnd = argc > 1;
  const int H = 256; const int64_t n = 65536; const int B = 48;
  double *pts, *covs, *w, *lam, *resp, *part;
  hipMalloc(&pts, sizeof(double) * H * n * 3);
  hipMalloc(&covs, sizeof(double) * H * n * 9);
  hipMalloc(&w, sizeof(double) * H * n);
  hipMalloc(&lam, sizeof(double) * H * n);
  hipMalloc(&resp, sizeof(double) * H * n * B);
  hipMalloc(&part, sizeof(double) * (size_t)128 * H * (B * 28 + 4));  // chunks <= 128 (groups >= 4)
  hipMemset(pts, 0, sizeof(double) * H * n * 3);
  hipMemset(covs, 0, sizeof(double) * H * n * 9);
  hipMemset(w, 0, sizeof(double) * H * n);
  hipMemset(lam, 0, sizeof(double) * H * n);
  hipMemset(resp, 0, sizeof(double) * H * n * B);
  if (rnd) {
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, pts, (int64_t)H * n * 3, 1, -20.0, 20.0);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, covs, (int64_t)H * n * 9, 2, 0.0, 1e-3);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, w, (int64_t)H * n, 3, 0.0, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, lam, (int64_t)H * n, 4, 0.5, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, resp, (int64_t)H * n * B, 5, 0.0, 0.04);
    hipDeviceSynchronize();
    printf("random data\n");
  }
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const double bytes = (double)H * n * (24 + 72 + 8 + 8 + 8 * B);
  auto timeit = [&](const char* name, auto fn) {
    for (int w = 0; w < 15; ++w) fn();  // clocks ramp over the first ~30 ms of sustained load
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) fn();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
    printf("%-36s %8.3f ms  %7.0f GB/s (contract bytes)\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  timeit("read resp only (16B/lane) g8192", [&] { hipLaunchKernelGGL(k_read, dim3(8192), dim3(256), 0, 0, (const dvec2*)resp, (int64_t)H * n * B / 2, part); });
  timeit("read resp only (16B/lane) g32768", [&] { hipLaunchKernelGGL(k_read, dim3(32768), dim3(256), 0, 0, (const dvec2*)resp, (int64_t)H * n * B / 2, part); });
  for (int groups : {4, 8, 16}) {
    const int64_t chunks = (n + 128 * groups - 1) / (128 * groups);
    if (chunks > 128) { printf("chunks %ld exceeds the partials buffer\n", (long)chunks); return 1; }
    const size_t sh = sizeof(double) * std::max<size_t>((size_t)4 * 32 * gc::kMomFS, (size_t)4 * B * 28);
    char nm[64]; snprintf(nm, 64, "k_moment_partials groups=%d", groups);
    timeit(nm, [&] { hipLaunchKernelGGL((gc::k_moment_partials<3, true, true, 1>), dim3(chunks, H), dim3(256), sh, 0, n, B, groups, pts, covs, w, resp, lam, 0.1, 0.2, 0.3, part); });
  }
  if (argc > 2) {  // interleave with the soft-assign contract kernel, as in the bench's roofline leg
    double *dirs, *bins, *sap; int32_t* idx;
    hipMalloc(&dirs, sizeof(double) * H * n * 3); hipMalloc(&bins, sizeof(double) * 3 * B);
    hipMalloc(&sap, sizeof(double) * 2 * 64 * H); hipMalloc(&idx, sizeof(int32_t) * H * n);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, dirs, (int64_t)H * n * 3, 7, -0.577, 0.577);
    hipLaunchKernelGGL(k_fill, dim3(1), dim3(256), 0, 0, bins, (int64_t)3 * B, 8, -0.577, 0.577);
    hipEvent_t ev[3]; for (auto& e : ev) hipEventCreate(&e);
    const size_t sh = sizeof(double) * std::max<size_t>((size_t)4 * 32 * gc::kMomFS, (size_t)4 * B * 28);
    for (int r = 0; r < 4; ++r) {
      hipEventRecord(ev[0]);
      hipLaunchKernelGGL((gc::k_soft_assign<3, true>), dim3(64, H), dim3(256), 0, 0, n, B, 4, dirs, bins, 10.0, resp, idx, sap);
      hipEventRecord(ev[1]);
      hipLaunchKernelGGL((gc::k_moment_partials<3, true, true, 1>), dim3(32, H), dim3(256), sh, 0, n, B, 16, pts, covs, w, resp, lam, 0.1, 0.2, 0.3, part);
      hipEventRecord(ev[2]); hipEventSynchronize(ev[2]);
      float a, b; hipEventElapsedTime(&a, ev[0], ev[1]); hipEventElapsedTime(&b, ev[1], ev[2]);
      printf("interleaved: soft_assign %.3f ms, moment_partials %.3f ms\n", a, b);
    }
  }
  return 0;
}
