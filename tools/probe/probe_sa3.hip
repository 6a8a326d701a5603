// Dev probe (not product): the soft-assign contract kernel variants (ex[] in registers vs the
// register-light recompute form) at C3 size, timed with events; FETCH/WRITE passes via rocprofv3.
// Build: hipcc -O3 --offload-arch=gfx950 -I include tools/probe/probe_sa3.hip -o tools/probe/probe_sa3
#include "../../fl-slam_amd/csrc/gc_points.hip"
#include <cstdio>
#include <vector>

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
  const double bytes = (double)H * (n * 24 + n * B * 8);
  auto timeit = [&](const char* name, auto fn) {
    for (int w = 0; w < 20; ++w) fn();  // clocks ramp over the first ~30 ms of sustained load
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) fn();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
    printf("%-34s %8.3f ms  %7.0f GB/s (algorithmic)\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  for (int iters : {4, 8}) {
    const int blocks = (int)((n + iters * 256 - 1) / (iters * 256));
    char nm[64];
    snprintf(nm, 64, "regs iters=%d", iters);
    timeit(nm, [&] { hipLaunchKernelGGL((gc::k_soft_assign<3, true, false>), dim3(blocks, H), dim3(256), 0, 0, n, B, iters, dirs, bins, 10.0, resp, idx, part); });
    snprintf(nm, 64, "recomp iters=%d", iters);
    timeit(nm, [&] { hipLaunchKernelGGL((gc::k_soft_assign<3, true, true>), dim3(blocks, H), dim3(256), 0, 0, n, B, iters, dirs, bins, 10.0, resp, idx, part); });
  }
  printf("%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
