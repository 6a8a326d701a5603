// Dev probe (not product): the fused a1->a6 bins kernel at C3 size (64k points x 256 hypotheses),
// built per tuning variant with -DGC_FUSED_OCC / -DGC_FUSED_NACC / -DGC_LP_OCC; times the
// bin-distributed kernel (k_bins_fused) and the lane-per-point product kernel (k_bins_fused_lp).
#include "../../fl-slam_amd/csrc/gc_points.hip"
#include <cstdio>
#include <vector>

int main() {
  const int H = 256; const int64_t n = 65536; const int B = 48;
  std::vector<double> hp(3 * n), ht(n), hw(n), hb(3 * B), hx(6 * H), hs(8, 0.0);
  for (int64_t i = 0; i < n; ++i) {
    const double az = 2 * M_PI * (i % 4096) / 4096.0, el = -0.26 + 0.035 * (i / 4096);
    const double r = 3.0 + 2.0 * std::fabs(std::sin(3 * az));
    hp[3 * i] = r * cos(el) * cos(az); hp[3 * i + 1] = r * cos(el) * sin(az); hp[3 * i + 2] = r * sin(el);
    ht[i] = 100.0 + 0.1 * (i % 4096) / 4096.0; hw[i] = 0.9;
  }
  for (int b = 0; b < B; ++b) {
    double z = 1.0 - (2.0 * b + 1.0) / B, rr = sqrt(1 - z * z), ph = b * 2.399963229728653;
    hb[3 * b] = rr * cos(ph); hb[3 * b + 1] = rr * sin(ph); hb[3 * b + 2] = z;
  }
  for (int h = 0; h < H; ++h) { hx[6 * h] = 0.1 + 1e-4 * h; hx[6 * h + 5] = 0.03; }
  hs[2] = 1.0; hs[5] = (double)n; hs[6] = 1.0;
  double *p, *t, *w, *bs, *xi, *bins, *part;
  hipMalloc(&p, 8 * 3 * n); hipMalloc(&t, 8 * n); hipMalloc(&w, 8 * n); hipMalloc(&bs, 64);
  hipMalloc(&xi, 8 * 6 * H); hipMalloc(&bins, 8 * 3 * B);
  const int iters = 8; const int64_t chunks = (n + iters * 256 - 1) / (iters * 256);
  const int RL = B * gc::NF_BASE + gc::REC_EXTRA;
  hipMalloc(&part, sizeof(double) * (size_t)H * chunks * RL);
  hipMemcpy(p, hp.data(), 8 * 3 * n, hipMemcpyHostToDevice); hipMemcpy(t, ht.data(), 8 * n, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), 8 * n, hipMemcpyHostToDevice); hipMemcpy(bs, hs.data(), 64, hipMemcpyHostToDevice);
  hipMemcpy(xi, hx.data(), 8 * 6 * H, hipMemcpyHostToDevice); hipMemcpy(bins, hb.data(), 8 * 3 * B, hipMemcpyHostToDevice);
  const size_t sh = sizeof(double) * std::max<size_t>(4 * gc::kFusedFS * (gc::NF_BASE + 4) + gc::kExpTab + 192, 4 * (size_t)B * gc::NF_BASE + 12);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&] { hipLaunchKernelGGL((gc::k_bins_fused<3, true>), dim3(chunks, H), dim3(256), sh, 0, n, B, iters, p, t, w, bs, 100.0, 100.1, xi, bins, 10.0, -0.06, -0.1, 0.1, part); };
  run(); hipDeviceSynchronize();
  hipEventRecord(e0); for (int r = 0; r < 10; ++r) run(); hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("k_bins_fused<3> occ=%d nacc=%d: %.3f ms/launch (%s)\n", GC_FUSED_OCC, GC_FUSED_NACC, ms / 10, hipGetErrorString(hipGetLastError()));
  // lane-per-point variant (product path)
  double* bsc; hipMalloc(&bsc, 8 * 3 * 64);
  hipLaunchKernelGGL(gc::k_scale_bins, dim3(1), dim3(192), 0, 0, B, 48, bins, 10.0, bsc);
  const size_t sh2 = sizeof(double) * (4 * gc::kFusedFS * gc::NF_BASE + 4 * 64 * 50 + gc::kExpTab);
  hipFuncSetAttribute((const void*)gc::k_bins_fused_lp<3, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh2);
  auto run2 = [&] { hipLaunchKernelGGL((gc::k_bins_fused_lp<3, true>), dim3(chunks, H), dim3(256), sh2, 0, n, B, iters, p, t, w, bs, 100.0, 100.1, xi, bsc, 10.0, -0.06, -0.1, 0.1, part); };
  run2(); hipDeviceSynchronize();
  hipEventRecord(e0); for (int r = 0; r < 10; ++r) run2(); hipEventRecord(e1); hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  printf("k_bins_fused_lp<3,full> occ=%d: %.3f ms/launch (%s)\n", GC_LP_OCC, ms / 10, hipGetErrorString(hipGetLastError()));
  return 0;
}
