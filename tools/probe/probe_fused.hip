// Dev probe (not product): the fused a1->a6 bins kernel at C3 size (64k points x 256 hypotheses),
// times the shipped configuration (kFusedOcc / kFusedNacc are constants of gc_points.hip: a variant is
// an edit of those constants, built here, never a knob of the product); times the
// bin-distributed product kernel (k_bins_fused) and the lane-per-point experiment (k_bins_fused_lp,
// kept here only).
#include "../../fl-slam_amd/csrc/gc_points.hip"
#include <cstdio>
#include <vector>

namespace gc {
// Lane-per-point fused kernel (experiment, not shipped: measured slower than k_bins_fused at one
// wave per SIMD). Phase A as in k_bins_fused (lane = point:
// budget gather, deskew, direction, 19 features). Phase B keeps the whole softmax of a point in
// its lane: the 16*BPL similarities against the 1/τ-prescaled bins (wave-uniform scalar loads),
// exps (LDS table), Z, the entropy partial and the max responsibility are lane-local, so there
// is no cross-lane butterfly and one reciprocal per point instead of one per 4-point step. The
// features are pre-multiplied by 1/Z (Σ_p e_pb (F_pk / Z_p) = Σ_p R_pb F_pk, rounding order
// only), so the MFMA A operand is the raw e. The point's e row is transposed through a
// wave-private LDS slab (row stride NB + 2: conflict-free ds_write_b128 rows and ds_read_b64
// columns) and consumed by 16 steps of BPL v_mfma_f64_16x16x4_f64 (features 0..15) plus VALU
// FMAs (16..18), 2*BPL independent accumulation chains. f64 MFMA and f64 VALU share the DP
// pipe on gfx950 (tools/probe/probe_rates.hip), so the kernel is bound by issued DP
// instructions; this layout issues ~1/3 fewer than k_bins_fused. The e row (2 NB VGPRs) and the
// full slab (36 KB per wave) size it for one wave per SIMD (up to 512 VGPR+AGPR); the next
// iteration's point loads are issued before the softmax to cover their latency.
#ifndef GC_LP_OCC
#define GC_LP_OCC 1
#endif
template <int BPL>
constexpr int lp_es() { return 16 * BPL + 2; }
template <int BPL, bool FULL>
__global__ void __launch_bounds__(256, GC_LP_OCC) k_bins_fused_lp(int64_t n_cap, int B, int iters,
                                                          const double* __restrict__ pts_raw,
                                                          const double* __restrict__ t_raw,
                                                          const double* __restrict__ w_raw,
                                                          const double* __restrict__ bscal, double t0, double t1,
                                                          const double* __restrict__ xi,
                                                          const double* __restrict__ bins_scaled, double inv_tau,
                                                          double o0, double o1, double o2, double* partials) {
  constexpr int NF = NF_BASE;
  constexpr int NX = NF - 16;  // features on the VALU
  constexpr int NB = 16 * BPL;
  constexpr int ES = lp_es<BPL>();
  typedef double dvec2 __attribute__((ext_vector_type(2)));
  extern __shared__ double lds[];
  const int h = blockIdx.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, bl = lane & 15;
  double* F = lds + wv * (NF * kFusedFS);                    // [feature][point] x 1/Z
  double* E = lds + 4 * NF * kFusedFS + wv * (64 * ES);       // [point][bin]
  double* Tx = lds + 4 * NF * kFusedFS + 4 * 64 * ES;         // exp table
  const double o[3] = {o0, o1, o2};
  double xr[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) xr[k] = xi[6 * h + k];
  const double scale = bscal[2];
  const int64_t n_sel = (int64_t)bscal[5];
  const int64_t stride = (int64_t)bscal[6];
  const double denom = fmax(t1 - t0, 1e-12);
  const double inv_denom = 1.0 / denom;
  const double inv_sig = 1.0 / fmax(0.1 * denom, 1e-6);
  exp_table_init(Tx);
  __syncthreads();
  v4d acc4[2][BPL];  // even / odd steps
  double accx[BPL][NX];
#pragma unroll
  for (int jt = 0; jt < BPL; ++jt) {
    acc4[0][jt] = v4d{0.0, 0.0, 0.0, 0.0};
    acc4[1][jt] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int t = 0; t < NX; ++t) accx[jt][t] = 0.0;
  }
  double sumw = 0.0, logacc = 0.0, entq = 0.0, mxr = 0.0;
  const double xmax = inv_tau;  // S <= 1 for unit vectors: exp never overflows
  const double Beps = (double)B * 1e-12;
  const int64_t chunk0 = (int64_t)blockIdx.x * iters * 256;
  // raw point of this lane for iteration `it` (clamped, branch-free; selection applied after)
  double np0, np1, np2, nt, nw;
  auto load_raw = [&](int it) {
    const int64_t j = chunk0 + (int64_t)it * 256 + wv * 64 + lane;
    const int64_t jj = j < n_sel ? j : (n_sel > 0 ? n_sel - 1 : 0);
    const int64_t i = jj * stride;
    np0 = pts_raw[3 * i]; np1 = pts_raw[3 * i + 1]; np2 = pts_raw[3 * i + 2];
    nt = t_raw[i];
    nw = w_raw[i];
  };
  load_raw(0);
  for (int it = 0; it < iters; ++it) {
    const int64_t wbase = chunk0 + (int64_t)it * 256 + wv * 64;
    // ---- phase A: lane = point
    const int64_t j = wbase + lane;
    const bool inr = j < n_cap;
    const bool sel = inr && j < n_sel;
    double p[3] = {sel ? np0 : 0.0, sel ? np1 : 0.0, sel ? np2 : 0.0};
    const double tt = sel ? nt : 0.0, ww = sel ? nw * scale : 0.0;
    if (it + 1 < iters) load_raw(it + 1);  // in flight across this iteration's softmax
    double q[3], d[3];
    deskew_point_fast(p, (tt - t0) * inv_denom, xr, q);
    const double wd = inr ? ww * window_weight_fast(tt, t0, t1, inv_sig, Tx) : 0.0;
    direction_fast(q, o, 1e-12, d);
    sumw += wd;
    lds_wave_sync();  // the previous iteration's operand reads are done
    {  // features parked in the lane's own slab column until 1/Z is known
      double f[NF];
      point_features(q, d, wd, f);
#pragma unroll
      for (int k = 0; k < NF; ++k) F[k * kFusedFS + lane] = f[k];
    }
    // ---- phase B: the point's softmax, lane-local
    const __attribute__((address_space(4))) double* bp = (const __attribute__((address_space(4))) double*)bins_scaled;
    double e[NB];
    double Z = 0.0, sl = 0.0, em = 0.0;
#pragma unroll
    for (int j0 = 0; j0 < NB; j0 += 8) {
      asm volatile("" : "+s"(bp));  // this group's scalar loads are issued here, not all up front
      double x[8], e8[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int b = j0 + jj;  // bins past B are zero: x = -1/τ stays finite, then masked
        x[jj] = fma(d[0], bp[3 * b], fma(d[1], bp[3 * b + 1], fma(d[2], bp[3 * b + 2], -xmax)));
      }
      exp_neg_n<8>(x, Tx, e8);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int b = j0 + jj;
        e[b] = (FULL || b < B) ? e8[jj] : 0.0;
        Z += e[b];
        sl = fma(e[b], x[jj], sl);
        em = e[b] > em ? e[b] : em;
      }
    }
#pragma unroll
    for (int qd = 0; qd < NB / 2; ++qd)
      *reinterpret_cast<dvec2*>(&E[lane * ES + 2 * qd]) = dvec2{e[2 * qd], e[2 * qd + 1]};
    const double rZ = recip(Z);
    if (inr) {
      logacc += log(Z);
      entq = fma(sl, rZ, entq);
      const double mr = em * rZ;
      mxr = mr > mxr ? mr : mxr;
    }
#pragma unroll
    for (int k = 0; k < NF; ++k) F[k * kFusedFS + lane] *= rZ;  // own column: no cross-lane hazard
    lds_wave_sync();
#pragma unroll 2
    for (int s = 0; s < 16; ++s) {
      const int pl = s * 4 + g;
      const double fb = F[bl * kFusedFS + pl];  // B: feature bl of point 4s + g
      double fk[NX];
#pragma unroll
      for (int t = 0; t < NX; ++t) fk[t] = F[(16 + t) * kFusedFS + pl];
#pragma unroll
      for (int jt = 0; jt < BPL; ++jt) {
        const double a = E[pl * ES + 16 * jt + bl];  // A: e of bin 16 jt + bl, point 4s + g
        acc4[s & 1][jt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, fb, acc4[s & 1][jt], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NX; ++t) accx[jt][t] = fma(a, fk[t], accx[jt][t]);
      }
    }
  }
  // entropy sum over the chunk's valid points: Σ log Z - Σ S/Z - B ε
  int64_t npts = n_cap - chunk0;
  npts = npts < 0 ? 0 : (npts > (int64_t)iters * 256 ? (int64_t)iters * 256 : npts);
  const double ent = logacc - entq - ((lane == 0) ? Beps * (double)npts * 0.25 : 0.0);
  const int RL = B * NF + REC_EXTRA;
#pragma unroll
  for (int jt = 0; jt < BPL; ++jt) acc4[0][jt] += acc4[1][jt];
  __syncthreads();
  write_partial_record_mfma<BPL, NX>(acc4[0], accx, ent, mxr, sumw, (double)npts, B, lds,
                                     partials + ((int64_t)h * gridDim.x + blockIdx.x) * RL);
}

// bins / τ, zero-padded to 16 * BPL rows (the lane-per-point kernel's scalar-load operand)
__global__ void k_scale_bins(int B, int NB, const double* __restrict__ bins, double inv_tau, double* out) {
  const int i = threadIdx.x;
  if (i < 3 * NB) out[i] = (i < 3 * B) ? bins[i] * inv_tau : 0.0;
}

}  // namespace gc

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
  const int iters = 16; const int64_t chunks = (n + iters * 256 - 1) / (iters * 256);
  const int RL = B * gc::NF_BASE + gc::REC_EXTRA;
  hipMalloc(&part, sizeof(double) * (size_t)H * chunks * RL);
  hipMemcpy(p, hp.data(), 8 * 3 * n, hipMemcpyHostToDevice); hipMemcpy(t, ht.data(), 8 * n, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), 8 * n, hipMemcpyHostToDevice); hipMemcpy(bs, hs.data(), 64, hipMemcpyHostToDevice);
  hipMemcpy(xi, hx.data(), 8 * 6 * H, hipMemcpyHostToDevice); hipMemcpy(bins, hb.data(), 8 * 3 * B, hipMemcpyHostToDevice);
  const size_t sh = sizeof(double) * std::max<size_t>(4 * gc::kFusedFS * (gc::NF_BASE + 4) + gc::kExpTab2 + 192, 4 * (size_t)B * gc::NF_BASE + 12);
  hipFuncSetAttribute((const void*)gc::k_bins_fused<3, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&] { hipLaunchKernelGGL((gc::k_bins_fused<3, true>), dim3(chunks, H), dim3(256), sh, 0, n, B, iters, p, t, w, bs, 100.0, 100.1, xi, bins, 10.0, -0.06, -0.1, 0.1, part); };
  for (int w = 0; w < 20; ++w) run(); hipDeviceSynchronize();
  hipEventRecord(e0); for (int r = 0; r < 10; ++r) run(); hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("k_bins_fused<3> occ=%d nacc=%d: %.3f ms/launch (%s)\n", gc::kFusedOcc, gc::kFusedNacc, ms / 10, hipGetErrorString(hipGetLastError()));
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
