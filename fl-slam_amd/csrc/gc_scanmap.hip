// gc_scanmap.hip — the C5 in-scan PrimitiveMap update (config C5, SURVEY §8d: "PoseCovInflation
// Pushforward map-update stress"; the reference's step 12b, pipeline.py:1236-1327, with
// transform_gaussian_to_world :1248-1256 and primitive_map_fuse, primitive_map.py:992-1163).
//
// BUILD-DEFINED (parity unpinned: the reference builds its measurement batch from camera splats /
// LiDAR surfels upstream of the OT association, outside this path, and PoseCovInflationPushforward's
// source is deleted, CHANGELOG.md:1246). Every budgeted point of the scan, deskewed with hypothesis
// 0's twist (a4), becomes one Gaussian row pushed to the world frame by hypothesis 0's recomposed
// pose z_t (t_z = 0, as the bin map), its covariance inflated by the pose covariance exactly as a13
// inflates a bin centroid:
//   μ_w = R p + t,   Σ_w = R Σ_lidar Rᵀ + J Σ_pose Jᵀ,   J = [R | −R [p]×],
//   Λ_w = Σ_w⁻¹,     θ_w = Λ_w μ_w,   η_w = [R d, 0, ..] (d = the unit ray direction),
// with Σ_lidar the measurement-IW LiDAR block's mode Ψ_2 / (ν_2 + 4) and the row's weight the
// deskewed point weight (a4). Its slot is the spatial hash of the world voxel of μ_w. The rows are
// fused with responsibility 1 and source LiDAR by the same reduce-by-key as gc_map.hip: a stable
// radix sort of (slot, row) and one thread per distinct slot summing its rows in row order, so the
// result is np.add.at's and bit-reproducible. LiDAR rows leave the camera accumulators unchanged,
// so the all-slot colour recompute (colors = rgb) runs only on the first update after the map is
// attached (gc_pipeline.cpp), when it may change colours an empty tile holds.
//
// Rows are never materialised: the key pass computes μ_w only, and the segment pass recomputes the
// row from the point index (40 B of point data per row instead of a 176 B row written and re-read).
// Every rank runs the update from the reduced record, so the maps stay bit-identical across ranks.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include "gc_internal.h"
#include "gc_math.h"
#include "gc_pipe.h"
#include "gc_scanmap.h"

namespace gc {
namespace {

constexpr int kSmapMaxLobes = 8;

struct ScanMapArgs {
  gc_primitive_map map;
  const double *pts, *t, *w_win, *bscal;  // the scan slot and predict's per-point w x window, budget
  const double* h0;                       // reduced record: [z_t 6, Σ_pose 36, ξ 6] of hypothesis 0
  const double *nu_meas, *Psi_meas;       // measurement IW state (LiDAR block 2)
  int64_t n_cap;
  double t0, t1, o0, o1, o2, voxel, timestamp, eps_mass;
  int64_t scan_seq;
};

// the row's deskewed body point and weight (false: padding or zero weight -> dropped)
GC_DEV bool smap_point(const ScanMapArgs& A, int64_t j, double* p0, double* w) {
  const int64_t n_sel = (int64_t)A.bscal[5], stride = (int64_t)A.bscal[6];
  if (j >= n_sel || j >= A.n_cap) return false;
  const int64_t i = j * stride;
  const double p[3] = {A.pts[3 * i], A.pts[3 * i + 1], A.pts[3 * i + 2]};
  const double alpha = (A.t[i] - A.t0) / fmax(A.t1 - A.t0, 1e-12);
  deskew_point(p, alpha, A.h0 + 42, p0);
  *w = A.w_win[j] * A.bscal[2];
  return *w > 0.0;
}

// μ_w = R p + t, left to right without contraction (the oracle's expression, so the voxel keys agree)
GC_DEV void smap_world_mean(const double* R, const double* tt, const double* p, double* mw) {
#pragma clang fp contract(off)
  for (int i = 0; i < 3; ++i) mw[i] = ((R[3 * i] * p[0] + R[3 * i + 1] * p[1]) + R[3 * i + 2] * p[2]) + tt[i];
}

GC_DEV uint32_t smap_slot(const double* mw, double voxel, int64_t M) {
  const int64_t vx = (int64_t)floor(mw[0] / voxel), vy = (int64_t)floor(mw[1] / voxel),
                vz = (int64_t)floor(mw[2] / voxel);
  const uint64_t h = ((uint64_t)vx * 73856093ull) ^ ((uint64_t)vy * 19349663ull) ^ ((uint64_t)vz * 83492791ull);
  return (uint32_t)(h % (uint64_t)M);
}

GC_DEV void smap_pose(const ScanMapArgs& A, double* R, double* tt) {
  so3_exp(A.h0 + 3, R);
  tt[0] = A.h0[0]; tt[1] = A.h0[1]; tt[2] = 0.0;  // planar map: t_z = 0 (CHANGELOG.md:575-578)
}

__global__ void k_smap_keys(ScanMapArgs A, uint32_t* keys, uint32_t* vals) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= A.n_cap) return;
  double R[9], tt[3], p0[3], mw[3], w;
  smap_pose(A, R, tt);
  uint32_t key = (uint32_t)A.map.m_slots;  // dropped rows sort after every slot
  if (smap_point(A, j, p0, &w)) {
    smap_world_mean(R, tt, p0, mw);
    key = smap_slot(mw, A.voxel, A.map.m_slots);
  }
  keys[j] = key;
  vals[j] = (uint32_t)j;
}

// One world row (the comment at the top): Λ_w (9), θ_w (3), η_w lobe 0 (3).
GC_DEV void smap_row(const ScanMapArgs& A, const double* R, const double* tt, const double* Sl, const double* p0,
                     double* Lw, double* th, double* e0) {
  double mw[3];
  smap_world_mean(R, tt, p0, mw);
  // Σ_w = R Σ_l Rᵀ + J Σ_pose Jᵀ, J = [R | −R K], K = [p0]×
  double M3[9], Sw[9];
  mat3_mul(R, Sl, M3);
  mat3_mul_nt(M3, R, Sw);
  const double K[9] = {0.0, -p0[2], p0[1], p0[2], 0.0, -p0[0], -p0[1], p0[0], 0.0};
  double RK[9], J[18];
  mat3_mul(R, K, RK);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) { J[i * 6 + j] = R[3 * i + j]; J[i * 6 + 3 + j] = -RK[3 * i + j]; }
  const double* Sp = A.h0 + 6;
  double JS[18];  // J Σ_pose (3 x 6)
  for (int i = 0; i < 3; ++i)
    for (int c = 0; c < 6; ++c) {
      double v = 0.0;
      for (int a = 0; a < 6; ++a) v += J[i * 6 + a] * Sp[a * 6 + c];
      JS[i * 6 + c] = v;
    }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double v = 0.0;
      for (int c = 0; c < 6; ++c) v += JS[i * 6 + c] * J[j * 6 + c];
      Sw[3 * i + j] += v;
    }
  for (int i = 0; i < 3; ++i)  // symmetric by construction up to rounding: symmetrise before inverting
    for (int j = i + 1; j < 3; ++j) {
      const double v = 0.5 * (Sw[3 * i + j] + Sw[3 * j + i]);
      Sw[3 * i + j] = v;
      Sw[3 * j + i] = v;
    }
  inv3(Sw, Lw);
  mat3_vec(Lw, mw, th);
  const double o[3] = {A.o0, A.o1, A.o2};
  double d[3];
  direction(p0, o, A.eps_mass, d);
  mat3_vec(R, d, e0);
}

__global__ void __launch_bounds__(256) k_smap_segments(ScanMapArgs A, const uint32_t* __restrict__ keys,
                                                       const uint32_t* __restrict__ vals,
                                                       unsigned long long* n_unique) {
#pragma clang fp contract(off)  // r·X then add, as the fuse and np.add.at
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t K = A.n_cap;
  if (i >= K) return;
  const uint32_t key = keys[i];
  if ((int64_t)key >= A.map.m_slots || (i > 0 && keys[i - 1] == key)) return;  // dropped / not a segment head
  const int L = A.map.n_lobes;
  const int64_t s = key;
  // the slot's current values first (their latency overlaps the row work)
  double mL[9], mth[3], met[3 * kSmapMaxLobes], mw, mlid = 0.0;
  for (int q = 0; q < 9; ++q) mL[q] = A.map.Lambdas[9 * s + q];
  for (int q = 0; q < 3; ++q) mth[q] = A.map.thetas[3 * s + q];
  for (int q = 0; q < 3 * L; ++q) met[q] = A.map.etas[(int64_t)3 * L * s + q];
  mw = A.map.weights[s];
  if (A.map.lidar_mass) mlid = A.map.lidar_mass[s];
  double R[9], tt[3], Sl[9];
  smap_pose(A, R, tt);
  {
    const double den = A.nu_meas[2] + 3.0 + 1.0;  // measurement_noise_mean_jax, LiDAR block
    for (int q = 0; q < 9; ++q) Sl[q] = A.Psi_meas[18 + q] / den;
  }
  double dL[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, dth[3] = {0, 0, 0}, de0[3] = {0, 0, 0}, dw = 0.0, dlid = 0.0;
  for (int64_t j = i; j < K && keys[j] == key; ++j) {
    const int64_t row = vals[j];
    double p0[3], w, Lw[9], th[3], e0[3];
    smap_point(A, row, p0, &w);  // a row with a key is valid
    smap_row(A, R, tt, Sl, p0, Lw, th, e0);
    const double r = 1.0;
    for (int q = 0; q < 9; ++q) dL[q] += r * Lw[q];
    for (int q = 0; q < 3; ++q) dth[q] += r * th[q];
    for (int q = 0; q < 3; ++q) de0[q] += r * e0[q];
    dw += r * w;
    dlid += r * w;
  }
  for (int q = 0; q < 9; ++q) A.map.Lambdas[9 * s + q] = mL[q] + dL[q];
  for (int q = 0; q < 3; ++q) A.map.thetas[3 * s + q] = mth[q] + dth[q];
  // lobes > 0 receive 0.0 per row: x + 0.0 = x for every x but -0.0, written as the fuse does
  for (int q = 0; q < 3; ++q) A.map.etas[(int64_t)3 * L * s + q] = met[q] + de0[q];
  for (int q = 3; q < 3 * L; ++q) A.map.etas[(int64_t)3 * L * s + q] = met[q] + 0.0;
  A.map.weights[s] = mw + dw;
  A.map.timestamps[s] = A.timestamp;
  A.map.last_supported_scan_seq[s] = A.scan_seq;
  A.map.last_update_scan_seq[s] = A.scan_seq;
  if (A.map.lidar_mass) A.map.lidar_mass[s] = mlid + dlid;
  atomicAdd(n_unique, 1ull);  // integer count: order-independent
}

inline int key_bits(int64_t M) {
  int b = 1;
  while (b < 32 && (M >> b) != 0) ++b;
  return b;
}

}  // namespace

int32_t scan_map_prepare(gc_ctx* ctx, ScanMapWork* W, int64_t n_cap, int64_t m_slots) {
  W->n_cap = n_cap;
  W->bits = key_bits(m_slots);
  size_t temp = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                         (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n_cap, 0, W->bits,
                                         ctx->stream) != hipSuccess) {
    set_error(ctx, "radix sort sizing failed");
    return GC_ERR_RUNTIME;
  }
  const size_t kv = ((size_t)n_cap * sizeof(uint32_t) + 255) / 256 * 256;
  const size_t bytes = 4 * kv + 256 + temp;
  if (bytes > W->bytes) {
    if (W->buf) GC_HIP(ctx, hipFree(W->buf));
    W->buf = nullptr;
    W->bytes = 0;
    GC_HIP(ctx, hipMalloc(&W->buf, bytes));
    W->bytes = bytes;
  }
  char* base = (char*)W->buf;
  W->keys_in = (uint32_t*)base;
  W->vals_in = (uint32_t*)(base + kv);
  W->keys = (uint32_t*)(base + 2 * kv);
  W->vals = (uint32_t*)(base + 3 * kv);
  W->count = (unsigned long long*)(base + 4 * kv);
  W->temp = base + 4 * kv + 256;
  W->temp_bytes = temp;
  return GC_OK;
}

int32_t scan_map_update(gc_ctx* ctx, hipStream_t st, ScanMapWork* W, const gc_primitive_map& map,
                        const PipeDev& P, const ScanMapInput& in) {
  ScanMapArgs A{};
  A.map = map;
  A.pts = in.pts; A.t = in.t; A.w_win = P.w_win; A.bscal = P.budget;
  A.h0 = P.send + rec_h0(P.B);  // the reduced record (k_combine_final, earlier on this stream)
  A.nu_meas = P.nu_meas; A.Psi_meas = P.Psi_meas;
  A.n_cap = P.n_cap;
  A.t0 = in.t0; A.t1 = in.t1;
  A.o0 = P.o0; A.o1 = P.o1; A.o2 = P.o2;
  A.voxel = in.voxel; A.timestamp = in.timestamp; A.eps_mass = P.eps_mass;
  A.scan_seq = in.scan_seq;
  const unsigned grid = (unsigned)((P.n_cap + 255) / 256);
  GC_HIP(ctx, hipMemsetAsync(W->count, 0, sizeof(unsigned long long), st));
  hipLaunchKernelGGL(k_smap_keys, dim3(grid), dim3(256), 0, st, A, W->keys_in, W->vals_in);
  GC_LAUNCH_CHECK(ctx);
  size_t temp = W->temp_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(W->temp, temp, W->keys_in, W->keys, W->vals_in, W->vals, (int)P.n_cap, 0,
                                         W->bits, st) != hipSuccess) {
    set_error(ctx, "radix sort failed");
    return GC_ERR_RUNTIME;
  }
  hipLaunchKernelGGL(k_smap_segments, dim3(grid), dim3(256), 0, st, A, (const uint32_t*)W->keys,
                     (const uint32_t*)W->vals, W->count);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

}  // namespace gc
