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
// fused with responsibility 1 and source LiDAR by a reduce-by-key: a stable radix sort of (slot,
// row), the rows gathered into that order, rocprim's deterministic reduce_by_key (a fixed
// association per run, so bit-reproducible run to run; within 1e-12 of np.add.at's sequential
// order) and one thread per distinct slot applying its sum. A scan's points crowd into few voxels
// (~65k rows into ~5k slots, runs of thousands near the sensor), so rows are computed one per
// thread and the runs reduced in parallel: one thread per run summing its rows serially took
// ~1 ms per scan. LiDAR rows leave the camera accumulators unchanged,
// so the all-slot colour recompute (colors = rgb) runs only on the first update after the map is
// attached (gc_pipeline.cpp), when it may change colours an empty tile holds.
//
// Every rank runs the update from the reduced record, so the maps stay bit-identical across ranks.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_reduce_by_key.hpp>
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

constexpr int kSmapRow = 16;  // [Λ_w 9, θ_w 3, η_w lobe 0 3, w]
struct SmapRow {
  double v[kSmapRow];
};
struct SmapRowSum {
  __host__ __device__ SmapRow operator()(const SmapRow& a, const SmapRow& b) const {
    SmapRow c;
#pragma unroll
    for (int q = 0; q < kSmapRow; ++q) c.v[q] = a.v[q] + b.v[q];
    return c;
  }
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

// one thread per row: its slot key (m_slots for a dropped row, sorted after every slot) and its
// world row [Λ_w 9, θ_w 3, η_w lobe 0 3, w] (zeros when dropped)
__global__ void k_smap_rows(ScanMapArgs A, uint32_t* keys, uint32_t* vals, SmapRow* rows) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= A.n_cap) return;
  double R[9], tt[3], p0[3], w, mw[3], Sl[9];
  smap_pose(A, R, tt);
  SmapRow row;
  for (int q = 0; q < kSmapRow; ++q) row.v[q] = 0.0;
  uint32_t key = (uint32_t)A.map.m_slots;
  if (smap_point(A, j, p0, &w)) {
    smap_world_mean(R, tt, p0, mw);
    key = smap_slot(mw, A.voxel, A.map.m_slots);
    const double den = A.nu_meas[2] + 3.0 + 1.0;  // measurement_noise_mean_jax, LiDAR block
    for (int q = 0; q < 9; ++q) Sl[q] = A.Psi_meas[18 + q] / den;
    smap_row(A, R, tt, Sl, p0, row.v, row.v + 9, row.v + 12);
    row.v[15] = w;
  }
  keys[j] = key;
  vals[j] = (uint32_t)j;
  rows[j] = row;
}

// the rows in sorted (slot, row) order, one double per thread (coalesced)
__global__ void k_smap_gather(int64_t n, const uint32_t* __restrict__ vals, const double* __restrict__ rows,
                              double* srows) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * kSmapRow) return;
  const int64_t i = e / kSmapRow, q = e % kSmapRow;
  srows[e] = rows[(int64_t)vals[i] * kSmapRow + q];
}

// one thread per run of the sorted keys: slot += its row sum (the fuse's read-modify-write)
__global__ void k_smap_apply(ScanMapArgs A, const uint32_t* __restrict__ unique, const SmapRow* __restrict__ agg,
                             const uint32_t* __restrict__ n_runs, unsigned long long* n_unique) {
#pragma clang fp contract(off)
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= (int64_t)*n_runs) return;
  const uint32_t key = unique[u];
  if ((int64_t)key >= A.map.m_slots) return;  // the dropped rows' run
  const int64_t s = key;
  const int L = A.map.n_lobes;
  const SmapRow d = agg[u];
  for (int q = 0; q < 9; ++q) A.map.Lambdas[9 * s + q] = A.map.Lambdas[9 * s + q] + d.v[q];
  for (int q = 0; q < 3; ++q) A.map.thetas[3 * s + q] = A.map.thetas[3 * s + q] + d.v[9 + q];
  // lobes > 0 receive 0.0 per row: x + 0.0 (as the fuse writes them)
  for (int q = 0; q < 3 * L; ++q)
    A.map.etas[(int64_t)3 * L * s + q] = A.map.etas[(int64_t)3 * L * s + q] + (q < 3 ? d.v[12 + q] : 0.0);
  A.map.weights[s] = A.map.weights[s] + d.v[15];
  A.map.timestamps[s] = A.timestamp;
  A.map.last_supported_scan_seq[s] = A.scan_seq;
  A.map.last_update_scan_seq[s] = A.scan_seq;
  if (A.map.lidar_mass) A.map.lidar_mass[s] = A.map.lidar_mass[s] + d.v[15];
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
  size_t t_sort = 0, t_red = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, t_sort, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                         (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n_cap, 0, W->bits,
                                         ctx->stream) != hipSuccess ||
      rocprim::deterministic_reduce_by_key(nullptr, t_red, (const uint32_t*)nullptr, (const SmapRow*)nullptr,
                                           (size_t)n_cap, (uint32_t*)nullptr, (SmapRow*)nullptr, (uint32_t*)nullptr,
                                           SmapRowSum(), rocprim::equal_to<uint32_t>(), ctx->stream) != hipSuccess) {
    set_error(ctx, "sort / reduce-by-key sizing failed");
    return GC_ERR_RUNTIME;
  }
  auto up = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t kv = up((size_t)n_cap * sizeof(uint32_t)), rv = up((size_t)n_cap * sizeof(SmapRow));
  const size_t bytes = 5 * kv + 3 * rv + 512 + up(t_sort) + up(t_red);
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
  W->unique = (uint32_t*)(base + 4 * kv);
  W->rows = (double*)(base + 5 * kv);
  W->srows = (double*)(base + 5 * kv + rv);
  W->agg = (double*)(base + 5 * kv + 2 * rv);
  W->count = (unsigned long long*)(base + 5 * kv + 3 * rv);
  W->n_runs = (uint32_t*)(base + 5 * kv + 3 * rv + 256);
  W->temp = base + 5 * kv + 3 * rv + 512;
  W->temp_bytes = up(t_sort);
  W->temp2 = (char*)W->temp + up(t_sort);
  W->temp2_bytes = up(t_red);
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
  const int64_t n = P.n_cap;
  const unsigned grid = (unsigned)((n + 255) / 256);
  GC_HIP(ctx, hipMemsetAsync(W->count, 0, sizeof(unsigned long long), st));
  hipLaunchKernelGGL(k_smap_rows, dim3(grid), dim3(256), 0, st, A, W->keys_in, W->vals_in, (SmapRow*)W->rows);
  GC_LAUNCH_CHECK(ctx);
  size_t t1 = W->temp_bytes, t2 = W->temp2_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(W->temp, t1, W->keys_in, W->keys, W->vals_in, W->vals, (int)n, 0, W->bits,
                                         st) != hipSuccess) {
    set_error(ctx, "radix sort failed");
    return GC_ERR_RUNTIME;
  }
  hipLaunchKernelGGL(k_smap_gather, dim3((unsigned)((n * kSmapRow + 255) / 256)), dim3(256), 0, st, n,
                     (const uint32_t*)W->vals, (const double*)W->rows, W->srows);
  GC_LAUNCH_CHECK(ctx);
  if (rocprim::deterministic_reduce_by_key(W->temp2, t2, (const uint32_t*)W->keys, (const SmapRow*)W->srows,
                                           (size_t)n, W->unique, (SmapRow*)W->agg, W->n_runs, SmapRowSum(),
                                           rocprim::equal_to<uint32_t>(), st) != hipSuccess) {
    set_error(ctx, "reduce-by-key failed");
    return GC_ERR_RUNTIME;
  }
  hipLaunchKernelGGL(k_smap_apply, dim3(grid), dim3(256), 0, st, A, (const uint32_t*)W->unique,
                     (const SmapRow*)W->agg, (const uint32_t*)W->n_runs, W->count);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

}  // namespace gc
