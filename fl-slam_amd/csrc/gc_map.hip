// gc_map.hip — C5 map update: world pushforward of measurement primitives and the
// PrimitiveMap Product-of-Experts fuse (a13 C5 analogue).
//
//  transform_gaussian_to_world   backend/pipeline.py:1248-1256
//  primitive_map_fuse            backend/structures/primitive_map.py:992-1163
//
// The fuse is a reduce-by-key of K measurement rows into M map slots. Rows are ordered by
// (slot, row) with a stable radix sort; one thread per distinct slot then sums its rows in row
// order and read-modify-writes the slot once. The per-slot sums are therefore formed in the same
// order as the reference's sequential scatter-add (bit-reproducible, no float atomics), and a
// slot's 176 B core record (Λ 9, θ 3, η 9, w 1) is touched exactly twice (read + write).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include "gc_internal.h"
#include "gc_math.h"

namespace gc {
namespace {

constexpr uint32_t kDropped = 0xFFFFFFFFu;

// key = slot, or M for a dropped row (sorts after every slot), so the radix sort needs only the
// bit width of M (21 bits for a 1M-slot map: 3 digit passes instead of 4)
__global__ void k_fuse_keys(int64_t K, int64_t M, const int32_t* __restrict__ slots, uint32_t* keys, uint32_t* vals) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const int32_t s = slots[k];
  keys[k] = (s >= 0 && (int64_t)s < M) ? (uint32_t)s : (uint32_t)M;  // out-of-range rows are dropped (JAX scatter)
  vals[k] = (uint32_t)k;
}

inline int key_bits(int64_t M) {  // bits of the largest key, M
  int b = 1;
  while (b < 32 && (M >> b) != 0) ++b;
  return b;
}

struct FuseArgs {
  gc_primitive_map map;
  gc_fuse_batch meas;
  double pose[6];  // world pose z_t = [t, rotvec] of the pushforward
  int world;       // apply transform_gaussian_to_world
  double eps_lift, timestamp;
  int64_t scan_seq;
};

// One measurement row in the world frame (pipeline.py:1248-1256): Λ_w = R Λ Rᵀ,
// μ_b = (Λ + ε I)⁻¹ θ, μ_w = R μ_b + t, θ_w = Λ_w μ_w, η_w = R η (each lobe).
GC_DEV void meas_world(const FuseArgs& A, const double* R, int64_t k, int L, double* Lw, double* th, double* et) {
  const double* Lb = A.meas.Lambdas + 9 * k;
  const double* tb = A.meas.thetas + 3 * k;
  const double* eb = A.meas.etas + (int64_t)3 * L * k;
  if (!A.world) {
    for (int q = 0; q < 9; ++q) Lw[q] = Lb[q];
    for (int q = 0; q < 3; ++q) th[q] = tb[q];
    for (int q = 0; q < 3 * L; ++q) et[q] = eb[q];
    return;
  }
  double M3[9], Lr[9], mu[3], mw[3];
  mat3_mul(R, Lb, M3);
  mat3_mul_nt(M3, R, Lw);
  for (int q = 0; q < 9; ++q) Lr[q] = Lb[q] + ((q % 4 == 0) ? A.eps_lift : 0.0);
  solve3(Lr, tb, mu);
  mat3_vec(R, mu, mw);
  for (int q = 0; q < 3; ++q) mw[q] += A.pose[q];
  mat3_vec(Lw, mw, th);
  for (int l = 0; l < L; ++l) mat3_vec(R, eb + 3 * l, et + 3 * l);
}

constexpr int kMaxLobes = 8;

__global__ void __launch_bounds__(256) k_fuse_segments(FuseArgs A, int64_t K, const uint32_t* __restrict__ keys,
                                                       const uint32_t* __restrict__ vals, unsigned long long* n_unique) {
#pragma clang fp contract(off)  // products rounded before the sums, as the reference's r * X then add
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K) return;
  const uint32_t key = keys[i];
  if ((int64_t)key >= A.map.m_slots || (i > 0 && keys[i - 1] == key)) return;  // dropped, or not a segment head
  const int L = A.map.n_lobes;
  const int64_t s = key;
  // the slot's current values are loaded first: they do not depend on the rows, so their latency
  // overlaps the row gathers (one dependent memory round trip fewer per slot)
  double mL[9], mth[3], met[3 * kMaxLobes], mw, mcam = 0.0, mlid = 0.0, macc[3] = {0, 0, 0}, mden = 0.0;
  for (int q = 0; q < 9; ++q) mL[q] = A.map.Lambdas[9 * s + q];
  for (int q = 0; q < 3; ++q) mth[q] = A.map.thetas[3 * s + q];
  for (int q = 0; q < 3 * L; ++q) met[q] = A.map.etas[(int64_t)3 * L * s + q];
  mw = A.map.weights[s];
  if (A.map.cam_mass) {
    mcam = A.map.cam_mass[s];
    mlid = A.map.lidar_mass[s];
    for (int q = 0; q < 3; ++q) macc[q] = A.map.rgb_cam_accum[3 * s + q];
    mden = A.map.rgb_cam_denom[s];
  }
  double dL[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, dth[3] = {0, 0, 0}, det[3 * kMaxLobes], dw = 0.0, dr = 0.0;
  double dcam = 0.0, dlid = 0.0, dacc[3] = {0, 0, 0}, dden = 0.0;
  for (int q = 0; q < 3 * L; ++q) det[q] = 0.0;
  double R[9];
  if (A.world) so3_exp(A.pose + 3, R);
  for (int64_t j = i; j < K && keys[j] == key; ++j) {
    const int64_t k = vals[j];
    const double r = A.meas.responsibilities[k] * ((A.meas.valid_mask && !A.meas.valid_mask[k]) ? 0.0 : 1.0);
    double Lw[9], th[3], et[3 * kMaxLobes];
    meas_world(A, R, k, L, Lw, th, et);
    for (int q = 0; q < 9; ++q) dL[q] += r * Lw[q];
    for (int q = 0; q < 3; ++q) dth[q] += r * th[q];
    for (int q = 0; q < 3 * L; ++q) det[q] += r * et[q];
    const double wm = A.meas.weights[k];
    dw += r * wm;
    dr += r;
    if (A.meas.sources) {
      const int src = A.meas.sources[k];
      const double wc = r * wm * (src == 0 ? 1.0 : 0.0), wl = r * wm * (src == 1 ? 1.0 : 0.0);
      dcam += wc;
      dlid += wl;
      if (A.meas.colors) {  // colour accumulators only with colours (primitive_map.py:1079-1083)
        for (int q = 0; q < 3; ++q) dacc[q] += clampd(A.meas.colors[3 * k + q], 0.0, 1.0) * wc;
        dden += wc;
      }
    }
  }
  double* Ls = A.map.Lambdas + 9 * s;
  for (int q = 0; q < 9; ++q) Ls[q] = mL[q] + dL[q];
  for (int q = 0; q < 3; ++q) A.map.thetas[3 * s + q] = mth[q] + dth[q];
  for (int q = 0; q < 3 * L; ++q) A.map.etas[(int64_t)3 * L * s + q] = met[q] + det[q];
  A.map.weights[s] = mw + dw;
  A.map.timestamps[s] = A.timestamp;  // every targeted slot (primitive_map.py:1109)
  if (dr > 0.0) {
    A.map.last_supported_scan_seq[s] = A.scan_seq;
    A.map.last_update_scan_seq[s] = A.scan_seq;
  }
  if (A.map.cam_mass) {
    A.map.cam_mass[s] = mcam + dcam;
    A.map.lidar_mass[s] = mlid + dlid;
    for (int q = 0; q < 3; ++q) A.map.rgb_cam_accum[3 * s + q] = macc[q] + dacc[q];
    A.map.rgb_cam_denom[s] = mden + dden;
  }
  atomicAdd(n_unique, 1ull);  // integer count: order-independent
}

// rgb = clip(accum / max(denom, ε), 0, 1) where cam_mass > 0 else gray; colors = rgb (all slots,
// primitive_map.py:1090-1098).
__global__ void k_fuse_colors(gc_primitive_map map, double eps_mass) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= map.m_slots) return;
  const bool cam = map.cam_mass[s] > 0.0;
  const double den = fmax(map.rgb_cam_denom[s], eps_mass);
  for (int q = 0; q < 3; ++q) {
    const double v = cam ? clampd(map.rgb_cam_accum[3 * s + q] / den, 0.0, 1.0) : 0.5;
    map.rgb[3 * s + q] = v;
    if (map.colors) map.colors[3 * s + q] = v;
  }
}

}  // namespace

// the all-slot colour estimate (rgb, colors) of primitive_map_fuse, for the in-scan update
hipError_t launch_fuse_colors(const gc_primitive_map& map, double eps_mass, hipStream_t st) {
  hipLaunchKernelGGL(k_fuse_colors, dim3((unsigned)((map.m_slots + 255) / 256)), dim3(256), 0, st, map, eps_mass);
  return hipGetLastError();
}
}  // namespace gc

using namespace gc;

extern "C" {

int32_t gc_primitive_map_fuse(gc_ctx* ctx, const gc_primitive_map* map, const gc_fuse_batch* meas,
                              const double* h_pose6, double eps_lift, double eps_mass, double timestamp,
                              int64_t scan_seq, int64_t* n_fused_out) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, map && meas, "NULL map or measurement batch");
  GC_CHECK_ARG(ctx, map->m_slots > 0 && map->m_slots < (int64_t)kDropped, "m_slots out of range");
  GC_CHECK_ARG(ctx, map->n_lobes >= 1 && map->n_lobes <= kMaxLobes, "n_lobes must be in [1, 8]");
  GC_CHECK_ARG(ctx, map->Lambdas && map->thetas && map->etas && map->weights && map->timestamps &&
                        map->last_supported_scan_seq && map->last_update_scan_seq,
               "NULL map field");
  const bool color = map->cam_mass != nullptr;
  GC_CHECK_ARG(ctx, !color || (map->lidar_mass && map->rgb_cam_accum && map->rgb_cam_denom && map->rgb),
               "colour fields must be all set or all NULL");
  GC_CHECK_ARG(ctx, meas->K >= 0 && meas->K < (int64_t)kDropped, "K out of range");
  if (n_fused_out) *n_fused_out = 0;
  const int64_t K = meas->K;
  if (K == 0) return GC_OK;  // exact no-op (primitive_map.py:1031-1039)
  GC_CHECK_ARG(ctx, meas->target_slots && meas->Lambdas && meas->thetas && meas->etas && meas->weights &&
                        meas->responsibilities,
               "NULL measurement field");
  FuseArgs A{};
  A.map = *map;
  A.meas = *meas;
  A.world = h_pose6 != nullptr;
  if (A.world)
    for (int q = 0; q < 6; ++q) A.pose[q] = h_pose6[q];
  A.eps_lift = eps_lift;
  A.timestamp = timestamp;
  A.scan_seq = scan_seq;
  // scratch: keys/vals in+out, the unique counter and the radix-sort temp storage
  size_t temp = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                         (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)K, 0,
                                         key_bits(map->m_slots), ctx->stream) != hipSuccess) {
    gc::set_error(ctx, "radix sort sizing failed");
    return GC_ERR_RUNTIME;
  }
  const size_t kv = ((size_t)K * sizeof(uint32_t) + 255) / 256 * 256;
  void* scr;
  if (int rc = gc::scratch(ctx, 4 * kv + 256 + temp, &scr)) return rc;
  char* base = (char*)scr;
  uint32_t* keys_in = (uint32_t*)base;
  uint32_t* vals_in = (uint32_t*)(base + kv);
  uint32_t* keys = (uint32_t*)(base + 2 * kv);
  uint32_t* vals = (uint32_t*)(base + 3 * kv);
  unsigned long long* cnt = (unsigned long long*)(base + 4 * kv);
  void* tmp = base + 4 * kv + 256;
  const unsigned grid = (unsigned)((K + 255) / 256);
  GC_HIP(ctx, hipMemsetAsync(cnt, 0, sizeof(unsigned long long), ctx->stream));
  hipLaunchKernelGGL(k_fuse_keys, dim3(grid), dim3(256), 0, ctx->stream, K, map->m_slots, meas->target_slots, keys_in,
                     vals_in);
  GC_LAUNCH_CHECK(ctx);
  if (hipcub::DeviceRadixSort::SortPairs(tmp, temp, keys_in, keys, vals_in, vals, (int)K, 0, key_bits(map->m_slots),
                                         ctx->stream) != hipSuccess) {
    gc::set_error(ctx, "radix sort failed");
    return GC_ERR_RUNTIME;
  }
  hipLaunchKernelGGL(k_fuse_segments, dim3(grid), dim3(256), 0, ctx->stream, A, K, keys, vals, cnt);
  GC_LAUNCH_CHECK(ctx);
  if (color) {
    hipLaunchKernelGGL(k_fuse_colors, dim3((unsigned)((map->m_slots + 255) / 256)), dim3(256), 0, ctx->stream, *map,
                       eps_mass);
    GC_LAUNCH_CHECK(ctx);
  }
  if (n_fused_out) {
    unsigned long long n = 0;
    GC_HIP(ctx, hipMemcpyAsync(&n, cnt, sizeof(n), hipMemcpyDeviceToHost, ctx->stream));
    GC_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *n_fused_out = (int64_t)n;
  }
  return GC_OK;
}

}  // extern "C"
