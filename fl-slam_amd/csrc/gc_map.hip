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
#include "gc_mapslot.h"

namespace gc {
namespace {

constexpr uint32_t kDropped = 0xFFFFFFFFu;

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
  double eps_lift, eps_mass, timestamp;
  int64_t scan_seq;
  int rec32;  // the map is the packed record of gc_primitive_map_record_layout with 3 lobes (fuse_slot32)
};

// One measurement row in the world frame (pipeline.py:1248-1256): Λ_w = R Λ Rᵀ,
// μ_b = (Λ + ε I)⁻¹ θ, μ_w = R μ_b + t, θ_w = Λ_w μ_w, η_w = R η (each lobe).
template <int LT>  // LT > 0: the lobe count at compile time (registers, no scratch); 0: A.map.n_lobes
GC_DEV void meas_world(const FuseArgs& A, const double* R, int64_t k, double* Lw, double* th, double* et) {
  const int L = LT > 0 ? LT : A.map.n_lobes;
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

// A measurement row's contribution, staged in row order as one record of kStage(L) doubles:
// [r Λ_w 9 | r θ_w 3 | r η_w 3L | r w | r | w_cam | w_lidar | clip(c) w_cam 3]. These are exactly the
// products the reference forms before its scatter-add (r * X, primitive_map.py:1074-1095), so the
// segment sums below add the same rounded terms in the same row order (bit-identical to summing
// them in place). The records are 128-B aligned: a segment gathers each of its rows as whole lines
// instead of one partial line per field of the reference's per-field row arrays.
__host__ __device__ constexpr int stage_doubles(int L) { return (19 + 3 * L + 15) / 16 * 16; }

// key = slot, or M for a dropped row (sorts after every slot), so the radix sort needs only the
// bit width of M (21 bits for a 1M-slot map: 3 digit passes instead of 4); plus the staged row
// Rows leave through a wave-private LDS slab (row stride SD + 2), so the wave's 64 consecutive staged
// records go out as one contiguous block, 16 B per lane (whole-line stores; lane-private records of
// 8-B stores left partially written lines in the L2s: ~3.4x the staged bytes reached HBM).
template <int LT>
__global__ void __launch_bounds__(256) k_fuse_keys(FuseArgs A, int64_t K, uint32_t* keys, uint32_t* vals,
                                                   double* stage) {
#pragma clang fp contract(off)  // the products rounded as the reference's r * X
  typedef double dvec2 __attribute__((ext_vector_type(2)));
  extern __shared__ __attribute__((aligned(16))) double fk_lds[];
  constexpr int LM = LT > 0 ? LT : kMaxLobes;
  const int L = LT > 0 ? LT : A.map.n_lobes;
  const int SD = stage_doubles(L), RS = SD + 2;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double* slab = fk_lds + wv * 64 * RS;
  const int64_t k0 = (int64_t)blockIdx.x * blockDim.x + wv * 64;  // the wave's first row
  const int64_t k = k0 + lane;
  double* o = slab + lane * RS;
  for (int q = 0; q < SD; ++q) o[q] = 0.0;
  if (k < K) {
    const int64_t M = A.map.m_slots;
    const int32_t sl = A.meas.target_slots[k];
    const bool in = sl >= 0 && (int64_t)sl < M;
    keys[k] = in ? (uint32_t)sl : (uint32_t)M;  // out-of-range rows are dropped (JAX scatter)
    vals[k] = (uint32_t)k;
    if (in) {
      double R[9];
      if (A.world) so3_exp(A.pose + 3, R);
      const double r = A.meas.responsibilities[k] * ((A.meas.valid_mask && !A.meas.valid_mask[k]) ? 0.0 : 1.0);
      double Lw[9], th[3], et[3 * LM];
      meas_world<LT>(A, R, k, Lw, th, et);
      for (int q = 0; q < 9; ++q) o[q] = r * Lw[q];
      for (int q = 0; q < 3; ++q) o[9 + q] = r * th[q];
      for (int q = 0; q < 3 * L; ++q) o[12 + q] = r * et[q];
      double* t = o + 12 + 3 * L;
      const double wm = A.meas.weights[k];
      t[0] = r * wm;
      t[1] = r;
      double wc = 0.0, wl = 0.0, ca[3] = {0.0, 0.0, 0.0};
      if (A.meas.sources) {
        const int src = A.meas.sources[k];
        wc = r * wm * (src == 0 ? 1.0 : 0.0);
        wl = r * wm * (src == 1 ? 1.0 : 0.0);
        if (A.meas.colors)
          for (int q = 0; q < 3; ++q) ca[q] = clampd(A.meas.colors[3 * k + q], 0.0, 1.0) * wc;
      }
      t[2] = wc;
      t[3] = wl;
      for (int q = 0; q < 3; ++q) t[4 + q] = ca[q];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (k0 >= K) return;
  const int64_t rows = K - k0 < 64 ? K - k0 : 64;
  double* dst = stage + k0 * SD;
  for (int e = 2 * lane; e < rows * SD; e += 128) {  // SD is even: a pair never straddles two rows
    const int row = e / SD, col = e - row * SD;
    *reinterpret_cast<dvec2*>(dst + e) = *reinterpret_cast<const dvec2*>(slab + row * RS + col);
  }
}

// rgb of one slot from its camera accumulators (primitive_map.py:1090-1098): clip(accum / max(denom,
// ε), 0, 1) where cam_mass > 0, else gray; colors = rgb
GC_DEV void slot_colour(const gc_primitive_map& m, int64_t s, double cam, const double* acc, double denom,
                        double eps_mass) {
  const bool on = cam > 0.0;
  const double den = fmax(denom, eps_mass);
  double* rgb = mRgb(m, s);
  for (int q = 0; q < 3; ++q) {
    const double v = on ? clampd(acc[q] / den, 0.0, 1.0) : 0.5;
    rgb[q] = v;
    if (m.colors) mCol(m, s)[q] = v;
  }
}

// The packed 3-lobe record (gc_mapslot.h): doubles [Λ 0-8 | θ 9-11 | w 12 | stamp 13 | supported seq 14 |
// update seq 15 | cam 16 | lidar 17 | accum 18-20 | denom 21 | η 22-30 | pad 31] in the record's first two
// lines, read and written as 16 16-B vectors (whole lines instead of 31 separate 8-B accesses), and the
// staged rows (19 + 9 doubles) likewise.
GC_DEV void fuse_segment32(const FuseArgs& A, int64_t i, int64_t K, uint32_t key, const uint32_t* __restrict__ keys,
                           const uint32_t* __restrict__ vals, const double* __restrict__ stage) {
#pragma clang fp contract(off)
  typedef double dvec2 __attribute__((ext_vector_type(2)));
  const gc_primitive_map& m = A.map;
  const int64_t s = key;
  dvec2* rp = reinterpret_cast<dvec2*>((char*)m.Lambdas + s * m.slot_bytes);
  double rec[32];
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const dvec2 x = rp[v];
    rec[2 * v] = x.x;
    rec[2 * v + 1] = x.y;
  }
  double d[28];
#pragma unroll
  for (int q = 0; q < 28; ++q) d[q] = 0.0;
  const bool src = A.meas.sources != nullptr, col = src && A.meas.colors;
  double dacc[3] = {0.0, 0.0, 0.0}, dden = 0.0;
  for (int64_t j = i; j < K && keys[j] == key; ++j) {
    const dvec2* o = reinterpret_cast<const dvec2*>(stage + (int64_t)vals[j] * 32);
    double t[28];
#pragma unroll
    for (int v = 0; v < 14; ++v) {
      const dvec2 x = o[v];
      t[2 * v] = x.x;
      t[2 * v + 1] = x.y;
    }
    // staged: [r Λ 0-8 | r θ 9-11 | r η 12-20 | r w 21 | r 22 | w_cam 23 | w_lidar 24 | c w_cam 25-27]
#pragma unroll
    for (int q = 0; q < 28; ++q) d[q] += t[q];
    if (col) {
#pragma unroll
      for (int q = 0; q < 3; ++q) dacc[q] += t[25 + q];
      dden += t[23];
    }
  }
#pragma unroll
  for (int q = 0; q < 12; ++q) rec[q] = rec[q] + d[q];        // Λ, θ
#pragma unroll
  for (int q = 0; q < 9; ++q) rec[22 + q] = rec[22 + q] + d[12 + q];  // η
  rec[12] = rec[12] + d[21];                                   // w
  rec[13] = A.timestamp;                                       // every targeted slot (primitive_map.py:1109)
  if (d[22] > 0.0) {
    rec[14] = __longlong_as_double((long long)A.scan_seq);
    rec[15] = __longlong_as_double((long long)A.scan_seq);
  }
  if (m.cam_mass) {
    if (src) {
      rec[16] = rec[16] + d[23];
      rec[17] = rec[17] + d[24];
    } else {  // x + 0.0, as the generic path
      rec[16] = rec[16] + 0.0;
      rec[17] = rec[17] + 0.0;
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) rec[18 + q] = rec[18 + q] + dacc[q];
    rec[21] = rec[21] + dden;
  }
#pragma unroll
  for (int v = 0; v < 16; ++v) rp[v] = dvec2{rec[2 * v], rec[2 * v + 1]};
  if (m.cam_mass && m.colors_current) slot_colour(m, s, rec[16], rec + 18, rec[21], A.eps_mass);
}

// the segment of sorted rows starting at i (its head) summed in row order and applied to its slot
template <int LT>
GC_DEV void fuse_segment(const FuseArgs& A, int64_t i, int64_t K, uint32_t key, const uint32_t* __restrict__ keys,
                         const uint32_t* __restrict__ vals, const double* __restrict__ stage) {
#pragma clang fp contract(off)
  constexpr int LM = LT > 0 ? LT : kMaxLobes;
  const gc_primitive_map& m = A.map;
  const int L = LT > 0 ? LT : m.n_lobes;
  const int64_t s = key;
  // the slot's current values are loaded first: they do not depend on the rows, so their latency
  // overlaps the row gathers (one dependent memory round trip fewer per slot)
  double mL[9], mth[3], met[3 * LM], mw, mcam = 0.0, mlid = 0.0, macc[3] = {0, 0, 0}, mden = 0.0;
  const double* Ls0 = mLam(m, s);
  const double* th0 = mTh(m, s);
  const double* et0 = mEta(m, s);
  for (int q = 0; q < 9; ++q) mL[q] = Ls0[q];
  for (int q = 0; q < 3; ++q) mth[q] = th0[q];
  for (int q = 0; q < 3 * L; ++q) met[q] = et0[q];
  mw = mW(m, s);
  if (m.cam_mass) {
    mcam = mCam(m, s);
    mlid = mLid(m, s);
    const double* a0 = mAcc(m, s);
    for (int q = 0; q < 3; ++q) macc[q] = a0[q];
    mden = mDen(m, s);
  }
  double dL[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, dth[3] = {0, 0, 0}, det[3 * LM], dw = 0.0, dr = 0.0;
  double dcam = 0.0, dlid = 0.0, dacc[3] = {0, 0, 0}, dden = 0.0;
  for (int q = 0; q < 3 * L; ++q) det[q] = 0.0;
  const bool col = A.meas.sources && A.meas.colors;  // colour accumulators only with colours (:1079-1083)
  const int SD = stage_doubles(L);
  for (int64_t j = i; j < K && keys[j] == key; ++j) {
    const double* o = stage + (int64_t)vals[j] * SD;
    for (int q = 0; q < 9; ++q) dL[q] += o[q];
    for (int q = 0; q < 3; ++q) dth[q] += o[9 + q];
    for (int q = 0; q < 3 * L; ++q) det[q] += o[12 + q];
    const double* t = o + 12 + 3 * L;
    dw += t[0];
    dr += t[1];
    if (A.meas.sources) {
      dcam += t[2];
      dlid += t[3];
      if (col) {
        for (int q = 0; q < 3; ++q) dacc[q] += t[4 + q];
        dden += t[2];
      }
    }
  }
  double* Ls = mLam(m, s);
  for (int q = 0; q < 9; ++q) Ls[q] = mL[q] + dL[q];
  double* ths = mTh(m, s);
  for (int q = 0; q < 3; ++q) ths[q] = mth[q] + dth[q];
  double* ets = mEta(m, s);
  for (int q = 0; q < 3 * L; ++q) ets[q] = met[q] + det[q];
  mW(m, s) = mw + dw;
  mTs(m, s) = A.timestamp;  // every targeted slot (primitive_map.py:1109)
  if (dr > 0.0) {
    mSup(m, s) = A.scan_seq;
    mUpd(m, s) = A.scan_seq;
  }
  if (m.cam_mass) {
    const double cam = mcam + dcam, den = mden + dden;
    const double acc[3] = {macc[0] + dacc[0], macc[1] + dacc[1], macc[2] + dacc[2]};
    mCam(m, s) = cam;
    mLid(m, s) = mlid + dlid;
    double* as = mAcc(m, s);
    for (int q = 0; q < 3; ++q) as[q] = acc[q];
    mDen(m, s) = den;
    // untouched slots already hold their estimate (colors_current): only this slot's can change
    if (m.colors_current) slot_colour(m, s, cam, acc, den, A.eps_mass);
  }
}

// one thread per sorted row; the head of each slot's segment fuses it
template <int LT, bool R32>  // R32: the packed 3-lobe record (A.rec32, fuse_segment32)
__global__ void __launch_bounds__(256) k_fuse_segments(FuseArgs A, int64_t K, const uint32_t* __restrict__ keys,
                                                       const uint32_t* __restrict__ vals,
                                                       const double* __restrict__ stage,
                                                       unsigned long long* n_unique) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t key = i < K ? keys[i] : 0u;
  // in range, and not a dropped row or the continuation of a segment
  const bool head = i < K && (int64_t)key < A.map.m_slots && (i == 0 || keys[i - 1] != key);
  if (head) {
    if constexpr (R32) fuse_segment32(A, i, K, key, keys, vals, stage);
    else fuse_segment<LT>(A, i, K, key, keys, vals, stage);
  }
  const unsigned long long b = __ballot(head);  // the distinct-slot count, one atomic per wave
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(n_unique, (unsigned long long)__popcll(b));
}

// every slot's colour estimate (primitive_map.py:1090-1098)
__global__ void k_fuse_colors(gc_primitive_map m, double eps_mass) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= m.m_slots) return;
  slot_colour(m, s, mCam(m, s), mAcc(m, s), mDen(m, s), eps_mass);
}

// rows x elem bytes between pitched buffers, one thread per 8-byte word (or per byte when the
// element, pitches or pointers are not 8-byte multiples)
template <class W>
__global__ void k_copy_strided(char* dst, int64_t dp, const char* __restrict__ src, int64_t sp, int64_t words,
                               int64_t rows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * words) return;
  const int64_t r = i / words, w = i - r * words;
  *(W*)(dst + r * dp + w * (int64_t)sizeof(W)) = *(const W*)(src + r * sp + w * (int64_t)sizeof(W));
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
  GC_CHECK_ARG(ctx, map->slot_bytes == 0 || (map->slot_bytes % 8 == 0 && map->slot_bytes >= 176 + 24 * map->n_lobes),
               "slot_bytes must be 0 (per-field arrays) or a packed record size");
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
  A.eps_mass = eps_mass;
  {  // the 3-lobe packed record, every field where gc_primitive_map_record_layout puts it
    int64_t off[gc::kRecFields], sb = 0;
    gc::map_record_layout(3, off, &sb);
    const char* b0 = (const char*)map->Lambdas;
    const void* f[gc::kRecFields] = {map->Lambdas, map->thetas, map->etas, map->weights, map->timestamps,
                                     map->last_supported_scan_seq, map->last_update_scan_seq, map->cam_mass,
                                     map->lidar_mass, map->rgb_cam_accum, map->rgb_cam_denom, map->rgb,
                                     map->colors, map->valid_mask, map->created_timestamps, map->primitive_ids};
    bool ok = map->n_lobes == 3 && map->slot_bytes == sb && ((uintptr_t)b0 % 16) == 0;
    for (int q = 0; q < 7 && ok; ++q) ok = (const char*)f[q] - b0 == off[q];  // the fuse's fields
    for (int q = 7; q < 11 && ok; ++q) ok = f[q] == nullptr || (const char*)f[q] - b0 == off[q];
    A.rec32 = ok ? 1 : 0;
  }
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
  const size_t sv = (size_t)K * stage_doubles(map->n_lobes) * sizeof(double);
  void* scr;
  if (int rc = gc::scratch(ctx, sv + 4 * kv + 256 + temp, &scr)) return rc;
  double* stage = (double*)scr;  // first: the scratch base is 256-B aligned, so every staged row is 128-B aligned
  char* base = (char*)scr + sv;
  uint32_t* keys_in = (uint32_t*)base;
  uint32_t* vals_in = (uint32_t*)(base + kv);
  uint32_t* keys = (uint32_t*)(base + 2 * kv);
  uint32_t* vals = (uint32_t*)(base + 3 * kv);
  unsigned long long* cnt = (unsigned long long*)(base + 4 * kv);
  void* tmp = base + 4 * kv + 256;
  const unsigned grid = (unsigned)((K + 255) / 256);
  GC_HIP(ctx, hipMemsetAsync(cnt, 0, sizeof(unsigned long long), ctx->stream));
  const size_t lds_keys = sizeof(double) * 4 * 64 * (stage_doubles(map->n_lobes) + 2);
  const bool l3 = map->n_lobes == 3;  // GC_VMF_N_LOBES: the compile-time lobe count
  const void* fk = l3 ? (const void*)k_fuse_keys<3> : (const void*)k_fuse_keys<0>;
  GC_HIP(ctx, gc::ensure_dyn_lds(fk, lds_keys));
  if (l3)
    hipLaunchKernelGGL(k_fuse_keys<3>, dim3(grid), dim3(256), lds_keys, ctx->stream, A, K, keys_in, vals_in, stage);
  else
    hipLaunchKernelGGL(k_fuse_keys<0>, dim3(grid), dim3(256), lds_keys, ctx->stream, A, K, keys_in, vals_in, stage);
  GC_LAUNCH_CHECK(ctx);
  if (hipcub::DeviceRadixSort::SortPairs(tmp, temp, keys_in, keys, vals_in, vals, (int)K, 0, key_bits(map->m_slots),
                                         ctx->stream) != hipSuccess) {
    gc::set_error(ctx, "radix sort failed");
    return GC_ERR_RUNTIME;
  }
  if (A.rec32)
    hipLaunchKernelGGL((k_fuse_segments<3, true>), dim3(grid), dim3(256), 0, ctx->stream, A, K, keys, vals,
                       (const double*)stage, cnt);
  else if (l3)
    hipLaunchKernelGGL((k_fuse_segments<3, false>), dim3(grid), dim3(256), 0, ctx->stream, A, K, keys, vals,
                       (const double*)stage, cnt);
  else
    hipLaunchKernelGGL((k_fuse_segments<0, false>), dim3(grid), dim3(256), 0, ctx->stream, A, K, keys, vals,
                       (const double*)stage, cnt);
  GC_LAUNCH_CHECK(ctx);
  if (color && !map->colors_current) {
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

int32_t gc_primitive_map_record_layout(int32_t n_lobes, int64_t* offsets_out, int64_t* slot_bytes_out) {
  GC_CHECK_ARG(nullptr, n_lobes >= 1 && n_lobes <= kMaxLobes, "n_lobes must be in [1, 8]");
  GC_CHECK_ARG(nullptr, offsets_out && slot_bytes_out, "NULL output");
  gc::map_record_layout(n_lobes, offsets_out, slot_bytes_out);
  return GC_OK;
}

int32_t gc_copy_strided(gc_ctx* ctx, void* d_dst, int64_t dst_pitch, const void* d_src, int64_t src_pitch,
                        int64_t elem_bytes, int64_t rows) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, elem_bytes >= 1 && rows >= 0 && dst_pitch >= elem_bytes && src_pitch >= elem_bytes,
               "bad element size, pitch or row count");
  if (rows == 0) return GC_OK;
  GC_CHECK_ARG(ctx, d_dst && d_src, "NULL buffer");
  const bool w8 = elem_bytes % 8 == 0 && dst_pitch % 8 == 0 && src_pitch % 8 == 0 && (uintptr_t)d_dst % 8 == 0 &&
                  (uintptr_t)d_src % 8 == 0;
  const int64_t words = w8 ? elem_bytes / 8 : elem_bytes;
  const unsigned grid = (unsigned)((rows * words + 255) / 256);
  if (w8)
    hipLaunchKernelGGL(k_copy_strided<uint64_t>, dim3(grid), dim3(256), 0, ctx->stream, (char*)d_dst, dst_pitch,
                       (const char*)d_src, src_pitch, words, rows);
  else
    hipLaunchKernelGGL(k_copy_strided<uint8_t>, dim3(grid), dim3(256), 0, ctx->stream, (char*)d_dst, dst_pitch,
                       (const char*)d_src, src_pitch, words, rows);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

}  // extern "C"
