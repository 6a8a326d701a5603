// gc_map.hip — C5 map update: world pushforward of measurement primitives and the
// PrimitiveMap Product-of-Experts fuse (a13 C5 analogue).
//
//  transform_gaussian_to_world   backend/pipeline.py:1248-1256
//  primitive_map_fuse            backend/structures/primitive_map.py:992-1163
//
// The fuse is a reduce-by-key of K measurement rows into M map slots (gc_runs.h): each block of
// 1024 rows is sorted by (slot, row) in LDS and its runs registered in per-slot entries; one owner thread
// per distinct slot then sums the slot's rows in row order (runs in block order) and
// read-modify-writes the slot once. The per-slot sums are therefore formed in the same order as the
// reference's sequential scatter-add (bit-reproducible, no float atomics); nothing is staged in HBM
// (each row is read once, by its slot's owner) and a slot's record is touched exactly twice (read +
// write).
#include <hip/hip_runtime.h>
#include <vector>
#include "gc_internal.h"
#include "gc_math.h"
#include "gc_mapslot.h"
#include "gc_runs.h"

namespace gc {
namespace {

constexpr uint32_t kDropped = 0xFFFFFFFFu;

// the packed record's apply with the sort block's rows staged in LDS (k_fuse_apply_blk), or gathered
// from HBM by 128-position workgroups (k_fuse_apply)
#ifndef GC_FUSE_STAGED
#define GC_FUSE_STAGED 1
#endif

struct FuseArgs {
  gc_primitive_map map;
  gc_fuse_batch meas;
  double pose[6];  // world pose z_t = [t, rotvec] of the pushforward
  int world;       // apply transform_gaussian_to_world
  double eps_lift, eps_mass, timestamp;
  int64_t scan_seq;
  int rec32;  // the map is the packed record of gc_primitive_map_record_layout with 3 lobes (fuse_slot32)
  int col32;  // rgb (and colors) at their layout offsets: written as whole 32-B sectors (slot_colour32)
};

// One measurement row in the world frame (pipeline.py:1248-1256): Λ_w = R Λ Rᵀ,
// μ_b = (Λ + ε I)⁻¹ θ, μ_w = R μ_b + t, θ_w = Λ_w μ_w, η_w = R η (each lobe). Lb / tb / eb: the row's
// Λ (9), θ (3) and η (3L), in HBM or staged in LDS.
template <int LT>  // LT > 0: the lobe count at compile time (registers, no scratch); 0: A.map.n_lobes
GC_DEV void meas_world(const FuseArgs& A, const double* R, const double* Lb, const double* tb, const double* eb,
                       double* Lw, double* th, double* et) {
  const int L = LT > 0 ? LT : A.map.n_lobes;
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

// A measurement row's contribution, formed exactly as the reference forms it before its scatter-add
// (r * X, primitive_map.py:1074-1095): [r Λ_w 9 | r θ_w 3 | r η_w 3L | r w | r | w_cam | w_lidar |
// clip(c) w_cam 3]. The owner of a slot adds these rounded terms in row order, so the slot's sums are
// bit-identical to a sequential scatter-add of them. r = responsibility x (valid ? 1 : 0), src < 0:
// no source column, col: the row's colour or NULL.
__host__ __device__ constexpr int row_terms_len(int L) { return 19 + 3 * L; }
template <int LT>
GC_DEV void row_terms_at(const FuseArgs& A, const double* R, const double* Lb, const double* tb, const double* eb,
                         double r, double wm, int src, const double* col, double* o) {
#pragma clang fp contract(off)  // the products rounded as the reference's r * X
  constexpr int LM = LT > 0 ? LT : kMaxLobes;
  const int L = LT > 0 ? LT : A.map.n_lobes;
  double Lw[9], th[3], et[3 * LM];
  meas_world<LT>(A, R, Lb, tb, eb, Lw, th, et);
  for (int q = 0; q < 9; ++q) o[q] = r * Lw[q];
  for (int q = 0; q < 3; ++q) o[9 + q] = r * th[q];
  for (int q = 0; q < 3 * L; ++q) o[12 + q] = r * et[q];
  double* t = o + 12 + 3 * L;
  t[0] = r * wm;
  t[1] = r;
  double wc = 0.0, wl = 0.0, ca[3] = {0.0, 0.0, 0.0};
  if (src >= 0) {
    wc = r * wm * (src == 0 ? 1.0 : 0.0);
    wl = r * wm * (src == 1 ? 1.0 : 0.0);
    if (col)
      for (int q = 0; q < 3; ++q) ca[q] = clampd(col[q], 0.0, 1.0) * wc;
  }
  t[2] = wc;
  t[3] = wl;
  for (int q = 0; q < 3; ++q) t[4 + q] = ca[q];
}
GC_DEV double row_r(const FuseArgs& A, int64_t k) {
  return A.meas.responsibilities[k] * ((A.meas.valid_mask && !A.meas.valid_mask[k]) ? 0.0 : 1.0);
}
// row k read from HBM
template <int LT>
GC_DEV void row_terms(const FuseArgs& A, const double* R, int64_t k, double* o) {
  const int L = LT > 0 ? LT : A.map.n_lobes;
  const int src = A.meas.sources ? A.meas.sources[k] : -1;
  row_terms_at<LT>(A, R, A.meas.Lambdas + 9 * k, A.meas.thetas + 3 * k, A.meas.etas + (int64_t)3 * L * k,
                   row_r(A, k), A.meas.weights[k], src, A.meas.colors ? A.meas.colors + 3 * k : nullptr, o);
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

// ---- pass 1: per block of kFuseBlk rows (one per thread), the (slot, row) sort and the run entries
// (gc_runs.h). 512-row blocks: 256 workgroups for a 131k-row fuse; 1024-row blocks left half the CUs
// idle (C5 fuse 0.081 -> 0.065 ms, profiles/r04/probe_soft_assign_store_only_and_fuse512.txt). The
// sort keeps one key per thread in a register (reg_bitonic_sort): 0.062 -> 0.054 ms against the
// all-LDS network, 256- and 512-row blocks alike (profiles/r04/ab_fuse_regsort.txt)
#ifndef GC_FUSE_BLK
#define GC_FUSE_BLK 256
#endif
constexpr int kFuseBlk = GC_FUSE_BLK;
__global__ void __launch_bounds__(kFuseBlk) k_fuse_runs(const int32_t* __restrict__ target, int64_t K, int64_t M,
                                                   RunTable T, uint32_t* sslot, uint32_t* order,
                                                   uint32_t* run_len, uint32_t* rank) {
  __shared__ uint64_t a[kFuseBlk];
  const int64_t base = (int64_t)blockIdx.x * kFuseBlk;
  {
    const int i = threadIdx.x;
    const int64_t k = base + i;
    uint32_t key = kNoRun;  // padding past K sorts last
    if (k < K) {
      const int32_t sl = target[k];
      key = (sl >= 0 && (int64_t)sl < M) ? (uint32_t)sl : (uint32_t)M;  // out of range: dropped (JAX scatter)
    }
    const uint64_t x = reg_bitonic_sort<kFuseBlk>(((uint64_t)key << 32) | (uint32_t)i, a);
    a[i] = x;  // the sort ended with a barrier after its last read of a
    __syncthreads();
  }
  for (int i = threadIdx.x; i < kFuseBlk; i += blockDim.x) {
    const int64_t p = base + i;
    if (p >= K) break;
    const uint32_t key = (uint32_t)(a[i] >> 32);
    order[p] = (uint32_t)(base + (uint32_t)a[i]);
    sslot[p] = key;
    uint32_t rk = kNoRun;
    if ((int64_t)key < M && (i == 0 || (uint32_t)(a[i - 1] >> 32) != key)) {
      int len = 1;
      while (i + len < kFuseBlk && (uint32_t)(a[i + len] >> 32) == key) ++len;
      run_len[p] = (uint32_t)len;
      rk = register_run(T, key, (uint32_t)p);
    }
    rank[p] = rk;
  }
}

// ---- pass 2: the owner of each slot sums its rows in row order and read-modify-writes the slot
// generic layout (any lobe count, per-field or packed record)
template <int LT>
GC_DEV void fuse_apply_slot(const FuseArgs& A, int64_t s, const double* d) {
#pragma clang fp contract(off)
  const gc_primitive_map& m = A.map;
  const int L = LT > 0 ? LT : m.n_lobes;
  const double* t = d + 12 + 3 * L;  // [rw, r, w_cam, w_lidar, c w_cam 3]
  double* Ls = mLam(m, s);
  for (int q = 0; q < 9; ++q) Ls[q] = Ls[q] + d[q];
  double* ths = mTh(m, s);
  for (int q = 0; q < 3; ++q) ths[q] = ths[q] + d[9 + q];
  double* ets = mEta(m, s);
  for (int q = 0; q < 3 * L; ++q) ets[q] = ets[q] + d[12 + q];
  mW(m, s) = mW(m, s) + t[0];
  mTs(m, s) = A.timestamp;  // every targeted slot (primitive_map.py:1109)
  if (t[1] > 0.0) {
    mSup(m, s) = A.scan_seq;
    mUpd(m, s) = A.scan_seq;
  }
  if (m.cam_mass) {
    const bool src = A.meas.sources != nullptr, col = src && A.meas.colors;
    const double cam = mCam(m, s) + (src ? t[2] : 0.0), den = mDen(m, s) + (col ? t[2] : 0.0);
    const double* a0 = mAcc(m, s);
    const double acc[3] = {a0[0] + (col ? t[4] : 0.0), a0[1] + (col ? t[5] : 0.0), a0[2] + (col ? t[6] : 0.0)};
    mCam(m, s) = cam;
    mLid(m, s) = mLid(m, s) + (src ? t[3] : 0.0);
    double* as = mAcc(m, s);
    for (int q = 0; q < 3; ++q) as[q] = acc[q];
    mDen(m, s) = den;
    // untouched slots already hold their estimate (colors_current): only this slot's can change
    if (m.colors_current) slot_colour(m, s, cam, acc, den, A.eps_mass);
  }
}

// slot_colour for the packed record: rgb and colors each as one 32-B sector (the value and a pad
// double), whole sectors for the memory controller (gc_mapslot.h)
GC_DEV void slot_colour32(const gc_primitive_map& m, int64_t s, double cam, const double* acc, double denom,
                          double eps_mass) {
  typedef double dvec2 __attribute__((ext_vector_type(2)));
  const bool on = cam > 0.0;
  const double den = fmax(denom, eps_mass);
  double v[3];
  for (int q = 0; q < 3; ++q) v[q] = on ? clampd(acc[q] / den, 0.0, 1.0) : 0.5;
  dvec2* rgb = reinterpret_cast<dvec2*>(mRgb(m, s));
  rgb[0] = dvec2{v[0], v[1]};
  rgb[1] = dvec2{v[2], 0.0};
  if (m.colors) {
    dvec2* col = reinterpret_cast<dvec2*>(mCol(m, s));
    col[0] = dvec2{v[0], v[1]};
    col[1] = dvec2{v[2], 0.0};
  }
}

// The packed 3-lobe record (gc_mapslot.h): doubles [Λ 0-8 | θ 9-11 | w 12 | stamp 13 | supported seq 14 |
// update seq 15 | cam 16 | lidar 17 | accum 18-20 | denom 21 | η 22-30 | pad 31] in the record's first two
// lines, read and written as 16 16-B vectors (whole lines instead of 31 separate 8-B accesses).
// the record rec (its first two lines, loaded) updated with the row sums d and stored back
GC_DEV void fuse_apply_rec32(const FuseArgs& A, int64_t s, double* rec, const double* d) {
#pragma clang fp contract(off)
  typedef double dvec2 __attribute__((ext_vector_type(2)));
  const gc_primitive_map& m = A.map;
  dvec2* rp = reinterpret_cast<dvec2*>((char*)m.Lambdas + s * m.slot_bytes);
  // d: [r Λ 0-8 | r θ 9-11 | r η 12-20 | r w 21 | r 22 | w_cam 23 | w_lidar 24 | c w_cam 25-27]
  const bool src = A.meas.sources != nullptr, col = src && A.meas.colors;
#pragma unroll
  for (int q = 0; q < 12; ++q) rec[q] = rec[q] + d[q];                // Λ, θ
#pragma unroll
  for (int q = 0; q < 9; ++q) rec[22 + q] = rec[22 + q] + d[12 + q];  // η
  rec[12] = rec[12] + d[21];                                          // w
  rec[13] = A.timestamp;                                              // every targeted slot (primitive_map.py:1109)
  if (d[22] > 0.0) {
    rec[14] = __longlong_as_double((long long)A.scan_seq);
    rec[15] = __longlong_as_double((long long)A.scan_seq);
  }
  if (m.cam_mass) {
    rec[16] = rec[16] + (src ? d[23] : 0.0);
    rec[17] = rec[17] + (src ? d[24] : 0.0);
#pragma unroll
    for (int q = 0; q < 3; ++q) rec[18 + q] = rec[18 + q] + (col ? d[25 + q] : 0.0);
    rec[21] = rec[21] + (col ? d[23] : 0.0);
  }
#pragma unroll
  for (int v = 0; v < 16; ++v) rp[v] = dvec2{rec[2 * v], rec[2 * v + 1]};
  if (m.cam_mass && m.colors_current) {
    if (A.col32) slot_colour32(m, s, rec[16], rec + 18, rec[21], A.eps_mass);
    else slot_colour(m, s, rec[16], rec + 18, rec[21], A.eps_mass);
  }
}
GC_DEV void fuse_apply_slot32(const FuseArgs& A, int64_t s, const double* d) {
  typedef double dvec2 __attribute__((ext_vector_type(2)));
  const dvec2* rp = reinterpret_cast<const dvec2*>((const char*)A.map.Lambdas + s * A.map.slot_bytes);
  double rec[32];
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const dvec2 x = rp[v];
    rec[2 * v] = x.x;
    rec[2 * v + 1] = x.y;
  }
  fuse_apply_rec32(A, s, rec, d);
}

// one thread per sorted position; the owner of each slot (the run its list ends on) fuses the slot
template <int LT, bool R32>  // R32: the packed 3-lobe record (A.rec32)
__global__ void __launch_bounds__(kApplyWG) k_fuse_apply(FuseArgs A, int64_t K, RunTable T,
                                                    const uint32_t* __restrict__ sslot,
                                                    const uint32_t* __restrict__ order,
                                                    const uint32_t* __restrict__ run_len,
                                                    const uint32_t* __restrict__ rank,
                                                    uint32_t* wg_count) {
#pragma clang fp contract(off)
  constexpr int LM = LT > 0 ? LT : kMaxLobes;
  constexpr int NT = row_terms_len(LM);
  const int64_t wgid = xcd_block(blockIdx.x, gridDim.x);  // a sort block's workgroups on one XCD
  const int64_t p = wgid * blockDim.x + threadIdx.x;
  bool own = false;
  uint32_t s = 0;
  if (p < K) {
    s = sslot[p];
    own = (int64_t)s < A.map.m_slots && rank[p] != kNoRun;  // the slot's entry index for its owner
  }
  if (own) {
    const int L = LT > 0 ? LT : A.map.n_lobes;
    const int nt = row_terms_len(L);
    double R[9];
    if (A.world) so3_exp(A.pose + 3, R);
    double d[NT], t[NT];
    for (int q = 0; q < NT; ++q) d[q] = 0.0;
    const auto add_run = [&](uint32_t r) {  // a run's rows in row order
      const uint32_t len = run_len[r];
      for (uint32_t q = 0; q < len; ++q) {
        row_terms<LT>(A, R, (int64_t)order[r + q], t);
        for (int e = 0; e < nt; ++e) d[e] += t[e];
      }
    };
    __shared__ uint32_t slices[kApplyWG * kRunCap];
    SlotRunList<kRunCap> rl(slices + threadIdx.x * kRunCap);
    const uint32_t s1 = T.succ[p];
    if (s1 == 0u) {  // the slot's rows all lie in one block (the common case)
      add_run((uint32_t)p);
    } else {
      rl.collect((uint32_t)p, s1, T.succ, (int)((K + kFuseBlk - 1) / kFuseBlk));
      uint32_t prev = 0;
      for (int i = 0; i < rl.n; ++i) {  // runs in block order
        const uint32_t r = rl.at(i, prev);
        if (r == kNoRun) break;  // only a corrupt entry: never index past the runs
        prev = r;
        add_run(r);
      }
    }
    if constexpr (R32) fuse_apply_slot32(A, s, d);
    else fuse_apply_slot<LT>(A, s, d);
    if (s1 != 0u) rl.clear();
    T.e[rank[p]] = 0ull;  // the entry and the chain empty for the next call
  }
  // the distinct-slot count per workgroup (an LDS sum: one global counter for every wave serialised
  // the kernel's end)
  __shared__ uint32_t owned;
  if (threadIdx.x == 0) owned = 0u;
  __syncthreads();
  const unsigned long long b = __ballot(own);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(&owned, (uint32_t)__popcll(b));
  __syncthreads();
  if (threadIdx.x == 0) wg_count[blockIdx.x] = owned;
}

// The packed 3-lobe record's apply with the rows staged: one workgroup per sort block (kFuseBlk
// positions = the block's rows, sorted by slot), whose rows are first read into LDS as coalesced
// field slices, so each owner takes its own block's rows from LDS instead of gathering them from HBM in
// sorted (random) order: with 128-position workgroups a block's row lines were fetched by four
// workgroups beside every other block's slot records in the same L2 and re-read (k_fuse_apply read
// ~1.5x the rows' and records' bytes). Runs in other blocks (a slot hit by several blocks) are read from
// HBM. Every term is formed by row_terms_at in the same order: bit-identical to k_fuse_apply.
constexpr int kBlkRunCap = 8;  // a position's run slice (more runs: SlotRunList's walk over the chain)
constexpr int kStageDoubles = (9 + 3 + 9 + 1 + 1 + 3) * kFuseBlk;
constexpr size_t kStageLds = sizeof(double) * kStageDoubles + sizeof(int32_t) * kFuseBlk +
                             sizeof(uint32_t) * kFuseBlk * kBlkRunCap;
// one workgroup's dynamic LDS on gfx950 (160 KiB per CU, all of it addressable by one workgroup once
// ensure_dyn_lds raises the limit): ~62 KB at GC_FUSE_BLK=256, ~125 KB at 512
static_assert(kStageLds <= 160 * 1024, "the staged fuse apply's rows do not fit one workgroup's LDS");
__global__ void __launch_bounds__(kFuseBlk) k_fuse_apply_blk(FuseArgs A, int64_t K, RunTable T,
                                                         const uint32_t* __restrict__ sslot,
                                                         const uint32_t* __restrict__ order,
                                                         const uint32_t* __restrict__ run_len,
                                                         const uint32_t* __restrict__ rank, uint32_t* wg_count) {
#pragma clang fp contract(off)
  constexpr int L = 3, NT = row_terms_len(L), NB = kFuseBlk;
  extern __shared__ double stg[];
  double* sL = stg;            // Λ   NB x 9
  double* sT = sL + 9 * NB;    // θ   NB x 3
  double* sE = sT + 3 * NB;    // η   NB x 9
  double* sR = sE + 9 * NB;    // r (masked)
  double* sW = sR + NB;        // w
  double* sC = sW + NB;        // colour NB x 3
  int32_t* sS = reinterpret_cast<int32_t*>(sC + 3 * NB);             // source
  uint32_t* slices = reinterpret_cast<uint32_t*>(sS + NB);           // NB x kBlkRunCap
  __shared__ double Rs[9];
  __shared__ uint32_t owned;
  const int64_t base = (int64_t)blockIdx.x * NB;
  const int nrow = (int)min<int64_t>(NB, K - base);
  const int t = threadIdx.x;
  // the position's slot and, for its owner, the slot's record (the first two lines) and chain link,
  // loaded before the staging so the record's HBM round trip overlaps it
  const int64_t p = base + t;
  bool own = false;
  uint32_t s = 0, s1 = 0;
  typedef double dvec2 __attribute__((ext_vector_type(2)));
  dvec2 rv[16];
  if (p < K) {
    s = sslot[p];
    own = (int64_t)s < A.map.m_slots && rank[p] != kNoRun;
  }
  if (own) {
    const dvec2* rp = reinterpret_cast<const dvec2*>((const char*)A.map.Lambdas + (int64_t)s * A.map.slot_bytes);
#pragma unroll
    for (int v = 0; v < 16; ++v) rv[v] = rp[v];
    s1 = T.succ[p];
  }
  // the block's rows as coalesced field slices, every load of a thread in flight at once
  {
    double vL[9], vE[9], vT[3], vC[3];
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int i = t + j * NB;
      vL[j] = i < 9 * nrow ? A.meas.Lambdas[9 * base + i] : 0.0;
      vE[j] = i < 9 * nrow ? A.meas.etas[9 * base + i] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int i = t + j * NB;
      vT[j] = i < 3 * nrow ? A.meas.thetas[3 * base + i] : 0.0;
      vC[j] = (A.meas.colors && i < 3 * nrow) ? A.meas.colors[3 * base + i] : 0.0;
    }
    const bool in = t < nrow;
    const double vR = in ? row_r(A, base + t) : 0.0, vW = in ? A.meas.weights[base + t] : 0.0;
    const int32_t vS = (in && A.meas.sources) ? A.meas.sources[base + t] : -1;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      sL[t + j * NB] = vL[j];
      sE[t + j * NB] = vE[j];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      sT[t + j * NB] = vT[j];
      sC[t + j * NB] = vC[j];
    }
    sR[t] = vR;
    sW[t] = vW;
    sS[t] = vS;
  }
  if (t == 0) {
    owned = 0u;
    if (A.world) so3_exp(A.pose + 3, Rs);
  }
  // the run hash is not read past the runs pass (owners follow the position-indexed links): the
  // grid zeroes it for the next call in coalesced 16-B stores, whole lines instead of one 8-B store
  // per owner at a random entry (each a partial-sector write the memory controller reads back)
  {
    typedef unsigned long long u64v2 __attribute__((ext_vector_type(2)));
    const int64_t n2 = ((int64_t)1 << T.bits) / 2;
    u64v2* e2 = reinterpret_cast<u64v2*>(T.e);
    for (int64_t i = (int64_t)blockIdx.x * NB + t; i < n2; i += (int64_t)gridDim.x * NB) e2[i] = u64v2{0ull, 0ull};
  }
  __syncthreads();
  if (own) {
    double R[9];
    for (int q = 0; q < 9; ++q) R[q] = Rs[q];
    double d[NT], tt[NT];
    for (int q = 0; q < NT; ++q) d[q] = 0.0;
    const auto add_run = [&](uint32_t r) {  // a run's rows in row order
      const uint32_t len = run_len[r];
      for (uint32_t q = 0; q < len; ++q) {
        const int64_t k = (int64_t)order[r + q];
        const int64_t i = k - base;
        if (i >= 0 && i < NB)
          row_terms_at<L>(A, R, sL + 9 * i, sT + 3 * i, sE + 9 * i, sR[i], sW[i], sS[i],
                          A.meas.colors ? sC + 3 * i : nullptr, tt);
        else
          row_terms<L>(A, R, k, tt);
        for (int e = 0; e < NT; ++e) d[e] += tt[e];
      }
    };
    SlotRunList<kBlkRunCap> rl(slices + t * kBlkRunCap);
    if (s1 == 0u) {
      add_run((uint32_t)p);
    } else {
      rl.collect((uint32_t)p, s1, T.succ, (int)((K + NB - 1) / NB));
      uint32_t prev = 0;
      for (int i = 0; i < rl.n; ++i) {
        const uint32_t r = rl.at(i, prev);
        if (r == kNoRun) break;
        prev = r;
        add_run(r);
      }
    }
    double rec[32];
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      rec[2 * v] = rv[v].x;
      rec[2 * v + 1] = rv[v].y;
    }
    fuse_apply_rec32(A, s, rec, d);
    if (s1 != 0u) rl.clear();
  }
  const unsigned long long b = __ballot(own);
  if ((t & 63) == 0 && b) atomicAdd(&owned, (uint32_t)__popcll(b));
  __syncthreads();
  if (t == 0) wg_count[blockIdx.x] = owned;
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
  if (int rc_j = gc::join_side(ctx)) return rc_j;
  GC_CHECK_ARG(ctx, map && meas, "NULL map or measurement batch");
  GC_CHECK_ARG(ctx, map->m_slots > 0 && map->m_slots < (int64_t)kDropped, "m_slots out of range");
  GC_CHECK_ARG(ctx, map->n_lobes >= 1 && map->n_lobes <= kMaxLobes, "n_lobes must be in [1, 8]");
  {
    const char* lay_ = gc::map_layout_error(*map);
    GC_CHECK_ARG(ctx, lay_ == nullptr, lay_ ? lay_ : "");
  }
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
    A.col32 = ok && (const char*)map->rgb - b0 == off[11] && (!map->colors || (const char*)map->colors - b0 == off[12]);
  }
  A.timestamp = timestamp;
  A.scan_seq = scan_seq;
  // scratch: the sorted slot, row order, run length and owner's entry of every position, the apply
  // launch's per-workgroup distinct-slot counts (the run hash and its links are the context's)
  const size_t kv = ((size_t)K * sizeof(uint32_t) + 255) / 256 * 256;
  const bool staged = A.rec32 && GC_FUSE_STAGED;  // k_fuse_apply_blk: one workgroup per sort block
  const unsigned nblk = (unsigned)((K + kFuseBlk - 1) / kFuseBlk);
  const unsigned grid = staged ? nblk : (unsigned)((K + kApplyWG - 1) / kApplyWG);
  void* scr;
  if (int rc = gc::scratch(ctx, 4 * kv + (size_t)grid * sizeof(uint32_t), &scr)) return rc;
  char* base = (char*)scr;
  uint32_t* sslot = (uint32_t*)base;
  uint32_t* order = (uint32_t*)(base + kv);
  uint32_t* run_len = (uint32_t*)(base + 2 * kv);
  uint32_t* rank = (uint32_t*)(base + 3 * kv);
  uint32_t* cnt = (uint32_t*)(base + 4 * kv);
  if (int rc = gc::run_table(ctx, ctx->stream, &ctx->runs, K)) return rc;
  const RunTable T{ctx->runs.entries(), ctx->runs.succ(), ctx->runs.bits};
  // from here a failed launch may leave entries set: the next call empties them
  ctx->runs.dirty = true;
  hipLaunchKernelGGL(k_fuse_runs, dim3(nblk), dim3(kFuseBlk), 0, ctx->stream,
                     (const int32_t*)meas->target_slots, K, map->m_slots, T, sslot, order, run_len, rank);
  GC_LAUNCH_CHECK(ctx);
  const bool l3 = map->n_lobes == 3;  // GC_VMF_N_LOBES: the compile-time lobe count
  if (staged) {
    GC_HIP(ctx, gc::ensure_dyn_lds((const void*)k_fuse_apply_blk, kStageLds));
    hipLaunchKernelGGL(k_fuse_apply_blk, dim3(grid), dim3(kFuseBlk), kStageLds, ctx->stream, A, K, T, sslot, order,
                       run_len, rank, cnt);
  } else if (A.rec32)
    hipLaunchKernelGGL((k_fuse_apply<3, true>), dim3(grid), dim3(kApplyWG), 0, ctx->stream, A, K, T, sslot, order,
                       run_len, rank, cnt);
  else if (l3)
    hipLaunchKernelGGL((k_fuse_apply<3, false>), dim3(grid), dim3(kApplyWG), 0, ctx->stream, A, K, T, sslot, order,
                       run_len, rank, cnt);
  else
    hipLaunchKernelGGL((k_fuse_apply<0, false>), dim3(grid), dim3(kApplyWG), 0, ctx->stream, A, K, T, sslot, order,
                       run_len, rank, cnt);
  GC_LAUNCH_CHECK(ctx);
  ctx->runs.dirty = false;  // every entry the runs pass set, its owner cleared
  if (color && !map->colors_current) {
    hipLaunchKernelGGL(k_fuse_colors, dim3((unsigned)((map->m_slots + 255) / 256)), dim3(256), 0, ctx->stream, *map,
                       eps_mass);
    GC_LAUNCH_CHECK(ctx);
  }
  if (n_fused_out) {
    std::vector<uint32_t> c(grid);
    GC_HIP(ctx, hipMemcpyAsync(c.data(), cnt, c.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
    if (int rc_w = gc::wait_stream(ctx, ctx->stream, "the touched-slot counts")) return rc_w;
    int64_t n = 0;
    for (uint32_t v : c) n += v;
    *n_fused_out = n;
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
  if (int rc_j = gc::join_side(ctx)) return rc_j;
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
