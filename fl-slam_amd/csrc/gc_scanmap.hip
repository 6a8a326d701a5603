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
// with Σ_lidar the measurement-IW LiDAR block's mode Ψ_2 / (ν_2 + 4) of the IW state the scan started
// from (before its own measurement-IW apply, as the reference's step 12b reads the scan's config) and the
// row's weight the
// deskewed point weight (a4). Its slot is the spatial hash of the world voxel of μ_w. The rows are
// fused with responsibility 1 and source LiDAR by a deterministic reduce-by-key (gc_runs.h): each
// 256-row block sorts its rows by slot in LDS and sums every run of one slot by a segmented scan
// (k_smap_block), the runs are registered per slot, and one owner thread per distinct slot sums its runs
// in block order and applies the sum (k_smap_apply): bit-reproducible, within 1e-12 of np.add.at's
// sequential order. A scan's points crowd into few voxels
// (~65k rows into ~5k slots, runs of thousands near the sensor), so rows are computed one per
// thread and the runs reduced in parallel: one thread per run summing its rows serially took
// ~1 ms per scan. LiDAR rows leave the camera accumulators unchanged,
// so the all-slot colour recompute (colors = rgb) runs only when the colours are stale: on the first
// update after the map is attached, and after a host operation wrote colour fields (an insert, a
// merge, a colour upload: gc_pipeline_map_colors_stale; gc_pipeline.cpp).
//
// Every rank runs the update from the reduced record, so the maps stay bit-identical across ranks.
#include <hip/hip_runtime.h>
#include <vector>
#include "gc_internal.h"
#include "gc_math.h"
#include "gc_mapslot.h"
#include "gc_pipe.h"
#include "gc_runs.h"
#include "gc_scanmap.h"

namespace gc {
namespace {

struct ScanMapArgs {
  gc_primitive_map map;
  const double *pts, *t, *w;  // the scan slot's raw points, times and weights
  const double* bscal;        // the scan's a1 budget scalars       } the scan's snapshot
  const double* h0;           // reduced record: [z_t 6, Σ_pose 36, ξ 6] of hypothesis 0 } (PipeDev::smap_snap,
  const double* lidar_iw;     // [ν_2, Ψ_2] before the scan's measurement-IW apply     } k_combine_final)
  int64_t n_cap;
  double t0, t1, o0, o1, o2, voxel, timestamp, eps_mass, eps_psd;
  int64_t scan_seq;
};

constexpr int kSmapRow = 16;  // [Λ_w 9, θ_w 3, η_w lobe 0 3, w]
struct SmapRow {
  double v[kSmapRow];
};

// the row's deskewed body point and weight (false: padding or zero weight -> dropped)
GC_DEV bool smap_point(const ScanMapArgs& A, int64_t j, double* p0, double* w) {
  const int64_t n_sel = (int64_t)A.bscal[5], stride = (int64_t)A.bscal[6];
  if (j >= n_sel || j >= A.n_cap) return false;
  const int64_t i = j * stride;
  const double p[3] = {A.pts[3 * i], A.pts[3 * i + 1], A.pts[3 * i + 2]};
  const double alpha = (A.t[i] - A.t0) / fmax(A.t1 - A.t0, 1e-12);
  deskew_point(p, alpha, A.h0 + 42, p0);
  // the point's w x time window as the predict launch forms it (window_points, gc_belief.hip), then
  // the budget's mass scale: from the slot, so the update reads nothing the next scan rewrites
  const double denom = fmax(A.t1 - A.t0, 1e-12);
  *w = (A.w[i] * window_weight(A.t[i], A.t0, A.t1, 0.1 * denom)) * A.bscal[2];
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
  // a power-of-two slot count (the C5 map's 2^20) takes the mask: the same key without the 64-bit
  // software division
  return (uint32_t)(((uint64_t)M & ((uint64_t)M - 1)) == 0 ? (h & ((uint64_t)M - 1)) : h % (uint64_t)M);
}

GC_DEV void smap_pose(const ScanMapArgs& A, double* R, double* tt) {
  so3_exp(A.h0 + 3, R);
  tt[0] = A.h0[0]; tt[1] = A.h0[1]; tt[2] = 0.0;  // planar map: t_z = 0 (CHANGELOG.md:575-578)
}

// One world row (the comment at the top), in the body frame first: with K = [p]× and the pose
// covariance blocks A = [[A_tt, A_tr], [A_rt, A_rr]], J Σ_pose Jᵀ = R M Rᵀ with
// M = A_tt + A_tr K − K A_rt − K A_rr K (J = R [I | −K], Kᵀ = −K), so Σ_w = R (Σ_lidar + M) Rᵀ,
// Λ_w = R (Σ_lidar + M)⁻¹ Rᵀ and θ_w = Λ_w μ_w = R (Σ_lidar + M)⁻¹ (p + Rᵀ t): one symmetric 3x3
// inverse and sparse skew products instead of the 3x6 Jacobian algebra. C: [R 9, Rᵀt 3, Σ_lidar 9,
// A 36] of the scan (LDS). Writes Λ_w (9), θ_w (3), η_w lobe 0 (3).
constexpr int kSmapC = 57;
GC_DEV void smap_row(const double* C, const double* o, double eps_mass, const double* p, double* Lw, double* th,
                     double* e0) {
  const double* R = C;
  const double* Rtt = C + 9;
  const double* Sl = C + 12;
  const double* A = C + 21;  // 6 x 6 row-major
  const double K[9] = {0.0, -p[2], p[1], p[2], 0.0, -p[0], -p[1], p[0], 0.0};
  double X[9], Y[9], Sb[9];
  // X = A_tr K, Y = K A_rt, then K A_rr K
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double x = 0.0, y = 0.0;
      for (int k = 0; k < 3; ++k) {
        x += A[i * 6 + 3 + k] * K[3 * k + j];
        y += K[3 * i + k] * A[(3 + k) * 6 + j];
      }
      X[3 * i + j] = x;
      Y[3 * i + j] = y;
    }
  double KA[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double v = 0.0;
      for (int k = 0; k < 3; ++k) v += K[3 * i + k] * A[(3 + k) * 6 + 3 + j];
      KA[3 * i + j] = v;
    }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double kak = 0.0;
      for (int k = 0; k < 3; ++k) kak += KA[3 * i + k] * K[3 * k + j];
      Sb[3 * i + j] = Sl[3 * i + j] + A[i * 6 + j] + X[3 * i + j] - Y[3 * i + j] - kak;
    }
  for (int i = 0; i < 3; ++i)  // symmetric by construction up to rounding: symmetrise before inverting
    for (int j = i + 1; j < 3; ++j) {
      const double v = 0.5 * (Sb[3 * i + j] + Sb[3 * j + i]);
      Sb[3 * i + j] = v;
      Sb[3 * j + i] = v;
    }
  double Ib[9], T[9];
  inv3(Sb, Ib);
  mat3_mul(R, Ib, T);
  mat3_mul_nt(T, R, Lw);
  const double q[3] = {p[0] + Rtt[0], p[1] + Rtt[1], p[2] + Rtt[2]};
  mat3_vec(T, q, th);
  double d[3];
  direction(p, o, eps_mass, d);
  mat3_vec(R, d, e0);
}

// Pass 1, one workgroup per block of kSmapBlk rows (gc_runs.h): every thread forms one row's slot key
// (m_slots for a dropped row, sorted after every slot) and world row [Λ_w 9, θ_w 3, η_w lobe 0 3, w]
// into LDS; the block sorts (key, row) and sums each run of equal keys by a segmented inclusive scan
// in sorted order (inside each wave by shuffles, then the carries across the waves in wave order; the
// order depends on the positions only); each run's last position holds the run's sum, written as the run's
// piece and registered with its slot's entry. A scan's points crowd into few voxels (~65k rows into
// ~5k slots), so most of the work is this in-block reduction; a slot gets at most one piece per block.
constexpr int kSmapBlk = 256;
__global__ void __launch_bounds__(kSmapBlk) k_smap_block(ScanMapArgs A, RunTable T, uint32_t* sslot,
                                                         uint32_t* rank, SmapRow* pieces) {
  __shared__ double C[kSmapC + 3];
  __shared__ double v[kSmapRow][kSmapBlk];
  __shared__ uint64_t a[kSmapBlk];
  __shared__ double wave_tail[kSmapBlk / 64][kSmapRow];
  __shared__ uint32_t wave_klast[kSmapBlk / 64], wave_kfirst[kSmapBlk / 64];
  const int t = threadIdx.x;
  // the scan's constants: Σ_pose and Σ_lidar by lanes of wave 0, R, tt and Rᵀ t by lane 0 of wave 1
  if (t < 36) {
    C[21 + t] = A.h0[6 + t];
  } else if (t == 36) {
    // measurement_noise_mean_jax's LiDAR block (operators/measurement_noise_iw_jax.py:50-56):
    // domain_projection_psd_core(Ψ / (ν + p + 1), eps_psd) (certified shortcut: S_sym when SPD)
    const double den = A.lidar_iw[0] + 3.0 + 1.0;
    double Sl[9];
    for (int q = 0; q < 9; ++q) Sl[q] = A.lidar_iw[1 + q] / den;
    psd_project3_fast(Sl, A.eps_psd, C + 12, nullptr);
  } else if (t == 64) {
    double R[9], tt[3];
    smap_pose(A, R, tt);
    for (int q = 0; q < 9; ++q) C[q] = R[q];
    mat3_tvec(R, tt, C + 9);
    for (int q = 0; q < 3; ++q) C[kSmapC + q] = tt[q];
  }
  // the row's point and its deskew (they need none of C) while thread 0 forms the constants
  const int64_t j = (int64_t)blockIdx.x * kSmapBlk + t;
  const int64_t M = A.map.m_slots;
  double p0[3], w = 0.0, mw[3];
  const bool live = j < A.n_cap && smap_point(A, j, p0, &w);
  __syncthreads();
  SmapRow row;
  for (int q = 0; q < kSmapRow; ++q) row.v[q] = 0.0;
  uint32_t key = j < A.n_cap ? (uint32_t)M : kNoRun;
  if (live) {
    smap_world_mean(C, C + kSmapC, p0, mw);
    key = smap_slot(mw, A.voxel, M);
    const double o[3] = {A.o0, A.o1, A.o2};
    smap_row(C, o, A.eps_mass, p0, row.v, row.v + 9, row.v + 12);
    row.v[15] = w;
  }
  for (int q = 0; q < kSmapRow; ++q) v[q][t] = row.v[q];
  {
    const uint64_t sx = reg_bitonic_sort<kSmapBlk>(((uint64_t)key << 32) | (uint32_t)t, a);
    a[t] = sx;  // the sort ended with a barrier after its last read of a
    __syncthreads();
  }
  // position t of the sorted block: its row's values, then the segmented scan in sorted order
  const uint32_t k_t = (uint32_t)(a[t] >> 32);
  const int src = (int)(uint32_t)a[t];
  double x[kSmapRow];
  for (int q = 0; q < kSmapRow; ++q) x[q] = v[q][src];
  // the segmented inclusive scan, first inside each wave by shuffles (Hillis-Steele: a position adds
  // the entry d back when that entry has its key; the keys are sorted, so that entry's segment is its)
  const int lane = t & 63, wv = t >> 6;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t kd = (uint32_t)__shfl_up((int)k_t, d, 64);
    const bool take = lane >= d && kd == k_t;
    for (int q = 0; q < kSmapRow; ++q) {
      const double y = __shfl_up(x[q], d, 64);
      if (take) x[q] = y + x[q];
    }
  }
  // then across the waves: the running sum of the segment open at each wave's end, in wave order,
  // enters the next wave's first segment (carry + partial)
  if (lane == 63) {
    for (int q = 0; q < kSmapRow; ++q) wave_tail[wv][q] = x[q];
    wave_klast[wv] = k_t;
  }
  if (lane == 0) wave_kfirst[wv] = k_t;
  __syncthreads();
  if (wv > 0 && wave_klast[wv - 1] == wave_kfirst[wv] && k_t == wave_kfirst[wv]) {
    double run[kSmapRow];
    for (int q = 0; q < kSmapRow; ++q) run[q] = wave_tail[0][q];
    for (int w = 1; w < wv; ++w) {
      const bool cont = wave_klast[w - 1] == wave_kfirst[w] && wave_kfirst[w] == wave_klast[w];
      for (int q = 0; q < kSmapRow; ++q) run[q] = cont ? run[q] + wave_tail[w][q] : wave_tail[w][q];
    }
    for (int q = 0; q < kSmapRow; ++q) x[q] = run[q] + x[q];
  }
  const int64_t p = (int64_t)blockIdx.x * kSmapBlk + t;
  const bool tail = (int64_t)k_t < M && (t == kSmapBlk - 1 || (uint32_t)(a[t + 1] >> 32) != k_t);
  uint32_t rk = kNoRun;
  if (tail) {
    SmapRow o;
    for (int q = 0; q < kSmapRow; ++q) o.v[q] = x[q];
    pieces[p] = o;
    rk = register_run(T, k_t, (uint32_t)p);
  }
  if (p < A.n_cap) {
    sslot[p] = k_t;
    rank[p] = rk;
  }
}

// Pass 2, one thread per position: the owner of each slot (its run of rank 0) adds the slot's pieces
// in block order and read-modify-writes the slot (the fuse with responsibility 1, source LiDAR)
__global__ void __launch_bounds__(kApplyWG) k_smap_apply(ScanMapArgs A, int64_t n, RunTable T,
                                                         const uint32_t* __restrict__ sslot,
                                                         const uint32_t* __restrict__ rank,
                                                         const SmapRow* __restrict__ pieces,
                                                         uint32_t* wg_count) {
#pragma clang fp contract(off)
  __shared__ uint32_t slices[kApplyWG * kRunCap];
  __shared__ double wave_sums[(kApplyWG / 64) * kSmapRow];
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t key = e < n ? sslot[e] : kNoRun;
  const bool own = (int64_t)key < A.map.m_slots && rank[e] != kNoRun;  // not dropped, the owner (its entry)
  // the touched-slot count per workgroup (an LDS sum; thousands of global atomics on one counter
  // serialised the kernel: ~20-40 us)
  __shared__ uint32_t owned;
  if (threadIdx.x == 0) owned = 0u;
  __syncthreads();
  const unsigned long long b = __ballot(own);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(&owned, (uint32_t)__popcll(b));
  __syncthreads();
  if (threadIdx.x == 0) wg_count[blockIdx.x] = owned;
  SmapRow d;
  for (int q = 0; q < kSmapRow; ++q) d.v[q] = 0.0;
  const auto add = [&](uint32_t r) {
    const SmapRow pc = pieces[r];
    for (int q = 0; q < kSmapRow; ++q) d.v[q] = d.v[q] + pc.v[q];
  };
  SlotRunList<kRunCap> rl(slices + threadIdx.x * kRunCap);
  bool heavy = false;
  uint32_t s1 = 0u;
  if (own) {
    T.e[rank[e]] = 0ull;  // empty for the next call (nothing probes the table in this pass)
    s1 = T.succ[e];
    if (s1 == 0u) {  // the slot's rows all lie in one block (the common case)
      add((uint32_t)e);
    } else {
      rl.collect((uint32_t)e, s1, T.succ, (int)((n + kSmapBlk - 1) / kSmapBlk));
      if (rl.spill) {  // more runs than a slice holds: correctness path, never at the C5 sizes
        uint32_t prev = 0;
        for (int i = 0; i < rl.n; ++i) {
          const uint32_t r = rl.at(i, prev);
          if (r == kNoRun) break;  // only a corrupt entry: never index past the runs
          prev = r;
          add(r);
        }
      } else if (rl.n <= 4) {
        for (int i = 0; i < rl.n; ++i) add(rl.buf[i]);
      } else {
        heavy = true;
      }
    }
  }
  // slots of many runs (the voxels next to the sensor): the whole wave sums them, lane c < 16 the
  // column c over the runs in block order (the same order and bits as one thread's), eight loads in
  // flight per lane, one owner at a time
  const int lane = threadIdx.x & 63;
  double* wsum = wave_sums + (threadIdx.x >> 6) * kSmapRow;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the owners' slices, then read by the wave
  __builtin_amdgcn_wave_barrier();
  for (unsigned long long hb = __ballot(heavy); hb; hb &= hb - 1) {
    const int src = __ffsll((long long)hb) - 1;
    const uint32_t* ids = slices + (threadIdx.x - lane + src) * kRunCap;
    const int m = __shfl(rl.n, src);
    if (lane < kSmapRow) {
      const double* col = reinterpret_cast<const double*>(pieces) + lane;
      double acc = 0.0;
      int i = 0;
      for (; i + 8 <= m; i += 8) {
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = col[(size_t)ids[i + u] * kSmapRow];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = acc + x[u];
      }
      for (; i < m; ++i) acc = acc + col[(size_t)ids[i] * kSmapRow];
      wsum[lane] = acc;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the sums in LDS, then read
    __builtin_amdgcn_wave_barrier();
    if (lane == src)
      for (int q = 0; q < kSmapRow; ++q) d.v[q] = wsum[q];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the sums in LDS, then read
    __builtin_amdgcn_wave_barrier();
  }
  if (!own) return;
  if (s1 != 0u) rl.clear();  // the chain's links zero for the next call
  const int64_t s = key;
  const int L = A.map.n_lobes;
  for (int q = 0; q < 9; ++q) mLam(A.map, s)[q] = mLam(A.map, s)[q] + d.v[q];
  for (int q = 0; q < 3; ++q) mTh(A.map, s)[q] = mTh(A.map, s)[q] + d.v[9 + q];
  // lobes > 0 receive 0.0 per row: x + 0.0 (as the fuse writes them)
  for (int q = 0; q < 3 * L; ++q)
    mEta(A.map, s)[q] = mEta(A.map, s)[q] + (q < 3 ? d.v[12 + q] : 0.0);
  mW(A.map, s) = mW(A.map, s) + d.v[15];
  mTs(A.map, s) = A.timestamp;
  mSup(A.map, s) = A.scan_seq;
  mUpd(A.map, s) = A.scan_seq;
  if (A.map.lidar_mass) mLid(A.map, s) = mLid(A.map, s) + d.v[15];
}

}  // namespace

int32_t scan_map_prepare(gc_ctx* ctx, ScanMapWork* W, int64_t n_cap, int64_t m_slots) {
  W->n_cap = n_cap;
  W->m_slots = m_slots;
  auto up = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t kv = up((size_t)n_cap * sizeof(uint32_t)), rv = up((size_t)n_cap * sizeof(SmapRow));
  W->n_wg = (n_cap + kApplyWG - 1) / kApplyWG;
  const size_t bytes = 2 * kv + rv + up((size_t)W->n_wg * sizeof(uint32_t));
  if (bytes > W->bytes) {
    if (W->buf) GC_HIP(ctx, hipFree(W->buf));
    W->buf = nullptr;
    W->bytes = 0;
    GC_HIP(ctx, hipMalloc(&W->buf, bytes));
    W->bytes = bytes;
  }
  char* base = (char*)W->buf;
  W->sslot = (uint32_t*)base;
  W->rank = (uint32_t*)(base + kv);
  W->pieces = (double*)(base + 2 * kv);
  W->wg_count = (uint32_t*)(base + 2 * kv + rv);
  return run_table(ctx, ctx->stream, &W->runs, n_cap);  // allocated (and emptied) now, outside any scan
}

int32_t scan_map_update(gc_ctx* ctx, hipStream_t st, ScanMapWork* W, const gc_primitive_map& map,
                        const PipeDev& P, const ScanMapInput& in) {
  ScanMapArgs A{};
  A.map = map;
  A.pts = in.pts; A.t = in.t; A.w = in.w;
  // the scan's snapshot, written by k_combine_final (ordered before this update by the caller)
  A.h0 = P.smap_snap;
  A.lidar_iw = P.smap_snap + kSnapIW;
  A.bscal = P.smap_snap + kSnapBudget;
  A.n_cap = P.n_cap;
  A.t0 = in.t0; A.t1 = in.t1;
  A.o0 = P.o0; A.o1 = P.o1; A.o2 = P.o2;
  A.voxel = in.voxel; A.timestamp = in.timestamp; A.eps_mass = P.eps_mass;
  A.eps_psd = P.eps_psd;
  A.scan_seq = in.scan_seq;
  const int64_t n = P.n_cap;
  if (int rc = run_table(ctx, st, &W->runs, n)) return rc;
  const RunTable T{W->runs.entries(), W->runs.succ(), W->runs.bits};
  W->runs.dirty = true;  // until both passes are enqueued
  hipLaunchKernelGGL(k_smap_block, dim3((unsigned)((n + kSmapBlk - 1) / kSmapBlk)), dim3(kSmapBlk), 0, st, A,
                     T, W->sslot, W->rank, (SmapRow*)W->pieces);
  GC_LAUNCH_CHECK(ctx);
  hipLaunchKernelGGL(k_smap_apply, dim3((unsigned)((n + kApplyWG - 1) / kApplyWG)), dim3(kApplyWG), 0, st, A, n,
                     T, (const uint32_t*)W->sslot, (const uint32_t*)W->rank, (const SmapRow*)W->pieces, W->wg_count);
  GC_LAUNCH_CHECK(ctx);
  W->runs.dirty = false;
  return GC_OK;
}

int32_t scan_map_count(gc_ctx* ctx, const ScanMapWork& W, int64_t* out, size_t* d2h_bytes) {
  std::vector<uint32_t> c((size_t)W.n_wg);
  GC_HIP(ctx, hipMemcpyAsync(c.data(), W.wg_count, c.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
  if (int rc_w = gc::wait_stream(ctx, ctx->stream, "a result download")) return rc_w;
  int64_t n = 0;
  for (uint32_t v : c) n += v;
  *out = n;
  *d2h_bytes = c.size() * sizeof(uint32_t);
  return GC_OK;
}

}  // namespace gc
