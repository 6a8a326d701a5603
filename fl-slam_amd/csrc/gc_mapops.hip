// gc_mapops.hip — PrimitiveMap maintenance on the device.
//
//  primitive_map_forget                 backend/structures/primitive_map.py:1314-1390
//  primitive_map_recency_inflate        :1400-1490
//  primitive_map_cull                   :1175-1305
//  primitive_map_insert_masked          :807-982 (+ _select_lowest_mass_slots_fixed :325-353)
//  primitive_map_merge_reduce           :1809-2030 (+ _merge_reduce_jax :1501-1807)
//
// One reference tile = the slot range [s0, s0 + n) of the flat device map (gc_map.hip). The
// per-slot work is one thread per slot (HBM-bound streaming of the 176 B core record). Sums are
// per-block partials in slot order reduced by one thread in block order (deterministic; the
// integer counts are exact). Orderings that the reference defines by a stable sort (eviction
// slots, merge candidates) use a stable radix sort on the same key, so ties resolve by index
// exactly as jax.lax.sort / jnp.argsort do. The greedy disjoint-pair selection of merge-reduce is
// inherently sequential and runs on one lane over the sorted candidates, stopping at the first
// distance >= threshold.
#include <hip/hip_runtime.h>
#include "gc_internal.h"
#include "gc_math.h"
#include "gc_mapslot.h"
#include "gc_sort.h"

namespace gc {
namespace {

constexpr int kMaxLobesOps = 8;
constexpr int kPartBlocks = 240;  // grid of the reduction passes (<= one wave of workgroups)

struct Tile {
  gc_primitive_map m;
  int64_t s0, n;
};

// Fixed-order block sum of NV per-thread values into part[blockIdx.x * NV + v].
template <int NV>
GC_DEV void block_partials(double (&v)[NV], double* part) {
  __shared__ double red[NV][4];
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    double x = v[q];
    for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
    if ((threadIdx.x & 63) == 0) red[q][threadIdx.x >> 6] = x;
  }
  __syncthreads();
  if ((int)threadIdx.x < NV)
    part[blockIdx.x * NV + threadIdx.x] =
        (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]);
}

template <int NV>
__global__ void k_sum_parts(const double* __restrict__ part, int blocks, double* out) {
  if ((int)threadIdx.x >= NV) return;
  double s = 0.0;
  for (int b = 0; b < blocks; ++b) s += part[b * NV + threadIdx.x];
  out[threadIdx.x] = s;
}

__global__ void k_forget(Tile T, double gamma) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < T.n) mW(T.m, T.s0 + s) = gamma * mW(T.m, T.s0 + s);
}

GC_DEV double recency_decay(int64_t seq, int64_t last, double lam) {
  const int64_t dt = seq - last > 0 ? seq - last : 0;
  return exp(-lam * (double)dt);
}

// part: [n_valid, Σ(1 - decay), Σ(1/decay - 1)] over valid slots
__global__ void __launch_bounds__(256) k_recency(Tile T, int64_t seq, double lam, double min_scale, double* part) {
  double acc[3] = {0.0, 0.0, 0.0};
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < T.n; s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = T.s0 + s;
    const bool valid = mValid(T.m, g) != 0;
    double decay = fmin(fmax(recency_decay(seq, mSup(T.m, g), lam), min_scale), 1.0);
    if (!valid) decay = 1.0;
    double* L = mLam(T.m, g);
#pragma unroll
    for (int q = 0; q < 9; ++q) L[q] = L[q] * decay;
#pragma unroll
    for (int q = 0; q < 3; ++q) mTh(T.m, g)[q] = mTh(T.m, g)[q] * decay;
    if (valid) {
      acc[0] += 1.0;
      acc[1] += 1.0 - decay;
      acc[2] += 1.0 / decay - 1.0;
    }
  }
  block_partials<3>(acc, part);
}

// part: [n_valid, n_below, mass_below, Σ w (all slots)]
__global__ void __launch_bounds__(256) k_cull_count(Tile T, double thr, double* part) {
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < T.n; s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = T.s0 + s;
    const double w = mW(T.m, g);
    const bool valid = mValid(T.m, g) != 0;
    const bool below = valid && w < thr;
    acc[0] += valid ? 1.0 : 0.0;
    acc[1] += below ? 1.0 : 0.0;
    acc[2] += w * (below ? 1.0 : 0.0);
    acc[3] += w;
  }
  block_partials<4>(acc, part);
}

__global__ void k_cull_keys(Tile T, double* keys) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < T.n) keys[s] = mW(T.m, T.s0 + s) * (mValid(T.m, T.s0 + s) ? 1.0 : 0.0);
}

__global__ void k_cull_apply(Tile T, double thr) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= T.n) return;
  const int64_t g = T.s0 + s;
  if (mValid(T.m, g) && mW(T.m, g) < thr) mValid(T.m, g) = 0;
}

__global__ void __launch_bounds__(256) k_count_valid(Tile T, double* part) {
  double acc[1] = {0.0};
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < T.n; s += (int64_t)gridDim.x * blockDim.x)
    acc[0] += mValid(T.m, T.s0 + s) ? 1.0 : 0.0;
  block_partials<1>(acc, part);
}

// eviction key (_select_lowest_mass_slots_fixed): retention w·exp(-λ dt) on valid slots, -inf on
// empty ones (selected first)
__global__ void k_insert_keys(Tile T, int64_t seq, double lam, double* keys, int32_t* vals) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= T.n) return;
  const int64_t g = T.s0 + s;
  const double ret = mW(T.m, g) * recency_decay(seq, mSup(T.m, g), lam);
  keys[s] = mValid(T.m, g) ? ret : -INFINITY;
  vals[s] = (int32_t)s;
}

// One workgroup: blocked exclusive prefix of the proposal mask (new ids), then each thread
// writes its proposals into their eviction slots.
__global__ void __launch_bounds__(256) k_insert_apply(Tile T, gc_insert_batch B, const int32_t* __restrict__ order,
                                                      double ts, int64_t seq, int64_t next_id, int32_t* slots_out,
                                                      int64_t* ids_out, double* n_ins_out) {
  __shared__ int64_t scan[256];
  const int t = threadIdx.x;
  const int64_t per = (B.K + 255) / 256;
  const int64_t k0 = t * per, k1 = k0 + per < B.K ? k0 + per : B.K;
  int64_t cnt = 0;
  for (int64_t k = k0; k < k1; ++k) cnt += B.valid_mask[k] ? 1 : 0;
  scan[t] = cnt;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {  // inclusive Hillis-Steele over the 256 chunk counts
    const int64_t v = t >= off ? scan[t - off] : 0;
    __syncthreads();
    scan[t] += v;
    __syncthreads();
  }
  int64_t run = scan[t] - cnt;
  const int L = T.m.n_lobes;
  const bool color = T.m.cam_mass != nullptr;
  for (int64_t k = k0; k < k1; ++k) {
    const int32_t slot = order[k];
    const bool ins = B.valid_mask[k] != 0;
    if (slots_out) slots_out[k] = slot;
    if (ids_out) ids_out[k] = ins ? next_id + run : -1;
    if (!ins) continue;
    const int64_t g = T.s0 + slot;
    for (int q = 0; q < 9; ++q) mLam(T.m, g)[q] = B.Lambdas[9 * k + q];
    for (int q = 0; q < 3; ++q) mTh(T.m, g)[q] = B.thetas[3 * k + q];
    for (int q = 0; q < 3 * L; ++q) mEta(T.m, g)[q] = B.etas[(int64_t)3 * L * k + q];
    const double w = B.weights[k];
    mW(T.m, g) = w;
    mTs(T.m, g) = ts;
    if (T.m.created_timestamps) mCreated(T.m, g) = ts;
    mSup(T.m, g) = seq;
    mUpd(T.m, g) = seq;
    if (T.m.primitive_ids) mPid(T.m, g) = next_id + run;
    mValid(T.m, g) = 1;
    if (color) {
      const int src = B.sources ? B.sources[k] : 1;
      const double cam = w * (src == 0 ? 1.0 : 0.0), lid = w * (src == 1 ? 1.0 : 0.0);
      mCam(T.m, g) = cam;
      mLid(T.m, g) = lid;
      mDen(T.m, g) = cam;
      for (int q = 0; q < 3; ++q) {
        const double c = B.colors ? B.colors[3 * k + q] : 0.0;
        const double rgb = cam > 0.0 ? clampd(c, 0.0, 1.0) : 0.5;
        mAcc(T.m, g)[q] = c * cam;
        mRgb(T.m, g)[q] = rgb;
        if (T.m.colors) mCol(T.m, g)[q] = rgb;
      }
    }
    ++run;
  }
  if (t == 255) *n_ins_out = (double)scan[255];
}

// ---- merge-reduce
// μ = solve(Λ + εI, θ), Σ = inv(Λ + εI), det Σ (primitive_map.py:1908-1911)
__global__ void k_merge_prep(Tile T, double eps_lift, double* mu, double* Sig, double* dets) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= T.n) return;
  const int64_t g = T.s0 + s;
  double Lr[9];
  for (int q = 0; q < 9; ++q) Lr[q] = mLam(T.m, g)[q] + ((q % 4 == 0) ? eps_lift : 0.0);
  solve3(Lr, mTh(T.m, g), mu + 3 * s);
  inv3(Lr, Sig + 9 * s);
  dets[s] = det3(Sig + 9 * s);
}

// pair p of jnp.triu_indices(n, k=1) (row-major, i < j)
GC_DEV void triu_pair(int64_t n, int64_t p, int64_t* i, int64_t* j) {
  const double b = 2.0 * (double)n - 1.0;
  int64_t r = (int64_t)floor((b - sqrt(b * b - 8.0 * (double)p)) * 0.5);
  if (r < 0) r = 0;
  auto off = [n](int64_t x) { return x * (2 * n - x - 1) / 2; };
  while (r > 0 && off(r) > p) --r;
  while (off(r + 1) <= p) ++r;
  *i = r;
  *j = p - off(r) + r + 1;
}

// Bhattacharyya distance of pair p (primitive_map.py:1921-1930)
__global__ void k_merge_dist(Tile T, int64_t P, const double* __restrict__ mu, const double* __restrict__ Sig,
                             const double* __restrict__ dets, double eps_lift, double* keys, uint32_t* vals) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  int64_t i, j;
  triu_pair(T.n, p, &i, &j);
  double S[9], Sr[9], Si[9];
  for (int q = 0; q < 9; ++q) S[q] = 0.5 * (Sig[9 * i + q] + Sig[9 * j + q]);
  const double detS = det3(S);
  for (int q = 0; q < 9; ++q) Sr[q] = S[q] + ((q % 4 == 0) ? eps_lift : 0.0);
  inv3(Sr, Si);
  const double dm[3] = {mu[3 * i] - mu[3 * j], mu[3 * i + 1] - mu[3 * j + 1], mu[3 * i + 2] - mu[3 * j + 2]};
  double rv[3];
  mat3_tvec(Si, dm, rv);  // dmuᵀ S⁻¹
  const double quad = 0.125 * dot3(rv, dm);
  const double logt = 0.5 * log(detS / sqrt(dets[i] * dets[j] + 1e-24));
  const bool pv = mValid(T.m, T.s0 + i) && mValid(T.m, T.s0 + j);
  keys[p] = pv ? quad + logt : INFINITY;
  vals[p] = (uint32_t)p;
}

// greedy disjoint selection over the sorted candidates (_merge_reduce_jax select_body)
__global__ void k_merge_select(int64_t n, int64_t P, const double* __restrict__ keys, const uint32_t* __restrict__ vals,
                               double thr, int max_pairs, uint8_t* used, int32_t* sel, int32_t* n_sel) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int ns = 0;
  for (int64_t k = 0; k < P && ns < max_pairs; ++k) {
    const double d = keys[k];
    if (d == INFINITY) break;   // the tail: +inf (invalid pairs), then NaN
    if (!isfinite(d)) continue;  // -inf / NaN: never selectable (jnp.isfinite)
    if (!(d < thr)) break;       // ascending: nothing later qualifies
    int64_t i, j;
    triu_pair(n, vals[k], &i, &j);
    if (used[i] || used[j]) continue;
    used[i] = 1;
    used[j] = 1;
    sel[2 * ns] = (int32_t)i;
    sel[2 * ns + 1] = (int32_t)j;
    ++ns;
  }
  *n_sel = ns;
}

// moment-matched merge of each selected (disjoint) pair into slot i (_merge_reduce_jax merge_body)
__global__ void k_merge_apply(Tile T, const double* __restrict__ mu, const double* __restrict__ Sig,
                              const int32_t* __restrict__ sel, const int32_t* __restrict__ n_sel, double eps_psd,
                              int max_pairs) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= max_pairs || k >= *n_sel) return;
  const int64_t i = sel[2 * k], j = sel[2 * k + 1];
  const int64_t gi = T.s0 + i, gj = T.s0 + j;
  const double w1 = mW(T.m, gi), w2 = mW(T.m, gj), ws = w1 + w2;
  if (!(ws > 0.0)) return;
  const double* m1 = mu + 3 * i;
  const double* m2 = mu + 3 * j;
  double mm[3], d1[3], d2[3], Sm[9], Lm[9], th[3];
  for (int q = 0; q < 3; ++q) mm[q] = (w1 * m1[q] + w2 * m2[q]) / ws;
  for (int q = 0; q < 3; ++q) { d1[q] = m1[q] - mm[q]; d2[q] = m2[q] - mm[q]; }
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      const int q = 3 * r + c;
      Sm[q] = (w1 * (Sig[9 * i + q] + d1[r] * d1[c]) + w2 * (Sig[9 * j + q] + d2[r] * d2[c])) / ws +
              (r == c ? eps_psd : 0.0);
    }
  inv3(Sm, Lm);
  mat3_vec(Lm, mm, th);
  for (int q = 0; q < 9; ++q) mLam(T.m, gi)[q] = Lm[q];
  for (int q = 0; q < 3; ++q) mTh(T.m, gi)[q] = th[q];
  const int L = T.m.n_lobes;
  double* ei = mEta(T.m, gi);
  const double* ej = mEta(T.m, gj);
  for (int q = 0; q < 3 * L; ++q) ei[q] = (w1 * ei[q] + w2 * ej[q]) / ws;
  mW(T.m, gi) = ws;
  if (T.m.cam_mass) {
    const double cm = mCam(T.m, gi) + mCam(T.m, gj);
    const double den = mDen(T.m, gi) + mDen(T.m, gj);
    mCam(T.m, gi) = cm;
    mLid(T.m, gi) = mLid(T.m, gi) + mLid(T.m, gj);
    mDen(T.m, gi) = den;
    for (int q = 0; q < 3; ++q) {
      const double acc = mAcc(T.m, gi)[q] + mAcc(T.m, gj)[q];
      const double rgb = cm > 0.0 ? clampd(acc / fmax(den, eps_psd), 0.0, 1.0) : 0.5;
      mAcc(T.m, gi)[q] = acc;
      mRgb(T.m, gi)[q] = rgb;
      if (T.m.colors) mCol(T.m, gi)[q] = rgb;
    }
  }
  mTs(T.m, gi) = fmax(mTs(T.m, gi), mTs(T.m, gj));
  if (T.m.created_timestamps) mCreated(T.m, gi) = fmin(mCreated(T.m, gi), mCreated(T.m, gj));
  const int64_t ls = mSup(T.m, gj), lu = mUpd(T.m, gj);
  if (ls > mSup(T.m, gi)) mSup(T.m, gi) = ls;
  if (lu > mUpd(T.m, gi)) mUpd(T.m, gi) = lu;
  mW(T.m, gj) = 0.0;
  mValid(T.m, gj) = 0;
}

unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }
unsigned part_blocks(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < kPartBlocks ? (b > 0 ? b : 1) : kPartBlocks);
}

int check_tile(gc_ctx* ctx, const gc_primitive_map* map, int64_t slot0, int64_t n_slots, bool need_valid) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  if (int rc_j = gc::join_side(ctx)) return rc_j;  // a pipeline's in-scan update may still write the map
  GC_CHECK_ARG(ctx, map != nullptr, "NULL map");
  GC_CHECK_ARG(ctx, map->m_slots > 0 && slot0 >= 0 && n_slots >= 0 && slot0 + n_slots <= map->m_slots,
               "tile range outside the map");
  GC_CHECK_ARG(ctx, map->n_lobes >= 1 && map->n_lobes <= kMaxLobesOps, "n_lobes must be in [1, 8]");
  {
    const char* lay_ = gc::map_layout_error(*map);
    GC_CHECK_ARG(ctx, lay_ == nullptr, lay_ ? lay_ : "");
  }
  GC_CHECK_ARG(ctx, map->Lambdas && map->thetas && map->etas && map->weights && map->timestamps &&
                        map->last_supported_scan_seq && map->last_update_scan_seq,
               "NULL map field");
  GC_CHECK_ARG(ctx, !need_valid || map->valid_mask, "valid_mask is required");
  const bool color = map->cam_mass != nullptr;
  GC_CHECK_ARG(ctx, !color || (map->lidar_mass && map->rgb_cam_accum && map->rgb_cam_denom && map->rgb),
               "colour fields must be all set or all NULL");
  return GC_OK;
}

// reduction pass: launch KER over the tile into part, then fixed-order finish into out (device)
template <int NV, typename Launch>
int reduce_into(gc_ctx* ctx, int64_t n, double* part, double* out, Launch launch) {
  const unsigned nb = part_blocks(n);
  launch(nb);
  GC_LAUNCH_CHECK(ctx);
  hipLaunchKernelGGL(k_sum_parts<NV>, dim3(1), dim3(64), 0, ctx->stream, part, (int)nb, out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int download(gc_ctx* ctx, void* h, const void* d, size_t bytes) {
  GC_HIP(ctx, hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, ctx->stream));
  if (int rc_w = gc::wait_stream(ctx, ctx->stream, "a result download")) return rc_w;
  return GC_OK;
}

}  // namespace
}  // namespace gc

using namespace gc;

extern "C" {

int32_t gc_primitive_map_forget(gc_ctx* ctx, const gc_primitive_map* map, int64_t slot0, int64_t n_slots,
                                double gamma) {
  if (int rc = check_tile(ctx, map, slot0, n_slots, false)) return rc;
  if (n_slots == 0) return GC_OK;
  hipLaunchKernelGGL(k_forget, dim3(blocks_for(n_slots)), dim3(256), 0, ctx->stream, Tile{*map, slot0, n_slots},
                     gamma);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_primitive_map_recency_inflate(gc_ctx* ctx, const gc_primitive_map* map, int64_t slot0, int64_t n_slots,
                                         int64_t scan_seq, double decay_lambda, double min_scale,
                                         double* h_stats3) {
  if (int rc = check_tile(ctx, map, slot0, n_slots, true)) return rc;
  if (h_stats3) h_stats3[0] = h_stats3[1] = h_stats3[2] = 0.0;
  if (n_slots == 0) return GC_OK;
  void* scr;
  if (int rc = gc::scratch(ctx, sizeof(double) * (3 * kPartBlocks + 8), &scr)) return rc;
  double* part = (double*)scr;
  double* out = part + 3 * kPartBlocks;
  const Tile T{*map, slot0, n_slots};
  if (int rc = reduce_into<3>(ctx, n_slots, part, out, [&](unsigned nb) {
        hipLaunchKernelGGL(k_recency, dim3(nb), dim3(256), 0, ctx->stream, T, scan_seq, decay_lambda, min_scale,
                           part);
      }))
    return rc;
  return h_stats3 ? download(ctx, h_stats3, out, 3 * sizeof(double)) : GC_OK;
}

int32_t gc_test_radix_sort(gc_ctx* ctx, const double* d_keys_in, const uint32_t* d_vals_in, int64_t n_seg, int64_t L,
                           int32_t descending, double* d_keys_out, uint32_t* d_vals_out) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, n_seg >= 0 && L >= 0 && n_seg * L < ((int64_t)1 << 32), "n_seg * L must be in [0, 2^32)");
  GC_CHECK_ARG(ctx, n_seg * L == 0 || (d_keys_in && d_keys_out), "NULL key buffer");
  GC_CHECK_ARG(ctx, !d_vals_in || d_vals_out, "NULL value output");
  if (n_seg * L == 0) return GC_OK;
  void* scr;
  if (int rc = gc::scratch(ctx, gc::sort_temp_bytes(n_seg, L, d_vals_in != nullptr), &scr)) return rc;
  GC_HIP(ctx, gc::radix_sort_pairs(ctx->stream, d_keys_in, d_keys_out, d_vals_in, d_vals_out, n_seg, L, descending != 0,
                                   scr));
  return GC_OK;
}

int32_t gc_primitive_map_cull(gc_ctx* ctx, const gc_primitive_map* map, int64_t slot0, int64_t n_slots,
                              double weight_threshold, int64_t max_primitives, double* h_out4) {
  if (int rc = check_tile(ctx, map, slot0, n_slots, true)) return rc;
  GC_CHECK_ARG(ctx, h_out4 != nullptr, "h_out4 is NULL");
  for (int q = 0; q < 4; ++q) h_out4[q] = 0.0;
  if (n_slots == 0) return GC_OK;
  const size_t temp = gc::sort_temp_bytes(1, n_slots, false);
  const size_t kb = ((size_t)n_slots * sizeof(double) + 255) / 256 * 256;
  void* scr;
  if (int rc = gc::scratch(ctx, sizeof(double) * (4 * kPartBlocks + 8) + 2 * kb + temp, &scr)) return rc;
  double* part = (double*)scr;
  double* out = part + 4 * kPartBlocks;
  double* keys_in = (double*)((char*)scr + sizeof(double) * (4 * kPartBlocks + 8));
  double* keys = (double*)((char*)keys_in + kb);
  void* tmp = (char*)keys + kb;
  const Tile T{*map, slot0, n_slots};
  auto count = [&](double thr, double* h4) -> int {
    if (int rc = reduce_into<4>(ctx, n_slots, part, out, [&](unsigned nb) {
          hipLaunchKernelGGL(k_cull_count, dim3(nb), dim3(256), 0, ctx->stream, T, thr, part);
        }))
      return rc;
    return download(ctx, h4, out, 4 * sizeof(double));
  };
  double c[4];
  if (int rc = count(weight_threshold, c)) return rc;
  const double n_valid = c[0];
  double thr = weight_threshold;
  // primitive_map.py:1222-1229: keep the top max_primitives by weight
  if (max_primitives >= 0 && n_valid - c[1] > (double)max_primitives && max_primitives < n_slots) {
    hipLaunchKernelGGL(k_cull_keys, dim3(blocks_for(n_slots)), dim3(256), 0, ctx->stream, T, keys_in);
    GC_LAUNCH_CHECK(ctx);
    if (gc::radix_sort_pairs(ctx->stream, keys_in, keys, nullptr, nullptr, 1, n_slots, true, tmp) != hipSuccess) {
      gc::set_error(ctx, "radix sort failed");
      return GC_ERR_RUNTIME;
    }
    if (int rc = download(ctx, &thr, keys + max_primitives, sizeof(double))) return rc;
    if (int rc = count(thr, c)) return rc;
  }
  if (c[1] > 0.0) {
    hipLaunchKernelGGL(k_cull_apply, dim3(blocks_for(n_slots)), dim3(256), 0, ctx->stream, T, thr);
    GC_LAUNCH_CHECK(ctx);
  }
  h_out4[0] = c[1];
  h_out4[1] = c[1] > 0.0 ? c[2] : 0.0;
  h_out4[2] = c[3];
  h_out4[3] = n_valid;
  return GC_OK;
}

int32_t gc_primitive_map_insert_masked(gc_ctx* ctx, const gc_primitive_map* map, int64_t slot0, int64_t n_slots,
                                       const gc_insert_batch* batch, double timestamp, int64_t scan_seq,
                                       double recency_decay_lambda, int64_t next_global_id,
                                       int32_t* d_target_slots_out, int64_t* d_new_ids_out, int64_t* h_out2) {
  if (int rc = check_tile(ctx, map, slot0, n_slots, true)) return rc;
  GC_CHECK_ARG(ctx, batch && h_out2, "NULL batch or h_out2");
  GC_CHECK_ARG(ctx, batch->K >= 1 && batch->K <= n_slots, "K must be in [1, n_slots]");
  GC_CHECK_ARG(ctx, n_slots < (int64_t)INT32_MAX, "tile too large");
  GC_CHECK_ARG(ctx, batch->Lambdas && batch->thetas && batch->etas && batch->weights && batch->valid_mask,
               "NULL proposal field");
  const size_t temp = gc::sort_temp_bytes(1, n_slots, true);
  const size_t kb = ((size_t)n_slots * sizeof(double) + 255) / 256 * 256;
  const size_t vb = ((size_t)n_slots * sizeof(int32_t) + 255) / 256 * 256;
  const size_t head = sizeof(double) * (kPartBlocks + 16);
  void* scr;
  if (int rc = gc::scratch(ctx, head + 2 * kb + 2 * vb + temp, &scr)) return rc;
  double* part = (double*)scr;
  double* out = part + kPartBlocks;  // [count_after, n_inserted]
  char* base = (char*)scr + head;
  double* keys_in = (double*)base;
  double* keys = (double*)(base + kb);
  int32_t* vals_in = (int32_t*)(base + 2 * kb);
  int32_t* vals = (int32_t*)(base + 2 * kb + vb);
  void* tmp = base + 2 * kb + 2 * vb;
  const Tile T{*map, slot0, n_slots};
  hipLaunchKernelGGL(k_insert_keys, dim3(blocks_for(n_slots)), dim3(256), 0, ctx->stream, T, scan_seq,
                     recency_decay_lambda, keys_in, vals_in);
  GC_LAUNCH_CHECK(ctx);
  if (gc::radix_sort_pairs(ctx->stream, keys_in, keys, (const uint32_t*)vals_in, (uint32_t*)vals, 1, n_slots, false,
                           tmp) != hipSuccess) {
    gc::set_error(ctx, "radix sort failed");
    return GC_ERR_RUNTIME;
  }
  hipLaunchKernelGGL(k_insert_apply, dim3(1), dim3(256), 0, ctx->stream, T, *batch, (const int32_t*)vals, timestamp,
                     scan_seq, next_global_id, d_target_slots_out, d_new_ids_out, out + 1);
  GC_LAUNCH_CHECK(ctx);
  if (int rc = reduce_into<1>(ctx, n_slots, part, out, [&](unsigned nb) {
        hipLaunchKernelGGL(k_count_valid, dim3(nb), dim3(256), 0, ctx->stream, T, part);
      }))
    return rc;
  double h[2];
  if (int rc = download(ctx, h, out, sizeof(h))) return rc;
  h_out2[0] = (int64_t)h[1];
  h_out2[1] = (int64_t)h[0];
  return GC_OK;
}

int32_t gc_primitive_map_merge_reduce(gc_ctx* ctx, const gc_primitive_map* map, int64_t slot0, int64_t n_slots,
                                      double merge_threshold, int32_t max_pairs, double eps_psd, double eps_lift,
                                      int64_t* h_out2) {
  if (int rc = check_tile(ctx, map, slot0, n_slots, true)) return rc;
  GC_CHECK_ARG(ctx, h_out2 != nullptr, "h_out2 is NULL");
  GC_CHECK_ARG(ctx, n_slots <= 65536, "merge-reduce tile larger than 65536 slots");
  h_out2[0] = 0;
  h_out2[1] = 0;
  const Tile T{*map, slot0, n_slots};
  const int64_t P = n_slots * (n_slots - 1) / 2;
  const size_t temp = P > 0 ? gc::sort_temp_bytes(1, P, true) : 0;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t head = sizeof(double) * (kPartBlocks + 16);
  const size_t b_mu = al(sizeof(double) * 3 * n_slots), b_sig = al(sizeof(double) * 9 * n_slots),
               b_det = al(sizeof(double) * n_slots), b_k = al(sizeof(double) * P), b_v = al(sizeof(uint32_t) * P),
               b_used = al(n_slots), b_sel = al(sizeof(int32_t) * (2 * (size_t)(max_pairs > 0 ? max_pairs : 1) + 1));
  void* scr;
  if (int rc = gc::scratch(ctx, head + b_mu + b_sig + b_det + 2 * b_k + 2 * b_v + b_used + b_sel + temp, &scr))
    return rc;
  double* part = (double*)scr;
  double* out = part + kPartBlocks;
  char* p = (char*)scr + head;
  double* mu = (double*)p; p += b_mu;
  double* Sig = (double*)p; p += b_sig;
  double* dets = (double*)p; p += b_det;
  double* keys_in = (double*)p; p += b_k;
  double* keys = (double*)p; p += b_k;
  uint32_t* vals_in = (uint32_t*)p; p += b_v;
  uint32_t* vals = (uint32_t*)p; p += b_v;
  uint8_t* used = (uint8_t*)p; p += b_used;
  int32_t* sel = (int32_t*)p; p += b_sel;
  void* tmp = p;
  auto count_valid = [&](double* h) -> int {
    if (int rc = reduce_into<1>(ctx, n_slots, part, out, [&](unsigned nb) {
          hipLaunchKernelGGL(k_count_valid, dim3(nb), dim3(256), 0, ctx->stream, T, part);
        }))
      return rc;
    return download(ctx, h, out, sizeof(double));
  };
  double nv = 0.0;
  if (n_slots > 0)
    if (int rc = count_valid(&nv)) return rc;
  h_out2[1] = (int64_t)nv;
  if (n_slots < 2 || nv < 2.0 || max_pairs <= 0) return GC_OK;  // primitive_map.py:1879-1880
  int32_t* n_sel = sel + 2 * max_pairs;
  GC_HIP(ctx, hipMemsetAsync(used, 0, (size_t)n_slots, ctx->stream));
  hipLaunchKernelGGL(k_merge_prep, dim3(blocks_for(n_slots)), dim3(256), 0, ctx->stream, T, eps_lift, mu, Sig, dets);
  GC_LAUNCH_CHECK(ctx);
  hipLaunchKernelGGL(k_merge_dist, dim3(blocks_for(P)), dim3(256), 0, ctx->stream, T, P, (const double*)mu,
                     (const double*)Sig, (const double*)dets, eps_lift, keys_in, vals_in);
  GC_LAUNCH_CHECK(ctx);
  if (gc::radix_sort_pairs(ctx->stream, keys_in, keys, vals_in, vals, 1, P, false, tmp) != hipSuccess) {
    gc::set_error(ctx, "radix sort failed");
    return GC_ERR_RUNTIME;
  }
  hipLaunchKernelGGL(k_merge_select, dim3(1), dim3(64), 0, ctx->stream, n_slots, P, (const double*)keys,
                     (const uint32_t*)vals, merge_threshold, (int)max_pairs, used, sel, n_sel);
  GC_LAUNCH_CHECK(ctx);
  hipLaunchKernelGGL(k_merge_apply, dim3((unsigned)((max_pairs + 255) / 256)), dim3(256), 0, ctx->stream, T,
                     (const double*)mu, (const double*)Sig, (const int32_t*)sel, (const int32_t*)n_sel, eps_psd,
                     (int)max_pairs);
  GC_LAUNCH_CHECK(ctx);
  int32_t ns = 0;
  if (int rc = download(ctx, &ns, n_sel, sizeof(ns))) return rc;
  if (int rc = count_valid(&nv)) return rc;
  h_out2[0] = ns;
  h_out2[1] = (int64_t)nv;
  return GC_OK;
}

}  // extern "C"
