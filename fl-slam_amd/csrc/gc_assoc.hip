// gc_assoc.hip — map view extraction and OT association on the device.
//
//  extract_atlas_map_view      backend/structures/primitive_map.py:356-451 (+ :304-322, :475-498)
//  associate_primitives_ot     backend/operators/primitive_association.py:239-553
//                              (+ _compute_sparse_cost_matrix_jax :152-197, _A_vmf_vec_jax :141-149,
//                               _sinkhorn_unbalanced_fixed_k_jax :105-138, tiling.py:148-186)
//
// View: one segmented stable radix sort ranks each view tile's slots by weight (invalid last,
// ties by slot), then one thread per view entry gathers it and evaluates the info-form means /
// covariances and the vMF resultant. Association: one wave per measurement row evaluates the
// cost of its whole stencil pool (n_stencil x m_tile_view candidates, 64 lanes strided), keeps a
// lane-local sorted top-K by (cost, pool position) — exactly the order of the reference's stable
// sort on cost — and merges the 64 lists with K wave-argmin rounds. The fixed-iteration unbalanced
// Sinkhorn couples all rows through the column sums, so it runs in one 1024-thread workgroup with
// fixed-order block reductions (deterministic), the N x K kernel matrix streamed from L2.
#include <hip/hip_runtime.h>
#include "gc_internal.h"
#include "gc_math.h"
#include "gc_mapslot.h"
#include "gc_sort.h"

namespace gc {
namespace {

constexpr int kMaxK = 16;          // k_assoc supported
constexpr int kMaxStencil = 128;   // n_z * n_xy stencil tiles per row
constexpr int kSinkT = 1024;       // Sinkhorn workgroup
constexpr int kMaxLobesA = 8;

struct OTCfg {
  int K, iters, row_min, wprop, r_xy, r_z;
  double beta, eps, tau_a, tau_b, eps_mass, h_tile, lam, eps_lift;
  int64_t seq;
};

// ---- view
__global__ void k_view_keys(gc_primitive_map map, int64_t m_tile, const int64_t* __restrict__ dense, int T,
                            double* keys, int32_t* vals, int* offsets) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= T) offsets[i] = (int)(i * m_tile);  // segment t = [t m_tile, (t+1) m_tile)
  if (i >= (int64_t)T * m_tile) return;
  const int t = (int)(i / m_tile);
  const int64_t s = i - (int64_t)t * m_tile;
  const int64_t d = dense[t];
  double key = 1e30;  // -score of an invalid slot (score -1e30)
  if (d >= 0) {
    const int64_t g = d * m_tile + s;
    if (mValid(map, g)) key = -mW(map, g);
  }
  keys[i] = key;
  vals[i] = (int32_t)s;
}

__global__ void k_view_gather(gc_primitive_map map, int64_t m_tile, const int64_t* __restrict__ dense,
                              const int32_t* __restrict__ order, gc_map_view V, double eps_lift, double eps_mass) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int k = V.m_tile_view;
  if (v >= (int64_t)V.n_tiles * k) return;
  const int t = (int)(v / k);
  const int j = (int)(v - (int64_t)t * k);
  const int64_t d = dense[t];
  const int32_t slot = order[(int64_t)t * m_tile + j];
  const int L = V.n_lobes;
  double Lr[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, th[3] = {0, 0, 0}, es[3] = {0, 0, 0};
  double w = 0.0, rgb[3] = {0.5, 0.5, 0.5};
  int64_t pid = 0, last = 0;
  uint8_t valid = 0;
  if (d >= 0) {
    const int64_t g = d * m_tile + slot;
    for (int q = 0; q < 9; ++q) Lr[q] = mLam(map, g)[q];
    for (int q = 0; q < 3; ++q) th[q] = mTh(map, g)[q];
    for (int l = 0; l < L; ++l) {
      for (int q = 0; q < 3; ++q) {
        const double e = mEta(map, g)[3 * l + q];
        V.etas[(v * L + l) * 3 + q] = e;
        es[q] += e;
      }
    }
    w = mW(map, g);
    pid = map.primitive_ids ? mPid(map, g) : 0;
    last = mSup(map, g);
    valid = mValid(map, g);
    if (map.rgb)
      for (int q = 0; q < 3; ++q) rgb[q] = mRgb(map, g)[q];
  } else {
    for (int q = 0; q < 3 * L; ++q) V.etas[v * 3 * L + q] = 0.0;
  }
  for (int q = 0; q < 9; q += 4) Lr[q] += eps_lift;
  double mu[3], S[9];
  solve3(Lr, th, mu);
  inv3(Lr, S);
  const double kap = sqrt(es[0] * es[0] + es[1] * es[1] + es[2] * es[2]);
  for (int q = 0; q < 3; ++q) {
    V.positions[3 * v + q] = mu[q];
    V.directions[3 * v + q] = es[q] / (kap + eps_mass);
    V.colors[3 * v + q] = rgb[q];
  }
  for (int q = 0; q < 9; ++q) V.covariances[9 * v + q] = S[q];
  V.kappas[v] = kap;
  V.weights[v] = w;
  V.primitive_ids[v] = pid;
  V.last_supported_scan_seq[v] = last;
  V.valid_mask[v] = valid;
  V.candidate_tile_ids[v] = V.tile_ids[t];
  V.candidate_slots[v] = slot;
}

// ---- association
GC_DEV double A_vmf(double k, double eps) {  // log(4π) + log sinh k - log k, stable
  k = fmax(k, eps);
  const double ls = k > 20.0 ? k - 0.69314718055994530942 : (k >= 1e-2 ? log(sinh(k)) : log(k + k * k * k / 6.0));
  return 2.5310242469692907 + ls - log(k);  // log(4π)
}

GC_DEV double ot_cost1(const double* mp, const double* md, double mk, const double* vp, const double* vd, double vk,
                       double beta) {
  const double d0 = mp[0] - vp[0], d1 = mp[1] - vp[1], d2 = mp[2] - vp[2];
  const double dpos = d0 * d0 + d1 * d1 + d2 * d2;
  const double e0 = mk * md[0] + vk * vd[0], e1 = mk * md[1] + vk * vd[1], e2 = mk * md[2] + vk * vd[2];
  const double km = 0.5 * sqrt(e0 * e0 + e1 * e1 + e2 * e2);
  const double eig = 1e-12;
  const double bc = exp(A_vmf(fmax(km, eig), eig) - 0.5 * (A_vmf(fmax(mk, eig), eig) + A_vmf(fmax(vk, eig), eig)));
  double ddir = fmax(0.0, 1.0 - bc);
  if (!(mk > 0.0 && vk > 0.0)) ddir = 0.0;
  return dpos + beta * ddir;
}

GC_DEV int64_t pack_tile(int64_t c1, int64_t c2, int64_t cz) {
  constexpr int64_t b = 1 << 20, m = (1 << 21) - 1;
  return (((c1 + b) & m) << 42) | (((c2 + b) & m) << 21) | ((cz + b) & m);
}

GC_DEV bool key_less(double ca, int pa, double cb, int pb) { return ca < cb || (ca == cb && pa < pb); }

// one wave per measurement row; 4 rows per 256-thread workgroup
__global__ void __launch_bounds__(256) k_assoc_rows(int64_t N, int L, const double* __restrict__ Lam,
                                                    const double* __restrict__ tht, const double* __restrict__ eta,
                                                    const uint8_t* __restrict__ valid, gc_map_view V, OTCfg c,
                                                    int32_t* cand_out, int64_t* ctile_out, int64_t* cslot_out,
                                                    double* cost_out, double* kmat) {
  __shared__ int st_tix[4][kMaxStencil];
  __shared__ int st_has[4][kMaxStencil];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 4 + wv;
  if (i >= N) return;  // whole wave exits together (no workgroup barrier below)
  const int K = c.K, kv = V.m_tile_view;
  // measurement mean position / direction / kappa (measurement_batch.py:389-411)
  double Lr[9], mp[3], es[3] = {0, 0, 0};
  for (int q = 0; q < 9; ++q) Lr[q] = Lam[9 * i + q] + ((q % 4 == 0) ? c.eps_lift : 0.0);
  solve3(Lr, tht + 3 * i, mp);
  for (int l = 0; l < L; ++l)
    for (int q = 0; q < 3; ++q) es[q] += eta[(i * L + l) * 3 + q];
  const double mk = sqrt(es[0] * es[0] + es[1] * es[1] + es[2] * es[2]);
  const double md[3] = {es[0] / (mk + c.eps_mass), es[1] / (mk + c.eps_mass), es[2] / (mk + c.eps_mass)};
  const bool vi = valid[i] != 0;
  // stencil tiles: z slab outer, sorted axial disk inner (primitive_association.py:307-348)
  const double h = fmax(c.h_tile, 1e-12);
  const int64_t c1 = (int64_t)floor(mp[0] / h);
  const int64_t c2 = (int64_t)floor((mp[0] * 0.5 + mp[1] * (1.7320508075688772 * 0.5)) / h);
  const int64_t cz = (int64_t)floor(mp[2] / h);
  const int r = c.r_xy;
  const int n_xy = 3 * r * (r + 1) + 1;  // hex disk size
  const int n_st = (2 * c.r_z + 1) * n_xy;
  for (int s = lane; s < n_st; s += 64) {
    const int zi = s / n_xy, xi = s - zi * n_xy;
    int qq = 0, rr = 0, cnt = 0;
    for (int q = -r; q <= r && cnt <= xi; ++q)  // xi-th entry of the sorted (q, r) disk
      for (int r2 = max(-r, -q - r); r2 <= min(r, -q + r); ++r2) {
        if (cnt == xi) { qq = q; rr = r2; }
        ++cnt;
      }
    const int64_t tid = pack_tile(c1 + qq, c2 + rr, cz + (zi - c.r_z));
    int tix = 0, has = 0;
    for (int t = 0; t < V.n_tiles; ++t)
      if (V.tile_ids[t] == tid) { tix = t; has = 1; break; }  // argmax of eq: first match
    st_tix[wv][s] = tix;
    st_has[wv][s] = has;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // lane-local top-K over the pool, ordered by (cost, pool position)
  double bc[kMaxK];
  int bp[kMaxK];
  for (int q = 0; q < kMaxK; ++q) { bc[q] = INFINITY; bp[q] = 0x7fffffff; }
  const int P = n_st * kv;
  for (int p = lane; p < P; p += 64) {
    const int s = p / kv, j = p - s * kv;
    const int64_t vix = (int64_t)st_tix[wv][s] * kv + j;
    double cst = 1e12;
    if (st_has[wv][s] && V.valid_mask[vix])
      cst = ot_cost1(mp, md, mk, V.positions + 3 * vix, V.directions + 3 * vix, V.kappas[vix], c.beta);
    if (isnan(cst)) cst = INFINITY;
    if (key_less(cst, p, bc[K - 1], bp[K - 1])) {  // insert (lists stay sorted)
      int q = K - 1;
      while (q > 0 && key_less(cst, p, bc[q - 1], bp[q - 1])) {
        bc[q] = bc[q - 1];
        bp[q] = bp[q - 1];
        --q;
      }
      bc[q] = cst;
      bp[q] = p;
    }
  }
  // merge: K rounds of wave argmin over the lane heads
  int head = 0, sel_p[kMaxK];
  for (int kk = 0; kk < K; ++kk) {
    double hc = head < K ? bc[head] : INFINITY;
    int hp = head < K ? bp[head] : 0x7fffffff;
    double mc = hc;
    int mpos = hp;
    for (int off = 32; off >= 1; off >>= 1) {
      const double oc = __shfl_xor(mc, off, 64);
      const int op = __shfl_xor(mpos, off, 64);
      if (key_less(oc, op, mc, mpos)) { mc = oc; mpos = op; }
    }
    sel_p[kk] = mpos;
    if (hp == mpos && head < K) ++head;  // pool positions are unique: exactly one lane pops
  }
  // selected candidates, their cost (recomputed as the reference does), recency, row min
  double cst = 0.0;
  int32_t cand = 0;
  if (lane < K) {
    int pp = 0;
    for (int kk = 0; kk < K; ++kk) if (kk == lane) pp = sel_p[kk];
    if (vi) {
      const int s = pp / kv, j = pp - s * kv;
      cand = st_tix[wv][s] * kv + j;
    }
    cst = ot_cost1(mp, md, mk, V.positions + 3 * (int64_t)cand, V.directions + 3 * (int64_t)cand, V.kappas[cand],
                   c.beta);
    const int64_t dt = c.seq - V.last_supported_scan_seq[cand] > 0 ? c.seq - V.last_supported_scan_seq[cand] : 0;
    cst = cst + c.eps * c.lam * (double)dt;
  }
  if (c.row_min) {
    double m = lane < K ? cst : INFINITY;
    for (int off = 32; off >= 1; off >>= 1) m = fmin(m, __shfl_xor(m, off, 64));
    cst = cst - m;
  }
  if (lane < K) {
    const int64_t o = i * K + lane;
    cand_out[o] = cand;
    ctile_out[o] = V.candidate_tile_ids[cand];
    cslot_out[o] = V.candidate_slots[cand];
    cost_out[o] = cst;
    kmat[o] = exp(-cst / fmax(c.eps, 1e-12));
  }
}

// fixed-order block reduction of NV values over kSinkT threads; result on every thread
template <int NV>
GC_DEV void block_sum_n(double (&v)[NV], double* red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    double x = v[q];
    for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
    v[q] = x;
  }
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < NV; ++q) red[wv * NV + q] = v[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    double s = 0.0;
    for (int w = 0; w < kSinkT / 64; ++w) s += red[w * NV + q];
    v[q] = s;
  }
  __syncthreads();
}

// unbalanced Sinkhorn, fixed iterations (_sinkhorn_unbalanced_fixed_k_jax) + outputs and certs
__global__ void __launch_bounds__(kSinkT) k_sinkhorn(int64_t N, const uint8_t* __restrict__ valid,
                                                     const double* __restrict__ wts, OTCfg c,
                                                     const double* __restrict__ kmat, const double* __restrict__ cost,
                                                     double* u, double* resp, double* rowm, double* cert) {
  __shared__ double red[(kSinkT / 64) * (kMaxK + 8)];
  __shared__ double vv[kMaxK];
  const int K = c.K;
  const double eps = fmax(c.eps, 1e-12);
  const double ua = 1.0 / (1.0 + c.tau_a / eps), vb = 1.0 / (1.0 + c.tau_b / eps);
  const double bk = 1.0 / (double)K;
  double s1[1] = {0.0};
  for (int64_t i = threadIdx.x; i < N; i += kSinkT)
    s1[0] += valid[i] ? (c.wprop ? wts[i] : 1.0) : 0.0;
  block_sum_n<1>(s1, red);
  const double sum_a = fmax(s1[0], c.eps_mass);
  if ((int)threadIdx.x < K) vv[threadIdx.x] = 1.0;
  __syncthreads();
  for (int it = 0; it < c.iters; ++it) {
    double cs[kMaxK];
    for (int q = 0; q < kMaxK; ++q) cs[q] = 0.0;
    for (int64_t i = threadIdx.x; i < N; i += kSinkT) {
      const double a = valid[i] ? (c.wprop ? wts[i] : 1.0) / sum_a : 0.0;
      const double* kr = kmat + i * K;
      double kvs = 0.0;
      for (int q = 0; q < K; ++q) kvs += kr[q] * vv[q];
      const double ui = pow(a / (kvs + 1e-12), ua);
      u[i] = ui;
      for (int q = 0; q < K; ++q) cs[q] += kr[q] * ui;
    }
    block_sum_n<kMaxK>(cs, red);
    if ((int)threadIdx.x < K) vv[threadIdx.x] = pow(bk / (cs[threadIdx.x] + 1e-12), vb);
    __syncthreads();
  }
  // π = u K v; responsibilities, row masses and the cert sums
  double acc[kMaxK + 7];  // [col sums (K) | transport, Σ(row - a)², Σ row², Σ max(a - row, 0), Σ π C, nonzero_a, n_valid]
  for (int q = 0; q < kMaxK + 7; ++q) acc[q] = 0.0;
  for (int64_t i = threadIdx.x; i < N; i += kSinkT) {
    const bool vi = valid[i] != 0;
    const double a = vi ? (c.wprop ? wts[i] : 1.0) / sum_a : 0.0;
    const double ui = u[i];
    double rm = 0.0, pc = 0.0;
    for (int q = 0; q < K; ++q) {
      const double pi = ui * kmat[i * K + q] * vv[q];
      resp[i * K + q] = vi ? pi : 0.0;
      acc[q] += pi;
      rm += pi;
      pc += pi * cost[i * K + q];
    }
    rowm[i] = rm;
    acc[kMaxK + 0] += rm;
    acc[kMaxK + 1] += (rm - a) * (rm - a);
    acc[kMaxK + 2] += rm * rm;
    acc[kMaxK + 3] += fmax(a - rm, 0.0);
    acc[kMaxK + 4] += pc;
    acc[kMaxK + 5] += a > c.eps_mass ? 1.0 : 0.0;
    acc[kMaxK + 6] += vi ? 1.0 : 0.0;
  }
  block_sum_n<kMaxK + 7>(acc, red);
  if (threadIdx.x == 0) {
    double db = 0.0;
    for (int q = 0; q < K; ++q) db += (acc[q] - bk) * (acc[q] - bk);
    const double tm = acc[kMaxK + 0];
    cert[0] = sqrt(acc[kMaxK + 1]);
    cert[1] = sqrt(db);
    cert[2] = tm;
    cert[3] = sum_a;
    cert[4] = (double)K * bk;
    cert[5] = tm;
    cert[6] = acc[kMaxK + 3];
    cert[7] = tm * tm / (acc[kMaxK + 2] + c.eps_mass);
    cert[8] = acc[kMaxK + 5];
    cert[9] = bk > c.eps_mass ? (double)K : 0.0;
    cert[10] = acc[kMaxK + 4];
    cert[11] = acc[kMaxK + 6];
  }
}

__global__ void k_count_u8(int64_t n, const uint8_t* __restrict__ m, unsigned long long* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // integer count: order-independent; one atomic per wave (one per element serialises on the counter)
  const unsigned long long b = __ballot(i < n && m[i] != 0);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(out, (unsigned long long)__popcll(b));
}

}  // namespace
}  // namespace gc

using namespace gc;

extern "C" {

int32_t gc_extract_map_view(gc_ctx* ctx, const gc_primitive_map* map, int64_t m_tile, const int64_t* h_dense_tiles,
                            const int64_t* h_tile_ids, double eps_lift, double eps_mass, const gc_map_view* view) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  if (int rc_j = gc::join_side(ctx)) return rc_j;
  GC_CHECK_ARG(ctx, map && view && h_dense_tiles && h_tile_ids, "NULL argument");
  {
    const char* lay_ = gc::map_layout_error(*map);
    GC_CHECK_ARG(ctx, lay_ == nullptr, lay_ ? lay_ : "");
  }
  const int T = view->n_tiles, k = view->m_tile_view;
  GC_CHECK_ARG(ctx, T >= 1 && k >= 1 && m_tile >= k && m_tile < (int64_t)INT32_MAX, "bad view shape");
  GC_CHECK_ARG(ctx, view->n_lobes == map->n_lobes && map->n_lobes <= kMaxLobesA, "n_lobes mismatch");
  GC_CHECK_ARG(ctx, map->valid_mask && map->Lambdas && map->thetas && map->etas && map->weights &&
                        map->last_supported_scan_seq,
               "NULL map field");
  for (int t = 0; t < T; ++t)
    GC_CHECK_ARG(ctx, h_dense_tiles[t] < 0 || (h_dense_tiles[t] + 1) * m_tile <= map->m_slots, "dense tile outside map");
  const int64_t n = (int64_t)T * m_tile;
  GC_CHECK_ARG(ctx, n < (int64_t)INT32_MAX, "view too large");
  const size_t temp = gc::sort_temp_bytes(T, m_tile, true);
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t bk = al(sizeof(double) * n), bv = al(sizeof(int32_t) * n), bo = al(sizeof(int) * (T + 1)),
               bd = al(sizeof(int64_t) * T);
  void* scr;
  if (int rc = gc::scratch(ctx, 2 * bk + 2 * bv + bo + bd + temp, &scr)) return rc;
  char* p = (char*)scr;
  double* keys_in = (double*)p; p += bk;
  double* keys = (double*)p; p += bk;
  int32_t* vals_in = (int32_t*)p; p += bv;
  int32_t* vals = (int32_t*)p; p += bv;
  int* offs = (int*)p; p += bo;
  int64_t* dense = (int64_t*)p; p += bd;
  void* tmp = p;
  GC_HIP(ctx, hipMemcpyAsync(dense, h_dense_tiles, sizeof(int64_t) * T, hipMemcpyHostToDevice, ctx->stream));
  GC_HIP(ctx, hipMemcpyAsync(view->tile_ids, h_tile_ids, sizeof(int64_t) * T, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_view_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, *map, m_tile,
                     (const int64_t*)dense, T, keys_in, vals_in, offs);
  GC_LAUNCH_CHECK(ctx);
  if (gc::radix_sort_pairs(ctx->stream, keys_in, keys, (const uint32_t*)vals_in, (uint32_t*)vals, T, m_tile, false,
                           tmp) != hipSuccess) {
    gc::set_error(ctx, "segmented sort failed");
    return GC_ERR_RUNTIME;
  }
  const int64_t V = (int64_t)T * k;
  hipLaunchKernelGGL(k_view_gather, dim3((unsigned)((V + 255) / 256)), dim3(256), 0, ctx->stream, *map, m_tile,
                     (const int64_t*)dense, (const int32_t*)vals, *view, eps_lift, eps_mass);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_associate_primitives_ot(gc_ctx* ctx, int64_t N, int32_t n_lobes, const double* d_Lambdas,
                                   const double* d_thetas, const double* d_etas, const double* d_weights,
                                   const uint8_t* d_valid, const gc_map_view* view, const double* h_cfg,
                                   double* d_resp_out, int32_t* d_cand_out, int64_t* d_cand_tile_out,
                                   int64_t* d_cand_slot_out, double* d_row_mass_out, double* d_cost_out,
                                   double* h_cert_out) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  if (int rc_j = gc::join_side(ctx)) return rc_j;
  GC_CHECK_ARG(ctx, view && h_cfg && h_cert_out, "NULL argument");
  GC_CHECK_ARG(ctx, N >= 1 && n_lobes >= 1 && n_lobes <= kMaxLobesA, "bad N or n_lobes");
  GC_CHECK_ARG(ctx, d_Lambdas && d_thetas && d_etas && d_valid && d_resp_out && d_cand_out && d_cand_tile_out &&
                        d_cand_slot_out && d_row_mass_out && d_cost_out,
               "NULL buffer");
  OTCfg c{};
  c.K = (int)h_cfg[0];
  c.iters = (int)h_cfg[1];
  c.beta = h_cfg[2];
  c.eps = h_cfg[3];
  c.tau_a = h_cfg[4];
  c.tau_b = h_cfg[5];
  c.row_min = h_cfg[6] != 0.0;
  c.wprop = h_cfg[7] != 0.0;
  c.eps_mass = h_cfg[8];
  c.h_tile = h_cfg[9];
  c.r_xy = (int)h_cfg[10];
  c.r_z = (int)h_cfg[11];
  c.seq = (int64_t)h_cfg[12];
  c.lam = h_cfg[13];
  c.eps_lift = h_cfg[14];
  GC_CHECK_ARG(ctx, c.K >= 1 && c.K <= kMaxK, "k_assoc must be in [1, 16]");
  GC_CHECK_ARG(ctx, c.iters >= 0 && c.r_xy >= 0 && c.r_z >= 0, "bad Sinkhorn / stencil config");
  const int n_xy = 3 * c.r_xy * (c.r_xy + 1) + 1;
  GC_CHECK_ARG(ctx, (2 * c.r_z + 1) * n_xy <= kMaxStencil, "stencil larger than 128 tiles");
  GC_CHECK_ARG(ctx, !c.wprop || d_weights, "weight_proportional needs weights");
  const int64_t V = (int64_t)view->n_tiles * view->m_tile_view;
  const int64_t pool = (2 * c.r_z + 1) * (int64_t)n_xy * view->m_tile_view;
  GC_CHECK_ARG(ctx, V >= 1 && pool >= c.K && pool < (int64_t)INT32_MAX, "bad view / pool smaller than k_assoc");
  for (int q = 0; q < GC_OT_CERT_LEN; ++q) h_cert_out[q] = 0.0;
  void* scr;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t bkm = al(sizeof(double) * N * c.K), bu = al(sizeof(double) * N), bc = al(64 * sizeof(double));
  if (int rc = gc::scratch(ctx, bkm + bu + bc + 256, &scr)) return rc;
  char* p = (char*)scr;
  double* kmat = (double*)p; p += bkm;
  double* u = (double*)p; p += bu;
  double* cert = (double*)p; p += bc;
  unsigned long long* cnt = (unsigned long long*)p;
  // the empty-input no-op (primitive_association.py:271-287) needs both valid counts
  GC_HIP(ctx, hipMemsetAsync(cnt, 0, 2 * sizeof(unsigned long long), ctx->stream));
  hipLaunchKernelGGL(k_count_u8, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, ctx->stream, N, d_valid, cnt);
  hipLaunchKernelGGL(k_count_u8, dim3((unsigned)((V + 255) / 256)), dim3(256), 0, ctx->stream, V,
                     (const uint8_t*)view->valid_mask, cnt + 1);
  GC_LAUNCH_CHECK(ctx);
  unsigned long long hc[2] = {0, 0};
  GC_HIP(ctx, hipMemcpyAsync(hc, cnt, sizeof(hc), hipMemcpyDeviceToHost, ctx->stream));
  if (int rc_w = gc::wait_stream(ctx, ctx->stream, "a result download")) return rc_w;
  if (hc[0] == 0 || hc[1] == 0) {
    const size_t nk = (size_t)N * c.K;
    GC_HIP(ctx, hipMemsetAsync(d_resp_out, 0, nk * sizeof(double), ctx->stream));
    GC_HIP(ctx, hipMemsetAsync(d_cand_out, 0, nk * sizeof(int32_t), ctx->stream));
    GC_HIP(ctx, hipMemsetAsync(d_cand_tile_out, 0, nk * sizeof(int64_t), ctx->stream));
    GC_HIP(ctx, hipMemsetAsync(d_cand_slot_out, 0, nk * sizeof(int64_t), ctx->stream));
    GC_HIP(ctx, hipMemsetAsync(d_row_mass_out, 0, (size_t)N * sizeof(double), ctx->stream));
    GC_HIP(ctx, hipMemsetAsync(d_cost_out, 0, nk * sizeof(double), ctx->stream));
    h_cert_out[11] = (double)hc[0];
    h_cert_out[12] = (double)hc[1];
    return GC_OK;
  }
  hipLaunchKernelGGL(k_assoc_rows, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, ctx->stream, N, (int)n_lobes,
                     d_Lambdas, d_thetas, d_etas, d_valid, *view, c, d_cand_out, d_cand_tile_out, d_cand_slot_out,
                     d_cost_out, kmat);
  GC_LAUNCH_CHECK(ctx);
  hipLaunchKernelGGL(k_sinkhorn, dim3(1), dim3(kSinkT), 0, ctx->stream, N, d_valid, d_weights, c,
                     (const double*)kmat, (const double*)d_cost_out, u, d_resp_out, d_row_mass_out, cert);
  GC_LAUNCH_CHECK(ctx);
  GC_HIP(ctx, hipMemcpyAsync(h_cert_out, cert, 12 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  if (int rc_w = gc::wait_stream(ctx, ctx->stream, "a result download")) return rc_w;
  h_cert_out[12] = (double)hc[1];
  return GC_OK;
}

}  // extern "C"
