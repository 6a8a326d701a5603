// gc_sort.hip — stable LSD radix sort of (double key, 32-bit value) pairs on the device, ascending or
// descending, over equal-length segments (one segment for a plain sort). It orders the PrimitiveMap
// maintenance keys (cull: the weight rank; insert: the replacement score; merge: the pair distances,
// primitive_map.py:1222-1229, :1037-1060, :1879-1920) and the association's per-tile map view
// (bin_atlas / association view: the top-k slots of each tile by weight), hand-written in place of a
// library radix sort.
//
// Key order: IEEE order of the doubles with -0.0 equal to +0.0 (the digits are taken from the usual
// order-preserving bit image, with the two zeros given one image), equal keys in input order (every
// pass is a stable counting sort), descending by the complemented image; the keys leave as they came
// in (bits unchanged). Eight 8-bit passes of three kernels:
//   k_sort_hist     per tile of 2048 keys: the digit histogram (LDS atomics) -> hist[seg][digit][tile]
//   k_sort_scan     per (segment, digit): the exclusive scan of its tiles' counts in place, and the total
//   k_sort_scatter  per tile: the digit bases (exclusive scan of the segment's totals + the tile's
//                   scanned count), then 8 rounds of 256 keys: a key's rank among the equal digits of
//                   its wave from 8 ballots (the lanes that agree on every digit bit), the waves' counts
//                   through LDS in wave order, so keys land in input order within each digit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gc_sort.h"

namespace gc {
namespace {

constexpr int kSortWG = 256, kSortItems = 8, kSortTile = kSortWG * kSortItems, kSortDigits = 256, kSortPasses = 8;

template <bool DESC>
__device__ __forceinline__ uint32_t sort_digit(uint64_t raw, int shift) {
  constexpr uint64_t kSign = 1ull << 63;
  uint64_t k = (raw & kSign) ? ~raw : (raw | kSign);
  if constexpr (DESC) {
    k = ~k;
    if (k == kSign) k = ~kSign;  // -0.0 -> the image of +0.0
  } else {
    if (k == ~kSign) k = kSign;
  }
  return (uint32_t)(k >> shift) & (kSortDigits - 1);
}

// exclusive scan of one value per thread over the workgroup (256 threads), the total in *tot
__device__ __forceinline__ uint32_t wg_excl_scan(uint32_t v, uint32_t* sh, uint32_t* tot) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint32_t pre = 0;
  for (int u = 0; u < w; ++u) pre += sh[u];
  const uint32_t all = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  *tot = all;
  return pre + x - v;
}

template <bool DESC>
__global__ void __launch_bounds__(kSortWG) k_sort_hist(const uint64_t* __restrict__ keys, int64_t L, int nbs,
                                                        int shift, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kSortDigits];
  const int t = threadIdx.x;
  const int64_t g = blockIdx.x / nbs, lb = blockIdx.x % nbs;
  const int64_t base = g * L + lb * kSortTile, end = (g * L + L < base + kSortTile) ? g * L + L : base + kSortTile;
  h[t] = 0u;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kSortItems; ++r) {
    const int64_t i = base + r * kSortWG + t;
    if (i < end) atomicAdd(&h[sort_digit<DESC>(keys[i], shift)], 1u);
  }
  __syncthreads();
  hist[(g * kSortDigits + t) * nbs + lb] = h[t];
}

// one workgroup per (segment, digit): its tiles' counts -> their exclusive prefix, totals[seg][digit]
__global__ void __launch_bounds__(kSortWG) k_sort_scan(uint32_t* __restrict__ hist, int nbs,
                                                        uint32_t* __restrict__ totals) {
  __shared__ uint32_t sh[4];
  uint32_t* row = hist + (int64_t)blockIdx.x * nbs;
  uint32_t run = 0;
  for (int c0 = 0; c0 < nbs; c0 += kSortWG) {
    const int c = c0 + threadIdx.x;
    const uint32_t v = c < nbs ? row[c] : 0u;
    uint32_t tot;
    const uint32_t ex = wg_excl_scan(v, sh, &tot);
    if (c < nbs) row[c] = run + ex;
    run += tot;
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = run;
}

template <bool DESC, bool VALS>
__global__ void __launch_bounds__(kSortWG) k_sort_scatter(const uint64_t* __restrict__ kin,
                                                           const uint32_t* __restrict__ vin, uint64_t* __restrict__ kout,
                                                           uint32_t* __restrict__ vout, int64_t L, int nbs, int shift,
                                                           const uint32_t* __restrict__ hist,
                                                           const uint32_t* __restrict__ totals) {
  __shared__ uint32_t dbase[kSortDigits], run[kSortDigits], wcnt[4][kSortDigits], sh[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t g = blockIdx.x / nbs, lb = blockIdx.x % nbs;
  const int64_t seg0 = g * L, base = seg0 + lb * kSortTile, end = (seg0 + L < base + kSortTile) ? seg0 + L : base + kSortTile;
  {
    uint32_t tot;
    const uint32_t ex = wg_excl_scan(totals[g * kSortDigits + t], sh, &tot);
    dbase[t] = ex + hist[(g * kSortDigits + t) * nbs + lb];
    run[t] = 0u;
  }
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int r = 0; r < kSortItems; ++r) {
    const int64_t i = base + r * kSortWG + t;
    const bool valid = i < end;
    const uint64_t key = valid ? kin[i] : 0ull;
    const uint32_t val = (VALS && valid) ? vin[i] : 0u;
    const uint32_t d = valid ? sort_digit<DESC>(key, shift) : 0u;
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const unsigned long long m = __ballot(valid && ((d >> b) & 1u));
      peers &= ((d >> b) & 1u) ? m : ~m;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & lt);
#pragma unroll
    for (int q = 0; q < 4; ++q) wcnt[q][t] = 0u;
    __syncthreads();
    if (valid && rank == 0u) wcnt[w][d] = (uint32_t)__popcll(peers);  // the group's first lane
    __syncthreads();
    if (valid) {
      uint32_t off = dbase[d] + run[d] + rank;
      for (int q = 0; q < w; ++q) off += wcnt[q][d];
      kout[seg0 + off] = key;
      if (VALS) vout[seg0 + off] = val;
    }
    __syncthreads();
    run[t] += (wcnt[0][t] + wcnt[1][t]) + (wcnt[2][t] + wcnt[3][t]);
    // the next round's zeroing follows a barrier after every read of wcnt / run above
    __syncthreads();
  }
}

}  // namespace

size_t sort_temp_bytes(int64_t n_seg, int64_t L, bool vals) {
  const int64_t nbs = (L + kSortTile - 1) / kSortTile, n = n_seg * L;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  return al(sizeof(uint64_t) * n) + (vals ? al(sizeof(uint32_t) * n) : 0) +
         al(sizeof(uint32_t) * (size_t)(n_seg * kSortDigits * nbs)) + al(sizeof(uint32_t) * (size_t)(n_seg * kSortDigits));
}

hipError_t radix_sort_pairs(hipStream_t st, const double* keys_in, double* keys_out, const uint32_t* vals_in,
                            uint32_t* vals_out, int64_t n_seg, int64_t L, bool descending, void* temp) {
  if (n_seg <= 0 || L <= 0) return hipSuccess;
  if (n_seg * L >= ((int64_t)1 << 32) || L >= ((int64_t)1 << 32)) return hipErrorInvalidValue;
  const int64_t nbs = (L + kSortTile - 1) / kSortTile, n = n_seg * L;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const bool vals = vals_in != nullptr;
  char* p = (char*)temp;
  uint64_t* kt = (uint64_t*)p; p += al(sizeof(uint64_t) * n);
  uint32_t* vt = nullptr;
  if (vals) { vt = (uint32_t*)p; p += al(sizeof(uint32_t) * n); }
  uint32_t* hist = (uint32_t*)p; p += al(sizeof(uint32_t) * (size_t)(n_seg * kSortDigits * nbs));
  uint32_t* totals = (uint32_t*)p;
  const unsigned tiles = (unsigned)(n_seg * nbs), scans = (unsigned)(n_seg * kSortDigits);
  for (int pass = 0; pass < kSortPasses; ++pass) {
    const int shift = 8 * pass;
    // even passes into the temporary buffers, odd ones into the outputs: the eighth pass ends there
    const uint64_t* ks = pass == 0 ? (const uint64_t*)keys_in : ((pass & 1) ? kt : (const uint64_t*)keys_out);
    const uint32_t* vs = pass == 0 ? vals_in : ((pass & 1) ? vt : vals_out);
    uint64_t* kd = (pass & 1) ? (uint64_t*)keys_out : kt;
    uint32_t* vd = (pass & 1) ? vals_out : vt;
    if (descending) hipLaunchKernelGGL(k_sort_hist<true>, dim3(tiles), dim3(kSortWG), 0, st, ks, L, (int)nbs, shift, hist);
    else hipLaunchKernelGGL(k_sort_hist<false>, dim3(tiles), dim3(kSortWG), 0, st, ks, L, (int)nbs, shift, hist);
    hipLaunchKernelGGL(k_sort_scan, dim3(scans), dim3(kSortWG), 0, st, hist, (int)nbs, totals);
#define GC_SCAT(D, V)                                                                                      \
  hipLaunchKernelGGL((k_sort_scatter<D, V>), dim3(tiles), dim3(kSortWG), 0, st, ks, vs, kd, vd, L, (int)nbs, shift, \
                     (const uint32_t*)hist, (const uint32_t*)totals)
    if (descending) {
      if (vals) GC_SCAT(true, true); else GC_SCAT(true, false);
    } else {
      if (vals) GC_SCAT(false, true); else GC_SCAT(false, false);
    }
#undef GC_SCAT
    if (hipError_t e = hipGetLastError()) return e;
  }
  return hipSuccess;
}

}  // namespace gc
