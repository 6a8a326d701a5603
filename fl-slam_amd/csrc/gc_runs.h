// gc_runs.h — the deterministic reduce-by-key of the map updates (gc_map.hip, gc_scanmap.hip).
//
// K rows each target one of M map slots; the rows of a slot must be summed in a fixed order and the
// slot read-modify-written once. Instead of a global radix sort of (slot, row):
//  1. each workgroup sorts its own block of rows by (slot, local row) (bitonic, reg_bitonic_sort), so a slot's
//     rows in the block form one contiguous run, and registers the run with its slot's entry of the
//     per-slot table (register_run): rank = atomicAdd(&cnt, 1), the run's position stored inline at
//     that rank (the first kInlRuns runs) or linked into the entry's overflow list;
//  2. the run of rank 0 belongs to the slot's owner thread, which reads the slot's runs from the
//     entry (no list walk for up to kInlRuns runs), orders them by position (= block
//     order), sums them in that order, applies the slot and clears the entry.
// The order of the atomics only decides ranks and ownership, never the order of the sums: results
// are bit-reproducible. Entries stay zero between calls (gc_ctx::slot_runs), so no pass over the M
// slots is needed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gc {

constexpr uint32_t kNoRun = 0xFFFFFFFFu;

// ascending bitonic sort of N (power of two) 64-bit keys, one per thread (N == blockDim.x), held in a register:
// the compare-exchange stages between lanes of one wave (j < 64, 39 of a 512-key sort's 45) are
// register shuffles with no workgroup barrier; only the stages across waves go through LDS (a[N]).
// Returns the thread's key of the sorted order (sorted position = threadIdx.x); a is scratch.
template <int N>
__device__ __forceinline__ uint64_t reg_bitonic_sort(uint64_t x, uint64_t* a) {
  const int i = threadIdx.x;
#pragma unroll
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      uint64_t y;
      if (j >= 64) {
        a[i] = x;
        __syncthreads();
        y = a[i ^ j];
        __syncthreads();
      } else {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, j);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), j);
        y = ((uint64_t)hi << 32) | lo;
      }
      // the lower element of a pair keeps the minimum in an ascending block, the maximum otherwise
      const bool take_min = ((i & j) == 0) == ((i & k) == 0);
      x = take_min ? (x < y ? x : y) : (x < y ? y : x);
    }
  }
  return x;
}

constexpr int kInlRuns = 62;
// a slot's entry: two 128-B lines, all zero between calls. 62 inline runs hold every slot of the C5
// scans (at most one run per 256-row block: ~45 at the busiest voxel of a dense 131k-point scan), so
// the overflow list is a correctness path only.
struct alignas(256) SlotRuns {
  uint32_t cnt;             // runs registered this call
  uint32_t ovf;             // overflow list head, as position + 1 (0 = none)
  uint32_t inl[kInlRuns];   // the positions of the first kInlRuns runs, in arrival order
};
static_assert(sizeof(SlotRuns) == 256, "two lines per slot");

// pass 1: register the run at position p with slot s; returns its rank (0: p's thread will own the slot)
__device__ __forceinline__ uint32_t register_run(SlotRuns* T, uint32_t s, uint32_t p, uint32_t* ovf_next) {
  const uint32_t r = atomicAdd(&T[s].cnt, 1u);
  if (r < (uint32_t)kInlRuns) T[s].inl[r] = p;
  else ovf_next[p] = atomicExch(&T[s].ovf, p + 1u);
  return r;
}

// pass 2, the owner: the slot's runs in ascending position order in a thread's LDS slice buf[0..CAP)
// (a register array indexed at run time would live in scratch memory). The inline runs are in arrival
// order and the overflow list in reverse arrival order; arrival order is close to block order (blocks
// are dispatched in order and register their runs as they finish), so after reversing the overflow
// part the insertion sort sees an almost ascending sequence. More than CAP runs (never at the C5
// sizes: at most one run per block, ~45 at the busiest voxel of a dense scan) fall back to a
// selection over the entry and its list, correct for any count. Clears the entry.
template <int CAP>
struct SlotRunList {
  uint32_t* buf;
  const SlotRuns* e = nullptr;
  const uint32_t* next = nullptr;
  int n = 0;
  bool spill = false;

  __device__ explicit SlotRunList(uint32_t* slice) : buf(slice) {}

  __device__ void collect(SlotRuns* T, uint32_t s, const uint32_t* __restrict__ ovf_next, int max_runs) {
    e = T + s;
    next = ovf_next;
    const uint32_t cnt = e->cnt;
    n = (int)(cnt < (uint32_t)max_runs ? cnt : (uint32_t)max_runs);
    spill = n > CAP;
    if (!spill) {
      const int ni = n < kInlRuns ? n : kInlRuns;
      for (int i = 0; i < ni; ++i) buf[i] = e->inl[i];
      int m = n;
      for (uint32_t r = e->ovf; r != 0u && m > ni; r = ovf_next[r - 1]) buf[--m] = r - 1;  // reversed
      for (int i = 1; i < n; ++i) {
        const uint32_t v = buf[i];
        int j = i - 1;
        while (j >= 0 && buf[j] > v) {
          buf[j + 1] = buf[j];
          --j;
        }
        buf[j + 1] = v;
      }
    }
  }

  // the i-th smallest run; with spill the i-th call in ascending i scans the entry and its list once
  __device__ uint32_t at(int i, uint32_t prev) const {
    if (!spill) return buf[i];
    uint32_t best = kNoRun;
    for (int k = 0; k < kInlRuns && k < n; ++k) {
      const uint32_t r = e->inl[k];
      if ((i == 0 || r > prev) && r < best) best = r;
    }
    int m = kInlRuns;
    for (uint32_t r1 = e->ovf; r1 != 0u && m < n; r1 = next[r1 - 1], ++m) {
      const uint32_t r = r1 - 1;
      if ((i == 0 || r > prev) && r < best) best = r;
    }
    return best;
  }

  // after the last at(): the entry is zero for the next call
  __device__ void clear(SlotRuns* T, uint32_t s) const {
    T[s].cnt = 0u;
    T[s].ovf = 0u;
  }
};

// XCD-aware workgroup order: workgroups are dispatched round-robin over the 8 XCDs (each with its own
// L2), so consecutive workgroup ids land on different XCDs. The apply kernels' workgroups that cover
// one sort block read the same block's rows (in sorted, i.e. random row order): mapping the ids so
// that the consecutive logical workgroups of one XCD take consecutive positions keeps a block's row
// lines in one L2. A bijection on [0, 8 floor(n / 8)); the tail keeps its id.
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t n) {
  constexpr int kXcd = 8;
  const int64_t full = n / kXcd * kXcd;
  if (b >= full) return b;
  return (b % kXcd) * (full / kXcd) + b / kXcd;
}

// the apply kernels' workgroup and per-thread slice capacity: 128 x 64 x 4 B = 32 KB of LDS
constexpr int kApplyWG = 128;
constexpr int kRunCap = 64;

}  // namespace gc
