// gc_runs.h — the deterministic reduce-by-key of the map updates (gc_map.hip, gc_scanmap.hip).
//
// K rows each target one of M map slots; the rows of a slot must be summed in a fixed order and the
// slot read-modify-written once. Instead of a global radix sort of (slot, row):
//  1. each workgroup sorts its own block of rows by (slot, local row) in LDS (bitonic), so a slot's
//     rows in the block form one contiguous run, and links the run into the slot's list:
//     next[run] = atomicExch(&head[slot], run), run = the run's global sorted position;
//  2. the one run left in head[slot] belongs to the slot's owner thread, which collects the slot's
//     runs (at most one per block), orders them by position (= block order), sums them in that order,
//     applies the slot and restores head[slot] = kNoRun.
// The order of the atomics only decides who owns a slot, never the order of the sums: results are
// bit-reproducible. Heads stay kNoRun between calls (gc_ctx::slot_head), so no pass over the M slots
// is needed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gc {

constexpr uint32_t kNoRun = 0xFFFFFFFFu;

// ascending bitonic sort of N (power of two) 64-bit keys in LDS by the whole workgroup; ends synchronised
template <int N>
__device__ __forceinline__ void lds_bitonic_sort(uint64_t* a) {
  __syncthreads();
  for (int k = 2; k <= N; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const uint64_t x = a[i], y = a[l];
          const bool up = (i & k) == 0;
          if ((x > y) == up) {
            a[i] = y;
            a[l] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}

// The runs of the list starting at `first`, in ascending order, into runs[0..n) (n returned). Lists
// longer than CAP are walked again per element (ascending selection): correct for any length, quadratic
// only past CAP runs of one slot.
template <int CAP>
struct RunList {
  uint32_t runs[CAP];
  int n = 0;
  bool spill = false;

  // max_runs: the number of blocks of the call (a slot has at most one run per block); the walk stops
  // there whatever the links hold, so no list can make a thread loop
  __device__ void collect(uint32_t first, const uint32_t* __restrict__ next, int max_runs) {
    n = 0;
    spill = false;
    for (uint32_t r = first; r != kNoRun && n < max_runs; r = next[r]) {
      if (n < CAP) runs[n] = r;
      else spill = true;
      ++n;
    }
    if (spill || n <= 1) return;
    for (int i = 1; i < n; ++i) {  // insertion sort (n is small: one run per block of the slot)
      const uint32_t v = runs[i];
      int j = i - 1;
      while (j >= 0 && runs[j] > v) {
        runs[j + 1] = runs[j];
        --j;
      }
      runs[j + 1] = v;
    }
  }

  // the i-th smallest run; with spill the i-th call in ascending i walks the list once more
  __device__ uint32_t at(int i, uint32_t first, const uint32_t* __restrict__ next, uint32_t prev) const {
    if (!spill) return runs[i];
    uint32_t best = kNoRun;
    int m = 0;
    for (uint32_t r = first; r != kNoRun && m < n; r = next[r], ++m)
      if ((i == 0 || r > prev) && r < best) best = r;
    return best;
  }
};

}  // namespace gc
