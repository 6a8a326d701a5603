// gc_runs.h — the deterministic reduce-by-key of the map updates (gc_map.hip, gc_scanmap.hip).
//
// K rows each target one of M map slots; the rows of a slot must be summed in a fixed order and the
// slot read-modify-written once. Instead of a global radix sort of (slot, row):
//  1. each workgroup sorts its own block of rows by (slot, local row) (bitonic, reg_bitonic_sort), so a slot's
//     rows in the block form one contiguous run, and registers the run in a row-sized open-addressing
//     hash of the touched slots (RunTable, register_run): an 8-B entry per touched slot, its slot claimed
//     by a compare-and-swap on the key word (one per slot and probe: no retry loop), the run pushed on
//     the slot's list by an exchange on the head word;
//  2. one thread per table entry (a coalesced sweep of the table, 4 B of key + 4 B of head per entry):
//     each occupied entry's thread walks the slot's list, orders the runs by position (= block order),
//     sums them in that order, applies the slot and empties the entry.
// The order of the atomics only decides the list order, never the order of the sums: results are
// bit-reproducible. The table holds 2^bits >= 4 x rows entries (load factor <= 1/4: ~1.2 probes per
// claim), 4 MB for a 131k-row call and all zero between calls: the 256 B per map slot of the previous
// direct-indexed run table (256 MB at the C5 map's 2^20 slots) and the per-position slot / rank arrays
// its owners were found by are gone.
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

// a touched slot's entry: low word slot + 1 (0 = empty), high word the head of its run list
// (position + 1 of the last registered run, 0 = none); all zero when empty
struct RunTable {
  unsigned long long* e;  // 2^bits entries
  uint32_t bits;
};

__device__ __forceinline__ uint32_t run_hash(uint32_t s, uint32_t bits) {
  return (uint32_t)(s * 2654435761u) >> (32u - bits);  // multiplicative (Fibonacci) hashing, top bits
}

// pass 1: register the run at position p with slot s (s < 2^32 - 1): claims (or finds) the slot's entry
// and pushes p on its list (next[p] = the previous head, position + 1; 0 ends the list)
__device__ __forceinline__ void register_run(RunTable T, uint32_t s, uint32_t p, uint32_t* next) {
  uint32_t* w = reinterpret_cast<uint32_t*>(T.e);
  const uint32_t mask = (1u << T.bits) - 1u, key = s + 1u;
  uint32_t e = run_hash(s, T.bits);
  for (uint32_t probes = 0; probes <= mask; ++probes) {
    const uint32_t k = atomicCAS(&w[2 * e], 0u, key);
    if (k == 0u || k == key) break;
    e = (e + 1u) & mask;  // another slot's entry: linear probing (never full: 4 x as many entries as runs)
  }
  next[p] = atomicExch(&w[2 * e + 1], p + 1u);
}

// pass 2, an occupied entry's thread: the slot's runs in ascending position order in a thread's LDS slice buf[0..CAP)
// (a register array indexed at run time would live in scratch memory). The list is in reverse arrival
// order, and arrival order is close to block order (blocks are dispatched in order and register their
// runs as they finish), so the collected positions are reversed and an insertion sort finishes an
// almost ascending sequence. More than CAP runs (never at the C5 sizes: at most one run per block,
// ~45 at the busiest voxel of a dense scan) fall back to a selection over the list, correct for any count.
template <int CAP>
struct SlotRunList {
  uint32_t* buf;
  uint32_t head = 0;
  const uint32_t* next = nullptr;
  int n = 0;
  bool spill = false;

  __device__ explicit SlotRunList(uint32_t* slice) : buf(slice) {}

  // head: the entry's low word; at most max_runs list nodes are visited (a bound for a corrupt list)
  __device__ void collect(uint32_t head_, const uint32_t* __restrict__ nxt, int max_runs) {
    head = head_;
    next = nxt;
    n = 0;
    for (uint32_t r = head; r != 0u && n < max_runs; r = nxt[r - 1]) {
      if (n < CAP) buf[n] = r - 1;
      ++n;
    }
    spill = n > CAP;
    if (!spill) {
      for (int i = 0, j = n - 1; i < j; ++i, --j) {  // arrival order
        const uint32_t x = buf[i];
        buf[i] = buf[j];
        buf[j] = x;
      }
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

  // the i-th smallest run; with spill the i-th call in ascending i walks the list once
  __device__ uint32_t at(int i, uint32_t prev) const {
    if (!spill) return buf[i];
    uint32_t best = kNoRun;
    int m = 0;
    for (uint32_t r1 = head; r1 != 0u && m < n; r1 = next[r1 - 1], ++m) {
      const uint32_t r = r1 - 1;
      if ((i == 0 || r > prev) && r < best) best = r;
    }
    return best;
  }
};

// the apply kernels' workgroup and per-thread slice capacity: 128 x 64 x 4 B = 32 KB of LDS
constexpr int kApplyWG = 128;
constexpr int kRunCap = 64;

}  // namespace gc
