// gc_runs.h — the deterministic reduce-by-key of the map updates (gc_map.hip, gc_scanmap.hip).
//
// K rows each target one of M map slots; the rows of a slot must be summed in a fixed order and the
// slot read-modify-written once. Instead of a global radix sort of (slot, row):
//  1. each workgroup sorts its own block of rows by (slot, local row) (bitonic, reg_bitonic_sort), so a slot's
//     rows in the block form one contiguous run, and registers the run in a row-sized open-addressing
//     hash of the touched slots (RunTable, register_run). An 8-B entry holds the slot and the last run
//     registered for it: the slot's first run claims an empty entry with one 64-bit compare-and-swap and
//     owns the slot; a later run swaps itself in as the entry's last run and links itself as its
//     predecessor's successor (succ), so the slot's runs form a chain in arrival order that starts at
//     the owner;
//  2. the owner thread (in position order: the rows a workgroup reads lie in one sort block) follows
//     the chain from its own position — succ is position-indexed, so a slot with one run (the common
//     case) costs a coalesced read and no table access — orders the runs by position (= block order),
//     sums them in that order, applies the slot, and empties its entry and the chain's links.
// The order of the atomics only decides ownership and the chain's order, never the order of the sums:
// results are bit-reproducible. The table holds 2^bits >= 4 x rows entries (load factor <= 1/4: ~1.2
// probes per claim), 4 MB for a 131k-row call, instead of the 256 B per map slot of the previous
// direct-indexed run table (256 MB at the C5 map's 2^20 slots); entries and links are zero between
// calls, so no pass over them is needed.
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

// a touched slot's entry: low word slot + 1 (0 = empty), high word position + 1 of the slot's last
// registered run; all zero when empty. succ[p]: position + 1 of the run registered after the run at
// p (0 = none), zero between calls like the entries (gc_ctx / ScanMapWork RunTableBuf).
struct RunTable {
  unsigned long long* e;  // 2^bits entries
  uint32_t* succ;         // per position
  uint32_t bits;
};

__device__ __forceinline__ uint32_t run_hash(uint32_t s, uint32_t bits) {
  return (uint32_t)(s * 2654435761u) >> (32u - bits);  // multiplicative (Fibonacci) hashing, top bits
}

// pass 1: register the run at position p with slot s (s < 2^32 - 1). Returns the slot's entry index
// when the run is the slot's first (its thread owns the slot), kNoRun otherwise.
__device__ __forceinline__ uint32_t register_run(RunTable T, uint32_t s, uint32_t p) {
  const uint32_t mask = (1u << T.bits) - 1u, key = s + 1u;
  const unsigned long long mine = ((unsigned long long)(p + 1u) << 32) | key;
  uint32_t e = run_hash(s, T.bits);
  for (uint32_t probes = 0; probes <= mask; ++probes) {
    const unsigned long long old = atomicCAS(&T.e[e], 0ull, mine);
    if (old == 0ull) return e;  // claimed: the slot's first run, no predecessor
    if ((uint32_t)old == key) {  // the slot's entry: become its last run, after the previous last
      const uint32_t prev = atomicExch(reinterpret_cast<uint32_t*>(T.e + e) + 1, p + 1u);
      T.succ[prev - 1u] = p + 1u;  // the one writer of that link this call
      return kNoRun;
    }
    e = (e + 1u) & mask;  // another slot's entry: linear probing (never full: 4 x as many entries as runs)
  }
  return kNoRun;  // unreachable
}

// pass 2, the owner: the slot's runs in ascending position order in a thread's LDS slice buf[0..CAP)
// (a register array indexed at run time would live in scratch memory). The chain is in arrival order,
// which is close to block order (blocks are dispatched in order and register their runs as they
// finish), so an insertion sort finishes an almost ascending sequence. More than CAP runs (never at
// the C5 sizes: at most one run per block, ~45 at the busiest voxel of a dense scan) fall back to a
// selection over the chain, correct for any count. clear() zeroes the chain's links after the last at().
template <int CAP>
struct SlotRunList {
  uint32_t* buf;
  uint32_t first = 0;
  uint32_t* succ = nullptr;
  int n = 0;
  bool spill = false;

  __device__ explicit SlotRunList(uint32_t* slice) : buf(slice) {}

  // the chain from the owner's position p0 (its successor link s1 already read); at most max_runs
  // links are followed (a bound for a corrupt chain)
  __device__ void collect(uint32_t p0, uint32_t s1, uint32_t* sc, int max_runs) {
    first = p0;
    succ = sc;
    buf[0] = p0;
    n = 1;
    for (uint32_t r = s1; r != 0u && n < max_runs; r = sc[r - 1]) {
      if (n < CAP) buf[n] = r - 1;
      ++n;
    }
    spill = n > CAP;
    if (!spill) {
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

  // the i-th smallest run; with spill the i-th call in ascending i walks the chain once
  __device__ uint32_t at(int i, uint32_t prev) const {
    if (!spill) return buf[i];
    uint32_t best = kNoRun;
    uint32_t r = first;
    for (int m = 0; m < n; ++m) {
      if ((i == 0 || r > prev) && r < best) best = r;
      const uint32_t nx = succ[r];
      if (nx == 0u) break;
      r = nx - 1;
    }
    return best;
  }

  // the chain's links back to zero for the next call
  __device__ void clear() const {
    if (!spill) {
      for (int i = 0; i < n; ++i) succ[buf[i]] = 0u;
      return;
    }
    uint32_t r = first;
    for (int m = 0; m < n; ++m) {
      const uint32_t nx = succ[r];
      if (nx == 0u) break;
      succ[r] = 0u;
      r = nx - 1;
    }
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
