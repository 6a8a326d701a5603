// gc_sort.h — the library's device radix sort (gc_sort.hip): stable, (double key, 32-bit value) pairs or
// keys alone, ascending or descending, over n_seg contiguous segments of L keys each.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace gc {
// device bytes of the temporary block radix_sort_pairs needs (ping-pong keys / values, tile counts)
size_t sort_temp_bytes(int64_t n_seg, int64_t L, bool vals);
// keys_in -> keys_out (and vals_in -> vals_out; vals_in null: keys only) on stream st; the inputs are
// not modified; n_seg * L < 2^32. Errors are launch errors (or hipErrorInvalidValue for the size).
hipError_t radix_sort_pairs(hipStream_t st, const double* keys_in, double* keys_out, const uint32_t* vals_in,
                            uint32_t* vals_out, int64_t n_seg, int64_t L, bool descending, void* temp);
}  // namespace gc
