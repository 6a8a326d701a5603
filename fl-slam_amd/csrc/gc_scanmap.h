// gc_scanmap.h — the in-scan PrimitiveMap update (gc_scanmap.hip) as the pipeline drives it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gc_pipe.h"
#include "../../include/gcslam.h"

struct gc_ctx;

namespace gc {

// device work buffers of one pipeline's update: keys / row indices in and sorted, the rows, the
// run-piece sums, the touched-slot counter and the sort's temporary storage (sized for n_cap rows
// and the map's key width)
struct ScanMapWork {
  void* buf = nullptr;
  size_t bytes = 0;
  uint32_t *keys_in = nullptr, *vals_in = nullptr, *keys = nullptr, *vals = nullptr;
  double *rows = nullptr, *pieces = nullptr;  // (n_cap, 16) rows by row index; run-piece sums by sorted index
  unsigned long long* count = nullptr;
  void* temp = nullptr;  // radix sort temporary storage
  size_t temp_bytes = 0;
  int64_t n_cap = 0;
  int bits = 0;
};

struct ScanMapInput {
  const double *pts, *t;  // the scan slot's raw points (n_in, 3) and times
  double t0, t1;          // scan window (a4)
  double voxel;           // world voxel edge of the slot hash (m)
  double timestamp;       // scan_end (primitive_map.py:1109)
  int64_t scan_seq;
};

// gc_map.hip: rgb = clip(accum / max(denom, eps)) where cam_mass > 0 else gray; colors = rgb
hipError_t launch_fuse_colors(const gc_primitive_map& map, double eps_mass, hipStream_t st);

int32_t scan_map_prepare(gc_ctx* ctx, ScanMapWork* W, int64_t n_cap, int64_t m_slots);
int32_t scan_map_update(gc_ctx* ctx, hipStream_t st, ScanMapWork* W, const gc_primitive_map& map,
                        const PipeDev& P, const ScanMapInput& in);

}  // namespace gc
