// gc_scanmap.h — the in-scan PrimitiveMap update (gc_scanmap.hip) as the pipeline drives it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gc_internal.h"
#include "gc_pipe.h"
#include "../../include/gcslam.h"

namespace gc {

// device work buffers of one pipeline's update (sized for n_cap rows): the sorted key of every block
// position and the owner's run-hash entry, the run-piece sums and the run hash with its links
// (gc_runs.h), the apply launch's per-workgroup touched-slot counts (summed on request). The
// pipeline's own run hash (not the context's) lets the update run on a stream of its own.
struct ScanMapWork {
  RunTableBuf runs;
  void* buf = nullptr;
  size_t bytes = 0;
  uint32_t *sslot = nullptr, *rank = nullptr;
  double* pieces = nullptr;  // (n_cap, 16) the run sums, at each run's last block position
  uint32_t* wg_count = nullptr;
  int64_t n_wg = 0;  // the apply launch's workgroups
  int64_t n_cap = 0, m_slots = 0;
};

struct ScanMapInput {
  const double *pts, *t, *w;  // the scan slot's raw points (n_in, 3), times and weights
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
// the touched-slot count of the last update (downloads the per-workgroup counts; synchronises ctx->stream)
int32_t scan_map_count(gc_ctx* ctx, const ScanMapWork& W, int64_t* out, size_t* d2h_bytes);

}  // namespace gc
