// gc_mapslot.h — slot addressing of a gc_primitive_map in either device layout (include/gcslam.h):
// the reference's per-field arrays (slot_bytes = 0) or one packed record per slot.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/gcslam.h"

namespace gc {

// slot s of a field of `width` elements
template <class T>
__host__ __device__ inline T* mslot(const gc_primitive_map& m, T* field, int64_t s, int width) {
  return m.slot_bytes ? (T*)((char*)field + s * m.slot_bytes) : field + s * (int64_t)width;
}

__host__ __device__ inline double* mLam(const gc_primitive_map& m, int64_t s) { return mslot(m, m.Lambdas, s, 9); }
__host__ __device__ inline double* mTh(const gc_primitive_map& m, int64_t s) { return mslot(m, m.thetas, s, 3); }
__host__ __device__ inline double* mEta(const gc_primitive_map& m, int64_t s) {
  return mslot(m, m.etas, s, 3 * m.n_lobes);
}
__host__ __device__ inline double& mW(const gc_primitive_map& m, int64_t s) { return *mslot(m, m.weights, s, 1); }
__host__ __device__ inline double& mTs(const gc_primitive_map& m, int64_t s) { return *mslot(m, m.timestamps, s, 1); }
__host__ __device__ inline int64_t& mSup(const gc_primitive_map& m, int64_t s) {
  return *mslot(m, m.last_supported_scan_seq, s, 1);
}
__host__ __device__ inline int64_t& mUpd(const gc_primitive_map& m, int64_t s) {
  return *mslot(m, m.last_update_scan_seq, s, 1);
}
__host__ __device__ inline double& mCam(const gc_primitive_map& m, int64_t s) { return *mslot(m, m.cam_mass, s, 1); }
__host__ __device__ inline double& mLid(const gc_primitive_map& m, int64_t s) { return *mslot(m, m.lidar_mass, s, 1); }
__host__ __device__ inline double* mAcc(const gc_primitive_map& m, int64_t s) {
  return mslot(m, m.rgb_cam_accum, s, 3);
}
__host__ __device__ inline double& mDen(const gc_primitive_map& m, int64_t s) {
  return *mslot(m, m.rgb_cam_denom, s, 1);
}
__host__ __device__ inline double* mRgb(const gc_primitive_map& m, int64_t s) { return mslot(m, m.rgb, s, 3); }
__host__ __device__ inline double* mCol(const gc_primitive_map& m, int64_t s) { return mslot(m, m.colors, s, 3); }
__host__ __device__ inline uint8_t& mValid(const gc_primitive_map& m, int64_t s) {
  return *mslot(m, m.valid_mask, s, 1);
}
__host__ __device__ inline double& mCreated(const gc_primitive_map& m, int64_t s) {
  return *mslot(m, m.created_timestamps, s, 1);
}
__host__ __device__ inline int64_t& mPid(const gc_primitive_map& m, int64_t s) {
  return *mslot(m, m.primitive_ids, s, 1);
}

// The packed record (gc_primitive_map_record_layout), in bytes. Everything the fuse reads and
// writes per touched slot (Λ, θ, w, stamp, both sequences, the camera / LiDAR masses and colour
// accumulators, η) comes first: 176 + 24 L bytes, the first two 128-B lines for L <= 3. The fields
// the fuse only writes (rgb, colors) and the maintenance fields follow on the next line.
constexpr int kRecFields = 16;
inline void map_record_layout(int n_lobes, int64_t* off, int64_t* slot_bytes) {
  auto up128 = [](int64_t b) { return (b + 127) / 128 * 128; };
  off[0] = 0;     // Lambdas 72
  off[1] = 72;    // thetas 24
  off[3] = 96;    // weights
  off[4] = 104;   // timestamps
  off[5] = 112;   // last_supported_scan_seq
  off[6] = 120;   // last_update_scan_seq
  off[7] = 128;   // cam_mass
  off[8] = 136;   // lidar_mass
  off[9] = 144;   // rgb_cam_accum 24
  off[10] = 168;  // rgb_cam_denom
  off[2] = 176;   // etas 24 L
  // rgb and colors each own a 32-B sector (24 B + pad): the fuse writes them as whole sectors, so the
  // memory controller never reads a sector back to merge a partial write (round 5: -8 MB of the C5
  // fuse's reads at 123k touched slots)
  const int64_t b2 = up128(176 + 24 * (int64_t)n_lobes);
  off[11] = b2;        // rgb 24 (+ 8 pad)
  off[12] = b2 + 32;   // colors 24 (+ 8 pad)
  off[14] = b2 + 64;   // created_timestamps
  off[15] = b2 + 72;   // primitive_ids
  off[13] = b2 + 80;   // valid_mask (1 byte)
  *slot_bytes = up128(b2 + 81);
}

// Host check of a map's layout before any kernel dereferences it: per-field arrays (slot_bytes 0),
// or exactly the packed record of map_record_layout(n_lobes) with every non-NULL field inside the
// record that Lambdas starts (a shorter slot_bytes would let a fuse write into the next slot's
// record). Returns nullptr when the layout is sound, else the reason.
inline const char* map_layout_error(const gc_primitive_map& m) {
  if (m.slot_bytes == 0) return nullptr;
  int64_t off[kRecFields], sb = 0;
  map_record_layout(m.n_lobes, off, &sb);
  if (m.slot_bytes != sb) return "slot_bytes must be 0 (per-field arrays) or gc_primitive_map_record_layout(n_lobes)";
  if (!m.Lambdas) return "NULL Lambdas";
  const char* b0 = (const char*)m.Lambdas;
  const void* f[kRecFields] = {m.Lambdas, m.thetas, m.etas, m.weights, m.timestamps, m.last_supported_scan_seq,
                               m.last_update_scan_seq, m.cam_mass, m.lidar_mass, m.rgb_cam_accum, m.rgb_cam_denom,
                               m.rgb, m.colors, m.valid_mask, m.created_timestamps, m.primitive_ids};
  const int64_t width[kRecFields] = {72, 24, 24 * (int64_t)m.n_lobes, 8, 8, 8, 8, 8, 8, 24, 8, 24, 24, 1, 8, 8};
  for (int k = 0; k < kRecFields; ++k) {
    if (!f[k]) continue;
    const int64_t d = (const char*)f[k] - b0;
    if (d < 0 || d + width[k] > sb) return "a packed field pointer lies outside its slot record";
  }
  return nullptr;
}

}  // namespace gc
