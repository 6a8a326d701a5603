// gc_cloud.hip — PointCloud2 (VLP-16 layout) parsing on the device:
// parse_pointcloud2_vlp16 (backend/backend_node.py:377-468) plus the no-TF base-frame transform
// p_base = R_base_lidar p + t_base_lidar (backend_node.py:1677-1690, _parse_T_base_sensor_6d
// :247-258). The raw message bytes go to HBM once; one thread per point reads its fields at
// their byte offsets (any PointField datatype, any alignment), applies nan_to_num with the
// ±GC_NONFINITE_SENTINEL, the range-sigmoid weight, the seconds/nanoseconds time rule and the
// extrinsic, and writes the pipeline's f64/u8 arrays. Byte work, HBM-bound: point_step bytes in,
// 42 bytes out per point.
#include <hip/hip_runtime.h>
#include "gc_internal.h"
#include "gc_math.h"

struct GcExtrinsic {  // p_base = R p + t (by value into the kernel)
  double R[9];
  double t[3];
};

namespace gc {

// sensor_msgs/PointField datatypes
enum { kI8 = 1, kU8 = 2, kI16 = 3, kU16 = 4, kI32 = 5, kU32 = 6, kF32 = 7, kF64 = 8 };

// little-endian field at an arbitrary byte address, converted to f64 (numpy astype(float64))
GC_DEV double load_field(const uint8_t* p, int type) {
  switch (type) {
    case kI8: return (double)(int8_t)p[0];
    case kU8: return (double)p[0];
    case kI16: { int16_t v; __builtin_memcpy(&v, p, 2); return (double)v; }
    case kU16: { uint16_t v; __builtin_memcpy(&v, p, 2); return (double)v; }
    case kI32: { int32_t v; __builtin_memcpy(&v, p, 4); return (double)v; }
    case kU32: { uint32_t v; __builtin_memcpy(&v, p, 4); return (double)v; }
    case kF32: { float v; __builtin_memcpy(&v, p, 4); return (double)v; }
    default: { double v; __builtin_memcpy(&v, p, 8); return v; }
  }
}

// ring as numpy astype(uint8): integer fields wrap modulo 256
GC_DEV uint8_t load_ring(const uint8_t* p, int type) {
  switch (type) {
    case kI8: case kU8: return p[0];
    case kI16: case kU16: { uint16_t v; __builtin_memcpy(&v, p, 2); return (uint8_t)v; }
    case kI32: case kU32: { uint32_t v; __builtin_memcpy(&v, p, 4); return (uint8_t)v; }
    case kF32: { float v; __builtin_memcpy(&v, p, 4); return (uint8_t)(int64_t)v; }
    default: { double v; __builtin_memcpy(&v, p, 8); return (uint8_t)(int64_t)v; }
  }
}

// np.nan_to_num(x, nan=s, posinf=s, neginf=-s)
GC_DEV double nan_to_num(double x, double s) {
  if (x != x) return s;
  if (isinf(x)) return x > 0.0 ? s : -s;
  return x;
}

// any(t_raw > 1e6): one integer flag (atomicOr: order-independent, deterministic)
__global__ void k_cloud_time_flag(const uint8_t* __restrict__ data, int64_t n, int32_t step, int32_t off,
                                  int32_t type, int32_t* flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool big = false;
  if (i < n) big = load_field(data + i * step + off, type) > 1e6;
  if (__any(big) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

__global__ void k_cloud_parse(const uint8_t* __restrict__ data, int64_t n, int32_t step, int4 fx, int4 fy,
                              int4 fz_ring, int2 ftime, const int32_t* __restrict__ flag, double stamp,
                              GcExtrinsic ex, double* pts, double* t, double* w, uint8_t* ring, uint8_t* tag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* p = data + i * step;
  const double s = 1e6;  // GC_NONFINITE_SENTINEL (constants.py:257)
  const double x = nan_to_num(load_field(p + fx.x, fx.y), s);
  const double y = nan_to_num(load_field(p + fy.x, fy.y), s);
  const double z = nan_to_num(load_field(p + fz_ring.x, fz_ring.y), s);
  ring[i] = load_ring(p + fz_ring.z, fz_ring.w);
  tag[i] = 0;
  if (ftime.x >= 0) {
    const double tr = load_field(p + ftime.x, ftime.y);
    t[i] = (*flag) ? tr * 1e-9 : tr;
  } else {
    t[i] = stamp;
  }
  // range weighting in the sensor frame (backend_node.py:448-459)
  const double dist = sqrt(x * x + y * y + z * z);
  const double a = (dist - 0.5) / 0.25, b = (50.0 - dist) / 0.25;
  const double wmin = 1.0 / (1.0 + exp(-a)), wmax = 1.0 / (1.0 + exp(-b));
  w[i] = (wmin * wmax) * (1.0 - 1e-12) + 1e-12;
  // p_base = R p + t
  pts[3 * i + 0] = (ex.R[0] * x + ex.R[1] * y + ex.R[2] * z) + ex.t[0];
  pts[3 * i + 1] = (ex.R[3] * x + ex.R[4] * y + ex.R[5] * z) + ex.t[1];
  pts[3 * i + 2] = (ex.R[6] * x + ex.R[7] * y + ex.R[8] * z) + ex.t[2];
}

}  // namespace gc

namespace gc {
// the parse on stream st with a caller-owned device flag word (the pipeline's copy stream and slot)
int32_t cloud_parse_on(gc_ctx* ctx, hipStream_t st, int32_t* flag, const uint8_t* d_data, int64_t n_points,
                       int32_t point_step, const int32_t* h_fields, double header_stamp, const double* h_R9,
                       const double* h_t3, double* d_points_out, double* d_t_out, double* d_w_out,
                       uint8_t* d_ring_out, uint8_t* d_tag_out) {
  GC_CHECK_ARG(ctx, n_points >= 0 && h_fields && h_R9 && h_t3, "bad arguments");
  if (n_points == 0) return GC_OK;
  GC_CHECK_ARG(ctx, d_data && d_points_out && d_t_out && d_w_out && d_ring_out && d_tag_out, "NULL buffer");
  GC_CHECK_ARG(ctx, point_step > 0, "point_step must be positive");
  auto size_of = [](int type) { return type <= 2 ? 1 : type <= 4 ? 2 : type <= 7 ? 4 : 8; };
  for (int f = 0; f < 4; ++f) {
    const int off = h_fields[2 * f], type = h_fields[2 * f + 1];
    GC_CHECK_ARG(ctx, type >= 1 && type <= 8, "unsupported PointField datatype for x/y/z/ring");
    GC_CHECK_ARG(ctx, off >= 0 && off + size_of(type) <= point_step, "field outside point_step");
  }
  const int toff = h_fields[8], ttype = h_fields[9];
  GC_CHECK_ARG(ctx, toff < 0 || (ttype >= 1 && ttype <= 8 && toff + size_of(ttype) <= point_step),
               "bad time field");
  GC_HIP(ctx, hipMemsetAsync(flag, 0, sizeof(int32_t), st));
  const unsigned blocks = (unsigned)((n_points + 255) / 256);
  if (toff >= 0)
    hipLaunchKernelGGL(k_cloud_time_flag, dim3(blocks), dim3(256), 0, st, d_data, n_points, point_step, toff, ttype,
                       flag);
  GcExtrinsic ex;
  for (int k = 0; k < 9; ++k) ex.R[k] = h_R9[k];
  for (int k = 0; k < 3; ++k) ex.t[k] = h_t3[k];
  hipLaunchKernelGGL(k_cloud_parse, dim3(blocks), dim3(256), 0, st, d_data, n_points, point_step,
                     make_int4(h_fields[0], h_fields[1], 0, 0), make_int4(h_fields[2], h_fields[3], 0, 0),
                     make_int4(h_fields[4], h_fields[5], h_fields[6], h_fields[7]), make_int2(toff, ttype), flag,
                     header_stamp, ex, d_points_out, d_t_out, d_w_out, d_ring_out, d_tag_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}
}  // namespace gc

extern "C" int32_t gc_pointcloud2_parse(gc_ctx* ctx, const uint8_t* d_data, int64_t n_points, int32_t point_step,
                                        const int32_t* h_fields, double header_stamp, const double* h_R9,
                                        const double* h_t3, double* d_points_out, double* d_t_out,
                                        double* d_w_out, uint8_t* d_ring_out, uint8_t* d_tag_out) {
  GC_CHECK_ARG(nullptr, ctx, "NULL ctx");
  void* scr;
  if (int rc = gc::scratch(ctx, sizeof(int32_t) * 4, &scr)) return rc;
  return gc::cloud_parse_on(ctx, ctx->stream, (int32_t*)scr, d_data, n_points, point_step, h_fields, header_stamp,
                            h_R9, h_t3, d_points_out, d_t_out, d_w_out, d_ring_out, d_tag_out);
}
