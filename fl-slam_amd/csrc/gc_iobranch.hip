// gc_iobranch.hip — per-operator entries of the IMU/odom evidence branch's 11 factors
// (gc_io_factor_batch, gc_imu_vmf_gravity_tr_batch). The batched pipeline's
// branch (_compute_imu_odom_branch, backend/pipeline.py:595-776) is io_branch_wg
// (gc_iobranch_wg.h), run inside the fused bins launch. Device code: gc_iofactors.h.
#include <hip/hip_runtime.h>
#include "gc_internal.h"
#include "gc_pipe.h"
#include "gc_iofactors.h"
#include "gc_opsdev.h"

namespace gc {

constexpr int N2 = kDZ * kDZ;

// ------------------------------------------------------------------ per-operator entries
// One thread per item; each item row: in GC_IOF_IN doubles, out L 484 | h 22 | extras 16.
__global__ void k_io_factor(int kind, int H, const double* __restrict__ in, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H) return;
  const double* x = in + (int64_t)i * GC_IOF_IN;
  double* L = out + (int64_t)i * GC_IOF_OUT;
  double* hv = L + N2;
  double* ex = hv + kDZ;
  for (int k = 0; k < GC_IOF_OUT; ++k) L[k] = 0.0;
  switch (kind) {
    case GC_IOF_ODOM_QUADRATIC:
      iof_odom_quadratic(x, x + 6, x + 12, x[48], x[49], L, hv, ex);
      break;
    case GC_IOF_IMU_GYRO_ROTATION:
      iof_gyro(x, x + 3, x + 6, x + 9, x[18], x[19], x[20], x[21], L, hv, ex);
      break;
    case GC_IOF_IMU_PREINT_FACTOR:
      iof_preint(x, x + 3, x + 6, x + 9, x + 12, x + 15, x + 18, x + 21, x[30], x[31], x[32], x[33], L, hv, ex);
      break;
    case GC_IOF_PLANAR_Z_PRIOR:
      iof_scalar_prior(2, x[6] - x[2], x[7], L, hv, ex);
      break;
    case GC_IOF_VELOCITY_Z_PRIOR:
      iof_scalar_prior(8, -x[0], x[1], L, hv, ex);
      ex[0] = x[0];
      break;
    case GC_IOF_ODOM_VELOCITY:
      iof_odom_velocity(x, x + 3, x + 12, x + 15, x[24], x[25], L, hv, ex);
      break;
    case GC_IOF_ODOM_YAWRATE:
      iof_scalar_prior(5, x[1] - x[0], x[2], L, hv, ex);
      break;
    case GC_IOF_KINEMATIC:
      iof_kinematic(x, x + 6, x + 12, x + 15, x[18], x + 19, x + 28, x[37], x[38], L, hv, ex);
      break;
    case GC_IOF_IMU_DEPENDENCE:
      ex[0] = dependence_scale(fmax(x[0], 0.0), x[1]);
      break;
    case GC_IOF_ODOM_DEPENDENCE:
      ex[0] = dependence_scale(norm3(x) + norm3(x + 3), x[6]);
      break;
    default:
      break;
  }
}

__global__ void __launch_bounds__(256) k_imu_vmf_tr(int M, const double* __restrict__ rotvec,
                                                    const double* __restrict__ accel, const double* __restrict__ gyro,
                                                    const double* __restrict__ w, const double* __restrict__ ba,
                                                    double g0, double g1, double g2, double dt, double eps_psd,
                                                    double eps_mass, double* out) {
  __shared__ double sc[1024];
  __shared__ double red[8];
  const int h = blockIdx.x;
  double* L = out + (int64_t)h * GC_IOF_OUT;
  for (int k = threadIdx.x; k < GC_IOF_OUT; k += kWG) L[k] = 0.0;
  __syncthreads();
  const double g[3] = {g0, g1, g2};
  double Lr[9], hr[3];
  wg_imu_vmf_tr(M, accel, gyro, w + (int64_t)h * M, rotvec + 3 * h, ba + 3 * h, g, dt, eps_psd, eps_mass, sc, red, Lr,
                hr, L + N2 + kDZ);
  if (threadIdx.x == 0)
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) L[(3 + i) * kDZ + 3 + j] = Lr[3 * i + j];
      L[N2 + 3 + i] = hr[i];
    }
}

}  // namespace gc

extern "C" {

int32_t gc_io_factor_batch(gc_ctx* ctx, int32_t kind, int32_t H, const double* d_in, double* d_out) {
  GC_CHECK_ARG(nullptr, ctx, "NULL ctx");
  GC_CHECK_ARG(ctx, kind >= 0 && kind < GC_IOF_NKINDS, "unknown factor kind");
  GC_CHECK_ARG(ctx, H >= 0 && (H == 0 || (d_in && d_out)), "bad batch");
  if (H == 0) return GC_OK;
  hipLaunchKernelGGL(gc::k_io_factor, dim3((H + 63) / 64), dim3(64), 0, ctx->stream, kind, H, d_in, d_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_imu_vmf_gravity_tr_batch(gc_ctx* ctx, int32_t H, int32_t M, const double* d_rotvec, const double* d_accel,
                                    const double* d_gyro, const double* d_w, const double* d_ba, const double* g3,
                                    double dt_imu, double eps_psd, double eps_mass, double* d_out) {
  GC_CHECK_ARG(nullptr, ctx, "NULL ctx");
  GC_CHECK_ARG(ctx, M >= 2 && M <= 512, "IMU slots M must be in [2, 512]");
  GC_CHECK_ARG(ctx, H >= 0 && g3 && (H == 0 || (d_rotvec && d_accel && d_gyro && d_w && d_ba && d_out)), "bad batch");
  if (H == 0) return GC_OK;
  hipLaunchKernelGGL(gc::k_imu_vmf_tr, dim3(H), dim3(256), 0, ctx->stream, M, d_rotvec, d_accel, d_gyro, d_w, d_ba,
                     g3[0], g3[1], g3[2], dt_imu, eps_psd, eps_mass, d_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

}  // extern "C"
