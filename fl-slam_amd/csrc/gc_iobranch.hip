// gc_iobranch.hip — the IMU/odom evidence branch on the GPU:
// _compute_imu_odom_branch (backend/pipeline.py:595-776) for every local hypothesis in one
// launch (k_io_branch, one 256-thread workgroup per hypothesis, between predict and the
// evidence kernel), and the per-operator entries of its 11 factors (gc_io_factor_batch,
// gc_imu_vmf_gravity_tr_batch). Device code: gc_iofactors.h.
#include <hip/hip_runtime.h>
#include "gc_internal.h"
#include "gc_pipe.h"
#include "gc_iofactors.h"
#include "gc_opsdev.h"

namespace gc {

constexpr int N2 = kDZ * kDZ;
constexpr int kNFac = 9;  // odom, imu, gyro, preint, planar, vz, odom_vel, odom_wz, kinematic

// LDS: factor L/h (9 x 506) | preint scratch A, Bm (256x9 each), V1, V2 (256x3) | sort scratch 1024
// | red 8 | misc 64 | extras 9 x 16
static size_t lds_io_branch() {
  return sizeof(double) * (kNFac * (N2 + kDZ) + 256 * 24 + 1024 + 8 + 64 + kNFac * kIofExtra);
}

__global__ void __launch_bounds__(256) k_io_branch(PipeDev P, ScanArgs S, const double* __restrict__ odom) {
  extern __shared__ double sm[];
  double* FL = sm;                          // factor k: L at FL + k*(N2+22), h after it
  double* A = FL + kNFac * (N2 + kDZ);
  double* Bm = A + 256 * 9;
  double* V1 = Bm + 256 * 9;
  double* V2 = V1 + 256 * 3;
  double* sc = V2 + 256 * 3;                // 1024
  double* red = sc + 1024;                  // 8
  double* misc = red + 8;                   // 64
  double* EX = misc + 64;                   // 9 x 16
  const int hl = blockIdx.x, t = threadIdx.x;
  const double* aux = P.mu_aux + (int64_t)hl * kMuAux;  // [mu_prev 22, mu_inc 22, pose0 6]
  const double* mu_prev = aux;
  const double* mu_inc = aux + 22;
  const double* pose0 = aux + 44;
  const double* pose_pred = P.pose_pred + (int64_t)hl * 6;
  const double* io = P.imu_out + (int64_t)hl * kImuOut;  // [ess, sigma_warp, dt_imu, omega 3]
  const double sigma_warp = io[1], dt_imu = io[2];
  const int M = P.M;
  for (int i = t; i < kNFac * (N2 + kDZ); i += kWG) FL[i] = 0.0;
  if (t == 0) {
    so3_exp(pose0 + 3, misc);  // R0 = Exp(rotvec0)
    // dt_int (compute_imu_integration_time, pipeline.py:262-313) computed below
  }
  // scan-to-scan window weights (unmasked: w_imu_int, pipeline.py:448-453)
  const int ia = 2 * t, ib = 2 * t + 1;
  const double ta = ia < M ? S.imu_t[ia] : 0.0, tb = ib < M ? S.imu_t[ib] : 0.0;
  const double wa = ia < M ? window_weight(ta, S.t_last, S.t_scan, sigma_warp) : 0.0;
  const double wb = ib < M ? window_weight(tb, S.t_last, S.t_scan, sigma_warp) : 0.0;
  // dt_int: Σ of the sorted in-window valid stamp intervals = max − min over them
  auto inwin = [&](double ts) { return ts > S.t_last - 1e-9 && ts <= S.t_scan + 1e-9 && ts > 0.0; };
  double cnt = 0.0, tmn = 1e308, tmx = -1e308;
  if (ia < M && inwin(ta)) { cnt += 1.0; tmn = fmin(tmn, ta); tmx = fmax(tmx, ta); }
  if (ib < M && inwin(tb)) { cnt += 1.0; tmn = fmin(tmn, tb); tmx = fmax(tmx, tb); }
  cnt = wg_sum(cnt, red);
  tmn = -wg_max(-tmn, red);
  tmx = wg_max(tmx, red);
  const double dt_int = cnt >= 2.0 ? fmax(0.0, fmin(tmx - tmn, S.t_scan - S.t_last)) : 0.0;
  __syncthreads();
  const double bg[3] = {mu_inc[9], mu_inc[10], mu_inc[11]};
  const double ba[3] = {mu_inc[12], mu_inc[13], mu_inc[14]};
  const double g[3] = {0.0, 0.0, -9.81 * P.gravity_scale};
  double* pre = misc + 16;  // kPreint = 25
  const ImuPair q = load_imu_pair(M, S.imu_t, S.imu_g, S.imu_a);
  wg_preintegrate(M, q, wa, wb, misc, bg, ba, g, A, Bm, V1, V2, pre);
  // time-resolved vMF gravity (imu_evidence.py:402-559): all threads; w = w_imu_int per slot
  {
    double* w = A;  // preint scratch is free again
    if (ia < M) w[ia] = wa;
    if (ib < M) w[ib] = wb;
    __syncthreads();
    double* F = FL + 1 * (N2 + kDZ);
    double Lr[9], hr[3];
    wg_imu_vmf_tr(M, S.imu_a, S.imu_g, w, pose_pred + 3, ba, g, dt_imu, P.eps_psd, P.eps_mass, sc, red, Lr, hr,
                  EX + 1 * kIofExtra);
    if (t == 0)
      for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) F[(3 + i) * kDZ + 3 + j] = Lr[3 * i + j];
        F[N2 + 3 + i] = hr[i];
      }
  }
  // Σ_g, Σ_a = measurement-IW modes (measurement_noise_iw_jax.py:38-56, backend_node.py:2021-2023)
  auto iw_mode = [&](int idx, double* out) {
    double Sg[9];
    const double den = P.nu_meas[idx] + 3.0 + 1.0;
    for (int k = 0; k < 9; ++k) Sg[k] = P.Psi_meas[9 * idx + k] / den;
    psd_project3_fast(Sg, P.eps_psd, out, nullptr);
  };
  const double* od_pose = odom;
  const double* od_cov = odom + 6;
  const double* tw = odom + 42;
  const double* twc = odom + 48;
  double twv[9], tww[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) { twv[3 * i + j] = twc[6 * i + j]; tww[3 * i + j] = twc[6 * (i + 3) + 3 + j]; }
  // one factor per lane of distinct waves (lanes 0, 64, 128, 192, then 1, 65, ...)
  const int lane = t & 63, wv = t >> 6;
  const int fac = (lane < 3) ? lane * 4 + wv : -1;  // 0..11
  if (fac >= 0) {
    double* F = nullptr;
    double* ex = nullptr;
    auto sel = [&](int k) { F = FL + k * (N2 + kDZ); ex = EX + k * kIofExtra; };
    switch (fac) {
      case 0:
        sel(0);
        iof_odom_quadratic<false>(pose_pred, od_pose, od_cov, P.eps_psd, P.eps_lift, F, F + N2, ex);
        break;
      case 1: {
        sel(2);
        double Sg[9], dR[9], drv[3];
        iw_mode(0, Sg);
        mat3_mul_tn(misc, pre, dR);  // R0ᵀ R_end
        so3_log(dR, drv);
        iof_gyro<false>(pose0 + 3, pose_pred + 3, drv, Sg, dt_int, P.eps_psd, P.eps_lift, P.eps_mass, F, F + N2, ex);
        break;
      }
      case 2: {
        sel(3);
        double Sa[9], dp[3], dv[3];
        iw_mode(1, Sa);
        mat3_tvec(misc, pre + 9, dp);
        mat3_tvec(misc, pre + 12, dv);
        iof_preint<false>(pose0, pose0 + 3, mu_prev + 6, pose_pred, mu_inc + 6, dv, dp, Sa, dt_int, P.eps_psd, P.eps_lift,
                   P.eps_mass, F, F + N2, ex);
        break;
      }
      case 3:
        sel(4);
        iof_scalar_prior(2, P.planar_z_ref - pose_pred[2], P.planar_z_sigma, F, F + N2, ex);
        break;
      case 4:
        sel(5);
        iof_scalar_prior(8, -mu_inc[8], P.planar_vz_sigma, F, F + N2, ex);
        ex[0] = mu_inc[8];
        break;
      case 5: {
        sel(6);
        double Rwb[9];
        so3_exp(pose_pred + 3, Rwb);
        iof_odom_velocity<false>(mu_inc + 6, Rwb, tw, twv, P.eps_psd, P.eps_lift, F, F + N2, ex);
        break;
      }
      case 6:
        sel(7);
        iof_scalar_prior(5, tw[5] - io[5], sqrt(fmax(twc[35], 1e-12)), F, F + N2, ex);
        break;
      case 7:
        sel(8);
        iof_kinematic<false>(pose0, pose_pred, tw, tw + 3, S.dt, twv, tww, P.eps_psd, P.eps_lift, F, F + N2, ex);
        break;
      default:
        break;
    }
  }
  __syncthreads();
  // dependence scalings, sum in the reference's order (pipeline.py:728-750)
  const double* ex_im = EX + 1 * kIofExtra;
  const double* ex_kc = EX + 8 * kIofExtra;
  const double si = dependence_scale(fmax(ex_im[4], 0.0), P.eps_mass);
  const double mag = norm3(ex_kc) + norm3(ex_kc + 3);
  const double so = dependence_scale(mag, P.eps_mass);
  const double sc9[kNFac] = {so, si, si, 1.0, 1.0, 1.0, so, so, 1.0};
  double* Lout = P.io_L + (int64_t)hl * N2;
  double* hout = P.io_h + (int64_t)hl * kDZ;
  for (int i = t; i < N2 + kDZ; i += kWG) {
    double v = 0.0;
    for (int k = 0; k < kNFac; ++k) v = v + FL[k * (N2 + kDZ) + i] * sc9[k];
    if (i < N2) Lout[i] = v; else hout[i - N2] = v;
  }
  if (t == 0) {
    const double* ex_od = EX;
    const double* ex_gy = EX + 2 * kIofExtra;
    const double* ex_pr = EX + 3 * kIofExtra;
    const double* ex_ov = EX + 6 * kIofExtra;
    // trigger magnitudes (certificates.py:439-455) of the 11 certs
    const double mer = ex_im[1] / (ex_im[2] + P.eps_mass);
    const double trig = ex_od[7] + (ex_im[8] + mer + fabs(1.0 - ex_im[3])) + fabs(1.0 - si) + ex_gy[4] + ex_pr[7] +
                        ex_ov[4] + ex_kc[7] + fabs(1.0 - so);
    double* c = P.io_cert + (int64_t)hl * kIoCert;
    c[0] = 0.0; c[1] = ex_im[1]; c[2] = 0.0;
    c[3] = 1.0; c[4] = ex_im[3]; c[5] = 1.0;
    c[6] = 0.0; c[7] = 0.0;
    c[8] = ex_od[6] + ex_im[7] + ex_gy[3];
    c[9] = trig;
    double* q = P.io_parts + (int64_t)hl * kIoParts;
    for (int k = 0; k < 6; ++k) q[k] = ex_od[k];
    for (int k = 0; k < 6; ++k) q[6 + k] = ex_im[k];  // kappa, ess_w, ess_raw, mean_rel, sigma, Rbar
    q[12] = si;
    for (int k = 0; k < 3; ++k) q[13 + k] = ex_gy[k];
    for (int k = 0; k < 6; ++k) q[16 + k] = ex_pr[k];
    q[22] = EX[4 * kIofExtra]; q[23] = EX[5 * kIofExtra];
    for (int k = 0; k < 3; ++k) q[24 + k] = ex_ov[k];
    q[27] = EX[7 * kIofExtra];
    for (int k = 0; k < 6; ++k) q[28 + k] = ex_kc[k];
    q[34] = so;
    q[35] = ex_od[6]; q[36] = ex_im[6]; q[37] = ex_gy[3]; q[38] = dt_int; q[39] = trig;
  }
}

hipError_t launch_io_branch(const PipeDev& P, const ScanArgs& S, const double* d_odom, hipStream_t st) {
  (void)hipFuncSetAttribute((const void*)k_io_branch, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_io_branch());
  hipLaunchKernelGGL(k_io_branch, dim3(P.Hl), dim3(256), lds_io_branch(), st, P, S, d_odom);
  return hipGetLastError();
}

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
