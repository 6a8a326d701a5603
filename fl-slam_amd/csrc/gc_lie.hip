// gc_lie.hip — the device Lie maps of gc_math.h as one batched entry (gc_lie_batch).
//
// Every kernel of the scan path reaches SO(3)/SE(3) through the same gc_math.h routines this entry
// runs: recompose and the world pose (se3_compose), anchor drift, ξ_body (se3_log), the MF δ and the
// IMU/odom residuals (so3_log). The entry exposes them on their own so the reference's fixed
// vectors (test_audit_invariants.py:224-328), including the near-π branch of so3_log
// (se3_jax.py:340-364), run on the device exactly as the pipeline evaluates them.
//
//  GC_LIE_SO3_EXP      in 3  (ω)          out 9  (R, row-major)        se3_jax.py:259-301
//  GC_LIE_SO3_LOG      in 9  (R)          out 3  (ω)                   se3_jax.py:304-366
//  GC_LIE_SE3_EXP      in 6  ([ρ, φ])     out 6  ([t, rotvec])         se3_jax.py:473-504
//  GC_LIE_SE3_LOG      in 6  ([t, rotvec]) out 6 ([ρ, φ])              se3_jax.py:220-256
//  GC_LIE_SE3_V        in 3  (φ)          out 9                        se3_jax.py:137-175
//  GC_LIE_SE3_V_INV    in 3  (φ)          out 9                        se3_jax.py:177-217
//  GC_LIE_SE3_COMPOSE  in 12 (a, b)       out 6  (a ∘ b)               se3_jax.py:420-438
//  GC_LIE_SE3_INVERSE  in 6  (a)          out 6  (a⁻¹)                 se3_jax.py:441-453
#include <hip/hip_runtime.h>
#include "gc_internal.h"
#include "gc_math.h"

namespace gc {
namespace {

constexpr int kLieIn[GC_LIE_NOPS] = {3, 9, 6, 6, 3, 3, 12, 6};
constexpr int kLieOut[GC_LIE_NOPS] = {9, 3, 6, 6, 9, 9, 6, 6};

template <int OP>
__global__ void __launch_bounds__(64) k_lie(int64_t n, const double* __restrict__ in, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  constexpr int ni = kLieIn[OP], no = kLieOut[OP];
  double a[ni], o[no];
#pragma unroll
  for (int k = 0; k < ni; ++k) a[k] = in[i * ni + k];
  if constexpr (OP == GC_LIE_SO3_EXP) so3_exp(a, o);
  else if constexpr (OP == GC_LIE_SO3_LOG) so3_log(a, o);
  else if constexpr (OP == GC_LIE_SE3_EXP) se3_exp(a, o);
  else if constexpr (OP == GC_LIE_SE3_LOG) se3_log(a, o);
  else if constexpr (OP == GC_LIE_SE3_V) se3_V(a, o);
  else if constexpr (OP == GC_LIE_SE3_V_INV) se3_V_inv(a, o);
  else if constexpr (OP == GC_LIE_SE3_COMPOSE) se3_compose(a, a + 6, o);
  else se3_inverse(a, o);
#pragma unroll
  for (int k = 0; k < no; ++k) out[i * no + k] = o[k];
}

template <int OP>
void launch(hipStream_t st, int64_t n, const double* in, double* out) {
  hipLaunchKernelGGL(k_lie<OP>, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, n, in, out);
}

}  // namespace
}  // namespace gc

extern "C" int32_t gc_lie_batch(gc_ctx* ctx, int32_t op, int64_t n, const double* d_in, double* d_out) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, op >= 0 && op < GC_LIE_NOPS, "unknown Lie op");
  GC_CHECK_ARG(ctx, n >= 0 && n <= (int64_t)0x7fffffff * 64, "n out of range");
  if (n == 0) return GC_OK;
  GC_CHECK_ARG(ctx, d_in && d_out, "NULL buffer");
  switch (op) {
    case GC_LIE_SO3_EXP: gc::launch<GC_LIE_SO3_EXP>(ctx->stream, n, d_in, d_out); break;
    case GC_LIE_SO3_LOG: gc::launch<GC_LIE_SO3_LOG>(ctx->stream, n, d_in, d_out); break;
    case GC_LIE_SE3_EXP: gc::launch<GC_LIE_SE3_EXP>(ctx->stream, n, d_in, d_out); break;
    case GC_LIE_SE3_LOG: gc::launch<GC_LIE_SE3_LOG>(ctx->stream, n, d_in, d_out); break;
    case GC_LIE_SE3_V: gc::launch<GC_LIE_SE3_V>(ctx->stream, n, d_in, d_out); break;
    case GC_LIE_SE3_V_INV: gc::launch<GC_LIE_SE3_V_INV>(ctx->stream, n, d_in, d_out); break;
    case GC_LIE_SE3_COMPOSE: gc::launch<GC_LIE_SE3_COMPOSE>(ctx->stream, n, d_in, d_out); break;
    default: gc::launch<GC_LIE_SE3_INVERSE>(ctx->stream, n, d_in, d_out); break;
  }
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

// Fail-fast test support: one thread that keeps the stream busy for `seconds` of device real time
// (s_memrealtime, 100 MHz) and then exits by itself, so a host wait with a shorter bound must time out
// while the kernel always drains (gc_test_device_spin; tests/test_gpu_failfast.py). Writes nothing.
namespace {
__global__ void k_test_spin(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
}  // namespace

extern "C" int32_t gc_test_device_spin(gc_ctx* ctx, double seconds) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, seconds >= 0.0 && seconds <= 10.0, "spin time must be in [0, 10] s");
  hipLaunchKernelGGL(k_test_spin, dim3(1), dim3(1), 0, ctx->stream, (uint64_t)(seconds * 1e8));
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}
