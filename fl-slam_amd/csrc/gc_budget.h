// gc_budget.h — a1 PointBudgetResample statistics (point_budget.py:60-113) as workgroup-level
// device helpers, shared by the stand-alone budget kernels (gc_points.hip) and the predict
// kernel's extra workgroups in the batched pipeline (gc_belief.hip).
#pragma once
#include "gc_pipe.h"
#include "gc_wgla.h"

namespace gc {

// Partial [Σw_in, Σw_sel, Σw_sel²] of block b (of kBudgetBlocks) into part[3b..3b+2].
GC_DEV void budget_partial_block(const double* __restrict__ w, int64_t n_in, int64_t stride, int b,
                                 double* part, double* red) {
  const int64_t n_sel = (n_in + stride - 1) / stride;
  double a = 0.0, bb = 0.0, c = 0.0;
  for (int64_t i = (int64_t)b * kWG + threadIdx.x; i < n_in; i += (int64_t)kBudgetBlocks * kWG) a += w[i];
  for (int64_t j = (int64_t)b * kWG + threadIdx.x; j < n_sel; j += (int64_t)kBudgetBlocks * kWG) {
    const double v = w[j * stride];
    bb += v;
    c += v * v;
  }
  a = wg_sum(a, red);
  bb = wg_sum(bb, red);
  c = wg_sum(c, red);
  if (threadIdx.x == 0) {
    part[3 * b] = a; part[3 * b + 1] = bb; part[3 * b + 2] = c;
  }
}

// The 8 budget scalars from the partials, summed in block order (one thread).
// ess = 1 / Σ_cap (ŵ² + ε) is evaluated as (scale/(m_in+ε))² Σw_sel² + cap·ε (algebraically the
// reference's sum, point_budget.py:100-101).
GC_DEV void budget_final_values(const double* part, int64_t n_in, int64_t n_cap, int64_t stride, double* out) {
  double a = 0.0, b = 0.0, c = 0.0;
  for (int k = 0; k < kBudgetBlocks; ++k) { a += part[3 * k]; b += part[3 * k + 1]; c += part[3 * k + 2]; }
  const int64_t n_sel = (n_in + stride - 1) / stride;
  const double scale = a / (b + 1e-12);
  const double f = scale / (a + 1e-12);
  out[0] = a;
  out[1] = b;
  out[2] = scale;
  out[3] = 1.0 / (f * f * c + (double)n_cap * 1e-12);
  out[4] = scale * b;
  out[5] = (double)n_sel;
  out[6] = (double)stride;
  out[7] = fmin(1.0, (double)n_cap / ((double)n_in + 1e-12));
}

__host__ __device__ inline int64_t budget_stride(int64_t n_in, int64_t n_cap) {
  const int64_t s = (n_in + n_cap - 1) / n_cap;
  return s < 1 ? 1 : s;
}

}  // namespace gc
