// gc_binfin.h — the a6 bin finalize shared by the split finalize kernel (gc_points.hip) and the
// evidence kernel's folded form (gc_evidence.hip): the chunk-record sums in chunk order and one bin's
// moments -> p̄, Σ_p (PSD-projected), κ (binning.py:139-209).
#pragma once
#include <hip/hip_runtime.h>
#include "gc_math.h"
#include "../../include/gcslam.h"

namespace gc {

constexpr int NF_BASE = 19;   // [1, d(3), dd(6: 00 01 02 11 12 22), p(3), pp(6)] x w
constexpr int REC_EXTRA = 4;  // [entropy_sum, max_resp, sum_w, n_points]
// k_evidence's per-bin table (64 x 16 doubles) also receives the folded finalize's summed record
// (B * NF_BASE + REC_EXTRA doubles): the fold is taken only when the record fits it (B <= 53), larger B
// keep the split finalize kernel (scan_bins_pipeline), so the sums never run into the table's neighbours
constexpr int kEvidenceTabDoubles = 64 * 16;
inline constexpr bool fold_record_fits(int B) { return B * NF_BASE + REC_EXTRA <= kEvidenceTabDoubles; }

// Chunk records of one hypothesis summed entry-wise in chunk order (the max entry by fmax), KE
// entries per thread and KU chunks per batch in flight; a ragged last batch loads zeros past the last
// chunk (+0 and fmax(·, 0) leave every entry, all >= 0 for the max, unchanged): one L2 round trip per
// batch. Entries past KE x blockDim go one chunk at a time (none at B <= 48 with the base features).
template <int KE, int KU>
GC_DEV void finalize_reduce(const double* __restrict__ P, int RL, int imax, int64_t chunks, double* sm) {
  const int nt = blockDim.x;
  int ie[KE];
  double v[KE];
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    ie[e] = threadIdx.x + e * nt;
    v[e] = 0.0;
  }
  for (int64_t c = 0; c < chunks; c += KU) {
    double x[KE][KU];
#pragma unroll
    for (int e = 0; e < KE; ++e)
#pragma unroll
      for (int u = 0; u < KU; ++u) x[e][u] = (ie[e] < RL && c + u < chunks) ? P[(c + u) * RL + ie[e]] : 0.0;
#pragma unroll
    for (int e = 0; e < KE; ++e)
#pragma unroll
      for (int u = 0; u < KU; ++u) v[e] = ie[e] == imax ? fmax(v[e], x[e][u]) : v[e] + x[e][u];
  }
#pragma unroll
  for (int e = 0; e < KE; ++e)
    if (ie[e] < RL) sm[ie[e]] = v[e];
  for (int i = threadIdx.x + KE * nt; i < RL; i += nt) {
    double w = 0.0;
    for (int64_t cc = 0; cc < chunks; ++cc) w = i == imax ? fmax(w, P[cc * RL + i]) : w + P[cc * RL + i];
    sm[i] = w;
  }
}
// One bin's finalize (binning.py:139-209): its NF summed moments a -> the GC_BIN_STATS row o
// (p̄, Σ_p PSD-projected, κ; N, s_dir, scatter and the raw sums), its projection delta and
// mass-epsilon ratio.
GC_DEV void finalize_bin(const double* a, int NF, double eps_psd, double eps_mass, double* o, double* psd_out,
                         double* er_out) {
  const double N = a[0];
  const double denom = N + eps_mass + kF64Eps;
  const double invN = 1.0 / denom, er = eps_mass / denom;
  const double sd[3] = {a[1], a[2], a[3]};
  const double Ssc[9] = {a[4], a[5], a[6], a[5], a[7], a[8], a[6], a[8], a[9]};
  const double sp[3] = {a[10], a[11], a[12]};
  const double Spp[9] = {a[13], a[14], a[15], a[14], a[16], a[17], a[15], a[17], a[18]};
  double pb[3] = {sp[0] * invN, sp[1] * invN, sp[2] * invN};
  double Sr[9], Sp[9], c6[6];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double v = Spp[3 * i + j] * invN - pb[i] * pb[j];
      if (NF > NF_BASE) v += a[NF_BASE + 3 * i + j] * invN;
      Sr[3 * i + j] = v;
    }
  // certified shortcut (as wg_psd_project_fast): Cholesky of Σ_sym - εI succeeds => the clamp
  // is inactive and the projection is Σ_sym itself (projection delta 0 up to rounding)
  {
    double S[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) S[3 * i + j] = 0.5 * (Sr[3 * i + j] + Sr[3 * j + i]);
    const double a00 = S[0] - eps_psd;
    const double l10 = S[3] / sqrt(fmax(a00, 1e-300)), l20 = S[6] / sqrt(fmax(a00, 1e-300));
    const double a11 = S[4] - eps_psd - l10 * l10;
    const double l21 = (S[7] - l20 * l10) / sqrt(fmax(a11, 1e-300));
    const double a22 = S[8] - eps_psd - l20 * l20 - l21 * l21;
    if (a00 > 0.0 && a11 > 0.0 && a22 > 0.0) {
      for (int k = 0; k < 9; ++k) Sp[k] = S[k];
      c6[0] = 0.0;
    } else {
      psd_project3(Sr, eps_psd, Sp, c6);
    }
  }
  const double Rbar = sqrt(sd[0] * sd[0] + sd[1] * sd[1] + sd[2] * sd[2]) * invN;
  const double kap = kappa_blend(Rbar, 1e-6, 3.0, 0.8, 0.03);
  o[0] = N;
  for (int k = 0; k < 3; ++k) o[1 + k] = sd[k];
  for (int k = 0; k < 9; ++k) o[4 + k] = Ssc[k];
  for (int k = 0; k < 3; ++k) o[13 + k] = pb[k];
  for (int k = 0; k < 9; ++k) o[16 + k] = Sp[k];
  o[25] = kap;
  for (int k = 0; k < 3; ++k) o[26 + k] = sp[k];
  for (int k = 0; k < 9; ++k) o[29 + k] = Spp[k];
  *psd_out = c6[0];
  *er_out = er;
}

}  // namespace gc
