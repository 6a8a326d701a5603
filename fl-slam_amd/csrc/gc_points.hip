// gc_points.hip — per-point / per-bin kernels of the GC-SLAM v2 hot path (gfx950).
//
//  a1 PointBudgetResample   backend/operators/point_budget.py:50-221
//  a4 DeskewConstantTwist   backend/operators/deskew_constant_twist.py:31-117 (+ pipeline.py:589-593)
//  a5 BinSoftAssign         archive/legacy_operators/binning.py:56-131
//  a6 ScanBinMomentMatch    archive/legacy_operators/binning.py:139-324, kappa.py:130-169
//
// Layout / mapping: a wave processes 4 points per step; its 64 lanes
// are 4 point-groups x 16 bin-lanes, bin-lane l owns bins {l, l+16, l+32, ...}. Per-point
// softmax sums are 16-lane butterflies; per-bin moment accumulators live in VGPRs for the
// whole chunk and are reduced across groups/waves once, in a fixed order, into one partial
// record per (hypothesis, chunk). A finalize kernel sums the records in chunk order, so every
// result is bit-reproducible run to run (no float atomics anywhere).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <type_traits>
#include "gc_internal.h"
#include "gc_wgla.h"
#include "gc_budget.h"
#include "gc_iobranch_wg.h"
#include "gc_binfin.h"

namespace gc {

typedef double v4d __attribute__((ext_vector_type(4)));  // f64 MFMA accumulator (4 per lane)

constexpr int NF_COV = 9;     // full 3x3 point covariance x w
// the moment kernel reads the responsibility stream exactly once: non-temporal loads for the 8-B
// per-lane tiles (A/B on one box, C3 contract launch: 1.548 -> 1.49 ms; the paired 16-B loads of bins
// 0-31 stay temporal: non-temporal there too measured 1.52, profiles/r02/ab_contract_pair_nt.txt)
#define GC_RESP_LOAD(ptr) __builtin_nontemporal_load(ptr)

// 16-lane (DPP row) butterflies: quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror,
// row_mirror. Every step pairs each lane with a distinct partner holding a disjoint partial, so
// all 16 lanes end with the bit-identical total; no LDS round trip (ds_bpermute) on the path.
template <int CTRL>
GC_DEV double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <int CTRL>
GC_DEV int dpp_i32(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;

GC_DEV double group16_sum(double v) {
  v += dpp_f64<kDppXor1>(v);
  v += dpp_f64<kDppXor2>(v);
  v += dpp_f64<kDppHalfMirror>(v);
  v += dpp_f64<kDppMirror>(v);
  return v;
}
// The same 16-lane sum for the issue-bound fused bins block, its exchanges on the LDS pipe: each
// ds_swizzle (bit mode, lane ^ XOR inside 32-lane halves) moves one 32-bit half of the partner's
// value through the LDS crossbar without touching memory, so a round costs the SIMD one f64 add
// instead of two DPP moves and an add (the block's VALU slots are its bound; the LDS pipe runs
// beside them). xor butterfly: lanes a and a ^ k add the same two partials, so all 16 lanes still
// end with the bit-identical total. GC_ZSUM: 0 = DPP (group16_sum), 1 = four swizzle rounds, 2 = two
// DPP rounds then two swizzle rounds.
#ifndef GC_ZSUM
#define GC_ZSUM 0
#endif
template <int XOR>
GC_DEV double swz_f64(double v) {
  constexpr int pat = (XOR << 10) | 0x1F;  // and_mask 0x1F, or_mask 0, xor_mask XOR
  const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), pat);
  const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), pat);
  return __hiloint2double(hi, lo);
}
GC_DEV double group16_sum_bins(double v) {
#if GC_ZSUM == 0
  return group16_sum(v);
#else
#if GC_ZSUM == 2
  v += dpp_f64<kDppXor1>(v);
  v += dpp_f64<kDppXor2>(v);
#else
  v += swz_f64<1>(v);
  v += swz_f64<2>(v);
#endif
  v += swz_f64<4>(v);
  v += swz_f64<8>(v);
  return v;
#endif
}
GC_DEV double group16_max(double v) {
  v = fmax(v, dpp_f64<kDppXor1>(v));
  v = fmax(v, dpp_f64<kDppXor2>(v));
  v = fmax(v, dpp_f64<kDppHalfMirror>(v));
  v = fmax(v, dpp_f64<kDppMirror>(v));
  return v;
}
template <int CTRL>
GC_DEV void argmax_step(double& best, int& bidx) {
  const double ob = dpp_f64<CTRL>(best);
  const int oi = dpp_i32<CTRL>(bidx);
  if (ob > best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
}
// (max, lowest index on ties) over the 16 lanes of a row
GC_DEV void group16_argmax(double& best, int& bidx) {
  argmax_step<kDppXor1>(best, bidx);
  argmax_step<kDppXor2>(best, bidx);
  argmax_step<kDppHalfMirror>(best, bidx);
  argmax_step<kDppMirror>(best, bidx);
}

// exp(x) for the softmax arguments x <= ~0 (x = (s - 1)/τ, |s| <= 1): 256-entry 2^(j/256)
// table in LDS, k = rint(x 256/ln2) by the round-to-integer magic constant (one FMA, k read
// from the low word), Cody-Waite reduction r = x - k ln2/256 (|r| <= ln2/512), degree-4 Taylor
// (truncation < 4e-17 relative), ldexp. ~12 f64 ops instead of ocml's general-range exp.
// Valid for x >= -5.8e6 (k fits in 32 bits; callers clamp).
constexpr int kExpTab = 256;
constexpr double kLn2OverTabHi = 0x1.62e42ffp-9;               // ln2/256, 24 trailing zero bits
constexpr double kLn2OverTabLo = -1.6409824502660487e-13;      // ln2/256 - hi
constexpr double kTabOverLn2 = 369.3299304675746;              // 256 / ln2
GC_DEV void exp_table_init(double* T) {  // needs blockDim.x >= 256
  if (threadIdx.x < kExpTab) T[threadIdx.x] = exp2((double)threadIdx.x / kExpTab);
}
constexpr double kRoundMagic = 6755399441055744.0;  // 1.5 * 2^52: fma(y, c, M) - M = rint(y c)
GC_DEV double exp_neg(double x, const double* T) {
  const double ks = fma(x, kTabOverLn2, kRoundMagic);  // k = rint(x 256/ln2) in the low word
  const double kf = ks - kRoundMagic;
  const int k = __double2loint(ks);
  const double r = fma(-kf, kLn2OverTabLo, fma(-kf, kLn2OverTabHi, x));
  double p = fma(r, 1.0 / 24.0, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(T[k & (kExpTab - 1)] * p, k >> 8);
}
// exp_neg over N independent arguments, phased so the N table reads are in flight together
// (one LDS round trip per step instead of one per bin). MAGIC: k by the rounding constant (one
// FMA + one add, k from the low word) instead of mul + rint + cvt; the soft-assign kernel keeps
// the rint form (its register budget at 3 waves/SIMD is tighter with the extra integer row).
template <int N, bool MAGIC = true>
GC_DEV void exp_neg_n(const double (&x)[N], const double* T, double (&out)[N]) {
  double kf[N], tv[N];
  int ki[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if constexpr (MAGIC) {
      const double ks = fma(x[j], kTabOverLn2, kRoundMagic);
      kf[j] = ks - kRoundMagic;
      ki[j] = __double2loint(ks);
    } else {
      kf[j] = rint(x[j] * kTabOverLn2);
      ki[j] = (int)kf[j];
    }
    tv[j] = T[ki[j] & (kExpTab - 1)];
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double r = fma(-kf[j], kLn2OverTabLo, fma(-kf[j], kLn2OverTabHi, x[j]));
    double p = fma(r, 1.0 / 24.0, 1.0 / 6.0);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    out[j] = ldexp(tv[j] * p, ki[j] >> 8);
  }
}
// 1/z for z > 0 in a normal range, one Newton step on the hardware reciprocal (a few ulp; the
// fused kernel's softmax normaliser, where it is one of ~140 issue slots per step)
GC_DEV double recip1(double z) {
  const double r = __builtin_amdgcn_rcp(z);
  return fma(r, fma(-z, r, 1.0), r);
}
// 1/z for z > 0 in a normal range: hardware reciprocal + two Newton steps (<= 1 ulp).
GC_DEV double recip(double z) {
  double r = __builtin_amdgcn_rcp(z);
  double e = fma(-z, r, 1.0);
  r = fma(r, e, r);
  e = fma(-z, r, 1.0);
  return fma(r, e, r);
}
// A double whose bits the compiler cannot see: two v_mov_b32 at the point of use. In a persistent
// kernel at 256 VGPRs a plain 64-bit constant is hoisted out of the task loop and spilled, and a
// polynomial then reloads each coefficient from scratch in a serial chain (the epilogue's log:
// six dependent scratch round trips per task)
template <int HI, int LO>
GC_DEV double vconst() {
  int h, l;
  asm volatile("v_mov_b32 %0, %1" : "=v"(l) : "i"(LO));
  asm volatile("v_mov_b32 %0, %1" : "=v"(h) : "i"(HI));
  return __hiloint2double(h, l);
}
// ln x for a positive normal x (the bins epilogue's log of Π Z): x = 2^k m with m in [√½, √2),
// f = m − 1, s = f/(2 + f), ln m = f − (f²/2 − s(f²/2 + R(s²))) with R the degree-7 minimax
// polynomial in s² of the classic fdlibm __ieee754_log; < 1 ulp there, within 2 ulp with the
// Newton reciprocal for 1/(2 + f). Every coefficient is a vconst.
GC_DEV double log_pos(double x) {
  int k;
  double m = frexp(x, &k);
  if (m < 0.70710678118654752440) {
    m *= 2.0;
    --k;
  }
  const double f = m - 1.0;
  const double s = f * recip(2.0 + f);
  const double z = s * s, w = z * z;
  const double t1 = w * (vconst<0x3FD99999, (int)0x9997FA04>() +
                         w * (vconst<0x3FCC71C5, 0x1D8E78AF>() + w * vconst<0x3FC39A09, (int)0xD078C69F>()));
  const double t2 = z * (vconst<0x3FE55555, 0x55555593>() +
                         w * (vconst<0x3FD24924, (int)0x94229359>() +
                              w * (vconst<0x3FC74664, (int)0x96CB03DE>() + w * vconst<0x3FC2F112, (int)0xDF3E5244>())));
  const double R = t2 + t1, hfsq = 0.5 * f * f, dk = (double)k;
  return dk * vconst<0x3FE62E42, (int)0xFEE00000>() -
         ((hfsq - (s * (hfsq + R) + dk * vconst<0x3DEA39EF, 0x35793C76>())) - f);
}
// the per-point entropy shift of the bins epilogue, (ymax ln2/2048 − B ε)/4 with ymax = ceil(2048/(τ ln2)),
// re-formed from the launch scalars each task (a loop-invariant double here is hoisted and spilled)
GC_DEV double ent_shift(double inv_tau, int B) {
  asm volatile("" : "+v"(inv_tau), "+v"(B));
  const double ymax = ceil(inv_tau * vconst<0x40A71547, 0x652B82FE>());  // 2048 / ln2
  return (ymax * vconst<0x3F362E42, (int)0xFEFA932F>() - (double)B * 1e-12) * 0.25;  // ln2 / 2048
}
// Fused-kernel exp: a 2048-entry table and arguments pre-scaled to y = x·2048/ln2. Entry j holds
// 2^(j/2048) with (j << 9) subtracted from its high word, so adding (k << 9) to the high word of
// T[k & 2047] yields 2^(j/2048)·2^(k >> 11) for any k (one integer add instead of a shift and a
// v_ldexp). r = y - rint(y) is exact (Sterbenz), |r| <= 1/2, and e^{r ln2/2048} needs only a
// cubic (truncation (ln2/4096)^4/24 = 3.5e-17). 13 VALU slots per exp with the 3-FMA logit
// (16 for exp_neg_n). Valid for y in [-2048·700/ln2, 0] (normal results).
constexpr int kExpTab2 = 2048;
constexpr double kTab2OverLn2 = 2954.6394437405970;     // 2048 / ln2
constexpr double kExp2C1 = 3.3845077175902435e-04;     // ln2 / 2048
constexpr double kExp2C2 = kExp2C1 * kExp2C1 * 0.5;
constexpr double kExp2C3 = kExp2C1 * kExp2C1 * kExp2C1 * (1.0 / 6.0);
GC_DEV void exp_table2_init(double* T) {
  for (int j = threadIdx.x; j < kExpTab2; j += blockDim.x) {
    const double v = exp2((double)j / kExpTab2);
    T[j] = __hiloint2double(__double2hiint(v) - (j << 9), __double2loint(v));
  }
}
// The table formed once per context on the device (gc_ctx_create -> init_exp_table) by the same
// exp_table2_init the workgroups used to run themselves: a workgroup now copies 16 KB from L2 instead
// of evaluating 2048 exp2 (~2 us at the start of every bins launch), the same bits.
__device__ __attribute__((aligned(16))) double g_exp_tab2[kExpTab2];
__global__ void __launch_bounds__(256) k_exp_table_init() { exp_table2_init(g_exp_tab2); }
GC_DEV void exp_table2_load(double* T) {
  typedef double dvec2 __attribute__((ext_vector_type(2)));
  for (int j = threadIdx.x; j < kExpTab2 / 2; j += blockDim.x)
    reinterpret_cast<dvec2*>(T)[j] = reinterpret_cast<const dvec2*>(g_exp_tab2)[j];
}
hipError_t init_exp_table(hipStream_t st) {
  hipLaunchKernelGGL(k_exp_table_init, dim3(1), dim3(256), 0, st);
  return hipGetLastError();
}
template <int N>
GC_DEV void exp2s_n(const double (&y)[N], const double* T, double (&out)[N]) {
  double r[N], tv[N];
  int ki[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double ks = y[j] + kRoundMagic;
    ki[j] = __double2loint(ks);
    r[j] = y[j] - (ks - kRoundMagic);
    tv[j] = T[ki[j] & (kExpTab2 - 1)];
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double p = fma(fma(fma(kExp2C3, r[j], kExp2C2), r[j], kExp2C1), r[j], 1.0);
    const double t = __hiloint2double(__double2hiint(tv[j]) + (ki[j] << 9), __double2loint(tv[j]));
    out[j] = t * p;
  }
}
// exp2s_n of y - m for an integer-valued shift m (Mp = kRoundMagic - m): ks = y + Mp rounds to
// Mp + rint(y), so r = y - (ks - Mp) = y - rint(y) exactly and lo(ks) = rint(y) - m. The shift rides
// in the rounding constant, so the fused logit needs no "- ymax" term of its own.
template <int N>
GC_DEV void exp2s_shift_n(const double (&y)[N], double Mp, const double* T, double (&out)[N]) {
  double r[N], tv[N];
  int ki[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double ks = y[j] + Mp;
    ki[j] = __double2loint(ks);
    r[j] = y[j] - (ks - Mp);
    tv[j] = T[ki[j] & (kExpTab2 - 1)];
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double p = fma(fma(fma(kExp2C3, r[j], kExp2C2), r[j], kExp2C1), r[j], 1.0);
    const double t = __hiloint2double(__double2hiint(tv[j]) + (ki[j] << 9), __double2loint(tv[j]));
    out[j] = t * p;
  }
}
// exp2s_shift_n reading the table at a fixed LDS byte address TAB. The kernels calling this have no
// static LDS (their dynamic block starts at address 0; the launchers check it, ensure_no_static_lds), so
// the table base folds into the ds_read's immediate offset: the entry's address is (k & 2047) << 3
// with no add of a relocated base per exp. Same values as exp2s_shift_n.
typedef const __attribute__((address_space(3))) char* lds_cptr;
template <int N, unsigned TAB>
GC_DEV void exp2s_shift_tab_n(const double (&y)[N], double Mp, double (&out)[N]) {
  double r[N], tv[N];
  int ki[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double ks = y[j] + Mp;
    ki[j] = __double2loint(ks);
    r[j] = y[j] - (ks - Mp);
    tv[j] = *reinterpret_cast<const __attribute__((address_space(3))) double*>(
        reinterpret_cast<lds_cptr>((uintptr_t)TAB) + ((unsigned)(ki[j] & (kExpTab2 - 1)) << 3));
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double p = fma(fma(fma(kExp2C3, r[j], kExp2C2), r[j], kExp2C1), r[j], 1.0);
    const double t = __hiloint2double(__double2hiint(tv[j]) + (ki[j] << 9), __double2loint(tv[j]));
    out[j] = t * p;
  }
}
// σ(x) = 1 / (1 + e^{-x}) on the 2048 table (e^{-|x|} clamped at e^{-700} ~ 1e-304)
GC_DEV double sigmoid2(double x, const double* T) {
  const double y[1] = {fmax(-fabs(x), -700.0) * kTab2OverLn2};
  double e[1];
  exp2s_n<1>(y, T, e);
  const double r = recip(1.0 + e[0]);
  return x >= 0.0 ? r : e[0] * r;
}


GC_DEV void lds_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Un-fused similarity: the bin-index integer contract (argmax of exactly this f64 expression).
GC_DEV double sim_nofma(double d0, double d1, double d2, double b0, double b1, double b2) {
#pragma clang fp contract(off)
  double s = d0 * b0 + d1 * b1;
  s = s + d2 * b2;
  return s;
}

// Fused-kernel variants of the three per-point helpers: reciprocals (hardware rcp + 2 Newton
// steps, <= 1 ulp) instead of IEEE divisions and the LDS-table exp in the window sigmoid.
// Results agree with the exact forms to a few ulps; they feed only floating-point moments
// (the bit-exact bin-index contract runs through direction() / k_point_dirs).
GC_DEV void deskew_point_fast(const double* p, double alpha, const double* xi, double* out) {
  const double rho[3] = {alpha * xi[0], alpha * xi[1], alpha * xi[2]};
  const double phi[3] = {alpha * xi[3], alpha * xi[4], alpha * xi[5]};
  const double ts = dot3(phi, phi);
  const double th = sqrt(ts);
  double Bv, Cv, a, b;
  if (th < kSmallAngle) {
    Bv = 0.5 - ts * (1.0 / 24.0);
    Cv = 1.0 / 6.0 - ts * (1.0 / 120.0);
    a = 1.0;
    b = 0.5;
  } else {
    double sn, c;
    sincos(th, &sn, &c);
    const double its = recip((ts < kSmallAngle * kSmallAngle) ? 1.0 : ts);
    const double ith = recip(th);
    Bv = (1.0 - c) * its;
    Cv = (th - sn) * its * ith;
    a = sn * ith;
    b = Bv;
  }
  double V[9], R[9], t[3], q[3];
  rodrigues_form(phi, Bv, Cv, V);
  mat3_vec(V, rho, t);
  rodrigues_form(phi, a, b, R);
  q[0] = p[0] - t[0]; q[1] = p[1] - t[1]; q[2] = p[2] - t[2];
  mat3_tvec(R, q, out);
}
// Series form for the fused kernel: a = sin θ/θ, B = (1 - cos θ)/θ², C = (θ - sin θ)/θ³ are
// power series in θ² (1/(2k+1)!, 1/(2k+2)!, 1/(2k+3)! of (-θ²)^k); ten terms reach < 1e-17 for
// θ² <= 1 — three independent Horner chains instead of sqrt + sincos + two reciprocals. Larger
// rotations (|α ω| > 1 rad within one scan) take the sincos form.
constexpr double kInvFact[22] = {1.0, 1.0, 0.5, 0.16666666666666666, 0.041666666666666664, 0.008333333333333333, 0.001388888888888889, 0.0001984126984126984, 2.48015873015873e-05, 2.7557319223985893e-06, 2.755731922398589e-07, 2.505210838544172e-08, 2.08767569878681e-09, 1.6059043836821613e-10, 1.1470745597729725e-11, 7.647163731819816e-13, 4.779477332387385e-14, 2.8114572543455206e-15, 1.5619206968586225e-16, 8.22063524662433e-18, 4.110317623312165e-19, 1.9572941063391263e-20};
GC_DEV void deskew_point_series(const double* p, double alpha, const double* xi, double* out) {
  const double phi[3] = {alpha * xi[3], alpha * xi[4], alpha * xi[5]};
  const double ts = dot3(phi, phi);
  if (ts > 1.0) {
    deskew_point_fast(p, alpha, xi, out);
    return;
  }
  const double rho[3] = {alpha * xi[0], alpha * xi[1], alpha * xi[2]};
  const double u = -ts;
  double a = kInvFact[19], Bv = kInvFact[20], Cv = kInvFact[21];
#pragma unroll
  for (int k = 8; k >= 0; --k) {
    a = fma(a, u, kInvFact[2 * k + 1]);
    Bv = fma(Bv, u, kInvFact[2 * k + 2]);
    Cv = fma(Cv, u, kInvFact[2 * k + 3]);
  }
  double V[9], R[9], t[3], q[3];
  rodrigues_form(phi, Bv, Cv, V);
  mat3_vec(V, rho, t);
  rodrigues_form(phi, a, Bv, R);
  q[0] = p[0] - t[0]; q[1] = p[1] - t[1]; q[2] = p[2] - t[2];
  mat3_tvec(R, q, out);
}
// Fused-kernel deskew in cross-product form: V ρ = ρ + B φ×ρ + C φ×(φ×ρ) and Rᵀ q = q − a φ×q + B φ×(φ×q)
// (the same Rodrigues matrices applied as vectors: 4 cross products instead of two 3x3 forms and two
// matrix-vector products). SHORT: the series for θ² <= kDeskewShortTs (six terms, first omitted term
// < 1e-18 relative), chosen wave-uniformly by the caller; otherwise ten terms (θ² <= 1), and the
// sincos form beyond.
constexpr double kDeskewShortTs = 0.04;
template <bool SHORT>
GC_DEV void deskew_point_cross(const double* p, double alpha, const double* xi, double* out) {
  const double phi[3] = {alpha * xi[3], alpha * xi[4], alpha * xi[5]};
  const double ts = dot3(phi, phi);
  if (!SHORT && ts > 1.0) {
    deskew_point_fast(p, alpha, xi, out);
    return;
  }
  const double rho[3] = {alpha * xi[0], alpha * xi[1], alpha * xi[2]};
  const double u = -ts;
  constexpr int K = SHORT ? 5 : 9;  // highest power of θ² kept
  double a = kInvFact[2 * K + 1], Bv = kInvFact[2 * K + 2], Cv = kInvFact[2 * K + 3];
#pragma unroll
  for (int k = K - 1; k >= 0; --k) {
    a = fma(a, u, kInvFact[2 * k + 1]);
    Bv = fma(Bv, u, kInvFact[2 * k + 2]);
    Cv = fma(Cv, u, kInvFact[2 * k + 3]);
  }
  double c1[3], c2[3], q[3];
  cross3(phi, rho, c1);
  cross3(phi, c1, c2);
#pragma unroll
  for (int k = 0; k < 3; ++k) q[k] = p[k] - fma(Cv, c2[k], fma(Bv, c1[k], rho[k]));
  cross3(phi, q, c1);
  cross3(phi, c1, c2);
#pragma unroll
  for (int k = 0; k < 3; ++k) out[k] = fma(Bv, c2[k], fma(-a, c1[k], q[k]));
}
// point_features with w folded into the first factor of each product (w d_i d_j as (w d_i) d_j)
GC_DEV void point_features_w(const double* p, const double* d, double w, double* f) {
  const double wd[3] = {w * d[0], w * d[1], w * d[2]};
  const double wp[3] = {w * p[0], w * p[1], w * p[2]};
  f[0] = w;
  f[1] = wd[0]; f[2] = wd[1]; f[3] = wd[2];
  f[4] = wd[0] * d[0]; f[5] = wd[0] * d[1]; f[6] = wd[0] * d[2];
  f[7] = wd[1] * d[1]; f[8] = wd[1] * d[2]; f[9] = wd[2] * d[2];
  f[10] = wp[0]; f[11] = wp[1]; f[12] = wp[2];
  f[13] = wp[0] * p[0]; f[14] = wp[0] * p[1]; f[15] = wp[0] * p[2];
  f[16] = wp[1] * p[1]; f[17] = wp[1] * p[2]; f[18] = wp[2] * p[2];
}
GC_DEV void direction_fast(const double* p, const double* o, double eps, double* d) {
  const double r0 = p[0] - o[0], r1 = p[1] - o[1], r2 = p[2] - o[2];
  const double inv = recip(sqrt(r0 * r0 + r1 * r1 + r2 * r2) + eps);
  d[0] = r0 * inv; d[1] = r1 * inv; d[2] = r2 * inv;
}
// σ(x) = 1 / (1 + e^{-x}) from e = exp(-|x|) (table exp; arguments below -745 underflow to 0)
GC_DEV double sigmoid_fast(double x, const double* T) {
  const double e = exp_neg(fmax(-fabs(x), -800.0), T);
  const double r = recip(1.0 + e);
  return x >= 0.0 ? r : e * r;
}
GC_DEV double window_weight_fast(double t, double t0, double t1, double inv_sig, const double* T) {
  const double wr = sigmoid_fast((t - t0) * inv_sig, T) * sigmoid_fast((t1 - t) * inv_sig, T);
  return wr * (1.0 - 1e-12) + 1e-12;
}

GC_DEV double window_weight2(double t, double t0, double t1, double inv_sig, const double* T) {
  const double wr = sigmoid2((t - t0) * inv_sig, T) * sigmoid2((t1 - t) * inv_sig, T);
  return wr * (1.0 - 1e-12) + 1e-12;
}

// Features g (pre-multiplied by w) for the moment sums of binning.py:160-173.
GC_DEV void point_features(const double* p, const double* d, double w, double* f) {
  f[0] = w;
  f[1] = w * d[0]; f[2] = w * d[1]; f[3] = w * d[2];
  f[4] = w * (d[0] * d[0]); f[5] = w * (d[0] * d[1]); f[6] = w * (d[0] * d[2]);
  f[7] = w * (d[1] * d[1]); f[8] = w * (d[1] * d[2]); f[9] = w * (d[2] * d[2]);
  f[10] = w * p[0]; f[11] = w * p[1]; f[12] = w * p[2];
  f[13] = w * (p[0] * p[0]); f[14] = w * (p[0] * p[1]); f[15] = w * (p[0] * p[2]);
  f[16] = w * (p[1] * p[1]); f[17] = w * (p[1] * p[2]); f[18] = w * (p[2] * p[2]);
}


// =============================================================================== a1 budget
// Two-level deterministic reduction: 64 workgroups write [Σw_in, Σw_sel, Σw_sel²] partials, one
// thread finishes (gc_budget.h).
__global__ void __launch_bounds__(256) k_budget_partials(const double* __restrict__ w, int64_t n_in,
                                                         int64_t stride, double* part) {
  __shared__ double red[4];
  budget_partial_block(w, n_in, stride, blockIdx.x, part, red);
}

__global__ void k_budget_final(const double* __restrict__ part, int64_t n_in, int64_t n_cap, int64_t stride,
                               double* out) {
  if (threadIdx.x != 0) return;
  budget_final_values(part, n_in, n_cap, stride, out);
}

__global__ void k_budget_gather(const double* __restrict__ pts, const double* __restrict__ t,
                                const double* __restrict__ w, const uint8_t* __restrict__ ring,
                                const uint8_t* __restrict__ tag, int64_t n_in, int64_t n_cap,
                                int64_t stride, const double* __restrict__ scal, double* pts_o,
                                double* t_o, double* w_o, uint8_t* ring_o, uint8_t* tag_o,
                                int64_t* idx_o) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_cap) return;
  const int64_t n_sel = (n_in + stride - 1) / stride;
  const bool sel = j < n_sel;
  const int64_t i = j * stride;
  pts_o[3 * j + 0] = sel ? pts[3 * i + 0] : 0.0;
  pts_o[3 * j + 1] = sel ? pts[3 * i + 1] : 0.0;
  pts_o[3 * j + 2] = sel ? pts[3 * i + 2] : 0.0;
  t_o[j] = sel ? t[i] : 0.0;
  w_o[j] = sel ? w[i] * scal[2] : 0.0;
  if (ring_o) ring_o[j] = (sel && ring) ? ring[i] : 0;
  if (tag_o) tag_o[j] = (sel && tag) ? tag[i] : 0;
  if (idx_o) idx_o[j] = sel ? i : -1;
}

// ============================================================================== a4 deskew
__global__ void __launch_bounds__(256) k_deskew(int64_t n, const double* __restrict__ pts,
                                                const double* __restrict__ t,
                                                const double* __restrict__ w, double t0, double t1,
                                                const double* __restrict__ xi, double* pts_o,
                                                double* w_o, double* partial) {
  __shared__ double red[4];
  const int h = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * kWG + threadIdx.x;
  double xr[6];
  for (int k = 0; k < 6; ++k) xr[k] = xi[6 * h + k];
  const double denom = fmax(t1 - t0, 1e-12);
  double wo = 0.0;
  if (j < n) {
    const double p[3] = {pts[3 * j], pts[3 * j + 1], pts[3 * j + 2]};
    const double alpha = (t[j] - t0) / denom;
    double q[3];
    deskew_point(p, alpha, xr, q);
    wo = w[j] * window_weight(t[j], t0, t1, 0.1 * denom);
    const int64_t o = (int64_t)h * n + j;
    pts_o[3 * o] = q[0]; pts_o[3 * o + 1] = q[1]; pts_o[3 * o + 2] = q[2];
    w_o[o] = wo;
  }
  const double s = wg_sum(wo, red);
  if (threadIdx.x == 0) partial[(int64_t)h * gridDim.x + blockIdx.x] = s;
}

// out[h] = Σ_c partial[h][c] (fixed order)
__global__ void k_sum_rows(const double* __restrict__ partial, int64_t cols, int rows, double* out) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= rows) return;
  double s = 0.0;
  for (int64_t c = 0; c < cols; ++c) s += partial[(int64_t)h * cols + c];
  out[h] = s;
}

__global__ void k_point_dirs(int64_t rows, const double* __restrict__ pts, double o0, double o1,
                             double o2, double eps, double* dirs) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= rows) return;
  const double p[3] = {pts[3 * j], pts[3 * j + 1], pts[3 * j + 2]};
  const double o[3] = {o0, o1, o2};
  double d[3];
  direction(p, o, eps, d);
  dirs[3 * j] = d[0]; dirs[3 * j + 1] = d[1]; dirs[3 * j + 2] = d[2];
}

// ============================================================================ a5 soft assign
// grid (chunks, H), chunk = iters*256 points; each wave owns 64 points per iteration with
// lane = point: the 16*BPL similarities, exps and the softmax sum of a point stay in one lane
// (no cross-lane reductions) and the bin directions are wave-uniform LDS reads.
// The bin index is a running argmax in bin order (lowest index on ties).
// FULL (B == 16 BPL <= 48): the normalised rows leave through a wave-private LDS slab one half-wave at a
// time: 32 rows of B doubles (row stride B + 2: the 8 lanes of a ds_write_b128 group hit disjoint
// banks) go out as the contiguous 32·B·8-byte block they form in HBM, 16 B per lane, 1 KiB per store
// instruction. Ragged B and B = 64: the rows are transposed one 16-bin block at a time (row stride 18) and leave
// as 128-B row segments, 8 B per lane.
// One 16-bin block of a wave's 64 normalised rows, from the LDS transpose slab (row stride 18) to
// HBM as 128-B row segments: 16 B per lane (FULL, B == 16 BPL) or 8 B per lane (ragged B).
template <int BPL, bool FULL>
GC_DEV void sa_store_block(const double* S, double* Rh, int64_t wbase, int64_t n, int B, int blk, int lane) {
  typedef double dvec2 __attribute__((ext_vector_type(2)));
  constexpr int NB = 16 * BPL, RS = 18;
  if constexpr (FULL) {
    // lane writes pieces (point 8m + lane/8, bins 16 blk + 2 (lane%8) +{0,1}); B == NB
    const int i0 = lane >> 3, q = lane & 7;
    double* rowp = Rh + (wbase + i0) * NB + 16 * blk + 2 * q;
    const int64_t lim = n - wbase - i0;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const dvec2 v = *reinterpret_cast<const dvec2*>(&S[(i0 + 8 * m) * RS + 2 * q]);
      if (8 * m < lim) *reinterpret_cast<dvec2*>(rowp + 8 * m * NB) = v;
    }
  } else {
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int e = lane + 64 * m, i = e >> 4, k = e & 15;
      const double v = S[i * RS + k];
      if (wbase + i < n && 16 * blk + k < B) Rh[(wbase + i) * B + 16 * blk + k] = v;
    }
  }
}
// 2 waves per SIMD: the 48 similarities / exps of a lane's point stay in registers with no spill
// (at 3, the 168-VGPR budget spilled ~12-27 VGPRs per point to scratch: 0.6 GB of extra HBM reads and
// 0.9 GB of extra writes per C3 launch, tools/probe/probe_sa3.hip; 1.74 -> 1.32 ms)
constexpr int kSaOcc = 2;
// the responsibility rows' store kind (A/B builds): 0 non-temporal (default), 1 plain, 2 sc1 write-through
// by inline asm. sc1 took the kernel 1.39 -> 1.33 ms (5.15 TB/s, 90 % of the plain-write probe) and the
// pair 0.673 -> 0.676 (profiles/r05/ab_soft_assign_store_and_moment_order.txt), but its asm form wrote
// wrong values on a ragged tail (test_soft_assign_matches_oracle[32-333]): not adopted
#ifndef GC_SA_STORE
#define GC_SA_STORE 0
#endif
// dynamic LDS of a soft-assign workgroup (doubles): exp table | bins (x, y, z rows of 64) | reduction |
// 4 wave slabs (FULL: 32 rows of 16 BPL + 2; ragged: 64 rows of 18)
__host__ __device__ constexpr bool sa_linear(int BPL, bool full) { return full && BPL <= 3; }  // B = 64: 16-bin blocks (register budget)
__host__ __device__ constexpr int sa_slab_doubles(int BPL, bool full) { return sa_linear(BPL, full) ? 32 * (16 * BPL + 2) : 64 * 18; }
__host__ __device__ constexpr int sa_lds_doubles(int BPL, bool full) { return kExpTab2 + 192 + 8 + 4 * sa_slab_doubles(BPL, full); }
template <int BPL, bool FULL>
__global__ void __launch_bounds__(256, kSaOcc) k_soft_assign(int64_t n, int B, int iters, const double* __restrict__ dirs,
                                                     const double* __restrict__ bins, double inv_tau,
                                                     double* resp, int32_t* bin_idx, double* partial) {
  constexpr int NB = 16 * BPL;
  constexpr int RS = 18;       // ragged slab row stride
  constexpr int RS2 = NB + 2;  // FULL slab row stride
  typedef double dvec2 __attribute__((ext_vector_type(2)));
  extern __shared__ __attribute__((aligned(16))) double sa_lds[];
  double* Tx = sa_lds;
  double* red = Tx + kExpTab2 + 192;  // (192 doubles after the table unused: the bins are scalar loads)
  exp_table2_load(Tx);
  __syncthreads();
  const int h = blockIdx.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double* Rh = resp + (int64_t)h * n * B;
  const double* Dh = dirs + (int64_t)h * n * 3;
  double* S = red + 8 + wv * sa_slab_doubles(BPL, FULL);
  const double Beps = (double)B * 1e-12;
  // Σ log Z is kept as a product of mantissas and a sum of exponents (frexp), one log at the end
  double zm = 1.0, entq = 0.0, mxr = 0.0;
  int ze = 0;
  // iteration it of workgroup b covers points [(it G + b) 256, +256) (G = gridDim.x): the
  // workgroups in flight write one contiguous window of the responsibility matrix instead of G
  // chunks spread over the whole hypothesis (DRAM page locality of the 6.4 GB write stream)
  const int64_t G256 = (int64_t)gridDim.x * 256;
  const int64_t chunk0 = (int64_t)blockIdx.x * 256;
  // directions of the wave's next 64 points: 192 contiguous doubles, three fully coalesced 512-B
  // loads (8 B per lane, any alignment), handed to lane = point through the LDS slab
  const int64_t nd = 3 * n;
  double nd0, nd1, nd2;
#define GC_LOAD_DIRS(WB)                                             \
  {                                                                  \
    const int64_t e0_ = 3 * (WB) + lane;                             \
    nd0 = Dh[e0_ < nd ? e0_ : nd - 1];                               \
    nd1 = Dh[e0_ + 64 < nd ? e0_ + 64 : nd - 1];                     \
    nd2 = Dh[e0_ + 128 < nd ? e0_ + 128 : nd - 1];                   \
  }
  GC_LOAD_DIRS(chunk0 + wv * 64)
  for (int it = 0; it < iters; ++it) {
    const int64_t wbase = chunk0 + (int64_t)it * G256 + wv * 64;
    if (wbase >= n) break;  // wave-uniform
    S[lane] = nd0; S[64 + lane] = nd1; S[128 + lane] = nd2;
    lds_wave_sync();
    const double d0 = S[3 * lane], d1 = S[3 * lane + 1], d2 = S[3 * lane + 2];
    lds_wave_sync();
    GC_LOAD_DIRS(wbase + G256)
    const int64_t pt = wbase + lane;
    const bool valid = pt < n;
    // pass 1: the exact un-fused similarities (kept in ex[]), their row maximum and the integer bin
    // index; pass 2 exponentiates x = (S - S_max)/τ in place, the reference's jax.nn.softmax shift
    // (binning.py:68-69): any τ > 0 and any direction norm. The bin directions are wave-uniform LDS
    // reads (broadcast, no bank conflicts).
    double ex[NB];
    double best = -1e308;
    int bidx = 0;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      // bin directions as wave-uniform scalar loads (SGPR operands; the LDS pipe keeps the exp table
      // and the row transposes)
      const double bx = FULL || j < B ? bins[3 * j] : 0.0, by = FULL || j < B ? bins[3 * j + 1] : 0.0,
                   bz = FULL || j < B ? bins[3 * j + 2] : 0.0;
      ex[j] = sim_nofma(d0, d1, d2, bx, by, bz);
      if ((FULL || j < B) && ex[j] > best) { best = ex[j]; bidx = j; }
    }
    // exponent in units of ln2/2048 (the 2048-entry table exp, exp2s_n): y = S ysc - S_max ysc by one
    // fma (the maximal bin gets y = the rounding error of S_max ysc, |y| < 1e-11, e = 1 within an ulp);
    // arguments below e^-700 are clamped there (R <= 1e-304 / Z instead of an underflow to 0)
    const double ysc = inv_tau * kTab2OverLn2;
    const double nbs = -(best * ysc);
    double Z = 0.0, sl = 0.0;
#pragma unroll
    for (int j0 = 0; j0 < NB; j0 += 8) {
      double y[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int j = j0 + jj;
        y[jj] = (FULL || j < B) ? fmax(fma(ex[j], ysc, nbs), -700.0 * kTab2OverLn2) : 0.0;
      }
      double e8[8];
      exp2s_n<8>(y, Tx, e8);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int j = j0 + jj;
        ex[j] = (FULL || j < B) ? e8[jj] : 0.0;
        Z += ex[j];
        sl = fma(ex[j], y[jj], sl);
      }
      asm volatile("" : "+v"(Z), "+v"(sl));  // accumulate now: the y of a group die here
    }
    sl *= kExp2C1;  // Σ e x in nats
    // the maximal bin has e = 1 (within an ulp): Z >= 1 and max_b R = 1/Z
    const double rZ = recip(Z);
    if (valid) {
      // entropy of the point: log Z - S/Z - B ε   (-Σ R log(R+ε) up to ≤ B·ε)
      int e;
      zm *= frexp(Z, &e);
      ze += e;
      entq += fma(sl, rZ, Beps);
      mxr = fmax(mxr, rZ);
      if (bin_idx) bin_idx[(int64_t)h * n + pt] = bidx;
    }
    if constexpr (sa_linear(BPL, FULL)) {
#pragma unroll
      for (int j = 0; j < NB; ++j) ex[j] *= rZ;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        if ((lane >> 5) == hf) {
          const int i = lane & 31;
#pragma unroll
          for (int q = 0; q < NB / 2; ++q)
            *reinterpret_cast<dvec2*>(&S[i * RS2 + 2 * q]) = dvec2{ex[2 * q], ex[2 * q + 1]};
        }
        lds_wave_sync();
        // the half's 32 rows are one contiguous block of 32 NB doubles in HBM: 1 KiB per instruction
        const int64_t pbase = wbase + 32 * hf;
        double* dst = Rh + pbase * NB;
        const auto put = [&](int o, const dvec2& v) {
#if GC_SA_STORE == 1
          *reinterpret_cast<dvec2*>(dst + o) = v;  // plain
#elif GC_SA_STORE == 2
          asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst + o), "v"(v) : "memory");  // write-through
#else
          __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(dst + o));
#endif
        };
        if (pbase + 32 <= n) {  // wave-uniform: the whole block is in range (every block but the tail's)
#pragma unroll
          for (int m = 0; m < NB / 4; ++m) {
            const int o = m * 128 + 2 * lane;
            const int row = o / NB, col = o - row * NB;
            put(o, *reinterpret_cast<const dvec2*>(&S[row * RS2 + col]));
          }
        } else {
          const int64_t lim = (n - pbase) * NB;  // doubles of the block that belong to points < n
#pragma unroll
          for (int m = 0; m < NB / 4; ++m) {
            const int o = m * 128 + 2 * lane;
            const int row = o / NB, col = o - row * NB;
            const dvec2 v = *reinterpret_cast<const dvec2*>(&S[row * RS2 + col]);
            if (o < lim) put(o, v);
          }
        }
        lds_wave_sync();
      }
    } else {
#pragma unroll
      for (int blk = 0; blk < BPL; ++blk) {
#pragma unroll
        for (int q = 0; q < 8; ++q)
          *reinterpret_cast<dvec2*>(&S[lane * RS + 2 * q]) =
              dvec2{ex[16 * blk + 2 * q] * rZ, ex[16 * blk + 2 * q + 1] * rZ};
        lds_wave_sync();
        sa_store_block<BPL, FULL>(S, Rh, wbase, n, B, blk, lane);
        lds_wave_sync();
      }
    }
    int e;
    zm = frexp(zm, &e);  // renormalise once per 64 points: |log2 zm| stays below ~64
    ze += e;
  }
  const double logacc = log(zm) + (double)ze * 0.69314718055994530942;
#undef GC_LOAD_DIRS
  const double es = wg_sum(logacc - entq, red);
  const double ms = wg_max(mxr, red);
  if (threadIdx.x == 0) {
    partial[((int64_t)h * gridDim.x + blockIdx.x) * 2] = es;
    partial[((int64_t)h * gridDim.x + blockIdx.x) * 2 + 1] = ms;
  }
}

__global__ void k_soft_assign_finalize(const double* __restrict__ partial, int64_t cols, int H,
                                       int64_t n, double* cert) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= H) return;
  double e = 0.0, m = 0.0;
  for (int64_t c = 0; c < cols; ++c) {
    e += partial[((int64_t)h * cols + c) * 2];
    m = fmax(m, partial[((int64_t)h * cols + c) * 2 + 1]);
  }
  cert[2 * h] = e / ((double)n + 1e-12);
  cert[2 * h + 1] = m;
}

// ===================================================================== a6 moment partials
// Contract variant: responsibilities streamed from HBM. grid (chunks, H), 4 waves per workgroup,
// each wave owns `groups` consecutive 32-point groups of the chunk. The moment sums
// Mom[b][k] = Σ_p R[p][b] F[p][k] run on the matrix core: per 4-point step s, bin tile j
// (16 bins) x feature tile t (16 features) is one v_mfma_f64_16x16x4_f64 with
// A[bin][point] = R (lane (g, l): point 4s + g, bin 16j + l) and B[point][feature] = F
// (lane (g, l): point 4s + g, feature 16t + l). The A operand is loaded from HBM straight into
// its lane (8 B per lane: four full 128-B row segments per load), a whole 32-point group ahead
// of its use (register double buffer, ~12 KiB of responsibilities in flight per wave); no LDS
// round trip. Features are computed lane = point for the next group and handed over through a
// wave-private LDS slab (feature-major, stride 34: the B-operand reads are bank-conflict free).
// NACC = 2: even and odd steps accumulate into separate tiles (2*BPL*NT independent MFMA chains)
// added in the epilogue. The 4 waves are reduced in a fixed order into one record per chunk.
constexpr int kMomFS = 34;
// PAIR (B >= 32, 16-B aligned rows): bins 0..31 arrive as one 16-B load per lane (bins 2l, 2l+1 of its
// point: four 256-B row segments per load instead of two loads of four 128-B segments); tile 0 holds
// the even bins, tile 1 the odd ones (row i of tile j < 2 is bin 2i + j), tiles >= 2 bins 16j + l.
#ifndef GC_MOM_FORWARD
constexpr bool kMomReverse = true;
#else
constexpr bool kMomReverse = false;
#endif
template <int BPL, bool COV, bool LAM, int NACC, bool PAIR>
__global__ void __launch_bounds__(256, 2) k_moment_partials(int64_t n, int B, int groups,
                                                           const double* __restrict__ pts,
                                                           const double* __restrict__ covs,
                                                           const double* __restrict__ w,
                                                           const double* __restrict__ resp,
                                                           const double* __restrict__ lam, double o0,
                                                           double o1, double o2, double* partials) {
  constexpr int NF = COV ? NF_BASE + NF_COV : NF_BASE;
  constexpr int NT = (NF + 15) / 16;  // feature tiles (zero-padded to 16 NT)
  extern __shared__ double lds[];
  // workgroups run the (hypothesis, chunk) grid from its end: the soft-assign before this kernel wrote
  // the responsibilities in ascending block order, so the last-written (still in the Infinity Cache /
  // L2) are read first (records, and so the sums, are the same in either order)
  const int bx = kMomReverse ? (int)(gridDim.x - 1 - blockIdx.x) : (int)blockIdx.x;
  const int h = kMomReverse ? (int)(gridDim.y - 1 - blockIdx.y) : (int)blockIdx.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, bl = lane & 15;
  double* F = lds + wv * (16 * NT * kMomFS);
  const double o[3] = {o0, o1, o2};
  const double* Rh = resp + (int64_t)h * n * B;
  const int64_t wbeg = ((int64_t)bx * 4 + wv) * groups * 32;
  int64_t wend = wbeg + (int64_t)groups * 32;
  wend = wend < n ? wend : n;
  const int ng = wbeg < n ? (int)((wend - wbeg + 31) / 32) : 0;
  v4d acc[NACC][BPL][NT];
#pragma unroll
  for (int e = 0; e < NACC; ++e)
#pragma unroll
    for (int j = 0; j < BPL; ++j)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[e][j][t] = v4d{0.0, 0.0, 0.0, 0.0};
  // this lane's responsibility column offsets (bins 16 j + l), clamped into the row
  int cb[BPL];
  bool cv[BPL];
#pragma unroll
  for (int j = 0; j < BPL; ++j) {
    cv[j] = bl + 16 * j < B;
    cb[j] = cv[j] ? bl + 16 * j : 0;
  }
  double Ra[8][BPL], Rb[8][BPL];  // group c (A operands of its 8 steps) and group c + 1
#define GC_LOAD_R(RR, BASE)                                                     \
  {                                                                             \
    _Pragma("unroll") for (int s_ = 0; s_ < 8; ++s_) {                          \
      int64_t p_ = (BASE) + 4 * s_ + g;                                         \
      p_ = p_ < wend ? p_ : wend - 1; /* prefetch past the range re-reads a line */ \
      const double* row_ = Rh + p_ * B;                                         \
      if constexpr (PAIR) {                                                     \
        typedef double dv2_ __attribute__((ext_vector_type(2)));                \
        const dv2_ v_ = *reinterpret_cast<const dv2_*>(row_ + 2 * bl);         \
        RR[s_][0] = v_.x;                                                       \
        RR[s_][1] = v_.y;                                                       \
      }                                                                         \
      _Pragma("unroll") for (int j_ = PAIR ? 2 : 0; j_ < BPL; ++j_) RR[s_][j_] = GC_RESP_LOAD(row_ + cb[j_]); \
    }                                                                           \
  }
  // raw inputs of one 32-point group (point = lane & 31), loaded by every lane into registers and
  // consumed branch-free a group later (no load is sunk into a lane-conditional block)
  double rp[3], rc[9], rw, rl;
  bool rok;
#define GC_LOAD_RAW(BASE)                                                       \
  {                                                                             \
    const int64_t pt_ = (BASE) + (lane & 31);                                   \
    rok = pt_ < wend;                                                           \
    const int64_t row_ = (int64_t)h * n + (rok ? pt_ : wend - 1);               \
    rw = w[row_];                                                               \
    if constexpr (LAM) rl = lam[row_];                                          \
    rp[0] = pts[3 * row_]; rp[1] = pts[3 * row_ + 1]; rp[2] = pts[3 * row_ + 2]; \
    if constexpr (COV) {                                                        \
      _Pragma("unroll") for (int k_ = 0; k_ < 9; ++k_) rc[k_] = covs[9 * row_ + k_]; \
    }                                                                           \
  }
  // lanes 0..31 write features 0..15 of their point, lanes 32..63 features 16..31
  // (pp[11 12 22], cov x w, zero padding)
#define GC_FEATURES()                                                           \
  {                                                                             \
    lds_wave_sync(); /* the previous group's B-operand reads are done */        \
    double wl_ = LAM ? rw * rl : rw;                                            \
    wl_ = rok ? wl_ : 0.0;                                                      \
    double d_[3], f_[NF_BASE];                                                  \
    direction(rp, o, 1e-12, d_);                                                \
    point_features(rp, d_, wl_, f_);                                            \
    const bool lo_ = lane < 32;                                                 \
    double* Fl_ = F + (lo_ ? 0 : 16 * kMomFS) + (lane & 31);                    \
    _Pragma("unroll") for (int k_ = 0; k_ < 16; ++k_) {                         \
      const int kk_ = 16 + k_;                                                  \
      double hi_ = 0.0;                                                         \
      if (kk_ < NF_BASE) hi_ = f_[kk_ < NF_BASE ? kk_ : 0];                      \
      else if (COV && kk_ < NF) hi_ = wl_ * rc[kk_ - NF_BASE < 9 ? kk_ - NF_BASE : 0]; \
      Fl_[k_ * kMomFS] = lo_ ? f_[k_] : hi_;                                    \
    }                                                                           \
    lds_wave_sync();                                                            \
  }
#define GC_CONSUME(RR)                                                          \
  {                                                                             \
    _Pragma("unroll") for (int s_ = 0; s_ < 8; ++s_) {                          \
      double fb_[NT];                                                           \
      _Pragma("unroll") for (int t_ = 0; t_ < NT; ++t_) fb_[t_] = F[(16 * t_ + bl) * kMomFS + 4 * s_ + g]; \
      _Pragma("unroll") for (int j_ = 0; j_ < BPL; ++j_) {                      \
        const double ra_ = cv[j_] ? RR[s_][j_] : 0.0;                           \
        _Pragma("unroll") for (int t_ = 0; t_ < NT; ++t_)                       \
          acc[s_ % NACC][j_][t_] = __builtin_amdgcn_mfma_f64_16x16x4f64(ra_, fb_[t_], acc[s_ % NACC][j_][t_], 0, 0, 0); \
      }                                                                         \
    }                                                                           \
  }
  if (ng > 0) {
    // loads past the wave's range are issued unconditionally (clamped rows, zero weights) so the
    // body is straight-line and every wait is a counted vmcnt, not a drain
    GC_LOAD_RAW(wbeg)
    __builtin_amdgcn_sched_barrier(0);
    GC_LOAD_R(Ra, wbeg)
    __builtin_amdgcn_sched_barrier(0);
    for (int c = 0; c < ng; c += 2) {
      GC_FEATURES()
      const int64_t b1 = wbeg + 32 * (int64_t)(c + 1);
      GC_LOAD_RAW(b1)  // raw first: the next features wait for these, not for the R stream
      __builtin_amdgcn_sched_barrier(0);
      GC_LOAD_R(Rb, b1)
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the consumption
      GC_CONSUME(Ra)
      __builtin_amdgcn_sched_barrier(0);
      GC_FEATURES()
      const int64_t b2 = wbeg + 32 * (int64_t)(c + 2);
      GC_LOAD_RAW(b2)
      __builtin_amdgcn_sched_barrier(0);
      GC_LOAD_R(Ra, b2)
      __builtin_amdgcn_sched_barrier(0);
      GC_CONSUME(Rb)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#undef GC_LOAD_R
#undef GC_LOAD_RAW
#undef GC_FEATURES
#undef GC_CONSUME
  // epilogue: even + odd tiles, then the 4 waves in a fixed order (LDS reused)
  __syncthreads();
  double* red = lds;  // [4][B][NF]
#pragma unroll
  for (int j = 0; j < BPL; ++j)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = (PAIR && j < 2) ? 2 * (g + 4 * r) + j : 16 * j + g + 4 * r, k = 16 * t + bl;  // D[row g + 4r][col l]
        if (b < B && k < NF) red[(wv * B + b) * NF + k] = NACC == 2 ? acc[0][j][t][r] + acc[NACC - 1][j][t][r] : acc[0][j][t][r];
      }
  __syncthreads();
  int64_t npts = n - (int64_t)bx * 4 * groups * 32;
  npts = npts < 0 ? 0 : (npts > (int64_t)4 * groups * 32 ? (int64_t)4 * groups * 32 : npts);
  const int RL = B * NF + REC_EXTRA;
  double* rec = partials + ((int64_t)h * gridDim.x + bx) * RL;
  for (int i = threadIdx.x; i < B * NF; i += kWG)
    rec[i] = (red[i] + red[B * NF + i]) + (red[2 * B * NF + i] + red[3 * B * NF + i]);
  if (threadIdx.x < REC_EXTRA) rec[B * NF + threadIdx.x] = threadIdx.x == 3 ? (double)npts : 0.0;
}

// MFMA epilogue: reduce per-lane tiles over the 4 waves (LDS, fixed order) into one partial
// record. Lane (g, l) holds D_j[row g + 4r][col l] = Σ R[·][16j + g + 4r] F[·][l] for the 16
// MFMA features, and per-group partial sums accx[j][t] (bin 16j + l, feature 16 + t).
// DF = 9: feature 9 (Σ R w d_z²) is not accumulated; the MFMA columns hold features 0..8, 10..16 and
// the VALU ones 17.. . It is recovered from the trace of the direction scatter, Σ R w |d|² = N − ε_d
// with ε_d = Σ R w (1 − |d|²) ≤ 2·1e-12 / range of N (|d| = |r| / (|r| + 1e-12)): d_z² = N − d_x² − d_y²,
// an absolute error ~1e-12 N in that one scatter entry; N, the resultant and κ stay exact sums.
struct NoHook {
  GC_DEV void operator()() const {}
};
// v + v^16 then + v^32 over the lane index (the value of lane l's column summed over the wave's four
// 16-lane rows) by gfx950's row and half swaps on the VALU instead of two LDS-routed shuffles; each
// step adds a lane pair in one order or the other, which is the same double (x + y == y + x)
GC_DEV double sum_rows4(double v) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const double w = __hiloint2double(h16[0], l16[0]) + __hiloint2double(h16[1], l16[1]);
  const unsigned wl = __double2loint(w), wh = __double2hiint(w);
  const auto l32 = __builtin_amdgcn_permlane32_swap(wl, wl, false, false);
  const auto h32 = __builtin_amdgcn_permlane32_swap(wh, wh, false, false);
  return __hiloint2double(h32[0], l32[0]) + __hiloint2double(h32[1], l32[1]);
}
#ifndef GC_EPI_PERMLANE
#define GC_EPI_PERMLANE 0
#endif
GC_DEV int64_t uniform_i64(int64_t v) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
// pre() runs before the barrier, mid() after it (the persistent bins form's next-task broadcast). Each wave
// stages its tiles, its two VALU features and its three certificate partials in its OWN slab (WS doubles
// from lds + wv WS: no other wave reads it during a task, so no barrier is needed before the writes),
// and computes its log-product and wave sums before the barrier: every latency-bound step of the
// epilogue runs before mid() issues the next task's loads (a later wait on scratch or on the staged
// values would otherwise wait for those loads' HBM round trip as well). One barrier, the 4-wave sum in
// a fixed order, and the caller's closing barrier.
template <int BPL, int NX, int DF = -1, bool FULL = false, int WS = 0, typename Pre = NoHook, typename Mid = NoHook>
GC_DEV void write_partial_record_mfma(const v4d (&acc4)[BPL], double (&accx)[BPL][NX], double ent, double mxr,
                                      double sumw, double npts, int B_, double* lds, double* rec,
                                      const Pre& pre = Pre(), const Mid& mid = Mid()) {
  const int B = FULL ? 16 * BPL : B_;  // FULL: a compile-time bin count (immediate LDS offsets, no bounds branches)
  constexpr int ND = DF >= 0 ? 1 : 0;
  constexpr int NF = ND + 16 + NX;
  static_assert(WS >= 16 * BPL * NF + 3, "a wave's slab holds its record tiles");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, bl = lane & 15;
  const int fcol = (DF >= 0 && bl >= DF) ? bl + 1 : bl;  // the feature of MFMA column bl
#pragma unroll
  for (int j = 0; j < BPL; ++j)
#pragma unroll
    for (int t = 0; t < NX; ++t) {
#if GC_EPI_PERMLANE
      accx[j][t] = sum_rows4(accx[j][t]);
#else
      double v = accx[j][t];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      accx[j][t] = v;
#endif
    }
  const double e = wave_sum(ent), m = wave_max(mxr), s = wave_sum(sumw);
  double* W = lds + wv * WS;
#pragma unroll
  for (int j = 0; j < BPL; ++j) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = 16 * j + g + 4 * r;
      if (b < B) W[b * NF + fcol] = acc4[j][r];
    }
    const int b = 16 * j + bl;
    if (g == 0 && b < B)
#pragma unroll
      for (int t = 0; t < NX; ++t) W[b * NF + ND + 16 + t] = accx[j][t];
  }
  if (lane == 0) {
    W[B * NF + 0] = e;
    W[B * NF + 1] = m;
    W[B * NF + 2] = s;
  }
  pre();
  __syncthreads();
  mid();
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // the per-lane addresses formed here, not hoisted out of the task loop and spilled
  const auto sum4 = [&](int e) { return (lds[e] + lds[WS + e]) + (lds[2 * WS + e] + lds[3 * WS + e]); };
  if constexpr (FULL) {
    // a compile-time entry count: every lane's entries summed with their LDS reads issued together (one
    // LDS round trip instead of one per entry), then stored; the complement entry's three sums are
    // selected, not branched to
    constexpr int NE = 16 * BPL * NF, NI = (NE + kWG - 1) / kWG;
    double v[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int i = min(tid + k * kWG, NE - 1);
      if constexpr (DF >= 0) {
        const bool df = i % NF == DF;
        const int i0 = i - (df ? DF : 0);  // N
        const double a = sum4(i0), b = sum4(df ? i0 + 4 : i0), c = sum4(df ? i0 + 7 : i0);
        v[k] = df ? (a - b) - c : a;  // N − xx − yy
      } else {
        v[k] = sum4(i);
      }
    }
    // the scheduler otherwise pairs each two reads with a wait for them: every read first
    __builtin_amdgcn_sched_group_barrier(0x100, (DF >= 0 ? 12 : 4) * NI, 0);
#pragma unroll
    for (int k = 0; k < NI; ++k)
      if (k < NI - 1 || tid + k * kWG < NE) rec[tid + k * kWG] = v[k];
  } else {
    for (int i = tid; i < B * NF; i += kWG) {
      if (DF >= 0 && i % NF == DF) rec[i] = (sum4(i - DF) - sum4(i - DF + 4)) - sum4(i - DF + 7);  // N − xx − yy
      else rec[i] = sum4(i);
    }
  }
  if (threadIdx.x == 0) {
    const double* ex = lds + B * NF;
    double x[4][3];
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int k = 0; k < 3; ++k) x[w][k] = ex[w * WS + k];
    __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
    rec[B * NF + 0] = (x[0][0] + x[1][0]) + (x[2][0] + x[3][0]);
    rec[B * NF + 1] = fmax(fmax(x[0][1], x[1][1]), fmax(x[2][1], x[3][1]));
    rec[B * NF + 2] = (x[0][2] + x[1][2]) + (x[2][2] + x[3][2]);
    rec[B * NF + 3] = npts;
  }
}

// =========================================================== fused a1 -> a4 -> a5 -> a6
// grid (chunks, H). Budget selection + deskew + directions + features in phase A (lane =
// point), soft assignment in phase B (lanes = 4 point-groups x 16 bin-lanes, 4 points per
// step). The moment sums are a GEMM, Mom[b][k] = Σ_p R[p][b] F[p][k]: the step's (16 bins x 4
// points) responsibility tile of bin block j is exactly the A operand of
// v_mfma_f64_16x16x4_f64 as the lanes already hold it, and F[p][k] for 4 points x 16 features
// is one LDS read per lane (B operand). The matrix core accumulates features 0..15 while the
// VALU does the exp/softmax; features 16..18 stay on the VALU. Responsibilities never leave
// registers.
// feature slab row stride: the B-operand read F[l][4s + g] of the 32 lanes of a ds_read_b64
// group lands on 32 distinct bank pairs (4 l + 2 g + 8 s mod 64)
constexpr int kFusedFS = 66;
constexpr int kFusedOcc = 2;   // waves per SIMD the register budget is sized for (3 spills: §5 of DESIGN.md)
constexpr int kFusedUnr = 8;   // softmax steps unrolled per block (Π Z renormalised after each block: exact)
constexpr int kFusedNacc = 2;  // MFMA accumulator sets (even / odd steps)
// Per-launch constants of the fused kernel and its LDS tables (exp table, scaled bins), set up once
// per workgroup by bins_prologue; a workgroup then runs one (grid form) or many (persistent form)
// (hypothesis, chunk) tasks with bins_task.
struct FusedArgs {
  int64_t n_cap;
  int B, iters;
  const double *pts_raw, *t_raw, *w_raw, *bscal;
  double t0, t1;
  const double *xi, *bins;
  double inv_tau, o0, o1, o2;
  double* partials;      // (H, chunks, RL) records
  const double* w_win;   // (n_cap) selected w x time window (the pipeline's predict), or NULL: per task
  // three chunk tiers: chunks [0, k1) hold iters x 256 points, the next k2 iters_s x 256, the rest
  // iters_t x 256 (the persistent form ends on ever shorter tasks, so the pullers finish together);
  // grid form: k1 = chunks
  int64_t k1;
  int iters_s;
  int64_t k2;
  int iters_t;
};
constexpr int kFusedNS = NF_BASE + 4;  // feature slab rows: 19 features + d(3) + valid flag
// Point-major softmax (GC_BINS_LP = 1, B <= 48; off: the A/B in profiles/r06/ab_bins_point_major.txt
// measured it neutral at H = 256 and 10 % slower at H = 32). The exp / softmax half runs with a quad of
// lanes per point (12 of its bins per lane, the quad's Z by two DPP rounds instead of the 16-lane
// butterfly), the responsibilities reach the matrix-core layout through a per-wave LDS slab of 16 points
// x B, and the moment half is bins_task's. ~14 % fewer VALU slots per block, but a slab round trip and
// a direction shuffle per 16 points on the chain. Per wave: 18 feature rows (the trace-complement
// feature DF has no row) of kFusedFS and the 16-row slab of stride 16 BPL + 2; the table after the four
// waves; no scaled-bins block (each lane holds its 12 bin directions).
#ifndef GC_BINS_LP
#define GC_BINS_LP 0
#endif
__host__ __device__ constexpr bool bins_lp(int BPL) { return GC_BINS_LP && BPL <= 3; }
constexpr int kLpFRows = NF_BASE - 1;
__host__ __device__ constexpr int lp_es(int BPL) { return 16 * BPL + 2; }
__host__ __device__ constexpr int lp_wave_doubles(int BPL) { return kLpFRows * kFusedFS + 16 * lp_es(BPL); }
__host__ __device__ constexpr int fused_tab_offset(int BPL) {
  return bins_lp(BPL) ? 4 * lp_wave_doubles(BPL) : 4 * kFusedFS * kFusedNS;
}
// dynamic LDS of a fused workgroup (doubles): 4 wave slabs | exp table | scaled bins (not LP) | epilogue
// reduction (aliases the slabs). LP at B = 48: 80,000 B, two workgroups per CU.
__host__ __device__ inline size_t fused_lds_doubles(int B) {
  const int bpl = (B + 15) / 16;
  const size_t a = (size_t)fused_tab_offset(bpl) + kExpTab2 + (bins_lp(bpl) ? 0 : 192),
               b = 4 * (size_t)B * NF_BASE + 12;
  return a > b ? a : b;
}
static_assert(4 * lp_wave_doubles(3) + kExpTab2 + 1 <= 81920 / 8, "LP bins workgroup beyond half a CU's LDS");

template <int BPL>
GC_DEV void bins_prologue(const FusedArgs& A, double* lds) {
  double* Tx = lds + fused_tab_offset(BPL);
  exp_table2_load(Tx);
  if constexpr (bins_lp(BPL)) {
    __syncthreads();
    return;
  }
  double* Lb = Tx + kExpTab2;  // bin directions pre-scaled by 2048/(τ ln2) (x, y, z rows of 64)
  const double ysc = A.inv_tau * kTab2OverLn2;
  if (threadIdx.x < 64) {
    const int b = threadIdx.x;
    Lb[b] = b < A.B ? A.bins[3 * b] * ysc : 0.0;
    Lb[64 + b] = b < A.B ? A.bins[3 * b + 1] * ysc : 0.0;
    Lb[128 + b] = b < A.B ? A.bins[3 * b + 2] * ysc : 0.0;
  }
  __syncthreads();
}

// the first point index of chunk c (the tiers of FusedArgs) and its iteration count
GC_DEV int64_t chunk_first(const FusedArgs& A, int64_t c, int* iters_out) {
  const bool big = c < A.k1, mid = !big && c < A.k1 + A.k2;
  *iters_out = big ? A.iters : (mid ? A.iters_s : A.iters_t);
  return big ? c * A.iters * 256
             : (mid ? (A.k1 * A.iters + (c - A.k1) * A.iters_s) * 256
                    : (A.k1 * A.iters + A.k2 * A.iters_s + (c - A.k1 - A.k2) * A.iters_t) * 256);
}
// A task's operands that its first iteration waits for: the hypothesis's twist and the lane's raw point
// of iteration 0. The persistent form loads the next task's during the current task's epilogue
// (TaskAhead::valid), so the HBM round trip overlaps the record's reduction instead of opening the task.
struct TaskAhead {
  double xr[6];
  double np[3], ntt, nww;
  unsigned t;   // the next task's ticket (all lanes), read back from the workgroup's task slot
  bool valid;
  bool ok;      // the lane's point is selected (np / ntt / nww are then the point's; zeroed at use otherwise)
};
// n_sel / stride: the a1 selection's count and stride (budget scalars), read once per launch. The raw point
// is loaded unconditionally from a clamped index, its validity applied where the next task uses it: no
// branch merge right behind the loads, so the epilogue issuing them never waits for their HBM round trip.
template <bool PRE>
GC_DEV void task_operands(const FusedArgs& A, int h, int64_t c, int64_t n_sel, int64_t stride, TaskAhead& ta) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int it_unused;
  const int64_t chunk0 = chunk_first(A, c, &it_unused);
#pragma unroll
  for (int k = 0; k < 6; ++k) ta.xr[k] = A.xi[6 * h + k];
  const int64_t j = chunk0 + wv * 64 + lane;
  const bool ok = j < A.n_cap && j < n_sel;
  const int64_t jc = ok ? j : 0, i = jc * stride;
  ta.np[0] = A.pts_raw[3 * i]; ta.np[1] = A.pts_raw[3 * i + 1]; ta.np[2] = A.pts_raw[3 * i + 2];
  ta.ntt = A.t_raw[i];
  ta.nww = PRE ? A.w_win[jc] : A.w_raw[i];
  ta.ok = ok;
  ta.valid = true;
}
// the budget scalars a launch's tasks share (read once per workgroup)
GC_DEV void selection_of(const FusedArgs& A, int64_t* n_sel, int64_t* stride) {
  *n_sel = (int64_t)A.bscal[5];
  *stride = (int64_t)A.bscal[6];
}

#ifdef GC_BINS_TIMING
// dev instrumentation: per workgroup of the last k_bins_io launch [start, prologue end, end, tasks] in
// device real-time ticks (100 MHz, one clock for every XCD); tasks = -1 for a branch workgroup
__device__ double g_bins_trace[4 * 8192];
__device__ double g_task_trace[4 * 16384];  // per task [start, end, puller, XCD id]
__device__ double g_task_ep[2 * 16384];  // per task [end of its first iteration, start of its epilogue] (wave 0)
__device__ double g_task_wv[4 * 16384];  // per task and wave: the end of its iterations
#define GC_BT_NOW() ((double)__builtin_amdgcn_s_memrealtime())
#endif
// bins_task in the point-major softmax form (bins_lp): the same task, records and ticket protocol.
// Per iteration of 64 points per wave:
//  phase A (lane = point): budget selection, deskew, direction, window weight and the 18 features,
//     as bins_task;
//  four sub-iterations of 16 points, lane = (point l >> 2, bin quarter l & 3):
//   B1: the lane's 12 logits against its bin directions (registers), exps (the 2048-entry table), the
//       quad's Z by two DPP rounds, 1/Z by one Newton step, Σ R x and max R, r = e / Z into the slab;
//   B2 (lanes = 4 points x 16 bins): the sub-iteration's 4 steps of BPL MFMAs (A = r of point 4s + g,
//       bin 16 j + l, from the slab; B = feature l of that point) and the two VALU features.
template <int BPL, bool FULL, bool PRE>
GC_DEV void bins_task_lp(const FusedArgs& A, int h, int64_t c, double* lds, double* rec, unsigned* ctr,
                         unsigned* task_slot, TaskAhead* ahead, unsigned T, int Hl, unsigned* late_next,
                         int64_t n_sel, int64_t stride) {
  typedef double dvec2 __attribute__((ext_vector_type(2)));
  constexpr int NF = NF_BASE;
  constexpr int DF = 9;
  constexpr int NX = NF - 16 - 1;
  constexpr int NB = 16 * BPL, ES = lp_es(BPL), WD = lp_wave_doubles(BPL);
  constexpr unsigned TAB = 8u * (unsigned)fused_tab_offset(BPL);
  constexpr int FS = kFusedFS;
  const int64_t n_cap = A.n_cap;
  const int B = A.B;
  int iters;
  const int64_t chunk0 = chunk_first(A, c, &iters);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, bl = lane & 15;
  double* F = lds + wv * WD;         // feature rows (row r = feature r, r + 1 past DF) x 64 points
  double* E = F + kLpFRows * FS;     // exp slab: 16 points x ES
  const double o[3] = {A.o0, A.o1, A.o2};
  TaskAhead ta_local;
  TaskAhead& ta = ahead ? *ahead : ta_local;
  if (!ahead || !ahead->valid) task_operands<PRE>(A, h, c, n_sel, stride, ta);
  double xr[6];  // the hypothesis's twist: wave-uniform, held in SGPRs
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const double v = ta.xr[k];
    xr[k] = __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                             __builtin_amdgcn_readfirstlane(__double2loint(v)));
  }
  const double* __restrict__ pts_raw = A.pts_raw;
  const double* __restrict__ t_raw = A.t_raw;
  const double* __restrict__ w_raw = A.w_raw;
  const double t0 = A.t0, t1 = A.t1;
  const double scale = A.bscal[2];
  const double denom = fmax(t1 - t0, 1e-12);
  const double inv_denom = 1.0 / denom;
  const double inv_sig = 1.0 / fmax(0.1 * denom, 1e-6);
  double* Tx = lds + fused_tab_offset(BPL);
  const double ysc = A.inv_tau * kTab2OverLn2;
  constexpr int NACC = 1;  // BPL independent MFMA chains per step suffice here (the slab round trip paces them)
  v4d acc4[NACC][BPL];
  double accx[BPL][NX];
#pragma unroll
  for (int j = 0; j < BPL; ++j) {
    acc4[0][j] = v4d{0.0, 0.0, 0.0, 0.0};
    acc4[NACC - 1][j] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int t = 0; t < NX; ++t) accx[j][t] = 0.0;
  }
  double sumw = 0.0, entq = 0.0, mxr = 0.0;
  double zst = 1.0;  // Π Z of the lane's points as mantissa x 2^zex (renormalised every iteration)
  int zex = 0;
  // x = (ysc d)·b <= ysc (1 + 1e-16) < ymax: the exp argument x - ymax <= 0, the shift riding in the
  // rounding constant (exp2s_shift_tab_n) and added back to the entropy below
  const double ymax = ceil(ysc);
  const double Mp = kRoundMagic - ymax;
  const double Beps = (double)B * 1e-12;
  double np[3] = {0.0, 0.0, 0.0}, ntt = 0.0, nww = 0.0;
  auto fetch = [&](int it2) {
    const int64_t j = chunk0 + (int64_t)it2 * 256 + wv * 64 + lane;
    np[0] = 0.0; np[1] = 0.0; np[2] = 0.0; ntt = 0.0; nww = 0.0;
    if (j < n_cap && j < n_sel) {
      const int64_t i = j * stride;
      np[0] = pts_raw[3 * i]; np[1] = pts_raw[3 * i + 1]; np[2] = pts_raw[3 * i + 2];
      ntt = t_raw[i];
      nww = PRE ? A.w_win[j] : w_raw[i];
    }
  };
  {
    const bool ok = ta.ok;  // applied here, a task after the loads were issued
    np[0] = ok ? ta.np[0] : 0.0; np[1] = ok ? ta.np[1] : 0.0; np[2] = ok ? ta.np[2] : 0.0;
    ntt = ok ? ta.ntt : 0.0; nww = ok ? ta.nww : 0.0;
  }
  unsigned next = 0;
  // this lane's bin set for the quad form: bins NQ c .. NQ c + NQ - 1 (c = lane & 3), pre-scaled by
  // ysc, in registers for the whole task (ragged B: the bins past B read as bin B - 1, masked below)
  constexpr int NQ = NB / 4;
  const int cq = lane & 3;
  double bq[NQ][3];
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const int b = min(NQ * cq + k, B - 1);
#pragma unroll
    for (int r = 0; r < 3; ++r) bq[k][r] = A.bins[3 * b + r] * ysc;
  }
  auto run_iters = [&](auto pad_tag) {
    constexpr bool PAD = decltype(pad_tag)::value;
    for (int it = 0; it < iters; ++it) {
      const int64_t wbase = chunk0 + (int64_t)it * 256 + wv * 64;
      if (ctr && !late_next && it == iters - 1 && threadIdx.x == 0) next = atomicAdd(ctr, 1u);
      // ---- phase A (lane = point): the point's features (w folded in) into the wave's feature rows
      double d[3];
      {
        const bool inr = !PAD || wbase + lane < n_cap;
        double p[3] = {np[0], np[1], np[2]};
        const double tt = ntt, ww = nww * scale;
        if (it + 1 < iters) fetch(it + 1);
        const double al = (tt - t0) * inv_denom;
        const double ph[3] = {al * xr[3], al * xr[4], al * xr[5]};
        double q[3];
        if (__all(dot3(ph, ph) <= kDeskewShortTs)) deskew_point_cross<true>(p, al, xr, q);
        else deskew_point_cross<false>(p, al, xr, q);
        const double wd = inr ? (PRE ? ww : ww * window_weight2(tt, t0, t1, inv_sig, Tx)) : 0.0;
        direction_fast(q, o, 1e-12, d);
        sumw += wd;
        double f[NF];
        point_features_w(q, d, wd, f);
#pragma unroll
        for (int k = 0; k < NF; ++k)
          if (k != DF) F[(k < DF ? k : k - 1) * FS + lane] = f[k];
      }
      // ---- four sub-iterations of 16 points: B1 with lane = (point p = l >> 2, bin quarter c = l & 3),
      // then B2 over the sub-iteration's 4 MFMA steps
#pragma unroll
      for (int sk = 0; sk < 4; ++sk) {
        const int pt = 16 * sk + (lane >> 2);  // the wave's point (its phase-A lane)
        const double dx = __shfl(d[0], pt), dy = __shfl(d[1], pt), dz = __shfl(d[2], pt);
        const double vf = (!PAD || wbase + pt < n_cap) ? 1.0 : 0.0;  // padding: no entropy / max / Π Z
        // B1: this lane's NQ logits, exps and partial Z, Σ e x, max e (groups of 4: all NQ table reads in
        // flight at once measured slower, profiles/r06/ab_bins_point_major.txt)
        double e[NQ];
        double Zl = 0.0, sl = 0.0, em = 0.0;
#pragma unroll
        for (int k0 = 0; k0 < NQ; k0 += 4) {
          double x[4], ex[4];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int k = k0 + kk;
            x[kk] = fma(dz, bq[k][2], fma(dy, bq[k][1], dx * bq[k][0]));
          }
          exp2s_shift_tab_n<4, TAB>(x, Mp, ex);
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int k = k0 + kk;
            e[k] = (FULL || NQ * cq + k < B) ? ex[kk] : 0.0;
            Zl += e[k];
            sl = fma(e[k], x[kk], sl);
            em = fmax(em, e[k]);
          }
        }
        // Z over the point's quad (two DPP rounds: the four lanes end bit-identical)
        double Z = Zl + dpp_f64<kDppXor1>(Zl);
        Z = Z + dpp_f64<kDppXor2>(Z);
        const double rZ = recip1(Z);
        entq = fma(sl * rZ, vf, entq);  // this lane's share of Σ R x
        mxr = fmax(mxr, em * rZ * vf);
        if (cq == 0) zst *= PAD ? fma(Z - 1.0, vf, 1.0) : Z;  // Π Z once per point
        // the responsibilities into the exp slab: row = the point within the sub-iteration
        {
          double* er = E + (lane >> 2) * ES + NQ * cq;
#pragma unroll
          for (int k = 0; k < NQ; k += 2) *reinterpret_cast<dvec2*>(er + k) = dvec2{e[k] * rZ, e[k + 1] * rZ};
        }
        lds_wave_sync();
        // B2 (lanes = 4 points x 16 bins): the sub-iteration's 4 MFMA steps
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int ss = 4 * sk + s;
          const int pl = 4 * ss + g;
          const double fb = F[bl * FS + pl];
          double fk[NX];
#pragma unroll
          for (int t = 0; t < NX; ++t) fk[t] = F[(16 + t) * FS + pl];
#pragma unroll
          for (int j = 0; j < BPL; ++j) {
            const double a = E[(4 * s + g) * ES + 16 * j + bl];
            acc4[ss % NACC][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, fb, acc4[ss % NACC][j], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < NX; ++t) accx[j][t] = fma(a, fk[t], accx[j][t]);
          }
        }
        lds_wave_sync();
      }
      int e8;
      zst = frexp(zst, &e8);
      zex += e8;
    }
  };
  if (chunk0 + (int64_t)iters * 256 <= n_cap) run_iters(std::false_type{});
  else run_iters(std::true_type{});
  int64_t npts = n_cap - chunk0;
  npts = npts < 0 ? 0 : (npts > (int64_t)iters * 256 ? (int64_t)iters * 256 : npts);
  // entropy over the chunk's valid points: Σ log Z' - Σ R x (x in units of ln2 / 2048) + ymax per valid
  // point - B ε per point; every lane holds its own points' Π Z (lane 0 of each wave adds the constants)
  const double logacc = log_pos(zst) + (double)zex * 0.69314718055994530942;
  const double ent = logacc - entq * kExp2C1 + ((lane == 0) ? (ymax * kExp2C1 - Beps) * (double)npts * 0.25 : 0.0);
#pragma unroll
  for (int j = 0; j < BPL; ++j)
    if (NACC == 2) acc4[0][j] += acc4[NACC - 1][j];
  if (ahead) ahead->valid = false;
  if (ctr && late_next && threadIdx.x == 0) *late_next = atomicAdd(ctr, 1u);
  const auto pre = [&]() {
    if (ctr && !late_next && threadIdx.x == 0) *task_slot = next;
  };
  const auto mid = [&]() {
    if (!ctr || late_next) return;
    const unsigned tn = *task_slot;
    ahead->t = tn;
    if (tn < T) task_operands<PRE>(A, (int)(tn % (unsigned)Hl), (int64_t)(tn / (unsigned)Hl), n_sel, stride, *ahead);
  };
  write_partial_record_mfma<BPL, NX, DF, FULL, WD>(acc4[0], accx, ent, mxr, sumw, (double)npts, B, lds, rec, pre, mid);
  __syncthreads();
}

// One task: hypothesis h, chunk c (its points: the tiers of FusedArgs) of the budgeted scan,
// its partial record written to rec. Ends with the workgroup synchronised (LDS free for the next task).
// Persistent form (ctr, task_slot, ahead non-null): the next task's ticket is taken by thread 0 at the
// start of the task's last iteration, broadcast through task_slot at the epilogue's first barrier, and
// the next task's operands are loaded into ahead during the rest of the epilogue (T tasks, H_l
// hypotheses: ticket t = chunk t / H_l, hypothesis t % H_l).
// SEL_CHECK: n_sel < 0 asks for the selection here (the non-look-ahead persistent form, which measured
// better with the launch's selection left in vector registers and this fallback: H = 256 1.1568 against
// 1.1592 ms with it scalar and given; profiles/r06/ab_bins_epilogue.txt)
template <int BPL, bool FULL, bool PRE, bool SEL_CHECK = false>
GC_DEV void bins_task(const FusedArgs& A, int h, int64_t c, double* lds, double* rec, unsigned* ctr,
                      unsigned* task_slot, TaskAhead* ahead, unsigned T, int Hl, unsigned* late_next, int bt_task,
                      int64_t n_sel, int64_t stride) {  // n_sel, stride: the launch's selection (selection_of)
  (void)bt_task;
  if constexpr (SEL_CHECK)
    if (n_sel < 0) selection_of(A, &n_sel, &stride);
  if constexpr (bins_lp(BPL)) {
    bins_task_lp<BPL, FULL, PRE>(A, h, c, lds, rec, ctr, task_slot, ahead, T, Hl, late_next, n_sel, stride);
    return;
  }
  constexpr int NF = NF_BASE;
  // features 0..8 and 10..16 on the matrix core, 17..18 on the VALU; feature 9 (w d_z²) is the trace
  // complement N − w d_x² − w d_y² (write_partial_record_mfma<.., 9>): one VALU feature fewer per step
  constexpr int DF = 9;
  constexpr int NX = NF - 16 - 1;
  constexpr int NS = kFusedNS;
  const int64_t n_cap = A.n_cap;
  const int B = A.B;
  int iters;
  const int64_t chunk0 = chunk_first(A, c, &iters);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, bl = lane & 15;
  const int fcol = bl >= DF ? bl + 1 : bl;  // the feature of this lane's MFMA column
  double* F = lds + wv * (NS * kFusedFS);
  const double o[3] = {A.o0, A.o1, A.o2};
  // the twist and iteration 0's raw point: loaded by the previous task's epilogue (persistent form), or
  // here
  TaskAhead ta_local;
  TaskAhead& ta = ahead ? *ahead : ta_local;
  if (!ahead || !ahead->valid) task_operands<PRE>(A, h, c, n_sel, stride, ta);
  double xr[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) xr[k] = ta.xr[k];
  const double* __restrict__ pts_raw = A.pts_raw;
  const double* __restrict__ t_raw = A.t_raw;
  const double* __restrict__ w_raw = A.w_raw;
  const double t0 = A.t0, t1 = A.t1;
  const double scale = A.bscal[2];
  const double denom = fmax(t1 - t0, 1e-12);
  const double inv_denom = 1.0 / denom;
  const double inv_sig = 1.0 / fmax(0.1 * denom, 1e-6);
  double* Tx = lds + 4 * kFusedFS * NS;
  double* Lb = Tx + kExpTab2;
  const double ysc = A.inv_tau * kTab2OverLn2;
  constexpr int NACC = kFusedNacc;
  v4d acc4[NACC][BPL];  // NACC = 2: even / odd steps, 2*BPL independent MFMA accumulation chains
  double accx[BPL][NX];
#pragma unroll
  for (int j = 0; j < BPL; ++j) {
    acc4[0][j] = v4d{0.0, 0.0, 0.0, 0.0};
    acc4[NACC - 1][j] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int t = 0; t < NX; ++t) accx[j][t] = 0.0;
  }
  double sumw = 0.0, entq = 0.0, mxr = 0.0;
  // Π Z of the lane's point group over the whole chunk as mantissa x 2^zex: renormalised every 8
  // points (Z >= e^{(S_max - 1)/τ} per point, so 8 factors stay normal for every τ the exp table
  // admits unless a direction lies almost opposite every bin), one log at the end
  double zst = 1.0;
  int zex = 0;
  // S <= 1 for unit vectors: the exp argument y - ymax = (S·ysc - ymax) <= 0 with an integer ymax
  // >= ysc (the shift cancels in R and is added back to the entropy below)
  const double ymax = ceil(ysc);
  const double Mp = kRoundMagic - ymax;  // the shift rides in the rounding constant (exp2s_shift_n)
  // raw point of the next iteration, loaded one iteration ahead (its HBM latency hides behind
  // this iteration's soft assignment)
  double np[3] = {0.0, 0.0, 0.0}, ntt = 0.0, nww = 0.0;
  auto fetch = [&](int it2) {
    const int64_t j = chunk0 + (int64_t)it2 * 256 + wv * 64 + lane;
    np[0] = 0.0; np[1] = 0.0; np[2] = 0.0; ntt = 0.0; nww = 0.0;
    if (j < n_cap && j < n_sel) {
      const int64_t i = j * stride;
      np[0] = pts_raw[3 * i]; np[1] = pts_raw[3 * i + 1]; np[2] = pts_raw[3 * i + 2];
      ntt = t_raw[i];
      nww = PRE ? A.w_win[j] : w_raw[i];  // PRE: the window is already applied (once per scan)
    }
  };
  {
    const bool ok = ta.ok;  // applied here, a task after the loads were issued
    np[0] = ok ? ta.np[0] : 0.0; np[1] = ok ? ta.np[1] : 0.0; np[2] = ok ? ta.np[2] : 0.0;
    ntt = ok ? ta.ntt : 0.0; nww = ok ? ta.nww : 0.0;
  }
  unsigned next = 0;
  // A chunk without padding points (all of it below n_cap: every chunk but the last) runs with
  // the valid flag folded to 1.0 — the masking multiplies vanish (x·1 = x, fma(Z−1, 1, 1) = Z
  // exactly), bit-identical to the masked form
  auto run_iters = [&](auto pad_tag) {
    constexpr bool PAD = decltype(pad_tag)::value;
    for (int it = 0; it < iters; ++it) {
      const int64_t wbase = chunk0 + (int64_t)it * 256 + wv * 64;
      // the next task's ticket, a whole iteration before the epilogue that broadcasts it (its round trip
      // is long done by then; the ticket is held one iteration, not the whole task)
      if (ctr && !late_next && it == iters - 1 && threadIdx.x == 0) next = atomicAdd(ctr, 1u);
      {  // phase A
        const int64_t j = wbase + lane;
        const bool inr = j < n_cap;
        double p[3] = {np[0], np[1], np[2]};
        const double tt = ntt, ww = nww * scale;
        if (it + 1 < iters) fetch(it + 1);
        double q[3], d[3], f[NF];
        const double al = (tt - t0) * inv_denom;
        {  // six series terms when every lane of the wave has θ² <= kDeskewShortTs (wave-uniform branch)
          const double ph[3] = {al * xr[3], al * xr[4], al * xr[5]};
          if (__all(dot3(ph, ph) <= kDeskewShortTs)) deskew_point_cross<true>(p, al, xr, q);
          else deskew_point_cross<false>(p, al, xr, q);
        }
        const double wd = inr ? (PRE ? ww : ww * window_weight2(tt, t0, t1, inv_sig, Tx)) : 0.0;
        direction_fast(q, o, 1e-12, d);
        point_features_w(q, d, wd, f);
        sumw += wd;
  #pragma unroll
        for (int k = 0; k < NF; ++k)
          if (k != DF) F[k * kFusedFS + lane] = f[k];
        F[(NF + 0) * kFusedFS + lane] = d[0];
        F[(NF + 1) * kFusedFS + lane] = d[1];
        F[(NF + 2) * kFusedFS + lane] = d[2];
        F[(NF + 3) * kFusedFS + lane] = inr ? 1.0 : 0.0;
      }
      lds_wave_sync();
      for (int s8 = 0; s8 < 16; s8 += kFusedUnr) {
  #pragma unroll
      for (int s = s8; s < s8 + kFusedUnr; ++s) {
        const int pl = s * 4 + g;
        const double d0 = F[(NF + 0) * kFusedFS + pl], d1 = F[(NF + 1) * kFusedFS + pl], d2 = F[(NF + 2) * kFusedFS + pl];
        const double vf = PAD ? F[(NF + 3) * kFusedFS + pl] : 1.0;  // 1 for a point of the chunk, 0 for padding
        const double fb = F[fcol * kFusedFS + pl];  // MFMA B operand: feature fcol of point 4s + g
        double e[BPL], x[BPL], ex[BPL];
  #pragma unroll
        for (int j = 0; j < BPL; ++j) {
          const int b = bl + 16 * j;  // Lb is zero past B: y = -ymax stays in range, then masked
          x[j] = fma(d0, Lb[b], fma(d1, Lb[64 + b], d2 * Lb[128 + b]));
        }
        exp2s_shift_tab_n<BPL, 8u * 4u * kFusedFS * kFusedNS>(x, Mp, ex);  // Tx at that absolute address
  #pragma unroll
        for (int j = 0; j < BPL; ++j) e[j] = (FULL || bl + 16 * j < B) ? ex[j] : 0.0;
        double zl = e[0];
  #pragma unroll
        for (int j = 1; j < BPL; ++j) zl += e[j];
        const double Z = group16_sum_bins(zl);
        const double rZ = recip1(Z);
        double r[BPL];
  #pragma unroll
        for (int j = 0; j < BPL; ++j) r[j] = e[j] * rZ;
        double rm = r[0];  // max responsibility: max(e) rZ == max(e rZ) exactly (monotone rounding)
  #pragma unroll
        for (int j = 1; j < BPL; ++j) rm = fmax(rm, r[j]);
        // padding points (vf = 0) add nothing: S/Z scaled by 0, r >= 0 scaled to 0 under the max,
        // and log Z replaced by log 1
  #pragma unroll
        for (int j = 0; j < BPL; ++j)  // lane partials of Σ R·x (in y units), summed over lanes at the end
          entq = fma(r[j] * vf, x[j], entq);
        mxr = fmax(mxr, rm * vf);
        zst *= PAD ? fma(Z - 1.0, vf, 1.0) : Z;  // Π Z of the group's points (<= 48^8 per renormalisation)
  #pragma unroll
        for (int j = 0; j < BPL; ++j)
          acc4[s % NACC][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(r[j], fb, acc4[s % NACC][j], 0, 0, 0);
  #pragma unroll
        for (int t = 0; t < NX; ++t) {
          const double fk = F[(17 + t) * kFusedFS + pl];
  #pragma unroll
          for (int j = 0; j < BPL; ++j) accx[j][t] = fma(r[j], fk, accx[j][t]);
        }
      }
        int e8;
        zst = frexp(zst, &e8);
        zex += e8;
      }
      lds_wave_sync();
#ifdef GC_BINS_TIMING
      if (it == 0 && threadIdx.x == 0 && bt_task >= 0 && bt_task < 16384) g_task_ep[2 * bt_task] = GC_BT_NOW();
#endif
    }
  };
  if (chunk0 + (int64_t)iters * 256 <= n_cap) run_iters(std::false_type{});
  else run_iters(std::true_type{});
#ifdef GC_BINS_TIMING
  if (threadIdx.x == 0 && bt_task >= 0 && bt_task < 16384) g_task_ep[2 * bt_task + 1] = GC_BT_NOW();
  if ((threadIdx.x & 63) == 0 && bt_task >= 0 && bt_task < 16384) g_task_wv[4 * bt_task + (threadIdx.x >> 6)] = GC_BT_NOW();
#endif
  // entropy sum over the chunk's valid points: Σ log Z - Σ S/Z - B ε
  int64_t npts = n_cap - chunk0;
  npts = npts < 0 ? 0 : (npts > (int64_t)iters * 256 ? (int64_t)iters * 256 : npts);
  // the 16 lanes of a point group hold the same product: only bin-lane 0 of each group contributes
  // its log. Σ log Z' (shifted by ymax) - Σ R y + ymax per valid point - B ε per point (lane 0 of
  // each wave)
  const double logacc = log_pos(zst) + (double)zex * 0.69314718055994530942;
  const double ent = (bl == 0 ? logacc : 0.0) - entq * kExp2C1 +
                     ((lane == 0) ? ent_shift(A.inv_tau, B) * (double)npts : 0.0);
#pragma unroll
  for (int j = 0; j < BPL; ++j)
    if (NACC == 2) acc4[0][j] += acc4[NACC - 1][j];
  if (ahead) ahead->valid = false;
  // without the look-ahead (late_next): the ticket taken here, its round trip overlapping the epilogue,
  // and broadcast by the caller after it
  if (ctr && late_next && threadIdx.x == 0) *late_next = atomicAdd(ctr, 1u);
  const auto pre = [&]() {  // before the epilogue's first barrier: the ticket into the task slot
    if (ctr && !late_next && threadIdx.x == 0) *task_slot = next;
  };
  const auto mid = [&]() {  // after it: every lane reads the ticket and loads the next task's operands
    if (!ctr || late_next) return;
    const unsigned tn = *task_slot;
    ahead->t = tn;
    if (tn < T) task_operands<PRE>(A, (int)(tn % (unsigned)Hl), (int64_t)(tn / (unsigned)Hl), n_sel, stride, *ahead);
  };
  write_partial_record_mfma<BPL, NX, DF, FULL, NS * kFusedFS>(acc4[0], accx, ent, mxr, sumw, (double)npts, B, lds, rec, pre, mid);
  __syncthreads();  // the epilogue's LDS reads are done before the next task writes the slabs
}

// Persistent form with the IMU/odom branch (the batched pipeline): workgroups [0, n_io) each run
// one hypothesis of the branch (io_branch_wg, independent of the bins); the rest stay resident and
// pull (hypothesis, chunk) tasks from a monotone counter until the H·chunks tasks are taken, so
// the branch's workgroups are dispatched first and the bin tasks balance over whatever CU slots
// remain — no stream fork / join and no partial last round of workgroups. Every task writes its
// own record, so the result does not depend on which workgroup ran it (bit-reproducible for a fixed
// device and shard size: the chunk geometry follows the CU count and H_l). ctr[0] is the task
// counter; the predict launch that precedes every k_bins_io on the stream zeroes it, so a launch
// never depends on how the previous one ended. No workgroup waits on another.
template <int BPL, bool FULL, bool AHEAD>
__global__ void __launch_bounds__(256, kFusedOcc) k_bins_io(FusedArgs A, PipeDev P, ScanArgs S,
                                                             const double* __restrict__ odom, int n_io, int io_on,
                                                             int H, int64_t chunks, unsigned* ctr) {
  extern __shared__ double lds[];
  unsigned& task_s = *reinterpret_cast<unsigned*>(lds + fused_lds_doubles(A.B));  // the launch's extra double
#ifdef GC_BINS_TIMING
  const double bt0 = GC_BT_NOW();
  double bt1 = bt0;
  int bt_n = 0;
#endif
  if ((int)blockIdx.x < n_io) {
    lpred_wg(P, S, blockIdx.x, lds);  // the predict's L_pred half (pred_mode 0), then the IMU/odom branch
    if (io_on) io_branch_wg(P, S, odom, blockIdx.x, lds);
#ifdef GC_BINS_TIMING
    if (threadIdx.x == 0 && blockIdx.x < 8192) {
      double* g = g_bins_trace + 4 * blockIdx.x;
      g[0] = bt0; g[1] = bt0; g[2] = GC_BT_NOW(); g[3] = -1.0;
    }
#endif
    return;
  }
  bins_prologue<BPL>(A, lds);
#ifdef GC_BINS_TIMING
  bt1 = GC_BT_NOW();
#endif
  const int RL = A.B * NF_BASE + REC_EXTRA;
  const unsigned T = (unsigned)(H * chunks);
  // the next task's ticket is taken inside the current task before its epilogue, so the atomic's
  // round trip overlaps the epilogue (bins_task ends with a barrier: task_s is read by all before it
  // is rewritten). Taken at the start of the task instead, a ticket was held for the whole task: at
  // the end of the launch a workgroup pairing a long task with another on its CU (each then runs at
  // half speed) started its reserved one ~180 us late (GC_BINS_TIMING task traces)
  if (threadIdx.x == 0) task_s = atomicAdd(ctr, 1u);
  __syncthreads();
  TaskAhead ahead;
  ahead.valid = false;
  ahead.ok = false;
  ahead.t = task_s;
  int64_t n_sel, stride;  // the a1 selection, shared by every task of the launch
  selection_of(A, &n_sel, &stride);
  // uniform values in scalar registers: held in VGPRs they were spilled, and each task's reload waited
  // (in-order vmcnt) on the previous epilogue's look-ahead loads
  if constexpr (AHEAD) {
    n_sel = uniform_i64(n_sel);
    stride = uniform_i64(stride);
  }
  for (;;) {
    // uniform: the task's record pointer lives in scalar registers (held in a VGPR it was spilled and
    // its reload waited on the look-ahead loads issued before it)
    const unsigned t = __builtin_amdgcn_readfirstlane(ahead.t);
    if (t >= T) break;
    // chunk-major: the workgroups in flight share a chunk's raw points across hypotheses (L2)
    const int64_t c = t / H;
    const int h = t % H;
#ifdef GC_BINS_TIMING
    const double tt0 = GC_BT_NOW();
#endif
    if constexpr (AHEAD) {
      bins_task<BPL, FULL, true>(A, h, c, lds, A.partials + ((int64_t)h * chunks + c) * RL, ctr, &task_s, &ahead, T, H,
                                 nullptr, (int)t, n_sel, stride);
    } else {
      unsigned next = 0;
      bins_task<BPL, FULL, true, true>(A, h, c, lds, A.partials + ((int64_t)h * chunks + c) * RL, ctr, &task_s, &ahead, T,
                                 H, &next, (int)t, n_sel, stride);
      if (threadIdx.x == 0) task_s = next;
      __syncthreads();
      ahead.t = task_s;
    }
#ifdef GC_BINS_TIMING
    ++bt_n;
    if (threadIdx.x == 0 && t < 16384) {
      unsigned xcc = 0;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      double* g = g_task_trace + 4 * t;
      g[0] = tt0; g[1] = GC_BT_NOW(); g[2] = (double)blockIdx.x; g[3] = (double)(xcc & 0xf);
    }
#endif
  }
#ifdef GC_BINS_TIMING
  if (threadIdx.x == 0 && blockIdx.x < 8192) {
    double* g = g_bins_trace + 4 * blockIdx.x;
    g[0] = bt0; g[1] = bt1; g[2] = GC_BT_NOW(); g[3] = (double)bt_n;
  }
#endif
}

// Grid form (the gc_scan_bins_fused entry): grid (chunks, H), one task per workgroup.
template <int BPL, bool FULL>
__global__ void __launch_bounds__(256, kFusedOcc) k_bins_fused(FusedArgs A) {
  extern __shared__ double lds[];
  bins_prologue<BPL>(A, lds);
  const int RL = A.B * NF_BASE + REC_EXTRA;
  int64_t n_sel, stride;
  selection_of(A, &n_sel, &stride);
  bins_task<BPL, FULL, false>(A, blockIdx.y, blockIdx.x, lds,
                       A.partials + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * RL, nullptr, nullptr, nullptr,
                       0u, 1, nullptr, -1, n_sel, stride);
}

// ================================================================ finalize (a6 + certs)
// One workgroup per hypothesis: chunk records summed in order, per-bin moments -> p̄, Σ_p
// (PSD-projected), κ; cert reductions in a fixed order.
// one hypothesis h (the whole workgroup); sm: B*NF + REC_EXTRA + 8 doubles
// One hypothesis h on a 1024-thread workgroup (kFinWG): the entry sums with 4x the loads in flight of
// a 256-thread one (the reduction is L2-latency-bound at small H), then per-bin moments -> p̄, Σ_p
// (PSD-projected), κ on lanes b < B of wave 0 (B <= 64) and the cert reductions on that wave.
// sm: B*NF + REC_EXTRA doubles.
constexpr int kFinWG = 1024;
GC_DEV void finalize_hyp(int h, int B, int NF, int64_t chunks, const double* __restrict__ partials, double eps_psd,
                         double eps_mass, double* stats, double* cert, double* sm) {
  const int RL = B * NF + REC_EXTRA;
  const double* P = partials + (int64_t)h * chunks * RL;
  const int imax = B * NF + 1;  // the max-responsibility entry reduces by fmax
  if (RL <= kFinWG) finalize_reduce<1, 32>(P, RL, imax, chunks, sm);
  else finalize_reduce<2, 16>(P, RL, imax, chunks, sm);
  __syncthreads();
  double Nl = 0.0, N2l = 0.0, psdl = 0.0, epsl = 0.0, sfl = 0.0;
  if ((int)threadIdx.x < B) {
    const int b = threadIdx.x;
    const double N = sm[b * NF];
    finalize_bin(sm + b * NF, NF, eps_psd, eps_mass, stats + ((int64_t)h * B + b) * GC_BIN_STATS, &psdl, &epsl);
    Nl = N; N2l = N * N; sfl = N / (N + eps_mass);
  }
  if (threadIdx.x >= 64) return;  // every bin lives on wave 0 (B <= 64)
  const double Nt = wave_sum(Nl);
  const double N2 = wave_sum(N2l);
  const double psd = wave_sum(psdl);
  const double mer = wave_max(epsl);
  const double sf = wave_sum(sfl);
  if (threadIdx.x == 0) {
    const double* ex = sm + B * NF;
    double* c = cert + (int64_t)h * GC_BIN_CERT;
    c[0] = Nt * Nt / (N2 + eps_mass);
    c[1] = sf / (double)B;
    c[2] = psd;
    c[3] = mer;
    c[4] = ex[0] / (ex[3] + eps_mass);
    c[5] = ex[1];
    c[6] = ex[2];
    c[7] = psd + mer;
  }
}
__global__ void __launch_bounds__(kFinWG) k_bins_finalize(int B, int NF, int64_t chunks,
                                                       const double* __restrict__ partials,
                                                       double eps_psd, double eps_mass,
                                                       double* stats, double* cert) {
  extern __shared__ double sm[];  // B*NF + 8 + 4
  finalize_hyp(blockIdx.x, B, NF, chunks, partials, eps_psd, eps_mass, stats, cert, sm);
}

// The batched pipeline's finalize, split over bins: grid (S, H), workgroup s of hypothesis h owns
// bins [s kFinBins, (s+1) kFinBins) (and, the last one, the record's extra entries). One lane per
// record entry sums the chunk records in chunk order (finalize_reduce's order and batching, so
// every sum is bit-identical to k_bins_finalize's), then one lane per bin runs finalize_bin. At
// small H this spreads a hypothesis's ~0.6 MB of records over S CUs instead of one (k_bins_finalize
// is bound by one CU's load rate there). The cross-bin certificate reductions need every bin: the
// per-bin projection delta and mass-epsilon ratio go to aux (H, B, 2) and k_evidence reduces them
// (finalize_cert), in k_bins_finalize's wave_sum order.
constexpr int kFinBins = 6;
// chunk records in flight per lane in the split finalize (one L2 round trip per batch)
#ifndef GC_FIN_KU
#define GC_FIN_KU 16
#endif
constexpr int kFinSplitWG = 128;
// up to this many chunk records per hypothesis (H = 256: 18, C5's 1024: 17) the evidence workgroup of
// each hypothesis sums its own records (one more L2 round trip per 8 chunks at its start) in place of
// this kernel's launch; more (H = 32: 80) keep the split kernel, which spreads them over 8 CUs
#ifndef GC_FOLD_CHUNKS
#define GC_FOLD_CHUNKS 32
#endif
constexpr int64_t kFoldChunks = GC_FOLD_CHUNKS;
static_assert(kFinBins * NF_BASE + REC_EXTRA <= kFinSplitWG, "one lane per record entry");
__global__ void __launch_bounds__(kFinSplitWG) k_bins_finalize_split(int B, int NF, int64_t chunks,
                                                                     const double* __restrict__ partials,
                                                                     double eps_psd, double eps_mass, double* stats,
                                                                     double* cert, double* aux, int64_t* done_word,
                                                                     int64_t ticket) {
  __shared__ double sm[kFinBins * NF_BASE + REC_EXTRA];
  // the bins launch before this one on the stream has completed, its reads of the scan slot
  // included: publish the scan's ticket to the host-coherent word the pipeline's staging checks.
  // Relaxed at system scope: one write-through store, no L2 writeback (nothing written before it
  // has to be visible to the host).
  if (done_word && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    __hip_atomic_store(done_word, ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const int h = blockIdx.y, s = blockIdx.x;
  const int RL = B * NF + REC_EXTRA;
  const int b0 = s * kFinBins, nb = min(kFinBins, B - b0);
  const bool last = s == (int)gridDim.x - 1;
  const int ne = nb * NF + (last ? REC_EXTRA : 0);
  const int e0 = b0 * NF, imax = B * NF + 1;
  const double* P = partials + (int64_t)h * chunks * RL;
  const int t = threadIdx.x;
  if (t < ne) {
    const int e = e0 + t;
    constexpr int KU = GC_FIN_KU;
    double v = 0.0;
    for (int64_t c = 0; c < chunks; c += KU) {
      double x[KU];
#pragma unroll
      for (int u = 0; u < KU; ++u) x[u] = c + u < chunks ? P[(c + u) * RL + e] : 0.0;
#pragma unroll
      for (int u = 0; u < KU; ++u) v = e == imax ? fmax(v, x[u]) : v + x[u];
    }
    sm[t] = v;
  }
  __syncthreads();
  if (t < nb) {
    double* ax = aux + ((int64_t)h * B + b0 + t) * 2;
    finalize_bin(sm + t * NF, NF, eps_psd, eps_mass, stats + ((int64_t)h * B + b0 + t) * GC_BIN_STATS, ax, ax + 1);
  } else if (last && t == 64) {
    const double* ex = sm + nb * NF;
    double* c = cert + (int64_t)h * GC_BIN_CERT;
    c[4] = ex[0] / (ex[3] + eps_mass);
    c[5] = ex[1];
    c[6] = ex[2];
  }
}

__global__ void k_kappa(int64_t n, const double* __restrict__ R, double eps_r, double d, double r0,
                        double tau, double* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = kappa_blend(R[i], eps_r, d, r0, tau);
}

__global__ void k_psd3(int batch, const double* __restrict__ M, double eps, double* Mo, double* cert) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch) return;
  double A[9], P[9], c[6];
  for (int k = 0; k < 9; ++k) A[k] = M[9 * i + k];
  psd_project3(A, eps, P, c);
  for (int k = 0; k < 9; ++k) Mo[9 * i + k] = P[k];
  for (int k = 0; k < 6; ++k) cert[6 * i + k] = c[k];
}

__global__ void __launch_bounds__(256) k_psd_wg(int d, const double* __restrict__ M, double eps,
                                                double* Mo, double* cert) {
  __shared__ double Ml[kDZ * kDZ], Mp[kDZ * kDZ], scr[2 * kDZ * kDZ + 4 * kDZ], red[4], c6[6];
  const int i = blockIdx.x;
  for (int k = threadIdx.x; k < d * d; k += kWG) Ml[k] = M[(int64_t)i * d * d + k];
  __syncthreads();
  wg_psd_project(Ml, Mp, eps, d, scr, red, c6);
  for (int k = threadIdx.x; k < d * d; k += kWG) Mo[(int64_t)i * d * d + k] = Mp[k];
  if (threadIdx.x < 6) cert[6 * i + threadIdx.x] = c6[threadIdx.x];
}

// domain_projection_psd_core (primitives.py:80-123) for any d (the per-operator drop-in; the
// pipeline uses the fixed-size forms above). An odd d is padded to even dp with a zero row and
// column: every Jacobi rotation touching the pad has a_pq = 0, so it is the identity, the pad stays
// decoupled with eigenvalue 0, contributes nothing to the d x d reconstruction (V[i][pad] = 0) and
// is left out of the certificate. Workspace: 3 dp² + 4 dp + 8 doubles of LDS (dp <= 64) or of
// global scratch (the same code on global pointers; __syncthreads orders the workgroup's accesses).
__host__ __device__ inline int psd_ws_len(int dp) { return 3 * dp * dp + 4 * dp + 8; }
__global__ void __launch_bounds__(256) k_psd_any(int d, const double* __restrict__ M, double eps, double* Mo,
                                                 double* cert, double* gws) {
  extern __shared__ double lds_psd[];
  const int dp = d + (d & 1);
  const int64_t i = blockIdx.x;
  double* A = gws ? gws + i * psd_ws_len(dp) : lds_psd;
  double* V = A + dp * dp;
  double* Ms = V + dp * dp;
  double* w = Ms + dp * dp;
  double* cs = w + dp;
  double* red = cs + 3 * dp;
  const double* Mi = M + i * d * d;
  double symloc = 0.0;
  for (int idx = threadIdx.x; idx < dp * dp; idx += kWG) {
    const int r = idx / dp, c = idx % dp;
    double sv = 0.0;
    if (r < d && c < d) {
      sv = 0.5 * (Mi[r * d + c] + Mi[c * d + r]);
      const double dd = sv - Mi[r * d + c];
      symloc += dd * dd;
    }
    A[idx] = sv;
    Ms[idx] = sv;
  }
  __syncthreads();
  const double symd = wg_sum(symloc, red);
  wg_jacobi_eigh(A, V, w, dp, cs, red);
  double mnl = 1e308, mxl = -1e308, nnl = 0.0;
  for (int k = threadIdx.x; k < dp; k += kWG) {
    const double wc = fmax(w[k], eps);
    w[k] = wc;
    if (k < d) {
      mnl = fmin(mnl, wc); mxl = fmax(mxl, wc); nnl += (wc < 10.0 * eps) ? 1.0 : 0.0;
    }
  }
  const double mn = -wg_max(-mnl, red);
  const double mx = wg_max(mxl, red);
  const double nn = wg_sum(nnl, red);
  double projloc = 0.0;
  for (int idx = threadIdx.x; idx < d * d; idx += kWG) {
    const int r = idx / d, c = idx % d;
    double v = 0.0;
    for (int k = 0; k < dp; ++k) v += V[r * dp + k] * w[k] * V[c * dp + k];
    const double dd = v - Ms[r * dp + c];
    projloc += dd * dd;
    Mo[i * d * d + idx] = v;
  }
  const double proj = wg_sum(projloc, red);
  if (threadIdx.x == 0) {
    double* c6 = cert + 6 * i;
    c6[0] = sqrt(proj); c6[1] = sqrt(symd); c6[2] = mn; c6[3] = mx; c6[4] = mx / mn; c6[5] = nn;
  }
}

// ------------------------------------------------------------------------ launch helpers
static int bpl_for(int B) { return (B + 15) / 16; }

}  // namespace gc

using namespace gc;

static int pick_iters(int64_t n, int H, int max_iters = 8, int64_t min_wgs = 2048) {
  // Aim for >= ~4 workgroups per CU-slot while keeping partial records small. The fused kernel
  // takes 16 (its per-workgroup prologue, the 16 KB exp table and the bin directions, and the
  // partial-record epilogue amortise over twice the points: 1.667 -> 1.604 ms/scan, 32 no better)
  // and halves only below 1024 workgroups (a 32-hypothesis shard: 8 iterations, 0.404 -> 0.395
  // ms/scan against 4).
  int iters = max_iters;
  while (iters > 1 && ((n + iters * 256 - 1) / (iters * 256)) * (int64_t)H < min_wgs) iters >>= 1;
  return iters;
}

namespace gc {
hipError_t launch_budget_stats(const double* d_w, int64_t n_in, int64_t n_cap, double* part, double* out,
                               hipStream_t st) {
  const int64_t stride = budget_stride(n_in, n_cap);
  hipLaunchKernelGGL(k_budget_partials, dim3(kBudgetBlocks), dim3(256), 0, st, d_w, n_in, stride, part);
  hipLaunchKernelGGL(k_budget_final, dim3(1), dim3(64), 0, st, (const double*)part, n_in, n_cap, stride, out);
  return hipGetLastError();
}
}  // namespace gc

extern "C" {


int32_t gc_budget_stats(gc_ctx* ctx, const double* d_w, int64_t n_in, int64_t n_cap, double* d_out) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, n_in > 0 && n_cap > 0, "n_in and n_cap must be positive");
  GC_CHECK_ARG(ctx, d_w && d_out, "NULL buffer");
  void* scr;
  if (int rc = gc::scratch(ctx, sizeof(double) * 3 * kBudgetBlocks, &scr)) return rc;
  GC_HIP(ctx, gc::launch_budget_stats(d_w, n_in, n_cap, (double*)scr, d_out, ctx->stream));
  return GC_OK;
}

int32_t gc_point_budget_resample(gc_ctx* ctx, const double* d_points, const double* d_t, const double* d_w,
                                 const uint8_t* d_ring, const uint8_t* d_tag, int64_t n_in, int64_t n_cap,
                                 double* d_points_out, double* d_t_out, double* d_w_out, uint8_t* d_ring_out,
                                 uint8_t* d_tag_out, int64_t* d_idx_out, double* d_scalars_out) {
  int32_t rc = gc_budget_stats(ctx, d_w, n_in, n_cap, d_scalars_out);
  if (rc) return rc;
  GC_CHECK_ARG(ctx, d_points && d_t && d_points_out && d_t_out && d_w_out, "NULL buffer");
  const int64_t stride = std::max<int64_t>(1, (n_in + n_cap - 1) / n_cap);
  hipLaunchKernelGGL(k_budget_gather, dim3((unsigned)((n_cap + 255) / 256)), dim3(256), 0, ctx->stream,
                     d_points, d_t, d_w, d_ring, d_tag, n_in, n_cap, stride, d_scalars_out, d_points_out,
                     d_t_out, d_w_out, d_ring_out, d_tag_out, d_idx_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_deskew_constant_twist(gc_ctx* ctx, int32_t H, int64_t n, const double* d_points, const double* d_t,
                                 const double* d_w, double t0, double t1, const double* d_xi,
                                 double* d_points_out, double* d_w_out, double* d_sum_w_out) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, H > 0 && n > 0, "H and n must be positive");
  GC_CHECK_ARG(ctx, d_points && d_t && d_w && d_xi && d_points_out && d_w_out && d_sum_w_out, "NULL buffer");
  const int64_t blocks = (n + 255) / 256;
  void* scr;
  if (int rc = gc::scratch(ctx, sizeof(double) * blocks * H, &scr)) return rc;
  hipLaunchKernelGGL(k_deskew, dim3((unsigned)blocks, H), dim3(256), 0, ctx->stream, n, d_points, d_t, d_w, t0,
                     t1, d_xi, d_points_out, d_w_out, (double*)scr);
  GC_LAUNCH_CHECK(ctx);
  hipLaunchKernelGGL(k_sum_rows, dim3((H + 63) / 64), dim3(64), 0, ctx->stream, (const double*)scr, blocks, H,
                     d_sum_w_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_point_directions(gc_ctx* ctx, int64_t rows, const double* d_points, const double* h_origin3,
                            double eps_mass, double* d_dirs_out) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, rows > 0 && d_points && h_origin3 && d_dirs_out, "bad arguments");
  hipLaunchKernelGGL(k_point_dirs, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, ctx->stream, rows,
                     d_points, h_origin3[0], h_origin3[1], h_origin3[2], eps_mass, d_dirs_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_bin_soft_assign(gc_ctx* ctx, int32_t H, int64_t n, int32_t B, const double* d_dirs,
                           const double* d_bins, double tau, double* d_resp_out, int32_t* d_bin_index_out,
                           double* d_cert_out) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, H > 0 && n > 0, "H and n must be positive");
  GC_CHECK_ARG(ctx, B >= 1 && B <= 64, "B must be in [1, 64]");
  GC_CHECK_ARG(ctx, tau > 0.0, "tau must be positive");
  GC_CHECK_ARG(ctx, d_dirs && d_bins && d_resp_out && d_cert_out, "NULL buffer");
  constexpr int kSaIters = 8;
  int iters = kSaIters;
  while (iters > 1 && ((n + iters * 256 - 1) / (iters * 256)) * (int64_t)H < 4096) iters >>= 1;
  const int64_t blocks = (n + iters * 256 - 1) / (iters * 256);
  void* scr;
  if (int rc = gc::scratch(ctx, sizeof(double) * 2 * blocks * H, &scr)) return rc;
  const double inv_tau = 1.0 / tau;
  dim3 grid((unsigned)blocks, H);
  const bool full = (B % 16) == 0 && ((uintptr_t)d_resp_out & 15) == 0;
#define GC_SA(BP)                                                                                        \
  do {                                                                                                   \
    const size_t sh = sizeof(double) * (size_t)sa_lds_doubles(BP, full);                                 \
    if (full) {                                                                                          \
      GC_HIP(ctx, gc::ensure_dyn_lds((const void*)k_soft_assign<BP, true>, sh));                          \
      hipLaunchKernelGGL((k_soft_assign<BP, true>), grid, dim3(256), sh, ctx->stream, n, B, iters, d_dirs, \
                         d_bins, inv_tau, d_resp_out, d_bin_index_out, (double*)scr);                    \
    } else {                                                                                             \
      GC_HIP(ctx, gc::ensure_dyn_lds((const void*)k_soft_assign<BP, false>, sh));                         \
      hipLaunchKernelGGL((k_soft_assign<BP, false>), grid, dim3(256), sh, ctx->stream, n, B, iters, d_dirs, \
                         d_bins, inv_tau, d_resp_out, d_bin_index_out, (double*)scr);                    \
    }                                                                                                    \
  } while (0)
  switch (bpl_for(B)) { case 1: GC_SA(1); break; case 2: GC_SA(2); break; case 3: GC_SA(3); break; default: GC_SA(4); }
#undef GC_SA
  GC_LAUNCH_CHECK(ctx);
  hipLaunchKernelGGL(k_soft_assign_finalize, dim3((H + 63) / 64), dim3(64), 0, ctx->stream, (const double*)scr,
                     blocks, H, n, d_cert_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

static int32_t launch_finalize(gc_ctx* ctx, int H, int B, int NF, int64_t chunks, const double* partials,
                               double eps_psd, double eps_mass, double* stats, double* cert) {
  const size_t sh = sizeof(double) * (B * NF + REC_EXTRA);
  hipLaunchKernelGGL(k_bins_finalize, dim3(H), dim3(kFinWG), sh, ctx->stream, B, NF, chunks, partials, eps_psd,
                     eps_mass, stats, cert);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_scan_bin_moment_match(gc_ctx* ctx, int32_t H, int64_t n, int32_t B, const double* d_points,
                                 const double* d_covs, const double* d_w, const double* d_resp,
                                 const double* d_lambda, const double* h_origin3, double eps_psd, double eps_mass,
                                 double* d_stats_out, double* d_cert_out) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, H > 0 && n > 0, "H and n must be positive");
  GC_CHECK_ARG(ctx, B >= 1 && B <= 64, "B must be in [1, 64]");
  GC_CHECK_ARG(ctx, d_points && d_w && d_resp && d_stats_out && d_cert_out, "NULL buffer");
  double o[3] = {0.0, 0.0, 0.0};
  if (h_origin3) { o[0] = h_origin3[0]; o[1] = h_origin3[1]; o[2] = h_origin3[2]; }
  // chunk = 4 waves x groups x 32 points; aim for >= ~8 workgroups per CU over the grid
  int groups = 16;
  while (groups > 1 && ((n + 128 * groups - 1) / (128 * groups)) * (int64_t)H < 4096) groups >>= 1;
  const int64_t chunks = (n + 128 * groups - 1) / (128 * groups);
  const bool cov = d_covs != nullptr;
  const int NF = cov ? NF_BASE + NF_COV : NF_BASE;
  const int RL = B * NF + REC_EXTRA;
  void* scr;
  if (int rc = gc::scratch(ctx, sizeof(double) * RL * chunks * H, &scr)) return rc;
  dim3 grid((unsigned)chunks, H);
  const int bpl = bpl_for(B);
  const int NT = (NF + 15) / 16;
  const size_t sh = sizeof(double) * std::max<size_t>((size_t)4 * 16 * NT * kMomFS, (size_t)4 * B * NF);
  const bool pair = B >= 32 && ((uintptr_t)d_resp & 15) == 0;
#define GC_MOM_L(BP, CV, LM, PR)                                                                                 \
  hipLaunchKernelGGL((k_moment_partials<BP, CV, LM, 1, PR>), grid, dim3(256), sh, ctx->stream, n, B, groups,    \
                     d_points, d_covs, d_w, d_resp, d_lambda, o[0], o[1], o[2], (double*)scr)
#define GC_MOM(BP, CV)                                                                                          \
  do {                                                                                                          \
    if (d_lambda) {                                                                                             \
      if (pair && BP >= 2) GC_MOM_L(BP, CV, true, (BP >= 2)); else GC_MOM_L(BP, CV, true, false);              \
    } else {                                                                                                    \
      if (pair && BP >= 2) GC_MOM_L(BP, CV, false, (BP >= 2)); else GC_MOM_L(BP, CV, false, false);            \
    }                                                                                                           \
  } while (0)
  if (cov) {
    switch (bpl) { case 1: GC_MOM(1, true); break; case 2: GC_MOM(2, true); break; case 3: GC_MOM(3, true); break; default: GC_MOM(4, true); }
  } else {
    switch (bpl) { case 1: GC_MOM(1, false); break; case 2: GC_MOM(2, false); break; case 3: GC_MOM(3, false); break; default: GC_MOM(4, false); }
  }
#undef GC_MOM
#undef GC_MOM_L
  GC_LAUNCH_CHECK(ctx);
  return launch_finalize(ctx, H, B, NF, chunks, (const double*)scr, eps_psd, eps_mass, d_stats_out, d_cert_out);
}

int32_t gc_scan_bins_fused(gc_ctx* ctx, int32_t H, int64_t n_in, int64_t n_cap, int32_t B,
                           const double* d_points_raw, const double* d_t_raw, const double* d_w_raw,
                           const double* d_budget_scalars, double t0, double t1, const double* d_xi,
                           const double* d_bins, double tau, const double* h_origin3, double eps_psd,
                           double eps_mass, double* d_stats_out, double* d_cert_out, int32_t iters) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, H > 0 && n_in > 0 && n_cap > 0, "H, n_in, n_cap must be positive");
  GC_CHECK_ARG(ctx, B >= 1 && B <= 64, "B must be in [1, 64]");
  // the table exp's exponent splice holds for arguments down to -2/τ (in units of ln 2 / 2048 that
  // is 2^-1022): below the floor the smallest responsibilities would wrap instead of underflowing
  GC_CHECK_ARG(ctx, tau >= GC_FUSED_TAU_MIN, "tau must be >= GC_FUSED_TAU_MIN (3e-3) for the fused kernel");
  GC_CHECK_ARG(ctx, iters >= 0 && iters <= 64, "iters must be in [0, 64] (0 = by grid size)");
  GC_CHECK_ARG(ctx, d_points_raw && d_t_raw && d_w_raw && d_budget_scalars && d_xi && d_bins && h_origin3 &&
                        d_stats_out && d_cert_out, "NULL buffer");
  (void)n_in;
  if (iters == 0) iters = pick_iters(n_cap, H, 16, 1024);
  const int64_t chunks = (n_cap + iters * 256 - 1) / (iters * 256);
  const int NF = NF_BASE;
  const int RL = B * NF + REC_EXTRA;
  const int bpl = bpl_for(B);
  void* scr;
  if (int rc = gc::scratch(ctx, sizeof(double) * RL * chunks * H, &scr)) return rc;
  const size_t sh = sizeof(double) * fused_lds_doubles(B);
  dim3 grid((unsigned)chunks, H);
  const FusedArgs FA{n_cap, B, iters, d_points_raw, d_t_raw, d_w_raw, d_budget_scalars, t0, t1, d_xi, d_bins,
                     1.0 / tau, h_origin3[0], h_origin3[1], h_origin3[2], (double*)scr, nullptr, chunks, iters,
                     0, iters};
#define GC_FUSED(BP, FULL)                                                                                     \
  GC_HIP(ctx, gc::ensure_dyn_lds((const void*)k_bins_fused<BP, FULL>, sh));                                   \
  if (int rc_ = gc::ensure_no_static_lds(ctx, (const void*)k_bins_fused<BP, FULL>)) return rc_;               \
  hipLaunchKernelGGL((k_bins_fused<BP, FULL>), grid, dim3(256), sh, ctx->stream, FA)
  const bool full = B == 16 * bpl;
  switch (bpl) {
    case 1: if (full) { GC_FUSED(1, true); } else { GC_FUSED(1, false); } break;
    case 2: if (full) { GC_FUSED(2, true); } else { GC_FUSED(2, false); } break;
    case 3: if (full) { GC_FUSED(3, true); } else { GC_FUSED(3, false); } break;
    default: if (full) { GC_FUSED(4, true); } else { GC_FUSED(4, false); } break;
  }
#undef GC_FUSED
  GC_LAUNCH_CHECK(ctx);
  return launch_finalize(ctx, H, B, NF, chunks, (const double*)scr, eps_psd, eps_mass, d_stats_out, d_cert_out);
}

}  // extern "C"

namespace gc {
// The batched pipeline's a1 -> a6 bins for its Hl local hypotheses, with the IMU/odom branch's
// workgroups in the same launch when io (k_bins_io), then the chunk-order finalize.
int32_t scan_bins_pipeline(gc_ctx* ctx, const PipeDev& P, const ScanArgs& S, const double* d_odom, bool io,
                           const double* d_pts, const double* d_t, const double* d_w, int64_t n_in,
                           int64_t* done_word, int64_t ticket, BinsFold* fold) {
  (void)n_in;
  if (ctx->cu_count == 0) {
    int cus = 0;
    GC_HIP(ctx, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    ctx->cu_count = cus > 0 ? cus : 1;
  }
  const int H = P.Hl, B = P.B;
  const int pullers = 2 * ctx->cu_count;  // 2 resident bin workgroups per CU (VGPR-bound)
  // the largest iteration count that still gives every puller >= 4 tasks (tail <= 1/4 task)
  // Two tiers of chunks, taken in order: long tasks (iters x 256 points, the prologue / epilogue
  // amortised) for the bulk, then short ones (2 x 256) that hold one long task of work per puller,
  // so the pullers run out of work together instead of one long task apart (A/B on one box against
  // half a long task: 1.2998/1.2984/1.2981 vs 1.3004/1.2997/1.2990 ms at H = 256, 0.342 vs 0.345 at 32)
  // (P.geom_H > 0: sized as for a shard of that many hypotheses, the summation order then being the
  // same for every shard size)
  const int64_t U = (P.n_cap + 255) / 256;  // 256-point units per hypothesis
  const int Hg = P.geom_H > 0 ? P.geom_H : H;
  // >= 2 long tasks per puller: with the late ticket and the tiny tier (below) the tail no longer
  // needs a third, and fewer, longer tasks amortise each task's set-up and record epilogue: H = 32
  // 4 -> 8 iterations, 92 -> 62 chunks, 0.2892 -> 0.2800 ms/scan (3 tasks: 0.2892, 1: 0.2848;
  // profiles/r04/ab_bins_tail.txt); H >= 64 keep 16
#ifndef GC_BINS_MIN_TASKS
#define GC_BINS_MIN_TASKS 2
#endif
  constexpr int kBinsMinTasks = GC_BINS_MIN_TASKS;
  // at most 32 iterations (8192 points) per long task: H = 256 1.1935 -> 1.1803 ms, H = 128 0.6706 ->
  // 0.6658 against 16; 64: 1.1872 (profiles/r04/ab_bins_tail.txt)
  int iters = 32;
  while (iters > 2 && (int64_t)Hg * U < kBinsMinTasks * (int64_t)pullers * iters) iters >>= 1;
#ifndef GC_BINS_SHORT_DIV
#define GC_BINS_SHORT_DIV 2
#endif
  constexpr int kShortDiv = GC_BINS_SHORT_DIV;
#ifndef GC_BINS_TINY_DIV
#define GC_BINS_TINY_DIV 4
#endif
#ifndef GC_BINS_TINY_PER_PULLER
#define GC_BINS_TINY_PER_PULLER 1
#endif
  constexpr int kTinyDiv = GC_BINS_TINY_DIV, kTinyPerPuller = GC_BINS_TINY_PER_PULLER;
  // short tasks of half a long one, at least 2 iterations: H = 256 8-iteration short tasks (interleaved
  // A/B on one box, 1.2499/1.2463 ms/scan with 4 -> 1.2377/1.2391 with 8); H = 32 (4-iteration long
  // tasks) 2, which stays best there (0.3013/0.3004/0.3003 ms against 0.305-0.313 for 8-iteration long
  // tasks with 2- or 4-iteration short ones and for 4-iteration tasks only; tools/ab32.sh)
  const int kItersShort = std::max(2, iters / kShortDiv);
  // a third tier of tiny tasks (a quarter of a short one) at the very end, about one per puller: with
  // the next ticket taken before each task's epilogue (k_bins_io) the pullers' end spread fell from
  // 57 to ~24 us at H = 256 (GC_BINS_TIMING traces); interleaved A/B against the two tiers and the
  // ticket taken at the task start, 1.1999 -> 1.1950 ms at H = 256, 0.2930 -> 0.2903 at H = 32
  // (profiles/r04/ab_bins_tail.txt; 2 tiny tasks per puller, or an eighth or a half of a short task,
  // no better)
  const int kItersTiny = std::max(1, kItersShort / kTinyDiv);
  int64_t Ut = ((int64_t)pullers * kItersTiny * kTinyPerPuller + Hg - 1) / Hg;
  Ut = std::min<int64_t>((Ut + kItersTiny - 1) / kItersTiny * kItersTiny, U);
  // the short tier's work: one long task per puller when every puller has at least 4 long tasks (H = 256),
  // three quarters of one with fewer 32-iteration tasks (H = 128: 0.6497 -> 0.6459 ms/scan), half of one when
  // the long tasks are shorter (H = 32's 8 iterations, H = 64's 16): with few long tasks per puller the
  // epilogues of the many short tasks cost more than the finer tail gains (H = 32 0.2586 -> 0.2548 ms/scan;
  // H = 256 1.1624 against 1.1656 with half, 1.1648 with three quarters; profiles/r05/ab_bins_short_share.txt)
#ifndef GC_BINS_SHORT_SHARE
#define GC_BINS_SHORT_SHARE 0.5
#endif
#ifndef GC_BINS_SHORT_SHARE_32
#define GC_BINS_SHORT_SHARE_32 0.75
#endif
  const bool many_long = (int64_t)Hg * U >= 4 * (int64_t)pullers * iters;
  const double short_share = many_long ? 1.0 : (iters >= 32 ? GC_BINS_SHORT_SHARE_32 : GC_BINS_SHORT_SHARE);
  int64_t Us = std::max<int64_t>(iters, (int64_t)(short_share * (double)pullers * iters + Hg - 1) / Hg);
  Us = std::min(Us, U - Ut);
  const int64_t k1 = (U - Ut - Us) / iters;  // long chunks; the short and tiny tiers take the rest
  const int64_t k2 = (U - Ut - k1 * iters) / kItersShort;
  Ut = U - k1 * iters - k2 * kItersShort;
  const int64_t chunks = k1 + k2 + (Ut + kItersTiny - 1) / kItersTiny;
  GC_CHECK_ARG(ctx, (int64_t)H * chunks < (int64_t)0xFFFFFFFF, "too many bin tasks");
  const int NF = NF_BASE;
  const int RL = B * NF + REC_EXTRA;
  void* scr;
  if (int rc = gc::scratch(ctx, sizeof(double) * RL * chunks * H, &scr)) return rc;
  const FusedArgs FA{P.n_cap, B, iters, d_pts, d_t, d_w, P.budget, S.t0, S.t1, P.xi, P.bins, 1.0 / P.tau,
                     P.o0, P.o1, P.o2, (double*)scr, P.w_win, k1, kItersShort, k2, kItersTiny};
  // one auxiliary workgroup per hypothesis first: the predict's L_pred half (lpred_wg), then, when io,
  // the IMU/odom branch
  const int n_io = H, io_on = io ? 1 : 0;
  // + 1: the pullers' task slot after the fused layout (no static LDS in k_bins_io: the dynamic block
  // starts at LDS address 0, so the exp table's addresses need no base add, exp2s_shift_tab_n)
  const size_t sh = sizeof(double) * (std::max<size_t>(std::max<size_t>(fused_lds_doubles(B), (size_t)kLpredLdsDoubles),
                                                       io ? (size_t)kIoLdsDoubles : 0) + 1);
  const dim3 grid((unsigned)(n_io + pullers));
  // the look-ahead instantiation (the next task's operands loaded during the current task's epilogue,
  // the ticket taken one iteration earlier) for short tasks: H = 32's 8-iteration tasks 0.2597 ->
  // 0.2582 ms; H = 256's 32-iteration tasks keep the late ticket (holding it an iteration longer cost
  // as much as the hidden loads gained, 1.1699 -> 1.1709; profiles/r05/ab_bins_ahead.txt). One
  // instantiation per form: both paths in one kernel raised its spills and cost H = 32 10 us.
  const bool ahead = iters < 32;
#define GC_BIO2(BP, FULL, AH)                                                                                  \
  GC_HIP(ctx, gc::ensure_dyn_lds((const void*)k_bins_io<BP, FULL, AH>, sh));                                  \
  if (int rc_ = gc::ensure_no_static_lds(ctx, (const void*)k_bins_io<BP, FULL, AH>)) return rc_;              \
  hipLaunchKernelGGL((k_bins_io<BP, FULL, AH>), grid, dim3(256), sh, ctx->stream, FA, P, S, d_odom, n_io, io_on, H,   \
                     chunks, P.task_ctr)
#define GC_BIO(BP, FULL)          \
  if (ahead) {                    \
    GC_BIO2(BP, FULL, true);      \
  } else {                        \
    GC_BIO2(BP, FULL, false);     \
  }
  const int bpl = bpl_for(B);
  const bool full = B == 16 * bpl;
  switch (bpl) {
    case 1: if (full) { GC_BIO(1, true); } else { GC_BIO(1, false); } break;
    case 2: if (full) { GC_BIO(2, true); } else { GC_BIO(2, false); } break;
    case 3: if (full) { GC_BIO(3, true); } else { GC_BIO(3, false); } break;
    default: if (full) { GC_BIO(4, true); } else { GC_BIO(4, false); } break;
  }
#undef GC_BIO
#undef GC_BIO2
  GC_LAUNCH_CHECK(ctx);
  if (fold && chunks <= kFoldChunks && fold_record_fits(B)) {  // k_evidence reduces the records (gc_evidence.hip)
    fold->part = (const double*)scr;
    fold->chunks = chunks;
    return GC_OK;
  }
  if (fold) fold->part = nullptr;
  const dim3 fgrid((unsigned)((B + kFinBins - 1) / kFinBins), (unsigned)H);
  hipLaunchKernelGGL(k_bins_finalize_split, fgrid, dim3(kFinSplitWG), 0, ctx->stream, B, NF, chunks,
                     (const double*)scr, P.eps_psd, P.eps_mass, P.stats, P.bincert, P.binaux, done_word, ticket);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}
}  // namespace gc

extern "C" {

#ifdef GC_BINS_TIMING
// dev: the last k_bins_io launch's per-workgroup trace (4 doubles each) into h_out
int32_t gc_dev_bins_trace(double* h_out, int64_t n_wg) {
  if (n_wg < 0 || n_wg > 8192) return GC_ERR_RUNTIME;
  return hipMemcpyFromSymbol(h_out, HIP_SYMBOL(gc::g_bins_trace), sizeof(double) * 4 * n_wg) == hipSuccess
             ? GC_OK : GC_ERR_RUNTIME;
}
int32_t gc_dev_task_wv_trace(double* h_out, int64_t n_tasks) {
  if (n_tasks < 0 || n_tasks > 16384) return GC_ERR_RUNTIME;
  return hipMemcpyFromSymbol(h_out, HIP_SYMBOL(gc::g_task_wv), sizeof(double) * 4 * n_tasks) == hipSuccess
             ? GC_OK : GC_ERR_RUNTIME;
}
int32_t gc_dev_task_ep_trace(double* h_out, int64_t n_tasks) {
  if (n_tasks < 0 || n_tasks > 16384) return GC_ERR_RUNTIME;
  return hipMemcpyFromSymbol(h_out, HIP_SYMBOL(gc::g_task_ep), sizeof(double) * 2 * n_tasks) == hipSuccess
             ? GC_OK : GC_ERR_RUNTIME;
}
int32_t gc_dev_task_trace(double* h_out, int64_t n_tasks) {
  if (n_tasks < 0 || n_tasks > 16384) return GC_ERR_RUNTIME;
  return hipMemcpyFromSymbol(h_out, HIP_SYMBOL(gc::g_task_trace), sizeof(double) * 4 * n_tasks) == hipSuccess
             ? GC_OK : GC_ERR_RUNTIME;
}
#endif

int32_t gc_kappa_from_resultant_batch(gc_ctx* ctx, int64_t n, const double* d_R, double eps_r, double d,
                                      double r0, double tau, double* d_kappa_out) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, n >= 0 && d_R && d_kappa_out, "bad arguments");
  if (n == 0) return GC_OK;
  hipLaunchKernelGGL(k_kappa, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, n, d_R, eps_r, d, r0,
                     tau, d_kappa_out);
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

int32_t gc_domain_projection_psd_batch(gc_ctx* ctx, int32_t batch, int32_t d, const double* d_M, double eps_psd,
                                       double* d_M_out, double* d_cert_out) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, batch >= 0 && d_M && d_M_out && d_cert_out, "bad arguments");
  GC_CHECK_ARG(ctx, d >= 1 && d <= 512, "d must be in [1, 512]");
  if (batch == 0) return GC_OK;
  if (d == 3) {
    hipLaunchKernelGGL(k_psd3, dim3((batch + 63) / 64), dim3(64), 0, ctx->stream, batch, d_M, eps_psd, d_M_out,
                       d_cert_out);
  } else if (d <= kDZ && d % 2 == 0) {
    hipLaunchKernelGGL(k_psd_wg, dim3(batch), dim3(256), 0, ctx->stream, d, d_M, eps_psd, d_M_out, d_cert_out);
  } else {
    const int dp = d + (d & 1);
    const size_t ws = sizeof(double) * (size_t)psd_ws_len(dp);
    if (dp <= 64) {
      GC_HIP(ctx, gc::ensure_dyn_lds((const void*)k_psd_any, ws));
      hipLaunchKernelGGL(k_psd_any, dim3(batch), dim3(256), ws, ctx->stream, d, d_M, eps_psd, d_M_out, d_cert_out,
                         (double*)nullptr);
    } else {
      void* scr;
      if (int rc = gc::scratch(ctx, ws * (size_t)batch, &scr)) return rc;
      hipLaunchKernelGGL(k_psd_any, dim3(batch), dim3(256), 0, ctx->stream, d, d_M, eps_psd, d_M_out, d_cert_out,
                         (double*)scr);
    }
  }
  GC_LAUNCH_CHECK(ctx);
  return GC_OK;
}

}  // extern "C"
