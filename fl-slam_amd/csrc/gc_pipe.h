// gc_pipe.h — device-resident state of the batched per-scan pipeline (one rank's shard of
// hypotheses) and the launch interface shared by gc_belief.hip and gc_pipeline.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gc {

constexpr int kMapRec = 26;   // [S_dir 3, S_dir_scatter 9, N_dir, N_pos, sum_p 3, sum_ppT 9]
constexpr int kMapDer = 17;   // [mu_dir 3, kappa, centroid 3, Sigma_c 9, pad]
constexpr int kPredCert = 8;  // [lift, psd_delta, eig_min, eig_max, cond, nnc, trace_cov, trigger]
constexpr int kImuOut = 8;    // [ess_scan, sigma_warp, dt_imu, omega_avg 3, pad 2]
constexpr int kIoCert = 10;   // [ess odom/imu/gyro, sf odom/imu/gyro, exc_dt, exc_ex, nll, trigger]
constexpr int kHypDiag = 40;
constexpr int kMuAux = 50;    // [mu_prev 22 (belief_prev increment), mu_inc 22 (belief_pred), pose0 6]
constexpr int kIoParts = 40;  // GC_IO_PARTS layout (include/gcslam.h)
constexpr int kOdomLen = 84;  // [pose 6, cov 36, twist 6, twist_cov 36]  // see include/gcslam.h GC_HYP_DIAG layout
constexpr int kCombCert = 16;
constexpr int kBudgetBlocks = 64;  // a1 budget partial workgroups (gc_budget.h)

// Partial-sum record exchanged between ranks once per scan (doubles).
constexpr int kPL = 0, kPH = 484, kPZ = 506, kPMU = 528, kPMU2 = 550, kPDPSIP = 551, kPDNUP = 803,
              kPDPSIM = 810, kPDNUM = 837, kPX0 = 841, kPSTAMP0 = 847, kPMAP = 848;
// after the map increments: hypothesis 0's [z_t 6 (recomposed world pose), Σ_post pose block 36,
// ξ_body 6] for the in-scan PrimitiveMap update every rank runs (gc_scanmap.hip)
constexpr int kH0Len = 48;
// the in-scan map update's snapshot (PipeDev::smap_snap): [reduced h0 record 48 | the measurement-IW
// LiDAR block [ν_2, Ψ_2 (9)] before the scan's IW apply 10 | the scan's 8 a1 budget scalars]
constexpr int kSnapIW = kH0Len, kSnapBudget = kSnapIW + 10, kSnapLen = 72;
__host__ __device__ inline int rec_h0(int B) { return kPMAP + B * kMapRec; }
__host__ __device__ inline int partial_len(int B) { return rec_h0(B) + kH0Len; }

struct PipeDev {
  int Hl;        // local hypotheses
  int H;         // total hypotheses
  int h_begin;   // global index of local hypothesis 0
  int B;         // bins
  int M;         // IMU slots (<= 512)
  int geom_H;    // bins chunk geometry as for this many hypotheses (0: Hl)
  int predict_route;  // 0: split predict (lift solves, L_pred in the bins launch) when certified; 1: always
                      // the factorised chain in the predict kernel (gc_pipeline_set_predict_route)
  int cus;       // compute units of the pipeline's device (ctx->device, queried once at create): every
                 // grid-size decision (predict's budget workgroups, the chain kernels' occupancy) uses it
  int64_t n_in, n_cap;
  double tau, o0, o1, o2;
  double eps_psd, eps_lift, eps_mass, lambda_ou, c_frob, forgetting, weight_floor;
  double power_beta_min, power_beta_exc_c, power_beta_z_c, alpha_min, alpha_max, c0_cond;
  double nu_max;
  double planar_z_ref, planar_z_sigma, planar_vz_sigma, gravity_scale;
  // per local hypothesis
  double *X, *z, *L, *h, *stamp;           // belief (in/out)
  double *Lpred, *hpred, *pred_cert, *pose_pred, *xi, *imu_out, *dPsiM;
  double *pred_mode;                       // (Hl) 0: L_pred / h_pred / pred_cert are formed by the bins
                                           // launch's workgroup of the hypothesis (lpred_wg); 1: by the
                                           // predict kernel itself (its factorised fallback route)
  double *stats, *bincert;                 // (Hl, B, 38), (Hl, 8)
  double *binaux;                          // (Hl, B, 2) per-bin [projection delta, mass-eps ratio]
  double *io_L, *io_h, *io_cert;           // IMU/odom-branch evidence (computed or given)
  double *mu_aux, *io_parts;               // (Hl, kMuAux), (Hl, kIoParts)
  double *dPsiP, *mu_fin, *diag;
  double *lpose;                           // (Hl, 36) pose block of L_evidence (diagnostics tape)
  double *Sig;                             // (Hl, 22, 22) Σ_post = (L_post + εI)⁻¹ of the last scan
  double *hcond;                           // (Hl, 2, 4) in-scan ConditioningCerts [L_pred, L_post] (gc_certs.hip)
  double *praw;                            // (Hl, 18) the unprojected MF L_rot and planar L_trans of the last
                                           // scan (k_evidence), for their projection certificates
  double *pcert;                           // (Hl (B + 2) + kScanCerts, 6) full projection certificates
                                           // (gc_certs.hip, layout GC_PCERT_* in include/gcslam.h)
  // shared
  double *weights;                         // (H)
  double *Q;                               // (22, 22)
  double *bins;                            // (B, 3)
  double *map, *map_der, *map_misc;        // (B, 26), (B, 17), [z_scale, N_dir_total, ...]
  double *map_inc;                         // (B, 26) written by hypothesis 0's owner
  double *h0rec;                           // (kH0Len) hypothesis 0's pose block (its owner's k_evidence)
  double *nu_proc, *Psi_proc, *nu_meas, *Psi_meas;  // (7), (7,36), (3), (3,9)
  double *smap_snap;                       // (kSnapLen) the in-scan map update's inputs of the scan, written by
                                           // k_combine_final (gc_scanmap.hip); the host alternates two blocks
                                           // per scan so the update can run on a stream of its own
  double *budget;                          // the scan's 8 a1 budget scalars: formed by the predict launch's
                                           // extra workgroups, or copied there from S.budget
  double *budget_part;                     // (64, 3) a1 partials of those workgroups
  unsigned *budget_ticket;                 // their arrival counter (reset by the last)
  unsigned *task_ctr;                      // k_bins_io task counter (zeroed by the predict launch)
  double *w_win;                           // (n_cap) selected points' w x time window, written by the predict
                                           // launch (per point, shared by every hypothesis)
  double *send, *gather;                   // (P), (G, P)
  int G;                                   // ranks
  double *comb;                            // combined belief: L 484, h 22, z 22, X 6, stamp, cert 16
  double *iw_cert;                         // [proc psd, proc nu, meas psd, meas nu]
  double *iwraw;                           // (kIwRawLen) the scan's unprojected IW blocks (k_combine_final):
                                           // process 7 x 6x6 masked, measurement 3 x 3x3 symmetrised
};

constexpr int kIwRawLen = 7 * 36 + 3 * 9;
// scan-level projection certificates after the per-hypothesis ones: the barycenter L, the 7 process-IW
// blocks, the 3 measurement-IW blocks, Q
constexpr int kScanCerts = 12;

struct ScanArgs {
  const double *imu_t, *imu_g, *imu_a;     // (M), (M,3), (M,3)
  double t0, t1, t_last, t_scan, dt;
  double w_process;                        // min(1, scan_count)
  const double* w_raw;                     // (n_in) raw point weights
  int64_t n_in;                            // raw points of this scan
  const double* budget;                    // (8) the a1 budget scalars of w_raw when they were formed at
                                           // staging (the slot's, !predict_budget_inline); read through P.budget
  const double* t_raw;                     // (n_in) raw point times (the window of P.w_win)
  int sig_cached;                          // P.Sig / P.mu_fin hold (P.L + εI)⁻¹ and its solve with P.h
  // the a6 finalize folded into k_evidence (few chunk records per hypothesis, BinsFold): the bins
  // launch's chunk records and count; null when the split finalize kernel ran
  const double* fin_part;
  int64_t fin_chunks;
  int64_t* done_word;                      // with fin_part: the ticket published by k_evidence
  int64_t ticket;
};

// dev instrumentation: -DGC_PHASE_TIMING records s_memtime at phase boundaries of workgroup wg
// (hypothesis 0's, or combine_final's IW workgroup) into io_parts[slot] (read with the pipeline in
// GC_IO_GIVEN mode; tools/phase_timing.py); compiled out otherwise
#ifdef GC_PHASE_TIMING
#define GC_PHASE_WG(P, i, wg)                                                             \
  do {                                                                                   \
    __syncthreads();                                                                     \
    if (blockIdx.x == (wg) && threadIdx.x == 0) (P).io_parts[i] = (double)__builtin_readcyclecounter(); \
  } while (0)
#else
#define GC_PHASE_WG(P, i, wg) \
  do {                        \
  } while (0)
#endif
#define GC_PHASE(P, i) GC_PHASE_WG(P, i, 0)

// launchers (gc_belief.hip)
hipError_t launch_predict_imu(const PipeDev& P, const ScanArgs& S, hipStream_t st);
// the predict launch forms the a1 budget itself (its extra workgroups fit beside Hl hypotheses);
// otherwise the staging must (S.budget)
bool predict_budget_inline(const PipeDev& P);
// a1 budget scalars into out (8) with 3 x 64 partials in part (gc_points.hip)
hipError_t launch_budget_stats(const double* d_w, int64_t n_in, int64_t n_cap, double* part, double* out,
                               hipStream_t st);
hipError_t launch_evidence(const PipeDev& P, const ScanArgs& S, hipStream_t st);
hipError_t launch_combine_local(const PipeDev& P, hipStream_t st);
hipError_t launch_combine_final(const PipeDev& P, const ScanArgs& S, hipStream_t st,
                                hipEvent_t done = nullptr);  // recorded at the launch's completion
hipError_t launch_map_derive(const PipeDev& P, hipStream_t st);
hipError_t launch_iw_Q(const PipeDev& P, hipStream_t st);
// the per-hypothesis ConditioningCerts of L_pred and L_post into P.hcond (gc_certs.hip)
hipError_t launch_hyp_certs(const PipeDev& P, hipStream_t st);
// the full projection certificates of the last scan into P.pcert (gc_certs.hip)
hipError_t launch_proj_certs(const PipeDev& P, hipStream_t st);
}  // namespace gc

struct gc_ctx;
namespace gc {
// a1 -> a6 bins of the local hypotheses (+ the IMU/odom branch's workgroups in the same launch when
// io) and their finalize into P.stats / P.bincert (gc_points.hip)
// (done_word: `ticket` stored once the bins have completed). With fold non-null and few chunk records
// per hypothesis the finalize is left to k_evidence: fold receives the records, and the evidence
// launch publishes the ticket
struct BinsFold {
  const double* part = nullptr;
  int64_t chunks = 0;
};
int32_t scan_bins_pipeline(gc_ctx* ctx, const PipeDev& P, const ScanArgs& S, const double* d_odom, bool io,
                           const double* d_pts, const double* d_t, const double* d_w, int64_t n_in,
                           int64_t* done_word = nullptr, int64_t ticket = 0, BinsFold* fold = nullptr);

}  // namespace gc
