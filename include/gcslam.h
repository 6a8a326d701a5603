/*
 * gcslam.h — C-ABI of libgcslam: the MI355X-native GC-SLAM v2 per-scan hot path.
 *
 * Drop-in boundary for the reference's operator API (fl_slam_poc.backend.operators,
 * docs/OPERATOR_CONTRACTS.md:3,35-38): every operator of the 14-step per-scan pipeline is an
 * `extern "C"` entry over plain pointers and sizes. The Python host package (gcslam) binds it
 * with ctypes and rebuilds the reference's (Result, CertBundle, ExpectedEffect) tuples.
 *
 * Conventions
 *  - All arithmetic is IEEE f64, as in the reference (jax_enable_x64, common/jax_init.py:32).
 *  - Array arguments named d_* are DEVICE pointers (gc_buffer_alloc), row-major, C-contiguous.
 *    Batched entries take H hypotheses stacked on the leading axis. Host pointers are h_*.
 *  - Every entry is enqueued on the context's HIP stream and returns immediately unless noted;
 *    gc_ctx_synchronize() waits. Entries never retain caller pointers.
 *  - Return codes: GC_OK, GC_ERR_ARG (shape/argument error -> Python ValueError),
 *    GC_ERR_RUNTIME (HIP/RCCL failure -> RuntimeError). gc_last_error() has the message.
 *  - Re-entrant: no global mutable state; one gc_ctx (stream) per calling thread
 *    (backend_node.py:1340-1381 worker-thread model).
 */
#ifndef GCSLAM_H_
#define GCSLAM_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GC_OK 0
#define GC_ERR_ARG 1
#define GC_ERR_RUNTIME 2

/* Per-bin statistics record written by the bin kernels (doubles per bin):
 * [0] N  [1:4] s_dir  [4:13] S_dir_scatter  [13:16] p_bar  [16:25] Sigma_p  [25] kappa
 * [26:29] sum_p  [29:38] sum_ppT   (ScanBinStats, archive/legacy_operators/binning.py:39-48) */
#define GC_BIN_STATS 38
/* Per-hypothesis bin certificate row (doubles):
 * [0] ess [1] support_frac [2] psd_projection_delta_total [3] max_mass_epsilon_ratio
 * [4] avg_entropy (soft-assign) [5] max_resp [6] sum of deskewed weights [7] trigger magnitude */
#define GC_BIN_CERT 8

typedef struct gc_ctx gc_ctx;
typedef struct gc_event gc_event;

/* ------------------------------------------------------------------ runtime */
int32_t gc_version(void);
/* Message of the last failing call on this ctx (ctx may be NULL for creation errors). */
const char* gc_last_error(const gc_ctx* ctx);
int32_t gc_device_count(int32_t* count);
int32_t gc_ctx_create(int32_t device, gc_ctx** out);
int32_t gc_ctx_destroy(gc_ctx* ctx);
int32_t gc_ctx_synchronize(gc_ctx* ctx);
int32_t gc_buffer_alloc(gc_ctx* ctx, uint64_t bytes, void** d_ptr);
int32_t gc_buffer_free(gc_ctx* ctx, void* d_ptr);
/* Synchronous copies (stream-ordered, then waited). */
int32_t gc_buffer_upload(gc_ctx* ctx, void* d_dst, const void* h_src, uint64_t bytes);
int32_t gc_buffer_download(gc_ctx* ctx, void* h_dst, const void* d_src, uint64_t bytes);
int32_t gc_buffer_copy(gc_ctx* ctx, void* d_dst, const void* d_src, uint64_t bytes);
int32_t gc_buffer_memset(gc_ctx* ctx, void* d_dst, int32_t value, uint64_t bytes);
/* HIP events on the ctx stream (for in-process kernel timing). */
int32_t gc_event_create(gc_ctx* ctx, gc_event** out);
int32_t gc_event_destroy(gc_event* ev);
int32_t gc_event_record(gc_ctx* ctx, gc_event* ev);
int32_t gc_event_elapsed_ms(gc_event* start, gc_event* stop, float* ms);

/* ------------------------------------------------------------------ a1 PointBudgetResample
 * Replaces backend/operators/point_budget.py:50-109 (_point_budget_resample_core) and the
 * stride of :160. stride = max(1, ceil(n_in / n_cap)); selection = arange(0, n_in, stride).
 * Outputs (n_cap rows, zero padded): d_points_out (n_cap,3), d_t_out, d_w_out (n_cap),
 * d_ring_out/d_tag_out (n_cap, u8; inputs may be NULL -> zeros), d_idx_out (n_cap, int64,
 * -1 padded). d_scalars_out (8): [mass_in, mass_selected, mass_scale, ess, sum_w_out,
 * n_selected, stride, support_frac]. */
int32_t gc_point_budget_resample(gc_ctx* ctx, const double* d_points, const double* d_t,
                                 const double* d_w, const uint8_t* d_ring, const uint8_t* d_tag,
                                 int64_t n_in, int64_t n_cap, double* d_points_out, double* d_t_out,
                                 double* d_w_out, uint8_t* d_ring_out, uint8_t* d_tag_out,
                                 int64_t* d_idx_out, double* d_scalars_out);

/* ------------------------------------------------------------------ a4 DeskewConstantTwist
 * Replaces backend/operators/deskew_constant_twist.py:31-69 for H twists over one point set:
 * p0 = Exp(α ξ_h)^{-1} p, α = (t - t0)/max(t1 - t0, 1e-12); w_out = w · window(t).
 * d_xi (H,6); d_points_out (H,n,3); d_w_out (H,n); d_sum_w_out (H) = Σ w_out (retained cert). */
int32_t gc_deskew_constant_twist(gc_ctx* ctx, int32_t H, int64_t n, const double* d_points,
                                 const double* d_t, const double* d_w, double t0, double t1,
                                 const double* d_xi, double* d_points_out, double* d_w_out,
                                 double* d_sum_w_out);

/* Ray directions (pipeline.py:589-593): d = (p - o) / (||p - o|| + eps_mass). (rows = H*n) */
int32_t gc_point_directions(gc_ctx* ctx, int64_t rows, const double* d_points, const double* h_origin3,
                            double eps_mass, double* d_dirs_out);

/* ------------------------------------------------------------------ a5 BinSoftAssign
 * Replaces archive/legacy_operators/binning.py:56-76 (_bin_soft_assign_core), batched over H.
 * d_dirs (H,n,3); d_bins (B,3), B <= 64; d_resp_out (H,n,B) = softmax(dirs·binsᵀ/τ);
 * d_bin_index_out (H,n) int32 = argmax_b of the un-fused f64 d0*b0+d1*b1+d2*b2 (lowest index
 * on ties; may be NULL); d_cert_out (H,2) = [avg_entropy, max_resp]. */
int32_t gc_bin_soft_assign(gc_ctx* ctx, int32_t H, int64_t n, int32_t B, const double* d_dirs,
                           const double* d_bins, double tau, double* d_resp_out,
                           int32_t* d_bin_index_out, double* d_cert_out);

/* ------------------------------------------------------------------ a6 ScanBinMomentMatch
 * Replaces binning.py:139-209 (_scan_bin_moment_match_core) incl. KappaFromResultant
 * (kappa.py:130-169) and InvMass (primitives.py:195-212), batched over H.
 * d_points (H,n,3), d_covs (H,n,3,3) or NULL (= zeros), d_w (H,n), d_resp (H,n,B),
 * d_lambda (H,n) or NULL (= ones), h_origin3 (host, 3). Outputs d_stats_out (H,B,GC_BIN_STATS)
 * and d_cert_out (H,GC_BIN_CERT) (entries [4:7] zero). */
int32_t gc_scan_bin_moment_match(gc_ctx* ctx, int32_t H, int64_t n, int32_t B, const double* d_points,
                                 const double* d_covs, const double* d_w, const double* d_resp,
                                 const double* d_lambda, const double* h_origin3, double eps_psd,
                                 double eps_mass, double* d_stats_out, double* d_cert_out);

/* Fused a1->a4->a5->a6 over H hypotheses of one raw scan (the batched pipeline's hot kernel):
 * budget selection (stride from n_in/n_cap, weights x d_budget_scalars[2]), per-hypothesis
 * deskew by d_xi (H,6), directions from h_origin3, soft assignment to d_bins (B,3) at tau and
 * moment accumulation — responsibilities never touch HBM. Same outputs as the contract pair
 * (d_stats_out (H,B,GC_BIN_STATS), d_cert_out (H,GC_BIN_CERT) incl. [4:7]).
 * d_budget_scalars: the 8 scalars written by gc_point_budget_resample / gc_budget_stats. */
int32_t gc_scan_bins_fused(gc_ctx* ctx, int32_t H, int64_t n_in, int64_t n_cap, int32_t B,
                           const double* d_points_raw, const double* d_t_raw, const double* d_w_raw,
                           const double* d_budget_scalars, double t0, double t1, const double* d_xi,
                           const double* d_bins, double tau, const double* h_origin3,
                           double eps_psd, double eps_mass, double* d_stats_out, double* d_cert_out);

/* Budget reduction only (no gather): writes the 8 budget scalars. */
int32_t gc_budget_stats(gc_ctx* ctx, const double* d_w, int64_t n_in, int64_t n_cap,
                        double* d_scalars_out);

/* kappa_from_resultant_batch (kappa.py:130-169). */
int32_t gc_kappa_from_resultant_batch(gc_ctx* ctx, int64_t n, const double* d_R, double eps_r,
                                      double d, double r0, double tau, double* d_kappa_out);

/* domain_projection_psd_core (primitives.py:80-123) over `batch` d x d matrices (d <= 22 even, or
 * d == 3). d_cert_out (batch,6) = [projection_delta, sym_delta, eig_min, eig_max, cond, nnc]. */
int32_t gc_domain_projection_psd_batch(gc_ctx* ctx, int32_t batch, int32_t d, const double* d_M,
                                       double eps_psd, double* d_M_out, double* d_cert_out);

/* ------------------------------------------------------------------ batched scan pipeline
 * Replaces the per-hypothesis loop + combine + IW apply of backend_node.py:2036-2119 (and
 * process_scan_single_hypothesis, pipeline.py:316-1591, with the legacy bin path a4-a8 of
 * SURVEY §3.2) by one device-resident driver over this rank's shard of hypotheses. */
typedef struct gc_pipeline gc_pipeline;
typedef struct gc_comm gc_comm;

typedef struct {
  int32_t H_total;   /* hypotheses per scan (all ranks) */
  int32_t h_begin;   /* first global hypothesis of this rank */
  int32_t h_count;   /* hypotheses on this rank (<= 1024) */
  int32_t B;         /* bins (<= 64) */
  int32_t M;         /* IMU slots (GC_MAX_IMU_PREINT_LEN = 512) */
  int32_t world_size;
  int32_t rank;
  int32_t pad_;
  int64_t n_in_max;  /* raw points per scan (max) */
  int64_t n_cap;     /* N_POINTS_CAP */
} gc_pipeline_dims;

/* configuration doubles (PipelineConfig, pipeline.py:96-160; constants.py) */
#define GC_PCFG_TAU 0
#define GC_PCFG_ORIGIN 1 /* 3: lidar origin in the base frame */
#define GC_PCFG_EPS_PSD 4
#define GC_PCFG_EPS_LIFT 5
#define GC_PCFG_EPS_MASS 6
#define GC_PCFG_LAMBDA_OU 7
#define GC_PCFG_C_FROB 8
#define GC_PCFG_FORGETTING 9
#define GC_PCFG_WEIGHT_FLOOR 10
#define GC_PCFG_POWER_BETA_MIN 11
#define GC_PCFG_POWER_BETA_EXC_C 12
#define GC_PCFG_POWER_BETA_Z_C 13
#define GC_PCFG_ALPHA_MIN 14
#define GC_PCFG_ALPHA_MAX 15
#define GC_PCFG_C0_COND 16
#define GC_PCFG_NU_MAX 17
#define GC_PCFG_LEN 18

#define GC_PIPE_MAX_SLOTS 8
/* map bin record (B x 26): [S_dir 3, S_dir_scatter 9, N_dir, N_pos, sum_p 3, sum_ppT 9] */
#define GC_MAP_REC 26
/* map-derived record (B x 17): [mu_dir 3, kappa, centroid 3, Sigma_c 9, pad] */
#define GC_MAP_DER 17
/* IMU/odom-branch cert row (10): ess odom/imu/gyro, support odom/imu/gyro, exc_dt, exc_ex,
 * nll_per_ess sum, trigger-magnitude sum */
#define GC_IO_CERT 10
/* per-hypothesis diagnostics (40): [0:6] world pose of the final belief, 6 T, 7 beta, 8 alpha,
 * 9 s_dt, 10 s_ex, 11 anchor rho, 12 frobenius strength, 13 cond_pose6, 14 ess_total,
 * 15 dt_asymmetry, 16 z_to_xy, 17 nll_per_ess, 18 MF trigger, 19 planar trigger,
 * 20 fusion psd delta, [21:24] t_wls, [24:27] log R_mf, [27:30] MF singular values,
 * [30:36] xi_body, 36 support_frac, 37 excitation_total */
#define GC_HYP_DIAG 40
/* combined output (GC_COMB_LEN): L 484, h 22, z_lin 22, X_anchor(hyp 0) 6, then
 * [stamp, psd_delta, eig_min, eig_max, cond, nnc, ess, support_frac, mass_eps_ratio,
 *  floor_adjustment, spread_proxy, 5 pad] */
#define GC_COMB_LEN (484 + 22 + 22 + 6 + 16)

int32_t gc_pipeline_create(gc_ctx* ctx, const gc_pipeline_dims* dims, const double* h_cfg, gc_pipeline** out);
int32_t gc_pipeline_destroy(gc_pipeline* p);
int32_t gc_pipeline_set_bins(gc_pipeline* p, const double* h_bins);
int32_t gc_pipeline_set_beliefs(gc_pipeline* p, const double* h_X, const double* h_z, const double* h_L,
                                const double* h_h, const double* h_stamp);
int32_t gc_pipeline_get_beliefs(gc_pipeline* p, double* h_X, double* h_z, double* h_L, double* h_h,
                                double* h_stamp);
int32_t gc_pipeline_set_weights(gc_pipeline* p, const double* h_weights);
int32_t gc_pipeline_set_io_evidence(gc_pipeline* p, const double* h_L, const double* h_h, const double* h_cert);
int32_t gc_pipeline_set_iw(gc_pipeline* p, const double* h_nu_proc7, const double* h_Psi_proc7x36,
                           const double* h_nu_meas3, const double* h_Psi_meas3x9);
int32_t gc_pipeline_get_iw(gc_pipeline* p, double* h_nu_proc7, double* h_Psi_proc7x36, double* h_nu_meas3,
                           double* h_Psi_meas3x9, double* h_Q22x22, double* h_cert4);
int32_t gc_pipeline_set_map(gc_pipeline* p, const double* h_map);
int32_t gc_pipeline_get_map(gc_pipeline* p, double* h_map, double* h_map_der, double* h_misc2);
int32_t gc_pipeline_stage_scan(gc_pipeline* p, int32_t slot, const double* h_points, const double* h_t,
                               const double* h_w, int64_t n_in, const double* h_imu_t, const double* h_imu_gyro,
                               const double* h_imu_accel);
/* Enqueue one scan (all local hypotheses, exchange, combine, IW apply, map update). */
int32_t gc_pipeline_run_scan(gc_pipeline* p, int32_t slot, double scan_start, double scan_end, double t_last,
                             double t_scan, double dt_sec, int64_t scan_count);
int32_t gc_pipeline_get_combined(gc_pipeline* p, double* h_out);
int32_t gc_pipeline_get_hyp_diag(gc_pipeline* p, double* h_diag);
int32_t gc_pipeline_get_bin_stats(gc_pipeline* p, double* h_stats, double* h_cert, double* h_xi);
int32_t gc_pipeline_attach_comm(gc_pipeline* p, gc_comm* comm);

/* ------------------------------------------------------------------ RCCL communicator */
#define GC_COMM_ID_BYTES 128
int32_t gc_comm_unique_id(uint8_t* h_id_out);
int32_t gc_comm_init(gc_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t* h_id, gc_comm** out);
int32_t gc_comm_destroy(gc_comm* comm);
int32_t gc_comm_allgather_f64(gc_ctx* ctx, gc_comm* comm, const double* d_send, double* d_recv, int64_t count);

#ifdef __cplusplus
}
#endif
#endif /* GCSLAM_H_ */
