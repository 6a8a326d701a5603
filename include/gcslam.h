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
/* Waits for everything enqueued on the ctx stream. Like every host wait in libgcslam it is bounded
 * (fail fast, backend_node.py:2205-2210 log and re-raise): after the context's wait timeout it returns
 * GC_ERR_RUNTIME, and an RCCL communicator initialised on this context is aborted first, so a rank whose
 * peer died does not stay in an all-gather. Its asynchronous error is polled during the wait. */
int32_t gc_ctx_synchronize(gc_ctx* ctx);
/* The bound of every host wait on this context, seconds (default: $GC_WAIT_TIMEOUT_S, else 300). */
int32_t gc_ctx_set_wait_timeout(gc_ctx* ctx, double seconds);
/* Test entries of the bounded wait. gc_test_bounded_wait runs the wait loop on a condition that
 * completes after ready_after_polls polls (< 0: never) with no device involved: GC_OK, or
 * GC_ERR_RUNTIME once timeout_s has passed; h_waited_ms receives the time spent. gc_test_device_spin
 * enqueues a one-thread kernel that keeps the stream busy for `seconds` (<= 10) and then exits. */
int32_t gc_test_bounded_wait(double timeout_s, int64_t ready_after_polls, double* h_waited_ms);
int32_t gc_test_device_spin(gc_ctx* ctx, double seconds);
/* Test entry of the library's device radix sort (the PrimitiveMap cull / insert / merge and the map view's
 * per-tile order): d_keys_in (n_seg x L doubles, n_seg * L < 2^32) sorted within each segment of L keys,
 * ascending (or descending), stable (equal keys, -0.0 and +0.0 included, in input order), into
 * d_keys_out, with d_vals_in (32-bit; NULL: keys only) permuted alike into d_vals_out. */
int32_t gc_test_radix_sort(gc_ctx* ctx, const double* d_keys_in, const uint32_t* d_vals_in, int64_t n_seg, int64_t L,
                           int32_t descending, double* d_keys_out, uint32_t* d_vals_out);
/* Device buffers from the context's arena (SURVEY §8b ownership): gc_buffer_free returns a block to a
 * per-size-class cache and the next allocation of that class takes it back, so a steady-state chain of
 * per-operator calls performs no hipMalloc / hipFree and no synchronisation. All work on arena buffers
 * must be ordered on the context's stream (as every libgcslam entry is). gc_ctx_trim returns the cached
 * blocks to HIP; gc_ctx_alloc_stats: [hipMalloc calls, hipFree calls, arena reuses, live buffers,
 * live bytes, cached bytes]. */
int32_t gc_buffer_alloc(gc_ctx* ctx, uint64_t bytes, void** d_ptr);
int32_t gc_buffer_free(gc_ctx* ctx, void* d_ptr);
int32_t gc_ctx_trim(gc_ctx* ctx);
int32_t gc_ctx_alloc_stats(gc_ctx* ctx, int64_t* h_out6);
/* Copies on the context's stream. An upload returns once the caller's buffer may be reused: up to
 * 512 KiB it is copied into the context's pinned staging ring and the DMA is left in flight (later work
 * on the stream is ordered after it), larger ones are waited for. A download is waited for. */
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

/* ------------------------------------------------------------- PointCloud2
 * parse_pointcloud2_vlp16 (backend/backend_node.py:377-468) + the no-TF base transform
 * p_base = R p + t (backend_node.py:1677-1690) on the device. d_data: the message's raw bytes
 * (n_points * point_step, little-endian). h_fields (10 int32): [x_off, x_type, y_off, y_type,
 * z_off, z_type, ring_off, ring_type, time_off, time_type] with sensor_msgs/PointField datatype
 * codes (1 INT8 .. 8 FLOAT64); time_off = -1 when the cloud has no t/time field (every point gets
 * header_stamp). Times are divided by 1e9 when any raw time exceeds 1e6 (ns-stamped drivers).
 * Non-finite coordinates become ±1e6 (GC_NONFINITE_SENTINEL); weights are the range sigmoid of
 * the sensor-frame distance; ring is the field cast to uint8; tag = 0. */
int32_t gc_pointcloud2_parse(gc_ctx* ctx, const uint8_t* d_data, int64_t n_points, int32_t point_step,
                             const int32_t* h_fields, double header_stamp, const double* h_R9, const double* h_t3,
                             double* d_points_out, double* d_t_out, double* d_w_out, uint8_t* d_ring_out,
                             uint8_t* d_tag_out);

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
 * d_dirs (H,n,3), any norm; d_bins (B,3), B <= 64; tau > 0;
 * d_resp_out (H,n,B) = softmax(dirs·binsᵀ/τ) shifted by the row maximum as jax.nn.softmax;
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
 * d_budget_scalars: the 8 scalars written by gc_point_budget_resample / gc_budget_stats.
 * tau >= GC_FUSED_TAU_MIN (the table exp's range; the contract gc_bin_soft_assign takes any tau).
 * iters: 256-point iterations per workgroup (launch geometry; it changes only the summation
 * order): 0 = chosen from the grid size (16 at 64k points x 256 hypotheses, 1 below ~1024
 * workgroups), 1..64 = forced. */
#define GC_FUSED_TAU_MIN 3e-3
int32_t gc_scan_bins_fused(gc_ctx* ctx, int32_t H, int64_t n_in, int64_t n_cap, int32_t B,
                           const double* d_points_raw, const double* d_t_raw, const double* d_w_raw,
                           const double* d_budget_scalars, double t0, double t1, const double* d_xi,
                           const double* d_bins, double tau, const double* h_origin3,
                           double eps_psd, double eps_mass, double* d_stats_out, double* d_cert_out,
                           int32_t iters);

/* Budget reduction only (no gather): writes the 8 budget scalars. */
int32_t gc_budget_stats(gc_ctx* ctx, const double* d_w, int64_t n_in, int64_t n_cap,
                        double* d_scalars_out);

/* kappa_from_resultant_batch (kappa.py:130-169). */
int32_t gc_kappa_from_resultant_batch(gc_ctx* ctx, int64_t n, const double* d_R, double eps_r,
                                      double d, double r0, double tau, double* d_kappa_out);

/* domain_projection_psd_core (primitives.py:80-123) over `batch` d x d matrices, any 1 <= d <= 512
 * (cyclic Jacobi; an odd d is padded with a decoupled zero row/column that the certificate
 * ignores). d_cert_out (batch,6) = [projection_delta, sym_delta, eig_min, eig_max, cond, nnc]. */
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
  int32_t geom_hyps; /* 0: the bins launch's chunk geometry follows h_count (and the CU count);
                        k > 0: as for a shard of k hypotheses, so shards of different sizes sum each
                        hypothesis's points in the same order (cross-world-size bit-reproducibility
                        of the per-hypothesis results) */
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
#define GC_PCFG_PLANAR_Z_REF 18    /* GC_PLANAR_Z_REF (constants.py:294) */
#define GC_PCFG_PLANAR_Z_SIGMA 19  /* GC_PLANAR_Z_SIGMA (constants.py:305) */
#define GC_PCFG_PLANAR_VZ_SIGMA 20 /* GC_PLANAR_VZ_SIGMA (constants.py:310) */
#define GC_PCFG_GRAVITY_SCALE 21   /* PipelineConfig.imu_gravity_scale (pipeline.py:141) */
#define GC_PCFG_LEN 22

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
 * [30:36] xi_body, 36 support_frac, 37 excitation_total, 38 |mu_final|^2 (barycenter spread),
 * 39 eigmin_pose6 (clipped at eps_psd, pipeline.py:1157-1168) */
#define GC_HYP_DIAG 40
/* combined output (GC_COMB_LEN): L 484, h 22, z_lin 22, X_anchor(hyp 0) 6, then
 * [stamp, psd_delta, eig_min, eig_max, cond, nnc, ess, support_frac, mass_eps_ratio,
 *  floor_adjustment, spread_proxy, 5 pad]. The conditioning fields are always filled: when the
 *  scan path certified the barycenter PSD by Cholesky, gc_pipeline_get_combined computes them from
 *  the stored combined L on demand (one extra launch, off the scan path). */
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
/* IMU/odom branch source: GC_IO_GIVEN uses the evidence of gc_pipeline_set_io_evidence (synthetic
 * input; calling it selects this mode); GC_IO_COMPUTED (default) evaluates _compute_imu_odom_branch (pipeline.py:595-776) on the
 * device each scan from the slot's odometry (gc_pipeline_stage_odom) and IMU window. */
#define GC_IO_GIVEN 0
#define GC_IO_COMPUTED 1
int32_t gc_pipeline_set_io_mode(gc_pipeline* p, int32_t mode);
/* Odometry of a scan slot (backend_node.py:1748-1765): relative pose [t, rotvec] (6), pose
 * covariance (6,6) in [trans, rot] order, body twist [v, ω] (6), twist covariance (6,6). */
int32_t gc_pipeline_stage_odom(gc_pipeline* p, int32_t slot, const double* h_pose6, const double* h_cov36,
                               const double* h_twist6, const double* h_twist_cov36);
/* Per-hypothesis IMU/odom-branch internals of the last scan (GC_IO_COMPUTED), (Hl, GC_IO_PARTS):
 * [0:6] odom se3 residual, 6 kappa, 7 ess_weighted, 8 ess_raw, 9 mean_reliability,
 * 10 transport_sigma, 11 Rbar, 12 imu dependence scale, [13:16] gyro r_rot, [16:19] preint r_vel,
 * [19:22] preint r_pos, 22 planar r_z, 23 v_z, [24:27] odom-velocity r_vel, 27 yaw-rate r_wz,
 * [28:31] kinematic r_trans, [31:34] kinematic r_rot, 34 odom dependence scale, 35 odom nll,
 * 36 imu nll, 37 gyro nll, 38 dt_int, 39 trigger-magnitude sum of the 11 certs.
 * gc_pipeline_get_io_evidence reads back (L_io, h_io, cert row) of the last scan. */
#define GC_IO_PARTS 40
int32_t gc_pipeline_get_io_parts(gc_pipeline* p, double* h_parts);
int32_t gc_pipeline_get_io_evidence(gc_pipeline* p, double* h_L, double* h_h, double* h_cert);
int32_t gc_pipeline_set_iw(gc_pipeline* p, const double* h_nu_proc7, const double* h_Psi_proc7x36,
                           const double* h_nu_meas3, const double* h_Psi_meas3x9);
int32_t gc_pipeline_get_iw(gc_pipeline* p, double* h_nu_proc7, double* h_Psi_proc7x36, double* h_nu_meas3,
                           double* h_Psi_meas3x9, double* h_Q22x22, double* h_cert4);
int32_t gc_pipeline_set_map(gc_pipeline* p, const double* h_map);
int32_t gc_pipeline_get_map(gc_pipeline* p, double* h_map, double* h_map_der, double* h_misc2);
/* Staging (stage_scan / stage_pointcloud2 / stage_odom) is the per-scan ingest
 * (backend_node.py:1679-1690): the host arrays are copied into the slot's pinned mirror before the
 * call returns (the caller may reuse them at once), then DMA'd into HBM on the pipeline's copy
 * stream, ordered after the last scan that read the slot; scan_local waits for the slot's copy. So
 * staging scan k+1 into a second slot overlaps scan k's compute. The call blocks only while the
 * slot's previous DMA is still reading its pinned mirror. */
int32_t gc_pipeline_stage_scan(gc_pipeline* p, int32_t slot, const double* h_points, const double* h_t,
                               const double* h_w, int64_t n_in, const double* h_imu_t, const double* h_imu_gyro,
                               const double* h_imu_accel);
/* Stage a scan slot straight from a PointCloud2 message (the on-wire format): the raw bytes are
 * uploaded once and parsed on the device into the slot (gc_pointcloud2_parse layout of h_fields;
 * h_R9/h_t3 = T_base_lidar). An empty cloud stages one zero-weight dummy point, as the node does
 * (backend_node.py:1700-1707). */
int32_t gc_pipeline_stage_pointcloud2(gc_pipeline* p, int32_t slot, const uint8_t* h_data, int64_t n_points,
                                      int32_t point_step, const int32_t* h_fields, double header_stamp,
                                      const double* h_R9, const double* h_t3, const double* h_imu_t,
                                      const double* h_imu_gyro, const double* h_imu_accel);
/* Enqueue one scan (all local hypotheses, exchange, combine, IW apply, map update) =
 * gc_pipeline_scan_local + gc_pipeline_scan_finish(p, NULL). */
int32_t gc_pipeline_run_scan(gc_pipeline* p, int32_t slot, double scan_start, double scan_end, double t_last,
                             double t_scan, double dt_sec, int64_t scan_count);
/* The two halves of a scan around the per-scan exchange (backend_node.py:2036-2119):
 *  scan_local   a1-a15 for this rank's hypotheses and its partial record (partial_len doubles:
 *               weighted L/h/z/μ sums, IW statistics, hypothesis-0 map increment, anchor).
 *  get_partial  reads that record back (synchronises the stream).
 *  scan_finish  the exchange and the combine: with h_gather (world_size x partial_len doubles, in
 *               rank order, gathered by the caller over any transport) the records are uploaded;
 *               with NULL the pipeline all-gathers over its RCCL communicator (world_size > 1, or a
 *               single rank with one attached) or reads its own record (one rank, none attached).
 *               Then the fixed rank-order reduction, barycenter, IW apply, Q and map update.
 * Every rank ends the scan with a bit-identical combined belief, IW state and map.
 * Between the two halves the state the combine reads or writes is locked: set_bins / set_beliefs /
 * set_weights / set_io_evidence / set_io_mode / set_iw / set_map, get_combined / get_iw / get_map,
 * attach_comm and a second scan_local return GC_ERR_ARG. Allowed: get_partial, the per-hypothesis
 * getters (beliefs, diag, bin stats, hyp stats, io evidence: final after scan_local) and staging
 * the next scan into any slot (ordered after the pending scan's reads of it) except, with a
 * PrimitiveMap attached, the pending scan's own slot (its map update reads it in scan_finish). */
int32_t gc_pipeline_scan_local(gc_pipeline* p, int32_t slot, double scan_start, double scan_end, double t_last,
                               double t_scan, double dt_sec, int64_t scan_count);
int32_t gc_pipeline_partial_len(const gc_pipeline* p);
int32_t gc_pipeline_get_partial(gc_pipeline* p, double* h_record);
int32_t gc_pipeline_scan_finish(gc_pipeline* p, const double* h_gather);
int32_t gc_pipeline_get_combined(gc_pipeline* p, double* h_out);
int32_t gc_pipeline_get_hyp_diag(gc_pipeline* p, double* h_diag);
/* Per-hypothesis ConditioningCert (Hl, 2, 4) of the last scan's two 22x22 PSD projections,
 * [L_pred (predict.py:183-188), L_post (fusion.py:150-230)] x [eig_min, eig_max, cond,
 * near_null_count] of the clamped spectrum. The scan certifies both by Cholesky and skips their
 * eigen-decompositions. With in-scan certificates on (gc_pipeline_set_inscan_certs) every scan
 * computes them right after its evidence kernel (Householder tridiagonalisation + Sturm
 * multisection, gc_certs.hip) and this getter reads them back; otherwise it computes them on demand
 * (Jacobi, off the scan path) from the stored matrices, so call it before the beliefs are set again.
 * Synchronises the stream. */
int32_t gc_pipeline_get_hyp_conditioning(gc_pipeline* p, double* h_out);
/* In-scan ConditioningCerts (off by default): on != 0 makes every later scan emit the certificates
 * gc_pipeline_get_hyp_conditioning reads, as the reference emits them on every predict / fusion call. */
int32_t gc_pipeline_set_inscan_certs(gc_pipeline* p, int32_t on);
/* The full certificate vector of every other PSD projection of the last scan, in the reference's
 * cert_vec layout [projection_delta, sym_delta, eig_min, eig_max, cond, near_null_count]
 * (domain_projection_psd_core, primitives.py:80-123; eigenvalues clamped at eps_psd, near-null =
 * clamped eigenvalues below 10 eps_psd), recomputed from the unprojected matrices by a full
 * eigen-decomposition (the scan certifies these projections by Cholesky and keeps only their deltas):
 *   h_hyp  (Hl, B + 2, 6): per hypothesis, GC_PCERT_BIN0 + b = the a6 Σ_p of bin b (binning.py:175-187),
 *          GC_PCERT_MF(B) = the a7 L_rot (matrix_fisher_evidence.py:330-331), GC_PCERT_PLANAR(B) = the
 *          a8 L_trans (matrix_fisher_evidence.py:609-610);
 *   h_scan (GC_PCERT_SCAN, 6): the a16 barycenter L (hypothesis.py:99), the 7 process-IW blocks
 *          (inverse_wishart_jax.py:168-172, each padded 6x6 block), the 3 measurement-IW blocks
 *          (measurement_noise_iw_jax.py:82-86) and Q (inverse_wishart_jax.py:67).
 * With in-scan certificates on, every scan computes them after its combine; otherwise this getter
 * does, from the last scan's stored matrices (call it before the next scan). Synchronises the stream. */
#define GC_PCERT_BIN0 0
#define GC_PCERT_MF(B) (B)
#define GC_PCERT_PLANAR(B) ((B) + 1)
#define GC_PCERT_SCAN 12
#define GC_PCERT_BARY 0
#define GC_PCERT_PROC0 1
#define GC_PCERT_MEAS0 8
#define GC_PCERT_Q 11
int32_t gc_pipeline_get_projection_certs(gc_pipeline* p, double* h_hyp, double* h_scan);
/* The a2 predict's route (predict.py:43-98). 0 (default): split at its first projection — when
 * Σ'_psd = Σ'_sym is certified, the predicted moments the bins need (μ_inc, σ_warp) are solved from Σ'
 * directly, (L_pred + ε_l I)⁻¹ L_pred = (I + ε_l(Σ' + ε_l I))⁻¹, and L_pred / h_pred / the predict cert
 * are formed in the bins launch beside the bin tasks; otherwise the factorised chain runs. 1: always the
 * factorised chain in the predict kernel (tests compare the two routes). */
int32_t gc_pipeline_set_predict_route(gc_pipeline* p, int32_t route);
/* L_evidence[pose, pose] (Hl, 6, 6) of the last scan, as the reference's MinimalScanTape.L_pose6
   (pipeline.py:1537). */
int32_t gc_pipeline_get_lpose6(gc_pipeline* p, double* h_lpose);
int32_t gc_pipeline_get_bin_stats(gc_pipeline* p, double* h_stats, double* h_cert, double* h_xi);
/* Per-hypothesis statistics of the last scan (any pointer may be NULL): process-IW sufficient
 * statistics dPsi (Hl,7,6,6) and measurement-IW dPsi (Hl,3,3,3) before the weighted accumulation
 * (backend_node.py:2085-2090), and the covariance of each updated belief Σ = (L + ε_lift I)⁻¹
 * (Hl,22,22) (BeliefGaussianInfo covariance, belief.py:373-386). */
int32_t gc_pipeline_get_hyp_stats(gc_pipeline* p, double* h_dPsi_proc, double* h_dPsi_meas, double* h_Sigma);
int32_t gc_pipeline_attach_comm(gc_pipeline* p, gc_comm* comm);
/* Size of the attached RCCL communicator (0 when none is attached). */
int32_t gc_pipeline_comm_size(const gc_pipeline* p);
/* Exchange timing (off by default): with on != 0, every later scan's exchange is bracketed by two
 * HIP events on the pipeline stream (each event between kernels costs the stream a few us, so the
 * timed product loop leaves it off). */
int32_t gc_pipeline_set_exchange_timing(gc_pipeline* p, int32_t on);
/* Device time (ms) of the last timed scan's exchange: the RCCL all-gather of the partial records,
 * or the upload of the host-gathered records. Synchronises on it. GC_ERR_ARG when no timed
 * exchange has run (timing off, or one rank without a communicator). */
int32_t gc_pipeline_exchange_ms(gc_pipeline* p, float* ms);

/* Per-stage device timing (off by default; the reference fills MinimalScanTape.t_*_ms per stage,
 * pipeline.py:383-394, :1560-1569). With on != 0 every later scan records GC_STAGE_N HIP events on the
 * pipeline stream, before predict and after each launch group; gc_pipeline_stage_ms returns the last
 * finished scan's stage times (ms) [predict (a1 scalars, a2, a3), bins (a1 selection, a4, a5, a6 and
 * the IMU/odom branch, + finalize), evidence (a7-a15), combine_local, exchange, combine_final (a16, IW
 * apply, bin-map update), map_update (the attached PrimitiveMap's, 0 without one), total]. Each event
 * between kernels costs the stream ~1-5 us, so the timed product loop leaves it off. stage_ms
 * synchronises on the last event. */
#define GC_STAGE_N 8
int32_t gc_pipeline_set_stage_timing(gc_pipeline* p, int32_t on);
int32_t gc_pipeline_stage_ms(gc_pipeline* p, float* h_ms_out);
/* Host-side accounting since creation or the last reset (GC_HOST_STATS doubles): the reference's
 * RuntimeCounters / DeviceRuntimeCert (common/runtime_counters.py:19-108, backend_node.py:2182-2190:
 * host syncs, host->device and device->host bytes, JIT recompiles = 0 for this AOT library), and the
 * split of the host time of every scan (scan_local + scan_finish) and every staging call into its
 * own work (argument checks, pinned copies, launch / DMA enqueue) and its waits on the device (slot
 * events, stream syncs). Times in ms. reset != 0 zeroes the counters after reading them. */
#define GC_HOST_STATS 16
#define GC_HS_SCANS 0
#define GC_HS_SCAN_ENQ_MS 1
#define GC_HS_SCAN_ENQ_MAX 2
#define GC_HS_SCAN_WAIT_MS 3
#define GC_HS_SCAN_WAIT_MAX 4
#define GC_HS_STAGES 5
#define GC_HS_STAGE_WORK_MS 6
#define GC_HS_STAGE_WORK_MAX 7
#define GC_HS_STAGE_WAIT_MS 8
#define GC_HS_STAGE_WAIT_MAX 9
#define GC_HS_HOST_SYNCS 10
#define GC_HS_H2D_BYTES 11
#define GC_HS_D2H_BYTES 12
#define GC_HS_JIT_RECOMPILES 13
int32_t gc_pipeline_host_stats(gc_pipeline* p, double* h_out, int32_t reset);

/* The C5 in-scan PrimitiveMap update (config C5; the reference's step 12b, pipeline.py:1236-1327,
 * transform_gaussian_to_world :1248-1256 + primitive_map_fuse, primitive_map.py:992-1163).
 * BUILD-DEFINED, parity unpinned (csrc/gc_scanmap.hip): with a map attached,
 * scan_finish fuses every budgeted point of the scan, deskewed with hypothesis 0's twist, as one
 * world-frame Gaussian row (pose z_t of hypothesis 0 with t_z = 0, covariance Σ_lidar inflated by
 * J Σ_pose Jᵀ) into the slot hashed from its voxel (edge voxel_m), responsibility 1, source
 * LiDAR, timestamp scan_end, scan_seq = scan_count. Σ_lidar is the measurement-IW LiDAR mode of the
 * state the scan started from (before its own IW apply). Which ranks run it is the scan-map mode
 * (gc_pipeline_set_scan_map_mode): by default only the rank whose shard holds hypothesis 0 (the
 * reference's owner, backend_node.py:2081-2083); replicated, every rank runs it from the reduced
 * record and the replicas stay bit-identical. The map's device arrays must outlive the attachment;
 * map == NULL detaches. */
struct gc_primitive_map; /* defined with the PrimitiveMap entries below */
int32_t gc_pipeline_attach_primitive_map(gc_pipeline* p, const struct gc_primitive_map* map, double voxel_m);
#define GC_SMAP_OWNER 0      /* default: the update runs on hypothesis 0's rank only */
#define GC_SMAP_REPLICATED 1 /* every rank updates its replica of the map */
/* Not while a scan is pending. A pipeline with world size 1 holds hypothesis 0: both modes update. */
int32_t gc_pipeline_set_scan_map_mode(gc_pipeline* p, int32_t mode);
/* The attached map's colour fields were written outside the pipeline (an insert, a merge, a colour
 * upload): the next in-scan update recomputes rgb / colors on every slot, as primitive_map_fuse does
 * on every fuse (primitive_map.py:1097-1105); while they stay current it only touches its rows' slots.
 * Allowed while a scan is pending (the pass then runs in that scan's finish). */
int32_t gc_pipeline_map_colors_stale(gc_pipeline* p);
/* Hypothesis 0's [z_t 6, Σ_post pose block 36 (row-major 6x6), ξ_body 6] that the last scan's
 * update used (from the reduced record). */
int32_t gc_pipeline_get_scan_map_pose(gc_pipeline* p, double* h_out48);
/* Distinct map slots the last in-scan update touched (synchronises the stream); 0 on a rank that does
 * not run the update. */
int32_t gc_pipeline_get_scan_map_count(gc_pipeline* p, int64_t* n_slots);

/* ------------------------------------------------------------------ RCCL communicator */
#define GC_COMM_ID_BYTES 128
int32_t gc_comm_unique_id(uint8_t* h_id_out);
int32_t gc_comm_init(gc_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t* h_id, gc_comm** out);
int32_t gc_comm_destroy(gc_comm* comm);
/* Abort the communicator (ncclCommAbort: its kernels exit; every later exchange fails fast). The
 * bounded waits of the context it was created on call this themselves on a timeout or an RCCL error. */
int32_t gc_comm_abort(gc_comm* comm);
/* *ok = 0 when the communicator has an asynchronous error or was aborted (gc_last_error has why). */
int32_t gc_comm_healthy(gc_comm* comm, int32_t* ok);
int32_t gc_comm_allgather_f64(gc_ctx* ctx, gc_comm* comm, const double* d_send, double* d_recv, int64_t count);

/* ------------------------------------------------------------------------------------------
 * Per-operator entries: each reference operator of the hot path as one launch over H
 * independent items (the gcslam.ops mirror calls them with H = 1 at the reference's
 * per-hypothesis call sites). Matrices are row-major f64; "belief" arrays are
 * X_anchor (H,6), z_lin (H,22), L (H,22,22), h (H,22). The same device code runs inside the
 * batched pipeline above.
 * ------------------------------------------------------------------------------------------ */
#define GC_PRED_CERT 8      /* [lift, psd_delta, eig_min, eig_max, cond, nnc, trace_cov, trigger] */
#define GC_PREINT_OUT 32    /* [delta_pose 6, delta_R 9, p_body 3, v_body 3, ess, a_body_mean 3,
                               a_world_nog_mean 3, a_world_mean 3, dt_eff_sum] */
#define GC_MF_OUT 66        /* [R_mf 9, L_rot 9, h_rot 3, delta_rot 3, svd 3, N_eff, nll_per_ess, psd_delta,
                               trigger, nll, map scatter 17, scan scatter 17]; scatter = [eigenvalues 3
                               (descending), eigenvectors 9 (row-major, columns = vectors), linearity,
                               planarity, sphericity, anisotropy, effective_rank] */
#define GC_PT_OUT 26        /* [t_wls 3, L_trans 9, h_trans 3, delta_trans 3, z_scale, N_eff, nll_per_ess,
                               psd_delta, trigger, xy_info_scale, z_info_scale, nll] */
#define GC_RECOMPOSE_OUT 19 /* [delta_pose 6, X_new 6, frobenius_strength, bch_correction 6] */
#define GC_DRIFT_OUT 3      /* [rho, drift_m, drift_r] */
#define GC_FUSION_ROW 8     /* in: [cond, ess_total, support_frac, excitation_total, dt_asymmetry,
                               z_to_xy_ratio, power_beta, nll_per_ess] */
#define GC_FUSION_OUT 4     /* [alpha, excitation_total, ess_to_excitation, cond_to_support] */
#define GC_BARY_CERT 16     /* [floor_adjustment, spread, ess, support_frac, mass_eps, psd cert 6, pad 5] */

/* IMU/odom-branch factors (pipeline.py:595-776), one thread per item.
 * Item rows: d_in (H, GC_IOF_IN) per kind below; d_out (H, GC_IOF_OUT) = L (22,22) | h (22) |
 * extras (16). Each kind replaces one reference operator:
 *  GC_IOF_ODOM_QUADRATIC    odom_quadratic_evidence (odom_evidence.py:87-154)
 *     in [pose_pred 6, odom_pose 6, cov 36, eps_psd, eps_lift]
 *     ex [delta_z_pose 6, nll, lift, eig_min, eig_max, cond, nnc]
 *  GC_IOF_IMU_GYRO_ROTATION imu_gyro_rotation_evidence (imu_gyro_evidence.py:103-163)
 *     in [rv_start 3, rv_end_pred 3, delta_rotvec 3, Sigma_g 9, dt_int, eps_psd, eps_lift, eps_mass]
 *     ex [r_rot 3, nll, lift, eig_min, eig_max, nnc]
 *  GC_IOF_IMU_PREINT_FACTOR imu_preintegration_factor (imu_preintegration_factor.py:46-180)
 *     in [p_start 3, rv_start 3, v_start 3, p_end_pred 3, v_end_pred 3, delta_v_body 3,
 *         delta_p_body 3, Sigma_a 9, dt_int, eps_psd, eps_lift, eps_mass]
 *     ex [r_vel 3, r_pos 3, nll, lift, eig_min, eig_max, cond, nnc]
 *  GC_IOF_PLANAR_Z_PRIOR    planar_z_prior (planar_prior.py:55-135): in [pose 6, z_ref, sigma_z]; ex [r_z, nll]
 *  GC_IOF_VELOCITY_Z_PRIOR  velocity_z_prior (planar_prior.py:138-195): in [v_z, sigma_vz]; ex [v_z, nll]
 *  GC_IOF_ODOM_VELOCITY     odom_velocity_evidence (odom_twist_evidence.py:58-154)
 *     in [v_pred_world 3, R_world_body 9, v_odom_body 3, Sigma_v 9, eps_psd, eps_lift]
 *     ex [r_vel 3, nll, lift, eig_min, eig_max, cond, nnc]
 *  GC_IOF_ODOM_YAWRATE      odom_yawrate_evidence (odom_twist_evidence.py:157-225)
 *     in [omega_z_pred, omega_z_odom, sigma_wz]; ex [r_wz, nll]
 *  GC_IOF_KINEMATIC         pose_twist_kinematic_consistency (odom_twist_evidence.py:251-397)
 *     in [pose_prev 6, pose_curr 6, v_body 3, omega_body 3, dt, Sigma_v 9, Sigma_omega 9, eps_psd, eps_lift]
 *     ex [r_trans 3, r_rot 3, nll, lift, eig_min, eig_max, cond]
 *  GC_IOF_IMU_DEPENDENCE    imu_dependence_inflation (imu_evidence.py:562-589): in [transport_sigma, eps_mass]; ex [scale]
 *  GC_IOF_ODOM_DEPENDENCE   odom_dependence_inflation (odom_twist_evidence.py:400-430):
 *     in [r_trans 3, r_rot 3, eps_mass]; ex [scale] */
#define GC_IOF_IN 64
#define GC_IOF_OUT (484 + 22 + 16)
#define GC_IOF_ODOM_QUADRATIC 0
#define GC_IOF_IMU_GYRO_ROTATION 1
#define GC_IOF_IMU_PREINT_FACTOR 2
#define GC_IOF_PLANAR_Z_PRIOR 3
#define GC_IOF_VELOCITY_Z_PRIOR 4
#define GC_IOF_ODOM_VELOCITY 5
#define GC_IOF_ODOM_YAWRATE 6
#define GC_IOF_KINEMATIC 7
#define GC_IOF_IMU_DEPENDENCE 8
#define GC_IOF_ODOM_DEPENDENCE 9
#define GC_IOF_NKINDS 10
int32_t gc_io_factor_batch(gc_ctx* ctx, int32_t kind, int32_t H, const double* d_in, double* d_out);
/* imu_vmf_gravity_evidence_time_resolved (imu_evidence.py:402-559), one workgroup per item over
 * the shared IMU window accel/gyro (M,3); rotvec (H,3), weights (H,M), accel_bias (H,3), g3 host.
 * d_out (H, GC_IOF_OUT), ex = [kappa, ess_weighted, ess_raw, mean_reliability, transport_sigma,
 * Rbar, nll, nll_per_ess, psd_delta, eig_min, eig_max, cond, nnc, xbar 3]. */
int32_t gc_imu_vmf_gravity_tr_batch(gc_ctx* ctx, int32_t H, int32_t M, const double* d_rotvec, const double* d_accel,
                                    const double* d_gyro, const double* d_w, const double* d_ba, const double* g3,
                                    double dt_imu, double eps_psd, double eps_mass, double* d_out);

/* SO(3)/SE(3) maps of common/geometry/se3_jax.py, batched: n items of the op's input row
 * (d_in (n, in)) to its output row (d_out (n, out)), one thread per item. These are the device
 * routines every kernel of the scan path uses (recompose, world pose, ξ_body, MF δ, IMU/odom
 * residuals). Rotations are row-major 3x3; poses [t 3, rotvec 3]; twists [ρ 3, φ 3].
 *   GC_LIE_SO3_EXP     so3_exp      (se3_jax.py:259-301)   in 3  out 9
 *   GC_LIE_SO3_LOG     so3_log      (se3_jax.py:304-366)   in 9  out 3  (softmax near-π axis)
 *   GC_LIE_SE3_EXP     se3_exp      (se3_jax.py:473-504)   in 6  out 6
 *   GC_LIE_SE3_LOG     se3_log      (se3_jax.py:220-256)   in 6  out 6
 *   GC_LIE_SE3_V       se3_V        (se3_jax.py:137-175)   in 3  out 9
 *   GC_LIE_SE3_V_INV   _se3_V_inv   (se3_jax.py:177-217)   in 3  out 9
 *   GC_LIE_SE3_COMPOSE se3_compose  (se3_jax.py:420-438)   in 12 (a, b) out 6
 *   GC_LIE_SE3_INVERSE se3_inverse  (se3_jax.py:441-453)   in 6  out 6 */
#define GC_LIE_SO3_EXP 0
#define GC_LIE_SO3_LOG 1
#define GC_LIE_SE3_EXP 2
#define GC_LIE_SE3_LOG 3
#define GC_LIE_SE3_V 4
#define GC_LIE_SE3_V_INV 5
#define GC_LIE_SE3_COMPOSE 6
#define GC_LIE_SE3_INVERSE 7
#define GC_LIE_NOPS 8
int32_t gc_lie_batch(gc_ctx* ctx, int32_t op, int64_t n, const double* d_in, double* d_out);

/* spd_cholesky_inverse_lifted_core (common/primitives.py:169-192): d_out = (L + eps_lift I)⁻¹ for H
 * n x n SPD matrices (n <= 22), by the Cholesky factor and C⁻ᵀ C⁻¹ as in the batched pipeline. */
int32_t gc_spd_inverse_lifted_batch(gc_ctx* ctx, int32_t H, int32_t n, const double* d_L, double eps_lift,
                                    double* d_out);
/* BeliefGaussianInfo.mean_increment + world pose X ∘ Exp(δz) (common/belief.py:373-425). */
int32_t gc_belief_world_pose_batch(gc_ctx* ctx, int32_t H, const double* d_X, const double* d_L, const double* d_h,
                                   double eps_lift, double* d_pose_out, double* d_mean_out);
/* predict_diffusion (backend/operators/predict.py:106-214 -> core :43-98); Q (22,22) shared. */
int32_t gc_predict_diffusion_batch(gc_ctx* ctx, int32_t H, const double* d_L, const double* d_h, const double* d_Q,
                                   double dt_sec, double eps_psd, double eps_lift, double lambda_ou, double* d_L_out,
                                   double* d_h_out, double* d_cert_out);
/* smooth_window_weights (backend/operators/imu_preintegration.py:20-43). */
int32_t gc_smooth_window_weights(gc_ctx* ctx, int32_t M, const double* d_stamps, double t0, double t1, double sigma,
                                 double* d_w_out);
/* preintegrate_imu_relative_pose_jax (imu_preintegration.py:47-147); M <= 512 samples shared by
   the H items; weights (H, weights_stride) or shared (stride 0); rotvec0/biases (H,3);
   h_gravity3 NULL = (0, 0, -9.81). out (H, GC_PREINT_OUT). */
int32_t gc_preintegrate_imu_batch(gc_ctx* ctx, int32_t H, int32_t M, const double* d_stamps, const double* d_gyro,
                                  const double* d_accel, const double* d_weights, int64_t weights_stride,
                                  const double* d_rotvec0, const double* d_gyro_bias, const double* d_accel_bias,
                                  const double* h_gravity3, double* d_out);
/* imu_gyro_meas_iw_suffstats_from_avg_rate_jax + imu_accel_meas_iw_suffstats_from_gravity_dir_jax
   (measurement_noise_iw_jax.py:131-218); out (H, 18) = [dPsi_gyro 9, dPsi_accel 9]. */
int32_t gc_imu_meas_iw_suffstats_batch(gc_ctx* ctx, int32_t H, int32_t M, const double* d_gyro, const double* d_accel,
                                       const double* d_weights, const double* d_gyro_bias, const double* d_accel_bias,
                                       const double* d_omega_avg, const double* d_rotvec0, double dt_imu,
                                       double eps_mass, double eps_psd, double* d_out);
/* matrix_fisher_rotation_evidence (archive/legacy_operators/matrix_fisher_evidence.py:264-394):
   pose_pred (H,6) = world pose of belief_pred; scan (H,B,*), map (B,*); scatter inputs may be
   NULL (metrics then use zero scatter). out (H, GC_MF_OUT). */
int32_t gc_matrix_fisher_batch(gc_ctx* ctx, int32_t H, int32_t B, const double* d_pose_pred, const double* d_scan_s_dir,
                               const double* d_scan_N, const double* d_scan_S_dir_scatter, const double* d_map_S_dir,
                               const double* d_map_N_dir, const double* d_map_S_dir_scatter, double eps_psd,
                               double eps_mass, double* d_out);
/* planar_translation_evidence (matrix_fisher_evidence.py:502-671); R_hat (H,9); out (H, GC_PT_OUT). */
int32_t gc_planar_translation_batch(gc_ctx* ctx, int32_t H, int32_t B, const double* d_pose_pred, const double* d_R_hat,
                                    const double* d_scan_p_bar, const double* d_scan_Sigma_p, const double* d_scan_N,
                                    const double* d_map_centroid, const double* d_map_Sigma_c,
                                    const double* d_map_N_pos, const double* d_map_S_dir_scatter,
                                    const double* d_map_N_dir, double eps_psd, double eps_mass, double* d_out);
/* compute_excitation_scales_jax + apply_excitation_prior_scaling_jax (backend/operators/excitation.py:15-64);
   s_out (H,2) = [s_dt, s_ex]. With d_L_ev == NULL, s_out is an input and only the scaling is applied. */
int32_t gc_excitation_scaling_batch(gc_ctx* ctx, int32_t H, const double* d_L_ev, const double* d_L_prior,
                                    const double* d_h_prior, double eps, double* d_s_out, double* d_L_out,
                                    double* d_h_out);
/* fusion_scale_from_certificates (backend/operators/fusion.py:46-142) over H certificate rows. */
int32_t gc_fusion_scale_batch(gc_ctx* ctx, int32_t H, const double* d_rows, double alpha_min, double alpha_max,
                              double c0_cond, double eps_mass, double* d_out);
/* info_fusion_additive (backend/operators/fusion.py:150-230); alpha (H); cert (H,6) PSD cert. */
int32_t gc_info_fusion_additive_batch(gc_ctx* ctx, int32_t H, const double* d_L_pred, const double* d_h_pred,
                                      const double* d_L_ev, const double* d_h_ev, const double* d_alpha,
                                      double eps_psd, double* d_L_out, double* d_h_out, double* d_cert_out);
/* pose_update_frobenius_recompose (backend/operators/recompose.py:94-205); T (H). */
int32_t gc_recompose_batch(gc_ctx* ctx, int32_t H, const double* d_X, const double* d_z, const double* d_L,
                           const double* d_h, const double* d_T, double c_frob, double eps_lift, double* d_X_out,
                           double* d_z_out, double* d_h_out, double* d_res_out);
/* anchor_drift_update (backend/operators/anchor_drift.py:93-191). */
int32_t gc_anchor_drift_batch(gc_ctx* ctx, int32_t H, const double* d_X, const double* d_z, const double* d_L,
                              const double* d_h, double eps_lift, double* d_X_out, double* d_z_out, double* d_h_out,
                              double* d_res_out);
/* process_noise_iw_suffstats_from_info_jax (inverse_wishart_jax.py:72-123): dPsi (H,7,6,6), dnu (H,7). */
int32_t gc_iw_process_suffstats_batch(gc_ctx* ctx, int32_t H, const double* d_L_pred, const double* d_h_pred,
                                      const double* d_L_post, const double* d_h_post, double eps_lift,
                                      double* d_dPsi_out, double* d_dnu_out);
/* process_noise_iw_apply_suffstats_jax (inverse_wishart_jax.py:127-185): nu (7), Psi (7,6,6);
   cert (2) = [psd_delta sum, nu projection sum]. Outputs may alias the inputs. */
int32_t gc_iw_process_apply(gc_ctx* ctx, const double* d_nu, const double* d_Psi, const double* d_dPsi,
                            const double* d_dnu, double eps_psd, double nu_max, double* d_nu_out, double* d_Psi_out,
                            double* d_cert_out);
/* process_noise_state_to_Q_jax (inverse_wishart_jax.py:36-68): Q (22,22). */
int32_t gc_iw_process_Q(gc_ctx* ctx, const double* d_nu, const double* d_Psi, double eps_psd, double* d_Q_out);
/* measurement_noise_apply_suffstats_jax (measurement_noise_iw_jax.py:60-100): nu (3), Psi (3,3,3). */
int32_t gc_iw_meas_apply(gc_ctx* ctx, const double* d_nu, const double* d_Psi, const double* d_dPsi,
                         const double* d_dnu, double eps_psd, double nu_max, double* d_nu_out, double* d_Psi_out,
                         double* d_cert_out);
/* hypothesis_barycenter_projection (backend/operators/hypothesis.py:125-236 -> core :52-122). */
int32_t gc_hypothesis_barycenter(gc_ctx* ctx, int32_t H, const double* d_L, const double* d_h, const double* d_z,
                                 const double* d_weights, double weight_floor, double eps_psd, double eps_lift,
                                 double* d_L_out, double* d_h_out, double* d_z_out, double* d_cert_out);

/* ------------------------------------------------------------------------------------------
 * C5 map update (a13 C5 analogue): transform_gaussian_to_world (backend/pipeline.py:1248-1256)
 * fused into primitive_map_fuse (backend/structures/primitive_map.py:992-1163). The map is one
 * flat tile of m_slots slots in device memory; tile t / local slot j of the reference map to slot
 * t * m_tile + j. Two layouts:
 *   slot_bytes = 0  the reference's per-field arrays (SoA, row-major per slot): slot s of a field
 *                   of width w at field + s * w;
 *   slot_bytes > 0  one packed record per slot (gc_primitive_map_record_layout): every field
 *                   pointer is the record array plus the field's offset, slot s of every field at
 *                   (char*)field + s * slot_bytes. The fuse's read-modify-write fields share the
 *                   record's first two 128-B lines, so a touched slot moves 2 lines each way
 *                   instead of one partial line per field.
 * Colour fields are all NULL (no camera colour tracking) or all set. All pointers inside the
 * structs are device pointers.
 * ------------------------------------------------------------------------------------------ */
typedef struct gc_primitive_map {
  int64_t m_slots;
  int32_t n_lobes;          /* GC_VMF_N_LOBES (3) */
  /* 1 when every slot's rgb and colors already equal the fuse's colour estimate of its camera
     accumulators (the state a fuse leaves): the fuse then recomputes the colour of the slots it
     touches only, which gives the same map as the reference's all-slot recompute
     (primitive_map.py:1090-1098). 0: the fuse recomputes every slot. */
  int32_t colors_current;
  double* Lambdas;          /* (M, 3, 3) */
  double* thetas;           /* (M, 3) */
  double* etas;             /* (M, n_lobes, 3) */
  double* weights;          /* (M) */
  double* timestamps;       /* (M) */
  int64_t* last_supported_scan_seq;  /* (M) */
  int64_t* last_update_scan_seq;     /* (M) */
  double* cam_mass;         /* (M) or NULL */
  double* lidar_mass;       /* (M) or NULL */
  double* rgb_cam_accum;    /* (M, 3) or NULL */
  double* rgb_cam_denom;    /* (M) or NULL */
  double* rgb;              /* (M, 3) or NULL */
  double* colors;           /* (M, 3) or NULL */
  /* maintenance fields (primitive_map_insert_masked / cull / recency / merge; the fuse ignores
     them): valid_mask is required by those entries, the other two may be NULL */
  uint8_t* valid_mask;      /* (M) */
  double* created_timestamps;        /* (M) or NULL */
  int64_t* primitive_ids;            /* (M) or NULL */
  int64_t slot_bytes;                /* 0 = per-field arrays; else the packed record's size */
} gc_primitive_map;

/* Packed slot record for n_lobes lobes (build-defined device layout; the reference's per-field
   arrays are honoured at upload / download through gc_copy_strided). offsets_out (host, 16) =
   byte offsets of Lambdas, thetas, etas, weights, timestamps, last_supported_scan_seq,
   last_update_scan_seq, cam_mass, lidar_mass, rgb_cam_accum, rgb_cam_denom, rgb, colors,
   valid_mask, created_timestamps, primitive_ids (the struct's field order); *slot_bytes_out = the
   record size, a multiple of 128 B. */
int32_t gc_primitive_map_record_layout(int32_t n_lobes, int64_t* offsets_out, int64_t* slot_bytes_out);
/* rows x elem_bytes copied between device buffers with the given pitches (bytes; pitch >=
   elem_bytes, elem_bytes a multiple of 1, rows >= 0): the transposes between a packed map and
   per-field arrays. Asynchronous on the context's stream. */
int32_t gc_copy_strided(gc_ctx* ctx, void* d_dst, int64_t dst_pitch, const void* d_src, int64_t src_pitch,
                        int64_t elem_bytes, int64_t rows);

typedef struct gc_fuse_batch {
  int64_t K;
  const int32_t* target_slots;      /* (K) slot per row; out-of-range rows are dropped */
  const double* Lambdas;            /* (K, 3, 3) body (or world) frame */
  const double* thetas;             /* (K, 3) */
  const double* etas;               /* (K, n_lobes, 3) */
  const double* weights;            /* (K) */
  const double* responsibilities;   /* (K) */
  const uint8_t* valid_mask;        /* (K) or NULL = all valid */
  const double* colors;             /* (K, 3) or NULL */
  const int32_t* sources;           /* (K) 0 = camera, 1 = lidar, or NULL */
} gc_fuse_batch;

/* Fuse K rows into the map in place. h_pose6 (host, [t, rotvec]) = world pose z_t of the
   pushforward, or NULL when the rows are already in the world frame. n_fused_out (host, may be
   NULL) = number of distinct in-range slots touched; it synchronises the stream. */
int32_t gc_primitive_map_fuse(gc_ctx* ctx, const gc_primitive_map* map, const gc_fuse_batch* meas,
                              const double* h_pose6, double eps_lift, double eps_mass, double timestamp,
                              int64_t scan_seq, int64_t* n_fused_out);

/* ------------------------------------------------------------------------------------------
 * PrimitiveMap maintenance. Each entry works on one reference tile: the slot
 * range [slot0, slot0 + n_slots) of the flat map (tile t -> slot0 = t * m_tile). Reductions are
 * fixed-order (no float atomics); host outputs synchronise the stream.
 * ------------------------------------------------------------------------------------------ */
/* primitive_map_forget (primitive_map.py:1314-1390): weights *= gamma on every slot. */
int32_t gc_primitive_map_forget(gc_ctx* ctx, const gc_primitive_map* map, int64_t slot0, int64_t n_slots,
                                double gamma);
/* primitive_map_recency_inflate (primitive_map.py:1400-1490) on one tile: decay =
   clip(exp(-lambda max(0, scan_seq - last_supported)), min_scale, 1) on valid slots (1 elsewhere);
   Lambdas, thetas *= decay. h_stats3 (host, may be NULL) = [n_valid, sum (1 - decay), sum (1/decay - 1)]
   over valid slots. */
int32_t gc_primitive_map_recency_inflate(gc_ctx* ctx, const gc_primitive_map* map, int64_t slot0, int64_t n_slots,
                                         int64_t scan_seq, double decay_lambda, double min_scale,
                                         double* h_stats3);
/* primitive_map_cull (primitive_map.py:1175-1305): clears valid on valid slots with weight <
   threshold; with max_primitives >= 0 (< 0 = None) and more survivors than that, the threshold
   becomes the (max_primitives+1)-th largest of weight*valid. h_out4 (host) = [n_culled,
   mass_dropped, sum of all tile weights, n_valid before]. */
int32_t gc_primitive_map_cull(gc_ctx* ctx, const gc_primitive_map* map, int64_t slot0, int64_t n_slots,
                              double weight_threshold, int64_t max_primitives, double* h_out4);

typedef struct gc_insert_batch {
  int64_t K;
  const double* Lambdas;            /* (K, 3, 3) */
  const double* thetas;             /* (K, 3) */
  const double* etas;               /* (K, n_lobes, 3) */
  const double* weights;            /* (K) */
  const uint8_t* valid_mask;        /* (K) proposals with 0 are ignored */
  const double* colors;             /* (K, 3) or NULL (zeros) */
  const int32_t* sources;           /* (K) 0 = camera, 1 = lidar, or NULL (all lidar) */
} gc_insert_batch;

/* primitive_map_insert_masked (primitive_map.py:807-982): proposal k goes to the k-th slot of the
   tile ordered by retention key (valid ? w exp(-lambda max(0, seq - last_supported)) : -inf),
   ties by slot (_select_lowest_mass_slots_fixed :325-353, a stable sort on the key). Inserted
   proposals get ids next_global_id + (number inserted before them). d_target_slots_out (K, tile-
   local) and d_new_ids_out (K, -1 where not inserted) may be NULL. h_out2 (host) = [n_inserted,
   valid count of the tile after]. Requires 1 <= K <= n_slots. */
int32_t gc_primitive_map_insert_masked(gc_ctx* ctx, const gc_primitive_map* map, int64_t slot0, int64_t n_slots,
                                       const gc_insert_batch* batch, double timestamp, int64_t scan_seq,
                                       double recency_decay_lambda, int64_t next_global_id,
                                       int32_t* d_target_slots_out, int64_t* d_new_ids_out, int64_t* h_out2);
/* primitive_map_merge_reduce (primitive_map.py:1809-2030 -> _merge_reduce_jax :1501-1807):
   Bhattacharyya distances of all slot pairs i < j (+inf unless both valid), a stable ascending
   sort, greedy disjoint selection of up to max_pairs pairs with finite distance < threshold, and
   moment-matched merges into the lower slot. The caller applies the reference's tile-size cap.
   h_out2 (host) = [n_merged, valid count after]. Requires n_slots <= 65536. */
int32_t gc_primitive_map_merge_reduce(gc_ctx* ctx, const gc_primitive_map* map, int64_t slot0, int64_t n_slots,
                                      double merge_threshold, int32_t max_pairs, double eps_psd, double eps_lift,
                                      int64_t* h_out2);

/* ------------------------------------------------------------------------------------------
 * Map view + OT association (the current PrimitiveMap pose-evidence path).
 * ------------------------------------------------------------------------------------------ */
/* AtlasMapView (primitive_map.py:236-300) in device memory: V = n_tiles * m_tile_view entries,
   tile-major. The caller allocates every array; tile_ids is a device copy of the view tile ids. */
typedef struct gc_map_view {
  int32_t n_tiles;
  int32_t m_tile_view;
  int32_t n_lobes;
  int32_t pad_;
  int64_t* tile_ids;                /* (T) packed MA-hex tile ids */
  int64_t* candidate_tile_ids;      /* (V) */
  int64_t* candidate_slots;         /* (V) tile-local slot */
  uint8_t* valid_mask;              /* (V) */
  double* positions;                /* (V, 3) solve(Λ + εI, θ) */
  double* covariances;              /* (V, 3, 3) inv(Λ + εI) */
  double* directions;               /* (V, 3) η_sum / (‖η_sum‖ + ε_mass) */
  double* kappas;                   /* (V) ‖η_sum‖ */
  double* weights;                  /* (V) */
  int64_t* primitive_ids;           /* (V) */
  int64_t* last_supported_scan_seq; /* (V) */
  double* etas;                     /* (V, n_lobes, 3) */
  double* colors;                   /* (V, 3) rgb (0.5 where the map has no colour fields) */
} gc_map_view;

/* extract_atlas_map_view (primitive_map.py:356-451): for view tile t, the top m_tile_view slots of
   dense map tile h_dense_tiles[t] (slot range [d * m_tile, (d+1) * m_tile); -1 = missing, an empty
   tile) by weight, invalid slots last, ties by slot (_select_topk_slots_fixed :304-322). */
int32_t gc_extract_map_view(gc_ctx* ctx, const gc_primitive_map* map, int64_t m_tile, const int64_t* h_dense_tiles,
                            const int64_t* h_tile_ids, double eps_lift, double eps_mass, const gc_map_view* view);

#define GC_OT_CFG_LEN 15  /* [k_assoc, k_sinkhorn, beta, epsilon, tau_a, tau_b, cost_subtract_row_min,
                             weight_proportional, eps_mass, h_tile, r_stencil_xy, r_stencil_z, scan_seq,
                             recency_decay_lambda, eps_lift] (AssociationConfig, primitive_association.py:205-236) */
#define GC_OT_CERT_LEN 13 /* [marginal_defect_a, marginal_defect_b, transport_mass_total, sum_a, sum_b, sum_m,
                             sum_novel, ess_ot, nonzero_a, nonzero_b, total_cost, n_valid_meas, n_valid_map] */
/* associate_primitives_ot (operators/primitive_association.py:239-553): N measurement primitives
   (info form + vMF lobes) against a map view. Outputs (device, caller-allocated, K = k_assoc <= 16):
   responsibilities (N, K), candidate pool indices int32 (N, K), candidate tile ids / slots int64
   (N, K), row masses (N), cost matrix (N, K). h_cert_out (host) = GC_OT_CERT_LEN values; with no
   valid measurement or map entry every output is zero and n_valid_* tell which. */
int32_t gc_associate_primitives_ot(gc_ctx* ctx, int64_t N, int32_t n_lobes, const double* d_Lambdas,
                                   const double* d_thetas, const double* d_etas, const double* d_weights,
                                   const uint8_t* d_valid, const gc_map_view* view, const double* h_cfg,
                                   double* d_resp_out, int32_t* d_cand_out, int64_t* d_cand_tile_out,
                                   int64_t* d_cand_slot_out, double* d_row_mass_out, double* d_cost_out,
                                   double* h_cert_out);

#ifdef __cplusplus
}
#endif
#endif /* GCSLAM_H_ */
