// gc_pipeline.cpp — the batched per-scan driver (replaces the hypothesis loop of
// backend_node.py:2036-2119): one rank's shard of hypotheses lives in HBM; gc_pipeline_run_scan
// enqueues the whole 14-step scan for all of them plus the combine/IW exchange on one stream.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>
#include "gc_internal.h"
#include "gc_mapslot.h"
#include "gc_pipe.h"
#include "gc_scanmap.h"

struct gc_comm;
namespace gc {
int comm_allgather(gc_comm* comm, gc_ctx* ctx, const double* d_send, double* d_recv, int64_t count);
int comm_size(const gc_comm* comm);
int32_t cloud_parse_on(gc_ctx* ctx, hipStream_t st, int32_t* flag, const uint8_t* d_data, int64_t n_points,
                       int32_t point_step, const int32_t* h_fields, double header_stamp, const double* h_R9,
                       const double* h_t3, double* d_points_out, double* d_t_out, double* d_w_out,
                       uint8_t* d_ring_out, uint8_t* d_tag_out);
}

// the period (in scans) of the combine_final completion events the slot staging orders on (0: none,
// every staging that must wait records an event on the compute stream; gc_pipeline::fin_ev)
#ifndef GC_BIND_EVERY
#define GC_BIND_EVERY 1
#endif
constexpr int64_t kBindEvery = GC_BIND_EVERY;

// the in-scan map update on a stream of its own (1), beside the next scan, or on the compute stream
// after the combine (0)
#ifndef GC_SMAP_SIDE
#define GC_SMAP_SIDE 1
#endif
constexpr bool kSmapSide = GC_SMAP_SIDE != 0;

struct gc_pipeline {
  gc_ctx* ctx = nullptr;
  gc::PipeDev P{};
  std::vector<void*> allocs;
  // Scan slots. Ingest runs on a copy stream of its own: the host arrays are copied into the slot's
  // pinned mirror, then one DMA per field moves them into the slot's device block, ordered after the
  // last kernel of the previous scan that read the slot (`consumed`); scan_local waits on `ready`.
  // So staging scan k+1 overlaps scan k's compute, and the caller's arrays are free on return.
  struct Slot {
    double* dev = nullptr;   // [pts 3n | t n | w n | imu_t M | imu_g 3M | imu_a 3M | odom kOdomLen]
    double* host = nullptr;  // pinned mirror of dev (same layout)
    double *pts = nullptr, *t = nullptr, *w = nullptr, *imu_t = nullptr, *imu_g = nullptr, *imu_a = nullptr;
    double* odom = nullptr;
    double *budget = nullptr, *bpart = nullptr;  // the staged scan's a1 budget scalars and partials
    bool has_odom = false;
    uint8_t *bytes = nullptr, *hbytes = nullptr, *ring = nullptr, *tag = nullptr;  // PointCloud2 staging
    int32_t* flag = nullptr;  // device word of the parse's seconds / nanoseconds test
    size_t bytes_cap = 0;
    int64_t n_in = 0;
    hipEvent_t ready = nullptr;      // copy stream: the slot's device block holds the staged scan
    hipEvent_t odom_done = nullptr;  // copy stream: the odometry DMA has read its pinned area
    hipEvent_t consumed = nullptr;   // compute stream: the last scan that read the slot is past it
    bool ready_rec = false, odom_rec = false, consumed_rec = false;
    // without a PrimitiveMap the slot's last reader is the bins launch of the scan with this ticket
    // (0 = not read since staged); see done_word
    int64_t consumed_ticket = 0;
  } slots[GC_PIPE_MAX_SLOTS];
  // Host-coherent pinned word: the ticket of the last scan whose bins have completed, written by that
  // scan's finalize kernel (one system-scope store). Staging into a slot whose last scan has already
  // published its ticket needs no ordering on the device at all; only otherwise is an event recorded
  // on the compute stream for the copy stream to wait on. A per-scan event between two kernels cost a
  // ~5 us gap before the next one; with three slots in rotation the word usually suffices.
  int64_t* done_word = nullptr;
  int64_t ticket = 0;
  bool stage_budget = false;  // the a1 budget is formed at staging (gc::predict_budget_inline false)
  // Completion events carried by the combine_final launch of every kBindEvery-th scan (ticket), the
  // newest two (hipExtLaunchKernelGGL's stop event: the kernel's own completion signal, no packet of
  // its own): staging into a slot whose scan has not published its ticket waits on the earliest
  // bound scan at or after it; with no bound scan far enough yet, `consumed` is recorded instead.
  // A signalled completion costs the next kernel a ~5 us start gap, as the recorded event does, but
  // the host then never enqueues into the compute stream at staging time: every scan bound gives
  // the shortest step and a host max within ~1.1x the mean (period 2 lets the copy of a slot wait a
  // scan too long at H = 256 with 3 slots, 1.195 -> 1.219 ms; profiles/r04/ab_slot_bind.txt)
  hipEvent_t fin_ev[2] = {nullptr, nullptr};
  int64_t fin_ticket[2] = {0, 0};
  int64_t pending_ticket = 0;
  hipStream_t cstream = nullptr;  // ingest (copy) stream
  int io_mode = GC_IO_COMPUTED;
  gc_comm* comm = nullptr;
  // P.Sig / P.mu_fin were written by the last scan's evidence kernel from the current P.L / P.h
  // (cleared whenever the beliefs are set from the host)
  bool sig_cached = false;
  // a scan whose local part (a1-a15 + partial record) is enqueued and whose exchange + combine
  // (gc_pipeline_scan_finish) is still due
  bool pending = false;
  gc::ScanArgs pending_S{};
  double* own_gather = nullptr;  // separate gather buffer of a single-rank pipeline with a communicator
  hipEvent_t x0 = nullptr, x1 = nullptr;  // around the last scan's all-gather (gc_pipeline_exchange_ms)
  bool x_rec = false;
  bool x_timing = false;  // gc_pipeline_set_exchange_timing
  // the in-scan PrimitiveMap update (gc_scanmap.hip), run by scan_finish after the combine
  bool smap_on = false;
  // GC_SMAP_OWNER: only the rank holding hypothesis 0 runs the in-scan update (backend_node.py:2081-2083:
  // hypothesis 0 writes the map); GC_SMAP_REPLICATED: every rank updates its own replica
  int32_t smap_mode = GC_SMAP_OWNER;
  gc_primitive_map smap{};
  double smap_voxel = 0.0;
  bool smap_colors = false;  // the colour pass is due (first update after attaching a map with colours not current)
  gc::ScanMapWork smapW;
  // With kSmapSide the update runs on mstream, started by combine_final's completion signal
  // (smap_go, the launch's own: no packet of its own), from the scan's snapshot block of
  // P.smap_snap (snap_base + (ticket & 1) x kSnapLen: the inputs the next scan rewrites, copied by
  // combine_final) and the slot (its restaging waits on `consumed`, recorded after the update). The
  // next scan's predict, bins and evidence run beside it; the compute stream waits for the update only
  // before the combine_final that rewrites its snapshot block, two scans later (smap_done), and
  // host access to the map through the context joins it first (gc::join_side).
  hipStream_t mstream = nullptr;
  hipEvent_t smap_go = nullptr;
  hipEvent_t smap_done[2] = {nullptr, nullptr};
  bool smap_done_rec[2] = {false, false};
  double* snap_base = nullptr;
  int pending_slot = -1;
  int64_t pending_seq = 0;
  // Host-side accounting (gc_pipeline_host_stats): the reference's RuntimeCounters
  // (common/runtime_counters.py:19-108: host syncs, host<->device bytes) and the split of every
  // scan's and every staging call's host time into enqueue / copy work and waits for the device.
  double hs[GC_HOST_STATS] = {};
  double wait_acc_ms = 0.0;  // host waits (event polls, stream syncs) since the current entry began
  double scan_enq_ms = 0.0, scan_wait_ms = 0.0;  // the pending scan's local half
  // per-stage device timing (gc_pipeline_set_stage_timing): events around each launch group
  bool st_timing = false, st_rec = false;
  hipEvent_t st_ev[GC_STAGE_N] = {};
  // in-scan ConditioningCerts (gc_pipeline_set_inscan_certs): launched after every scan's evidence;
  // hcond_scan: P.hcond holds the certificates of the current L_pred / L (cleared by a belief upload)
  bool inscan_certs = false, hcond_scan = false;
  // P.pcert holds the projection certificates of the last finished scan (computed inside it)
  bool pcert_scan = false;
  // getter workspace (conditioning certificates), allocated with the pipeline: no hipMalloc / hipFree
  // (device-synchronising) on a getter a live node calls every scan
  double* ws = nullptr;
};

namespace {

int dalloc(gc_pipeline* p, size_t count, double** out) {
  void* ptr = nullptr;
  GC_HIP(p->ctx, hipMalloc(&ptr, (count ? count : 1) * sizeof(double)));
  GC_HIP(p->ctx, hipMemsetAsync(ptr, 0, (count ? count : 1) * sizeof(double), p->ctx->stream));
  p->allocs.push_back(ptr);
  *out = static_cast<double*>(ptr);
  return GC_OK;
}

double now_ms() {
  return 1e-6 * (double)std::chrono::duration_cast<std::chrono::nanoseconds>(
                    std::chrono::steady_clock::now().time_since_epoch()).count();
}

// a stream synchronisation on the host, counted as a host sync and as waiting time
int sync_counted(gc_pipeline* p) {
  double ms = 0.0;
  const int rc = gc::wait_stream(p->ctx, p->ctx->stream, "the pipeline stream", &ms);
  p->wait_acc_ms += ms;
  p->hs[GC_HS_HOST_SYNCS] += 1.0;
  return rc;
}

int up(gc_pipeline* p, double* d, const double* h, size_t count) {
  if (!h || count == 0) return GC_OK;
  GC_HIP(p->ctx, hipMemcpyAsync(d, h, count * sizeof(double), hipMemcpyHostToDevice, p->ctx->stream));
  p->hs[GC_HS_H2D_BYTES] += (double)(count * sizeof(double));
  return sync_counted(p);
}

int down(gc_pipeline* p, double* h, const double* d, size_t count) {
  if (!h || count == 0) return GC_OK;
  GC_HIP(p->ctx, hipMemcpyAsync(h, d, count * sizeof(double), hipMemcpyDeviceToHost, p->ctx->stream));
  p->hs[GC_HS_D2H_BYTES] += (double)(count * sizeof(double));
  return sync_counted(p);
}

// Host wait for a copy-stream event by polling: hipEventSynchronize may sleep on an interrupt and
// take tens to hundreds of microseconds to wake, enough to make the host, not the device, the
// bottleneck of a 0.3 ms scan. ~10^5 busy polls, then short sleeps, bounded by the context's wait
// timeout (fail fast: a stuck device or a dead peer ends in GC_ERR_RUNTIME, never an unbounded wait).
// An event already complete costs one query and is not counted as a sync.
int wait_event(gc_pipeline* p, hipEvent_t e) {
  gc_ctx* ctx = p->ctx;
  hipError_t q = hipEventQuery(e);
  if (q == hipSuccess) return GC_OK;
  if (q != hipErrorNotReady) GC_HIP(ctx, q);
  p->hs[GC_HS_HOST_SYNCS] += 1.0;
  double ms = 0.0;
  const int rc = gc::wait_event(ctx, e, "a scan slot's ingest copy", &ms, 100000);
  p->wait_acc_ms += ms;
  return rc;
}

// host time of one entry split into work and waits: sum / max per kind (GC_HS_* layout)
void account(gc_pipeline* p, int base, double t_entry0) {
  const double total = now_ms() - t_entry0, w = p->wait_acc_ms, e = total - w;
  double* h = p->hs;
  h[base] += 1.0;
  h[base + 1] += e;
  h[base + 2] = std::max(h[base + 2], e);
  h[base + 3] += w;
  h[base + 4] = std::max(h[base + 4], w);
}

int stage_event(gc_pipeline* p, int i) {
  if (!p->st_timing) return GC_OK;
  GC_HIP(p->ctx, hipEventRecord(p->st_ev[i], p->ctx->stream));
  return GC_OK;
}

// slot block layout (doubles): pts 3n | t n | w n | imu_t M | imu_g 3M | imu_a 3M | odom | a1 budget
// scalars 8 | their 3 x 64 partials (written on the device at staging; the pinned mirror's copy of
// this tail is unused)
struct SlotLayout {
  size_t t, w, imu, odom, budget, bpart, len;
  explicit SlotLayout(const gc::PipeDev& P) {
    const size_t n = (size_t)P.n_in, M = (size_t)P.M;
    t = 3 * n; w = 4 * n; imu = 5 * n; odom = imu + 7 * M; budget = odom + gc::kOdomLen;
    bpart = budget + 8; len = bpart + 3 * gc::kBudgetBlocks;
  }
};

int slot_alloc(gc_pipeline* p, gc_pipeline::Slot& s) {
  if (s.dev) return GC_OK;
  const SlotLayout Ly(p->P);
  GC_HIP(p->ctx, hipMalloc((void**)&s.dev, Ly.len * sizeof(double)));
  GC_HIP(p->ctx, hipHostMalloc((void**)&s.host, Ly.len * sizeof(double), hipHostMallocDefault));
  for (hipEvent_t* e : {&s.ready, &s.odom_done})
    GC_HIP(p->ctx, hipEventCreateWithFlags(e, hipEventDisableTiming));
  // recorded between two compute kernels: no system-scope fence (nothing is published by it, the copy
  // stream only needs the reads ordered before its writes): ~1 us of device time instead of ~3-6
  // (tools/probe/probe_sync.hip)
  GC_HIP(p->ctx, hipEventCreateWithFlags(&s.consumed, hipEventDisableTiming | hipEventDisableSystemFence));
  s.pts = s.dev; s.t = s.dev + Ly.t; s.w = s.dev + Ly.w;
  s.imu_t = s.dev + Ly.imu; s.imu_g = s.imu_t + p->P.M; s.imu_a = s.imu_g + 3 * p->P.M;
  s.odom = s.dev + Ly.odom;
  s.budget = s.dev + Ly.budget;
  s.bpart = s.dev + Ly.bpart;
  return GC_OK;
}

#define GC_TRY(expr)             \
  do {                           \
    int _rc = (expr);            \
    if (_rc != GC_OK) return _rc; \
  } while (0)

// the copy stream may overwrite the slot's device block only after the last scan that read it
// with a PrimitiveMap attached the pending scan's last read of its slot (the map update) is only
// enqueued by scan_finish, so that slot cannot be restaged before then
// the in-scan map update runs on this rank (a map attached, and this rank its owner or every rank updating)
bool smap_active(const gc_pipeline* p) {
  return p->smap_on && (p->smap_mode == GC_SMAP_REPLICATED || p->P.h_begin == 0);
}

int slot_check_restage(gc_pipeline* p, int slot) {
  GC_CHECK_ARG(p->ctx, !(p->pending && smap_active(p) && slot == p->pending_slot),
               "the slot is read by the pending scan's map update (gc_pipeline_scan_finish first)");
  return GC_OK;
}

int slot_wait_consumed(gc_pipeline* p, gc_pipeline::Slot& s) {
  if (s.consumed_ticket > 0) {
    const int64_t k = s.consumed_ticket;
    if (__atomic_load_n(p->done_word, __ATOMIC_ACQUIRE) < k) {
      // its bins may still be running: order the DMA after the earliest enqueued scan >= k whose
      // combine_final carries a completion event (fin_ev), or else after everything enqueued on the
      // compute stream. (A host poll of the word instead costs more than the gap it removes: H = 32
      // 0.2924 -> 0.2977 ms with 3 or 4 slots, H = 256 1.212 -> 1.221, profiles/r04/ab_slot_poll.txt;
      // so does a stream wait on the word, whose blit kernel spins on a CU: profiles/r04/ab_slot_bind.txt)
      int e = -1;
      for (int i = 0; i < 2; ++i)
        if (p->fin_ticket[i] >= k && (e < 0 || p->fin_ticket[i] < p->fin_ticket[e])) e = i;
      if (e >= 0) {
        GC_HIP(p->ctx, hipStreamWaitEvent(p->cstream, p->fin_ev[e], 0));
      } else {
        GC_HIP(p->ctx, hipEventRecord(s.consumed, p->ctx->stream));
        s.consumed_rec = true;
      }
    }
    s.consumed_ticket = 0;
  }
  if (s.consumed_rec) GC_HIP(p->ctx, hipStreamWaitEvent(p->cstream, s.consumed, 0));
  s.consumed_rec = false;
  return GC_OK;
}

// a1 budget scalars of the staged weights (point_budget.py:60-113), on the copy stream after them, when
// the predict launch has no room for its budget workgroups beside the hypotheses (stage_budget): they
// depend on the scan's weights and sizes only, so that launch is left its hypotheses (and the window
// of the points, which needs the scan window). H = 256: predict 46 -> ~41 us, 1.2010 -> 1.1984 ms per
// scan; at H = 32 the budget workgroups run beside the hypotheses for free and stay there (staged,
// 0.2873 -> 0.2890: profiles/r04/ab_staged_budget.txt)
int slot_budget(gc_pipeline* p, gc_pipeline::Slot& s, int64_t n_in) {
  if (p->stage_budget) GC_HIP(p->ctx, gc::launch_budget_stats(s.w, n_in, p->P.n_cap, s.bpart, s.budget, p->cstream));
  return GC_OK;
}

// host arrays -> the slot's pinned mirror (the previous DMA out of it has finished) -> device, on the
// copy stream; imu block = [imu_t M | imu_g 3M | imu_a 3M]
int slot_stage_imu_host(gc_pipeline* p, gc_pipeline::Slot& s, const double* h_imu_t, const double* h_imu_g,
                        const double* h_imu_a) {
  const SlotLayout Ly(p->P);
  const size_t M = (size_t)p->P.M;
  double* h = s.host + Ly.imu;
  std::memcpy(h, h_imu_t, M * sizeof(double));
  std::memcpy(h + M, h_imu_g, 3 * M * sizeof(double));
  std::memcpy(h + 4 * M, h_imu_a, 3 * M * sizeof(double));
  return GC_OK;
}

}  // namespace

extern "C" {

int32_t gc_pipeline_create(gc_ctx* ctx, const gc_pipeline_dims* dims, const double* cfg, gc_pipeline** out) {
  GC_CHECK_ARG(nullptr, ctx && dims && cfg && out, "NULL argument");
  GC_CHECK_ARG(ctx, dims->H_total > 0 && dims->h_count > 0 && dims->h_begin >= 0 &&
                        dims->h_begin + dims->h_count <= dims->H_total, "bad hypothesis shard");
  GC_CHECK_ARG(ctx, dims->h_count <= 1024, "at most 1024 hypotheses per rank");
  GC_CHECK_ARG(ctx, dims->B >= 1 && dims->B <= 64, "B must be in [1, 64]");
  GC_CHECK_ARG(ctx, dims->M >= 2 && dims->M <= 512, "IMU slots M must be in [2, 512]");
  GC_CHECK_ARG(ctx, dims->n_in_max > 0 && dims->n_cap > 0, "point counts must be positive");
  GC_CHECK_ARG(ctx, dims->world_size >= 1 && dims->rank >= 0 && dims->rank < dims->world_size, "bad rank");
  GC_CHECK_ARG(ctx, dims->geom_hyps >= 0 && dims->geom_hyps <= 65536, "geom_hyps must be in [0, 65536]");
  GC_CHECK_ARG(ctx, cfg[GC_PCFG_TAU] >= GC_FUSED_TAU_MIN, "tau must be >= GC_FUSED_TAU_MIN (3e-3)");
  GC_HIP(ctx, hipSetDevice(ctx->device));
  if (ctx->cu_count == 0) {
    int cus = 0;
    GC_HIP(ctx, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    ctx->cu_count = cus > 0 ? cus : 1;
  }
  gc_pipeline* p = new gc_pipeline();
  p->ctx = ctx;
  gc::PipeDev& P = p->P;
  P.Hl = dims->h_count; P.H = dims->H_total; P.h_begin = dims->h_begin; P.B = dims->B; P.M = dims->M;
  P.n_in = dims->n_in_max; P.n_cap = dims->n_cap; P.G = dims->world_size;
  P.geom_H = dims->geom_hyps;
  P.cus = ctx->cu_count;
  P.tau = cfg[GC_PCFG_TAU]; P.o0 = cfg[GC_PCFG_ORIGIN]; P.o1 = cfg[GC_PCFG_ORIGIN + 1]; P.o2 = cfg[GC_PCFG_ORIGIN + 2];
  P.eps_psd = cfg[GC_PCFG_EPS_PSD]; P.eps_lift = cfg[GC_PCFG_EPS_LIFT]; P.eps_mass = cfg[GC_PCFG_EPS_MASS];
  P.lambda_ou = cfg[GC_PCFG_LAMBDA_OU]; P.c_frob = cfg[GC_PCFG_C_FROB]; P.forgetting = cfg[GC_PCFG_FORGETTING];
  P.weight_floor = cfg[GC_PCFG_WEIGHT_FLOOR]; P.power_beta_min = cfg[GC_PCFG_POWER_BETA_MIN];
  P.power_beta_exc_c = cfg[GC_PCFG_POWER_BETA_EXC_C]; P.power_beta_z_c = cfg[GC_PCFG_POWER_BETA_Z_C];
  P.alpha_min = cfg[GC_PCFG_ALPHA_MIN]; P.alpha_max = cfg[GC_PCFG_ALPHA_MAX]; P.c0_cond = cfg[GC_PCFG_C0_COND];
  P.nu_max = cfg[GC_PCFG_NU_MAX];
  P.planar_z_ref = cfg[GC_PCFG_PLANAR_Z_REF]; P.planar_z_sigma = cfg[GC_PCFG_PLANAR_Z_SIGMA];
  P.planar_vz_sigma = cfg[GC_PCFG_PLANAR_VZ_SIGMA]; P.gravity_scale = cfg[GC_PCFG_GRAVITY_SCALE];
  const int Hl = P.Hl, B = P.B, NN = 484;
  const int PL = gc::partial_len(B);
  int rc = GC_OK;
  double** fields[] = {&P.X, &P.z, &P.L, &P.h, &P.stamp, &P.Lpred, &P.hpred, &P.pred_cert, &P.pose_pred, &P.xi,
                       &P.imu_out, &P.dPsiM, &P.stats, &P.bincert, &P.io_L, &P.io_h, &P.io_cert, &P.dPsiP,
                       &P.mu_fin, &P.diag, &P.mu_aux, &P.io_parts, &P.lpose, &P.Sig, &P.binaux, &P.hcond,
                       &P.pred_mode, &P.praw, &P.pcert};
  const size_t sizes[] = {(size_t)Hl * 6, (size_t)Hl * 22, (size_t)Hl * NN, (size_t)Hl * 22, (size_t)Hl,
                          (size_t)Hl * NN, (size_t)Hl * 22, (size_t)Hl * gc::kPredCert, (size_t)Hl * 6,
                          (size_t)Hl * 6, (size_t)Hl * gc::kImuOut, (size_t)Hl * 27, (size_t)Hl * B * 38,
                          (size_t)Hl * 8, (size_t)Hl * NN, (size_t)Hl * 22, (size_t)Hl * gc::kIoCert,
                          (size_t)Hl * 252, (size_t)Hl * 22, (size_t)Hl * gc::kHypDiag, (size_t)Hl * gc::kMuAux,
                          (size_t)Hl * gc::kIoParts, (size_t)Hl * 36, (size_t)Hl * NN, (size_t)Hl * B * 2,
                          (size_t)Hl * 8, (size_t)Hl, (size_t)Hl * 18,
                          ((size_t)Hl * (B + 2) + gc::kScanCerts) * 6};
  for (size_t i = 0; i < sizeof(sizes) / sizeof(sizes[0]) && rc == GC_OK; ++i) rc = dalloc(p, sizes[i], fields[i]);
  double** shared[] = {&P.weights, &P.Q, &P.bins, &P.map, &P.map_der, &P.map_misc, &P.map_inc, &P.nu_proc,
                       &P.Psi_proc, &P.nu_meas, &P.Psi_meas, &P.budget, &P.send, &P.gather, &P.comb, &P.iw_cert,
                       &P.h0rec, &P.smap_snap, &P.iwraw};
  const size_t ssz[] = {(size_t)P.H, (size_t)NN, (size_t)B * 3, (size_t)B * gc::kMapRec, (size_t)B * gc::kMapDer, 8,
                        (size_t)B * gc::kMapRec, 7, 7 * 36, 3, 27, 8, (size_t)PL, (size_t)PL * P.G,
                        GC_COMB_LEN, 4, gc::kH0Len, 2 * gc::kSnapLen, gc::kIwRawLen};
  for (size_t i = 0; i < sizeof(ssz) / sizeof(ssz[0]) && rc == GC_OK; ++i) rc = dalloc(p, ssz[i], shared[i]);
  if (rc != GC_OK) {
    gc_pipeline_destroy(p);
    return rc;
  }
  if (P.G == 1) {  // single rank: the combine reads its own partial record in place
    P.gather = P.send;
  }
  if (rc == GC_OK) rc = dalloc(p, 3 * gc::kBudgetBlocks, &P.budget_part);
  double* ticket = nullptr;
  if (rc == GC_OK) rc = dalloc(p, 1, &ticket);  // zeroed: the predict grid's budget arrival counter
  P.budget_ticket = reinterpret_cast<unsigned*>(ticket);
  p->stage_budget = !gc::predict_budget_inline(P);
  double* ctr = nullptr;
  if (rc == GC_OK) rc = dalloc(p, 1, &ctr);  // zeroed: k_bins_io's task counter + finished pullers
  P.task_ctr = reinterpret_cast<unsigned*>(ctr);
  if (rc == GC_OK) rc = dalloc(p, (size_t)P.n_cap, &P.w_win);
  if (rc == GC_OK) rc = dalloc(p, (size_t)2 * Hl * (NN + 6), &p->ws);  // getter workspace (conditioning certs)
  if (rc == GC_OK && hipHostMalloc((void**)&p->done_word, sizeof(int64_t), hipHostMallocCoherent) != hipSuccess) {
    gc::set_error(ctx, "hipHostMalloc failed for the slot completion word");
    rc = GC_ERR_RUNTIME;
  }
  if (p->done_word) *p->done_word = 0;
  for (hipEvent_t& e : p->fin_ev)
    if (rc == GC_OK && hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess)
      rc = GC_ERR_RUNTIME;
  if (rc == GC_OK && hipStreamCreateWithFlags(&p->cstream, hipStreamNonBlocking) != hipSuccess) {
    gc::set_error(ctx, "hipStreamCreateWithFlags failed for the ingest stream");
    rc = GC_ERR_RUNTIME;
  }
  p->snap_base = P.smap_snap;
  if (rc == GC_OK) rc = gc::wait_stream(ctx, ctx->stream, "the pipeline's zero fills");  // before any launch
  if (rc != GC_OK) {
    gc_pipeline_destroy(p);
    return rc;
  }
  *out = p;
  return GC_OK;
}

int32_t gc_pipeline_destroy(gc_pipeline* p) {
  if (!p) return GC_OK;
  // bounded (a stream stuck behind a failed peer's all-gather is still torn down)
  (void)gc::wait_stream(p->ctx, p->ctx->stream, "the pipeline stream at destruction");
  if (p->cstream) (void)gc::wait_stream(p->ctx, p->cstream, "the ingest stream at destruction");
  if (p->mstream) (void)gc::wait_stream(p->ctx, p->mstream, "the map-update stream at destruction");
  for (hipEvent_t e : p->smap_done)
    if (e && p->ctx->side_ev == e) {
      p->ctx->side_ev = nullptr;
      p->ctx->side_pending = false;
    }
  for (void* a : p->allocs) (void)hipFree(a);
  for (auto& s : p->slots) {
    for (void* d : {(void*)s.dev, (void*)s.bytes, (void*)s.ring, (void*)s.tag, (void*)s.flag})
      if (d) (void)hipFree(d);
    for (void* h : {(void*)s.host, (void*)s.hbytes})
      if (h) (void)hipHostFree(h);
    for (hipEvent_t e : {s.ready, s.odom_done, s.consumed})
      if (e) (void)hipEventDestroy(e);
  }
  for (hipEvent_t e : {p->x0, p->x1, p->fin_ev[0], p->fin_ev[1], p->smap_go, p->smap_done[0], p->smap_done[1]})
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : p->st_ev)
    if (e) (void)hipEventDestroy(e);
  if (p->smapW.buf) (void)hipFree(p->smapW.buf);
  if (p->smapW.runs.ptr) (void)hipFree(p->smapW.runs.ptr);
  if (p->cstream) (void)hipStreamDestroy(p->cstream);
  if (p->mstream) (void)hipStreamDestroy(p->mstream);
  if (p->done_word) (void)hipHostFree(p->done_word);
  delete p;
  return GC_OK;
}

int32_t gc_pipeline_set_bins(gc_pipeline* p, const double* h_bins) {
  GC_CHECK_ARG(nullptr, p && h_bins, "NULL argument");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  return up(p, p->P.bins, h_bins, (size_t)p->P.B * 3);
}

int32_t gc_pipeline_set_beliefs(gc_pipeline* p, const double* h_X, const double* h_z, const double* h_L,
                                const double* h_h, const double* h_stamp) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  const size_t Hl = p->P.Hl;
  p->sig_cached = false;
  p->hcond_scan = false;
  GC_TRY(up(p, p->P.X, h_X, Hl * 6));
  GC_TRY(up(p, p->P.z, h_z, Hl * 22));
  GC_TRY(up(p, p->P.L, h_L, Hl * 484));
  GC_TRY(up(p, p->P.h, h_h, Hl * 22));
  return up(p, p->P.stamp, h_stamp, Hl);
}

int32_t gc_pipeline_get_beliefs(gc_pipeline* p, double* h_X, double* h_z, double* h_L, double* h_h,
                                double* h_stamp) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  const size_t Hl = p->P.Hl;
  GC_TRY(down(p, h_X, p->P.X, Hl * 6));
  GC_TRY(down(p, h_z, p->P.z, Hl * 22));
  GC_TRY(down(p, h_L, p->P.L, Hl * 484));
  GC_TRY(down(p, h_h, p->P.h, Hl * 22));
  return down(p, h_stamp, p->P.stamp, Hl);
}

int32_t gc_pipeline_set_weights(gc_pipeline* p, const double* h_w) {
  GC_CHECK_ARG(nullptr, p && h_w, "NULL argument");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  return up(p, p->P.weights, h_w, p->P.H);
}

int32_t gc_pipeline_set_io_evidence(gc_pipeline* p, const double* h_L, const double* h_h, const double* h_cert) {
  GC_CHECK_ARG(nullptr, p && h_L && h_h && h_cert, "NULL argument");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  const size_t Hl = p->P.Hl;
  GC_TRY(up(p, p->P.io_L, h_L, Hl * 484));
  GC_TRY(up(p, p->P.io_h, h_h, Hl * 22));
  p->io_mode = GC_IO_GIVEN;
  return up(p, p->P.io_cert, h_cert, Hl * gc::kIoCert);
}

int32_t gc_pipeline_set_io_mode(gc_pipeline* p, int32_t mode) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  GC_CHECK_ARG(p->ctx, mode == GC_IO_GIVEN || mode == GC_IO_COMPUTED, "io mode must be GC_IO_GIVEN or GC_IO_COMPUTED");
  p->io_mode = mode;
  return GC_OK;
}

static int32_t gc_pipeline_stage_odom_impl(gc_pipeline* p, int32_t slot, const double* h_pose6, const double* h_cov36,
                               const double* h_twist6, const double* h_twist_cov36) {
  GC_CHECK_ARG(p->ctx, slot >= 0 && slot < GC_PIPE_MAX_SLOTS, "slot out of range");
  GC_TRY(slot_check_restage(p, slot));
  GC_CHECK_ARG(p->ctx, h_pose6 && h_cov36 && h_twist6 && h_twist_cov36, "NULL odometry array");
  auto& s = p->slots[slot];
  GC_TRY(slot_alloc(p, s));
  if (s.odom_rec) GC_TRY(wait_event(p, s.odom_done));  // the last odometry DMA read its area
  double* buf = s.host + SlotLayout(p->P).odom;
  std::memcpy(buf, h_pose6, 6 * sizeof(double));
  std::memcpy(buf + 6, h_cov36, 36 * sizeof(double));
  std::memcpy(buf + 42, h_twist6, 6 * sizeof(double));
  std::memcpy(buf + 48, h_twist_cov36, 36 * sizeof(double));
  GC_TRY(slot_wait_consumed(p, s));
  GC_HIP(p->ctx, hipMemcpyAsync(s.odom, buf, gc::kOdomLen * sizeof(double), hipMemcpyHostToDevice, p->cstream));
  p->hs[GC_HS_H2D_BYTES] += (double)(gc::kOdomLen * sizeof(double));
  GC_HIP(p->ctx, hipEventRecord(s.odom_done, p->cstream));
  GC_HIP(p->ctx, hipEventRecord(s.ready, p->cstream));  // scan_local's wait covers the odometry too
  s.odom_rec = s.ready_rec = true;
  s.has_odom = true;
  return GC_OK;
}

int32_t gc_pipeline_stage_odom(gc_pipeline* p, int32_t slot, const double* h_pose6, const double* h_cov36,
                               const double* h_twist6, const double* h_twist_cov36) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  const double t0 = now_ms();
  p->wait_acc_ms = 0.0;
  const int32_t rc = gc_pipeline_stage_odom_impl(p, slot, h_pose6, h_cov36, h_twist6, h_twist_cov36);
  account(p, GC_HS_STAGES, t0);
  return rc;
}

int32_t gc_pipeline_get_io_parts(gc_pipeline* p, double* h_parts) {
  GC_CHECK_ARG(nullptr, p && h_parts, "NULL argument");
  return down(p, h_parts, p->P.io_parts, (size_t)p->P.Hl * gc::kIoParts);
}

int32_t gc_pipeline_get_io_evidence(gc_pipeline* p, double* h_L, double* h_h, double* h_cert) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  const size_t Hl = p->P.Hl;
  GC_TRY(down(p, h_L, p->P.io_L, Hl * 484));
  GC_TRY(down(p, h_h, p->P.io_h, Hl * 22));
  return down(p, h_cert, p->P.io_cert, Hl * gc::kIoCert);
}

int32_t gc_pipeline_set_iw(gc_pipeline* p, const double* nu_proc, const double* Psi_proc, const double* nu_meas,
                           const double* Psi_meas) {
  GC_CHECK_ARG(nullptr, p && nu_proc && Psi_proc && nu_meas && Psi_meas, "NULL argument");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  GC_TRY(up(p, p->P.nu_proc, nu_proc, 7));
  GC_TRY(up(p, p->P.Psi_proc, Psi_proc, 252));
  GC_TRY(up(p, p->P.nu_meas, nu_meas, 3));
  GC_TRY(up(p, p->P.Psi_meas, Psi_meas, 27));
  GC_HIP(p->ctx, gc::launch_iw_Q(p->P, p->ctx->stream));
  return GC_OK;
}

int32_t gc_pipeline_get_iw(gc_pipeline* p, double* nu_proc, double* Psi_proc, double* nu_meas, double* Psi_meas,
                           double* Q, double* cert4) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  GC_TRY(down(p, nu_proc, p->P.nu_proc, 7));
  GC_TRY(down(p, Psi_proc, p->P.Psi_proc, 252));
  GC_TRY(down(p, nu_meas, p->P.nu_meas, 3));
  GC_TRY(down(p, Psi_meas, p->P.Psi_meas, 27));
  GC_TRY(down(p, Q, p->P.Q, 484));
  return down(p, cert4, p->P.iw_cert, 4);
}

int32_t gc_pipeline_set_map(gc_pipeline* p, const double* h_map) {
  GC_CHECK_ARG(nullptr, p && h_map, "NULL argument");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  GC_TRY(up(p, p->P.map, h_map, (size_t)p->P.B * gc::kMapRec));
  GC_HIP(p->ctx, gc::launch_map_derive(p->P, p->ctx->stream));
  return GC_OK;
}

int32_t gc_pipeline_get_map(gc_pipeline* p, double* h_map, double* h_map_der, double* h_misc2) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  GC_TRY(down(p, h_map, p->P.map, (size_t)p->P.B * gc::kMapRec));
  GC_TRY(down(p, h_map_der, p->P.map_der, (size_t)p->P.B * gc::kMapDer));
  return down(p, h_misc2, p->P.map_misc, 2);
}

static int32_t gc_pipeline_stage_scan_impl(gc_pipeline* p, int32_t slot, const double* h_pts, const double* h_t,
                               const double* h_w, int64_t n_in, const double* h_imu_t, const double* h_imu_g,
                               const double* h_imu_a) {
  GC_CHECK_ARG(p->ctx, slot >= 0 && slot < GC_PIPE_MAX_SLOTS, "slot out of range");
  GC_TRY(slot_check_restage(p, slot));
  GC_CHECK_ARG(p->ctx, n_in > 0 && n_in <= p->P.n_in, "n_in must be in [1, n_in_max]");
  GC_CHECK_ARG(p->ctx, h_pts && h_t && h_w && h_imu_t && h_imu_g && h_imu_a, "NULL scan array");
  auto& s = p->slots[slot];
  GC_TRY(slot_alloc(p, s));
  if (s.ready_rec) GC_TRY(wait_event(p, s.ready));  // the last DMA out of the mirror is done
  const SlotLayout Ly(p->P);
  const size_t n = (size_t)n_in, M = (size_t)p->P.M;
  std::memcpy(s.host, h_pts, 3 * n * sizeof(double));
  std::memcpy(s.host + Ly.t, h_t, n * sizeof(double));
  std::memcpy(s.host + Ly.w, h_w, n * sizeof(double));
  GC_TRY(slot_stage_imu_host(p, s, h_imu_t, h_imu_g, h_imu_a));
  GC_TRY(slot_wait_consumed(p, s));
  const hipMemcpyKind k = hipMemcpyHostToDevice;
  if (n == (size_t)p->P.n_in) {  // a full scan: points, times, weights and IMU are one contiguous block
    GC_HIP(p->ctx, hipMemcpyAsync(s.pts, s.host, (Ly.imu + 7 * M) * sizeof(double), k, p->cstream));
  } else {
    GC_HIP(p->ctx, hipMemcpyAsync(s.pts, s.host, 3 * n * sizeof(double), k, p->cstream));
    GC_HIP(p->ctx, hipMemcpyAsync(s.t, s.host + Ly.t, n * sizeof(double), k, p->cstream));
    GC_HIP(p->ctx, hipMemcpyAsync(s.w, s.host + Ly.w, n * sizeof(double), k, p->cstream));
    GC_HIP(p->ctx, hipMemcpyAsync(s.imu_t, s.host + Ly.imu, 7 * M * sizeof(double), k, p->cstream));
  }
  GC_TRY(slot_budget(p, s, n_in));
  GC_HIP(p->ctx, hipEventRecord(s.ready, p->cstream));
  p->hs[GC_HS_H2D_BYTES] += (double)((5 * n + 7 * M) * sizeof(double));
  s.ready_rec = true;
  s.n_in = n_in;
  return GC_OK;
}

int32_t gc_pipeline_stage_scan(gc_pipeline* p, int32_t slot, const double* h_pts, const double* h_t,
                               const double* h_w, int64_t n_in, const double* h_imu_t, const double* h_imu_g,
                               const double* h_imu_a) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  const double t0 = now_ms();
  p->wait_acc_ms = 0.0;
  const int32_t rc = gc_pipeline_stage_scan_impl(p, slot, h_pts, h_t, h_w, n_in, h_imu_t, h_imu_g, h_imu_a);
  account(p, GC_HS_STAGES, t0);
  return rc;
}

static int32_t gc_pipeline_stage_pointcloud2_impl(gc_pipeline* p, int32_t slot, const uint8_t* h_data, int64_t n_points,
                                      int32_t point_step, const int32_t* h_fields, double header_stamp,
                                      const double* h_R9, const double* h_t3, const double* h_imu_t,
                                      const double* h_imu_g, const double* h_imu_a) {
  GC_CHECK_ARG(p->ctx, slot >= 0 && slot < GC_PIPE_MAX_SLOTS, "slot out of range");
  GC_TRY(slot_check_restage(p, slot));
  GC_CHECK_ARG(p->ctx, n_points >= 0 && n_points <= p->P.n_in, "n_points must be in [0, n_in_max]");
  GC_CHECK_ARG(p->ctx, h_fields && h_R9 && h_t3 && h_imu_t && h_imu_g && h_imu_a, "NULL argument");
  GC_CHECK_ARG(p->ctx, n_points == 0 || (h_data && point_step > 0), "NULL message data");
  if (n_points == 0) {  // one zero-weight dummy point (backend_node.py:1700-1707)
    const double z3[3] = {0.0, 0.0, 0.0}, z1 = 0.0;
    return gc_pipeline_stage_scan_impl(p, slot, z3, &z1, &z1, 1, h_imu_t, h_imu_g, h_imu_a);
  }
  auto& s = p->slots[slot];
  GC_TRY(slot_alloc(p, s));
  if (!s.ring) {
    GC_HIP(p->ctx, hipMalloc((void**)&s.ring, (size_t)p->P.n_in));
    GC_HIP(p->ctx, hipMalloc((void**)&s.tag, (size_t)p->P.n_in));
    GC_HIP(p->ctx, hipMalloc((void**)&s.flag, 4 * sizeof(int32_t)));
  }
  if (s.ready_rec) GC_TRY(wait_event(p, s.ready));  // the last DMA / parse from this slot is done
  const size_t nb = (size_t)n_points * (size_t)point_step;
  if (s.bytes_cap < nb) {
    if (s.bytes) GC_HIP(p->ctx, hipFree(s.bytes));
    if (s.hbytes) GC_HIP(p->ctx, hipHostFree(s.hbytes));
    s.bytes = s.hbytes = nullptr;
    s.bytes_cap = 0;
    GC_HIP(p->ctx, hipMalloc((void**)&s.bytes, nb));
    GC_HIP(p->ctx, hipHostMalloc((void**)&s.hbytes, nb, hipHostMallocDefault));
    s.bytes_cap = nb;
  }
  std::memcpy(s.hbytes, h_data, nb);
  GC_TRY(slot_stage_imu_host(p, s, h_imu_t, h_imu_g, h_imu_a));
  GC_TRY(slot_wait_consumed(p, s));
  GC_HIP(p->ctx, hipMemcpyAsync(s.bytes, s.hbytes, nb, hipMemcpyHostToDevice, p->cstream));
  GC_TRY(gc::cloud_parse_on(p->ctx, p->cstream, s.flag, s.bytes, n_points, point_step, h_fields, header_stamp, h_R9,
                            h_t3, s.pts, s.t, s.w, s.ring, s.tag));
  GC_TRY(slot_budget(p, s, n_points));
  GC_HIP(p->ctx, hipMemcpyAsync(s.imu_t, s.host + SlotLayout(p->P).imu, 7 * (size_t)p->P.M * sizeof(double),
                                hipMemcpyHostToDevice, p->cstream));
  GC_HIP(p->ctx, hipEventRecord(s.ready, p->cstream));
  p->hs[GC_HS_H2D_BYTES] += (double)(nb + 7 * (size_t)p->P.M * sizeof(double));
  s.ready_rec = true;
  s.n_in = n_points;
  return GC_OK;
}

int32_t gc_pipeline_stage_pointcloud2(gc_pipeline* p, int32_t slot, const uint8_t* h_data, int64_t n_points,
                                      int32_t point_step, const int32_t* h_fields, double header_stamp,
                                      const double* h_R9, const double* h_t3, const double* h_imu_t,
                                      const double* h_imu_g, const double* h_imu_a) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  const double t0 = now_ms();
  p->wait_acc_ms = 0.0;
  const int32_t rc = gc_pipeline_stage_pointcloud2_impl(p, slot, h_data, n_points, point_step, h_fields, header_stamp, h_R9, h_t3, h_imu_t, h_imu_g, h_imu_a);
  account(p, GC_HS_STAGES, t0);
  return rc;
}

int32_t gc_pipeline_attach_comm(gc_pipeline* p, gc_comm* comm) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  GC_CHECK_ARG(p->ctx, comm == nullptr || gc::comm_size(comm) == p->P.G, "communicator size != world_size");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  p->comm = comm;
  if (p->P.G == 1) {
    // a single-rank pipeline with a communicator runs the real all-gather into a buffer of its own
    // (without one the combine reads its partial record in place)
    if (comm && !p->own_gather) GC_TRY(dalloc(p, (size_t)gc::partial_len(p->P.B), &p->own_gather));
    p->P.gather = comm ? p->own_gather : p->P.send;
  }
  return GC_OK;
}

int32_t gc_pipeline_partial_len(const gc_pipeline* p) { return p ? gc::partial_len(p->P.B) : 0; }

int32_t gc_pipeline_run_scan(gc_pipeline* p, int32_t slot, double scan_start, double scan_end, double t_last,
                             double t_scan, double dt_sec, int64_t scan_count) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  GC_CHECK_ARG(p->ctx, p->P.G == 1 || p->comm, "world_size > 1 needs gc_pipeline_attach_comm");
  GC_TRY(gc_pipeline_scan_local(p, slot, scan_start, scan_end, t_last, t_scan, dt_sec, scan_count));
  return gc_pipeline_scan_finish(p, nullptr);
}

int32_t gc_pipeline_get_partial(gc_pipeline* p, double* h_record) {
  GC_CHECK_ARG(nullptr, p && h_record, "NULL argument");
  GC_CHECK_ARG(p->ctx, p->pending, "no pending scan (gc_pipeline_scan_local)");
  return down(p, h_record, p->P.send, (size_t)gc::partial_len(p->P.B));
}

static int32_t scan_finish_impl(gc_pipeline* p, const double* h_gather) {
  GC_CHECK_ARG(p->ctx, p->pending, "no pending scan (gc_pipeline_scan_local)");
  GC_CHECK_ARG(p->ctx, h_gather || p->P.G == 1 || p->comm,
               "world_size > 1 needs a communicator or the host-gathered records");
  gc_ctx* ctx = p->ctx;
  gc::PipeDev& P = p->P;
  const int64_t PL = gc::partial_len(P.B);
  if (h_gather || p->comm) {
    if (p->x_timing) {
      if (!p->x0) {
        GC_HIP(ctx, hipEventCreate(&p->x0));
        GC_HIP(ctx, hipEventCreate(&p->x1));
      }
      GC_HIP(ctx, hipEventRecord(p->x0, ctx->stream));
    }
    if (h_gather) {  // the G records of this scan, gathered by the caller (rank order)
      GC_TRY(up(p, P.gather, h_gather, (size_t)PL * P.G));
    } else {
      GC_TRY(gc::comm_allgather(p->comm, ctx, P.send, P.gather, PL));
    }
    if (p->x_timing) {
      GC_HIP(ctx, hipEventRecord(p->x1, ctx->stream));
      p->x_rec = true;
    }
  }
  GC_TRY(stage_event(p, 5));
  p->pending = false;
  // every kBindEvery-th scan's combine_final carries a completion event for the slot staging
  // (fin_ev; with a map attached the slots order on the map update instead)
  hipEvent_t fin = nullptr;
  int fin_e = -1;
  const bool smap = smap_active(p);
  if (kBindEvery > 0 && !smap && p->pending_ticket > 0 && p->pending_ticket % kBindEvery == 0) {
    fin_e = (int)((p->pending_ticket / kBindEvery) & 1);
    fin = p->fin_ev[fin_e];
    p->fin_ticket[fin_e] = 0;  // the event is re-armed by this launch: unusable until it succeeds
  }
  const int par = (int)(p->pending_ticket & 1);
  P.smap_snap = p->snap_base + par * gc::kSnapLen;
  if (smap && p->smap_done_rec[par]) {
    // the map update two scans back read this snapshot block: rewritten only after it (long done
    // by now, the wait costs the stream a barrier)
    GC_HIP(ctx, hipStreamWaitEvent(ctx->stream, p->smap_done[par], 0));
    p->smap_done_rec[par] = false;
  }
  const bool side = smap && p->mstream;
  if (side) fin = p->smap_go;
  GC_HIP(ctx, gc::launch_combine_final(P, p->pending_S, ctx->stream, fin));
  // only a launch that carries the event makes it cover this ticket (a failed launch leaves it
  // cleared, so slot_wait_consumed falls back to an event recorded on the compute stream)
  if (fin_e >= 0) p->fin_ticket[fin_e] = p->pending_ticket;
  // the scan's remaining projection certificates (the record and IW blocks combine_final just used)
  if (p->inscan_certs) GC_HIP(ctx, gc::launch_proj_certs(P, ctx->stream));
  p->pcert_scan = p->inscan_certs;
  GC_TRY(stage_event(p, 6));
  if (smap) {
    auto& s = p->slots[p->pending_slot];
    const gc::ScanArgs& S = p->pending_S;
    const gc::ScanMapInput in{s.pts, s.t, s.w, S.t0, S.t1, p->smap_voxel, S.t1, p->pending_seq};
    hipStream_t ms = side ? p->mstream : ctx->stream;
    if (side) GC_HIP(ctx, hipStreamWaitEvent(ms, p->smap_go, 0));
    if (side && ctx->side_pending && ctx->side_ev != p->smap_done[0] && ctx->side_ev != p->smap_done[1]) {
      // the context keeps one side event: another pipeline's update is still pending on it, so this
      // update orders after it and the event recorded below covers both (join_side then joins every
      // pipeline's update, not only the last one's)
      GC_HIP(ctx, hipStreamWaitEvent(ms, ctx->side_ev, 0));
    }
    int rc = gc::scan_map_update(ctx, ms, &p->smapW, p->smap, P, in);
    if (rc == GC_OK && p->smap_colors) {
      // primitive_map_fuse ends with colors = rgb = the estimate from the camera accumulators on
      // every slot (primitive_map.py:1090-1098); LiDAR rows leave those inputs unchanged, so the
      // assignment is idempotent until a host operation (insert, merge, a colour upload) writes the
      // colour fields and marks them stale again (gc_pipeline_map_colors_stale)
      const hipError_t e = gc::launch_fuse_colors(p->smap, P.eps_mass, ms);
      if (e != hipSuccess) {
        gc::set_error(ctx, std::string("HIP error ") + hipGetErrorString(e) + " in the map colour pass");
        rc = GC_ERR_RUNTIME;
      } else {
        p->smap_colors = false;
      }
    }
    // the map update was the slot's last reader: the next staging into the slot orders after this
    // event on every path, a failed launch of the update included (its earlier kernels may be queued)
    hipError_t er = hipEventRecord(s.consumed, ms);
    s.consumed_rec = er == hipSuccess;
    s.consumed_ticket = 0;
    if (side && er == hipSuccess) {
      er = hipEventRecord(p->smap_done[par], ms);
      p->smap_done_rec[par] = er == hipSuccess;
      ctx->side_ev = p->smap_done[par];
      ctx->side_pending = er == hipSuccess;
    }
    if (rc != GC_OK) return rc;
    GC_HIP(ctx, er);
  }
  GC_TRY(stage_event(p, 7));
  p->st_rec = p->st_timing;
  return GC_OK;
}

int32_t gc_pipeline_scan_finish(gc_pipeline* p, const double* h_gather) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  const double t0 = now_ms();
  p->wait_acc_ms = 0.0;
  const bool was_pending = p->pending;
  const int32_t rc = scan_finish_impl(p, h_gather);
  if (was_pending) {
    // one scan = its local half and this finish: enqueue work and waits, each summed and maxed per scan
    const double enq = p->scan_enq_ms + (now_ms() - t0 - p->wait_acc_ms), w = p->scan_wait_ms + p->wait_acc_ms;
    double* h = p->hs;
    h[GC_HS_SCANS] += 1.0;
    h[GC_HS_SCAN_ENQ_MS] += enq;
    h[GC_HS_SCAN_ENQ_MAX] = std::max(h[GC_HS_SCAN_ENQ_MAX], enq);
    h[GC_HS_SCAN_WAIT_MS] += w;
    h[GC_HS_SCAN_WAIT_MAX] = std::max(h[GC_HS_SCAN_WAIT_MAX], w);
  }
  return rc;
}

int32_t gc_pipeline_map_colors_stale(gc_pipeline* p) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  GC_CHECK_ARG(p->ctx, p->smap_on, "no PrimitiveMap attached");
  p->smap_colors = p->smap.cam_mass != nullptr;
  return GC_OK;
}

int32_t gc_pipeline_attach_primitive_map(gc_pipeline* p, const gc_primitive_map* map, double voxel_m) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  if (!map) {
    p->smap_on = false;
    return GC_OK;
  }
  GC_CHECK_ARG(p->ctx, map->m_slots > 0 && map->m_slots < (int64_t)0xFFFFFFFF, "m_slots out of range");
  GC_CHECK_ARG(p->ctx, map->n_lobes >= 1 && map->n_lobes <= 8, "n_lobes must be in [1, 8]");
  {
    const char* lay_ = gc::map_layout_error(*map);
    GC_CHECK_ARG(p->ctx, lay_ == nullptr, lay_ ? lay_ : "");
  }
  GC_CHECK_ARG(p->ctx, map->Lambdas && map->thetas && map->etas && map->weights && map->timestamps &&
                           map->last_supported_scan_seq && map->last_update_scan_seq,
               "NULL map field");
  GC_CHECK_ARG(p->ctx, voxel_m > 0.0, "voxel_m must be positive");
  if (p->mstream) GC_TRY(gc::wait_stream(p->ctx, p->mstream, "the map-update stream before re-attaching"));
  GC_TRY(gc::scan_map_prepare(p->ctx, &p->smapW, p->P.n_cap, map->m_slots));
  if (kSmapSide && !p->mstream) {
    // the start signal orders device work only; the done events keep the system-scope release (a
    // host copy of the map joined after them reads memory the update wrote)
    GC_HIP(p->ctx, hipEventCreateWithFlags(&p->smap_go, hipEventDisableTiming | hipEventDisableSystemFence));
    for (hipEvent_t* e : {&p->smap_done[0], &p->smap_done[1]})
      GC_HIP(p->ctx, hipEventCreateWithFlags(e, hipEventDisableTiming));
    GC_HIP(p->ctx, hipStreamCreateWithFlags(&p->mstream, hipStreamNonBlocking));
  }
  p->smap = *map;
  p->smap_voxel = voxel_m;
  p->smap_colors = map->cam_mass != nullptr && !map->colors_current;
  GC_CHECK_ARG(p->ctx, !p->smap_colors || (map->rgb_cam_accum && map->rgb_cam_denom && map->rgb),
               "colour fields must be all set or all NULL");
  p->smap_on = true;
  return GC_OK;
}

int32_t gc_pipeline_set_scan_map_mode(gc_pipeline* p, int32_t mode) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  GC_CHECK_ARG(p->ctx, mode == GC_SMAP_OWNER || mode == GC_SMAP_REPLICATED, "mode must be GC_SMAP_OWNER or GC_SMAP_REPLICATED");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  p->smap_mode = mode;
  return GC_OK;
}

int32_t gc_pipeline_get_scan_map_pose(gc_pipeline* p, double* h_out) {
  GC_CHECK_ARG(nullptr, p && h_out, "NULL argument");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  return down(p, h_out, p->P.send + gc::rec_h0(p->P.B), gc::kH0Len);
}

int32_t gc_pipeline_get_scan_map_count(gc_pipeline* p, int64_t* n_slots) {
  GC_CHECK_ARG(nullptr, p && n_slots, "NULL argument");
  GC_CHECK_ARG(p->ctx, p->smap_on, "no PrimitiveMap attached");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  if (!smap_active(p)) {  // not this rank's map to update (GC_SMAP_OWNER on a rank without hypothesis 0)
    *n_slots = 0;
    return GC_OK;
  }
  GC_TRY(gc::join_side(p->ctx));  // the counts of the last update (its stream)
  size_t bytes = 0;
  const int32_t rc = gc::scan_map_count(p->ctx, p->smapW, n_slots, &bytes);
  p->hs[GC_HS_HOST_SYNCS] += 1.0;
  p->hs[GC_HS_D2H_BYTES] += (double)bytes;
  return rc;
}

static int32_t scan_local_impl(gc_pipeline* p, int32_t slot, double scan_start, double scan_end, double t_last,
                               double t_scan, double dt_sec, int64_t scan_count) {
  GC_CHECK_ARG(p->ctx, !p->pending, "the previous scan's exchange is pending (gc_pipeline_scan_finish)");
  GC_CHECK_ARG(p->ctx, slot >= 0 && slot < GC_PIPE_MAX_SLOTS && p->slots[slot].n_in > 0, "scan slot not staged");
  GC_CHECK_ARG(p->ctx, p->io_mode == GC_IO_GIVEN || p->slots[slot].has_odom,
               "GC_IO_COMPUTED needs the slot's odometry (gc_pipeline_stage_odom)");
  gc_ctx* ctx = p->ctx;
  auto& s = p->slots[slot];
  // the slot's staged scan must have landed. The host waits for the copy rather than the compute
  // stream: a cross-queue barrier costs ~6 us of device time per scan, while the host is normally a
  // scan or more ahead of the device and the copy (ordered after an earlier scan's bins) long done
  if (s.ready_rec) GC_TRY(wait_event(p, s.ready));
  gc::ScanArgs S{s.imu_t, s.imu_g, s.imu_a, scan_start, scan_end, t_last, t_scan, dt_sec,
                 scan_count >= 1 ? 1.0 : 0.0, s.w, s.n_in, p->stage_budget ? s.budget : nullptr, s.t, p->sig_cached ? 1 : 0};
  gc::PipeDev& P = p->P;
  const bool io = p->io_mode == GC_IO_COMPUTED;
  // a2 + a3 (and the points' time window; the a1 budget scalars the fused kernel reads the
  // selection / mass scale from were formed when the slot was staged)
  GC_TRY(stage_event(p, 0));
  GC_HIP(ctx, gc::launch_predict_imu(P, S, ctx->stream));
  GC_TRY(stage_event(p, 1));
  // a1 -> a4 -> a5 -> a6 fused over all local hypotheses, and the a9a IMU/odom evidence branch
  // (pipeline.py:595-776: it needs the prediction, not the bins) as extra workgroups of the same
  // launch
  // nothing after the bins reads the slot (but the in-scan map update in scan_finish, when a map
  // is attached): the next staging into it may proceed once the bins are done, which the finalize
  // kernel publishes as this scan's ticket (done_word)
  ++p->ticket;
  gc::BinsFold fold;
  int64_t* dw = smap_active(p) ? nullptr : p->done_word;
  GC_TRY(gc::scan_bins_pipeline(ctx, P, S, s.odom, io, s.pts, s.t, s.w, s.n_in, dw, p->ticket, &fold));
  gc::ScanArgs Se = S;  // the evidence launch's: with the finalize folded in, its records and the ticket
  Se.fin_part = fold.part;
  Se.fin_chunks = fold.chunks;
  Se.done_word = fold.part ? dw : nullptr;
  Se.ticket = p->ticket;
  if (!smap_active(p)) s.consumed_ticket = p->ticket;
  p->pending_ticket = p->ticket;
  GC_TRY(stage_event(p, 2));
  // a7 .. a15
  GC_HIP(ctx, gc::launch_evidence(P, Se, ctx->stream));
  p->sig_cached = true;
  if (p->inscan_certs) GC_HIP(ctx, gc::launch_hyp_certs(P, ctx->stream));
  p->hcond_scan = p->inscan_certs;
  GC_TRY(stage_event(p, 3));
  // a16 local part: this rank's partial record (weighted sums, IW statistics, map increment)
  GC_HIP(ctx, gc::launch_combine_local(P, ctx->stream));
  GC_TRY(stage_event(p, 4));
  p->pending_S = S;
  p->pending_slot = slot;
  p->pending_seq = scan_count;
  p->pending = true;
  return GC_OK;
}

int32_t gc_pipeline_scan_local(gc_pipeline* p, int32_t slot, double scan_start, double scan_end, double t_last,
                               double t_scan, double dt_sec, int64_t scan_count) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  const double t0 = now_ms();
  p->wait_acc_ms = 0.0;
  const int32_t rc = scan_local_impl(p, slot, scan_start, scan_end, t_last, t_scan, dt_sec, scan_count);
  p->scan_wait_ms = p->wait_acc_ms;
  p->scan_enq_ms = now_ms() - t0 - p->wait_acc_ms;
  return rc;
}

int32_t gc_pipeline_get_combined(gc_pipeline* p, double* h_out) {
  GC_CHECK_ARG(nullptr, p && h_out, "NULL argument");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  GC_TRY(down(p, h_out, p->P.comb, GC_COMB_LEN));
  double* cc = h_out + 484 + 22 + 22 + 6;
  if (cc[2] != cc[2]) {
    // the combine certified the barycenter PSD by Cholesky (the projection is then the identity and
    // its eigen-decomposition was skipped on the scan path); the reference's ConditioningCert of the
    // combined belief (hypothesis.py:186-202) is the clamped spectrum of that same matrix, computed
    // here on demand by the Jacobi projection of the stored combined L
    double* ws = p->ws;  // the pipeline's workspace (>= 2 Hl (484 + 6) doubles): no allocation here
    GC_TRY(gc_domain_projection_psd_batch(p->ctx, 1, 22, p->P.comb, p->P.eps_psd, ws, ws + 484));
    double c6[6];
    GC_TRY(down(p, c6, ws + 484, 6));
    cc[2] = c6[2]; cc[3] = c6[3]; cc[4] = c6[4]; cc[5] = c6[5];
  }
  return GC_OK;
}

int32_t gc_pipeline_set_exchange_timing(gc_pipeline* p, int32_t on) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  p->x_timing = on != 0;
  return GC_OK;
}

int32_t gc_pipeline_exchange_ms(gc_pipeline* p, float* ms) {
  GC_CHECK_ARG(nullptr, p && ms, "NULL argument");
  GC_CHECK_ARG(p->ctx, p->x_rec, "no timed exchange has run (timing off, or one rank without a communicator)");
  if (int rc = gc::wait_event(p->ctx, p->x1, "the timed exchange")) return rc;
  GC_HIP(p->ctx, hipEventElapsedTime(ms, p->x0, p->x1));
  return GC_OK;
}

int32_t gc_pipeline_comm_size(const gc_pipeline* p) { return p ? (p->comm ? gc::comm_size(p->comm) : 0) : 0; }

int32_t gc_pipeline_get_hyp_conditioning(gc_pipeline* p, double* h_out) {
  GC_CHECK_ARG(nullptr, p && h_out, "NULL argument");
  GC_CHECK_ARG(p->ctx, p->sig_cached, "no scan has run since the beliefs were set");
  // The batched scan certifies these projections by Cholesky (their eigen-decompositions are skipped
  // on the scan path); the reference's ConditioningCert of each is the clamped spectrum of the same
  // stored matrix, computed here on demand by the Jacobi projection (off the scan path, as
  // gc_pipeline_get_combined does for the combined belief)
  const int Hl = p->P.Hl, NN = 484;
  if (p->hcond_scan) return down(p, h_out, p->P.hcond, (size_t)Hl * 8);  // computed inside the scan
  double* ws = p->ws;  // 2 Hl (NN + 6) doubles, allocated with the pipeline
  const size_t len = (size_t)Hl * (NN + 6);
  const double* mats[2] = {p->P.Lpred, p->P.L};
  int32_t rc = GC_OK;
  for (int m = 0; m < 2 && rc == GC_OK; ++m)
    rc = gc_domain_projection_psd_batch(p->ctx, Hl, 22, mats[m], p->P.eps_psd, ws + m * len,
                                        ws + m * len + (size_t)Hl * NN);
  std::vector<double> c6((size_t)2 * Hl * 6);
  if (rc == GC_OK) rc = down(p, c6.data(), ws + (size_t)Hl * NN, (size_t)Hl * 6);
  if (rc == GC_OK) rc = down(p, c6.data() + (size_t)Hl * 6, ws + len + (size_t)Hl * NN, (size_t)Hl * 6);
  if (rc != GC_OK) return rc;
  for (int h = 0; h < Hl; ++h)
    for (int m = 0; m < 2; ++m)
      for (int k = 0; k < 4; ++k) h_out[((size_t)h * 2 + m) * 4 + k] = c6[((size_t)m * Hl + h) * 6 + 2 + k];
  return GC_OK;
}

int32_t gc_pipeline_get_projection_certs(gc_pipeline* p, double* h_hyp, double* h_scan) {
  GC_CHECK_ARG(nullptr, p && h_hyp && h_scan, "NULL argument");
  GC_CHECK_ARG(p->ctx, p->sig_cached, "no scan has run since the beliefs were set");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  const gc::PipeDev& P = p->P;
  // computed inside the scan (in-scan certificates), or now from the last scan's stored operands
  if (!p->pcert_scan) GC_HIP(p->ctx, gc::launch_proj_certs(P, p->ctx->stream));
  const size_t nh = (size_t)P.Hl * (P.B + 2) * 6;
  GC_TRY(down(p, h_hyp, P.pcert, nh));
  return down(p, h_scan, P.pcert + nh, (size_t)gc::kScanCerts * 6);
}

int32_t gc_pipeline_get_hyp_diag(gc_pipeline* p, double* h_diag) {
  GC_CHECK_ARG(nullptr, p && h_diag, "NULL argument");
  return down(p, h_diag, p->P.diag, (size_t)p->P.Hl * gc::kHypDiag);
}

int32_t gc_pipeline_get_lpose6(gc_pipeline* p, double* h_lpose) {
  GC_CHECK_ARG(nullptr, p && h_lpose, "NULL argument");
  return down(p, h_lpose, p->P.lpose, (size_t)p->P.Hl * 36);
}

int32_t gc_pipeline_get_hyp_stats(gc_pipeline* p, double* h_dPsi_proc, double* h_dPsi_meas, double* h_Sigma) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  const size_t Hl = p->P.Hl;
  GC_TRY(down(p, h_dPsi_proc, p->P.dPsiP, Hl * 252));
  GC_TRY(down(p, h_dPsi_meas, p->P.dPsiM, Hl * 27));
  GC_CHECK_ARG(p->ctx, h_Sigma == nullptr || p->sig_cached, "no scan has run since the beliefs were set");
  return down(p, h_Sigma, p->P.Sig, Hl * 484);
}

int32_t gc_pipeline_get_bin_stats(gc_pipeline* p, double* h_stats, double* h_cert, double* h_xi) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  GC_TRY(down(p, h_stats, p->P.stats, (size_t)p->P.Hl * p->P.B * 38));
  GC_TRY(down(p, h_cert, p->P.bincert, (size_t)p->P.Hl * 8));
  return down(p, h_xi, p->P.xi, (size_t)p->P.Hl * 6);
}

int32_t gc_pipeline_set_stage_timing(gc_pipeline* p, int32_t on) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  if (on && !p->st_ev[0])
    for (hipEvent_t& e : p->st_ev) GC_HIP(p->ctx, hipEventCreate(&e));
  p->st_timing = on != 0;
  p->st_rec = false;
  return GC_OK;
}

int32_t gc_pipeline_stage_ms(gc_pipeline* p, float* h_ms) {
  GC_CHECK_ARG(nullptr, p && h_ms, "NULL argument");
  GC_CHECK_ARG(p->ctx, p->st_rec, "no scan has finished with stage timing on (gc_pipeline_set_stage_timing)");
  double wms = 0.0;
  if (int rc = gc::wait_event(p->ctx, p->st_ev[GC_STAGE_N - 1], "the stage-timing events", &wms)) return rc;
  p->wait_acc_ms += wms;
  p->hs[GC_HS_HOST_SYNCS] += 1.0;
  for (int i = 0; i + 1 < GC_STAGE_N; ++i)
    GC_HIP(p->ctx, hipEventElapsedTime(&h_ms[i], p->st_ev[i], p->st_ev[i + 1]));
  GC_HIP(p->ctx, hipEventElapsedTime(&h_ms[GC_STAGE_N - 1], p->st_ev[0], p->st_ev[GC_STAGE_N - 1]));
  return GC_OK;
}

int32_t gc_pipeline_set_predict_route(gc_pipeline* p, int32_t route) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  GC_CHECK_ARG(p->ctx, route == 0 || route == 1, "route must be 0 (split) or 1 (factorised)");
  p->P.predict_route = route;
  return GC_OK;
}

int32_t gc_pipeline_set_inscan_certs(gc_pipeline* p, int32_t on) {
  GC_CHECK_ARG(nullptr, p, "NULL pipeline");
  GC_CHECK_ARG(p->ctx, !p->pending, "a scan's exchange is pending (gc_pipeline_scan_finish)");
  p->inscan_certs = on != 0;
  return GC_OK;
}

int32_t gc_pipeline_host_stats(gc_pipeline* p, double* h_out, int32_t reset) {
  GC_CHECK_ARG(nullptr, p && h_out, "NULL argument");
  for (int i = 0; i < GC_HOST_STATS; ++i) h_out[i] = p->hs[i];
  if (reset)
    for (double& v : p->hs) v = 0.0;
  return GC_OK;
}

}  // extern "C"
