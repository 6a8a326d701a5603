// gc_internal.h — host-side internals shared by the libgcslam translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include "../../include/gcslam.h"

struct gc_comm;

namespace gc {
// a device run hash (gc_runs.h RunTable): 2^bits 8-B entries (>= 2^kRunLoadShift x the rows) and
// the 2^(bits - kRunLoadShift) position-indexed successor links after them, all zero between uses
#ifndef GC_RUN_LOAD_SHIFT
#define GC_RUN_LOAD_SHIFT 2
#endif
constexpr uint32_t kRunLoadShift = GC_RUN_LOAD_SHIFT;
// the linear probe (gc_runs.h) relies on a table strictly larger than its runs
static_assert(kRunLoadShift >= 1, "the run hash needs more entries than rows");
struct RunTableBuf {
  void* ptr = nullptr;
  uint32_t bits = 0;
  unsigned long long* entries() const { return (unsigned long long*)ptr; }
  uint32_t* succ() const { return (uint32_t*)((char*)ptr + ((size_t)8 << bits)); }
  bool dirty = true;  // a fill is due (new, grown, or a call that failed between its two passes)
};
}  // namespace gc

struct gc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  void* scratch = nullptr;  // growable device scratch (per ctx, stream-ordered use only)
  size_t scratch_bytes = 0;
  int cu_count = 0;  // compute units of the device (queried on first use)
  // the run hash of gc_primitive_map_fuse's reduce-by-key (gc_runs.h RunTable)
  gc::RunTableBuf runs;
  // device work of this context left running on a stream of its own (a pipeline's in-scan map
  // update, gc_pipeline.cpp): every entry point that may touch its data orders ctx->stream after it
  // first (gc::join_side); the event belongs to the pipeline, which clears it before destroying it
  hipEvent_t side_ev = nullptr;
  bool side_pending = false;
  // Fail-fast bound on every host wait for this context's device work (gc_ctx_set_wait_timeout;
  // GC_WAIT_TIMEOUT_S in the environment, default 300 s). A wait that runs out aborts `comm` (the
  // RCCL communicator last initialised on this context) so a peer that died cannot hold this rank in
  // an all-gather, and returns GC_ERR_RUNTIME (backend_node.py:2205-2210: log and re-raise).
  double wait_timeout_s = 300.0;
  gc_comm* comm = nullptr;
  // Device buffer arena behind gc_buffer_alloc / gc_buffer_free (device buffers are owned
  // by the context's arena): a freed block goes back to a per-size-class free list and is handed to
  // the next allocation of its class with no hipMalloc / hipFree and no synchronisation. Every use of
  // an arena buffer is ordered on this context's stream (the entries, uploads and downloads all run
  // there), so a block freed while a queued kernel still reads it is only rewritten by work queued
  // after that kernel. Blocks are returned to HIP at gc_ctx_trim / gc_ctx_destroy, or at once when the
  // cache would exceed arena_cap bytes.
  std::mutex arena_mu;
  std::multimap<size_t, void*> arena_free;     // class size -> cached block
  std::unordered_map<void*, size_t> arena_live;  // block -> class size
  size_t arena_cached = 0, arena_live_bytes = 0, arena_cap = (size_t)16 << 30;
  int64_t arena_hip_allocs = 0, arena_hip_frees = 0, arena_reuses = 0;
  // Pinned staging ring of gc_buffer_upload (uploads of at most kStageSeg bytes): the caller's bytes are
  // copied into the current segment of a pinned host ring and the DMA is enqueued on the stream with
  // no wait, so the caller's buffer is free on return and a chain of small uploads and launches
  // never drains the stream (the per-operator drop-ins upload a few hundred small operands per scan).
  // A segment is reused only after the event recorded when the ring last left it has completed.
  static constexpr int kStageSegs = 8;
  static constexpr size_t kStageSeg = (size_t)512 << 10;
  char* stage_host = nullptr;
  hipEvent_t stage_ev[kStageSegs] = {};
  bool stage_rec[kStageSegs] = {};
  int stage_seg = 0;
  size_t stage_off = 0;
  int64_t stage_uploads = 0;
};

namespace gc {

// thread-local fallback message for errors raised before a ctx exists
void set_error(gc_ctx* ctx, const std::string& msg);

// orders ctx->stream after the context's pending side-stream work (side_ev), once
int join_side(gc_ctx* ctx);

// device scratch of at least `bytes` (synchronises the stream before growing)
int scratch(gc_ctx* ctx, size_t bytes, void** out);

// a run hash (gc_runs.h RunTable) of at least 2^kRunLoadShift x rows entries, every entry empty on return
// (stream-ordered: a fill is enqueued on st when the table is new, grown or dirty)
int run_table(gc_ctx* ctx, hipStream_t st, RunTableBuf* T, int64_t rows);

// the table exp's 2048-entry table in device memory (gc_points.hip), enqueued once per context
hipError_t init_exp_table(hipStream_t st);

// Bounded host waits (fail fast). Poll the stream / event: ~spin_polls busy polls first (the wake-up
// latency of a blocking wait can exceed a 0.3 ms scan), then short sleeps, until the device work is
// done or ctx->wait_timeout_s runs out; the attached communicator's asynchronous error is polled on
// the way. On a timeout or an RCCL error the communicator is aborted (its kernels see the abort flag
// and exit) and GC_ERR_RUNTIME is returned with the reason in gc_last_error. ctx may be NULL (the
// environment's default bound, no communicator). waited_ms (optional) receives the time spent.
int wait_stream(gc_ctx* ctx, hipStream_t st, const char* what, double* waited_ms = nullptr, long spin_polls = 2000);
int wait_event(gc_ctx* ctx, hipEvent_t ev, const char* what, double* waited_ms = nullptr, long spin_polls = 2000);
// the default bound (GC_WAIT_TIMEOUT_S or 300 s)
double default_wait_timeout_s();
// RCCL hooks (gc_comm.cpp): the communicator's asynchronous error (false and why set if it failed),
// abort it (idempotent), and forget the context it was created on
bool comm_healthy(gc_comm* c, std::string* why);
void comm_abort(gc_comm* c);
void comm_detach_ctx(gc_comm* c);

// hipFuncSetAttribute(fn, MaxDynamicSharedMemorySize, bytes) only when fn has not yet been allowed that
// much: the runtime call is not free (it waited for an in-flight ingest copy on another stream,
// delaying the next launch by its duration), so the per-scan launches skip it after the first
hipError_t ensure_dyn_lds(const void* fn, size_t bytes);

// GC_OK when kernel fn has no static LDS (its dynamic block starts at LDS address 0, which the fused
// bins kernels' absolute table addressing relies on, gc_points.hip exp2s_shift8_n); checked once per
// kernel and device
int ensure_no_static_lds(gc_ctx* ctx, const void* fn);

}  // namespace gc

#define GC_CHECK_ARG(ctx, cond, msg)                   \
  do {                                                 \
    if (!(cond)) {                                     \
      gc::set_error((ctx), std::string("invalid argument: ") + (msg)); \
      return GC_ERR_ARG;                               \
    }                                                  \
  } while (0)

#define GC_HIP(ctx, expr)                                                              \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess) {                                                            \
      gc::set_error((ctx), std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + " (" #expr ")"); \
      return GC_ERR_RUNTIME;                                                           \
    }                                                                                  \
  } while (0)

#define GC_LAUNCH_CHECK(ctx) GC_HIP(ctx, hipGetLastError())
