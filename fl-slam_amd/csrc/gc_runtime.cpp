// gc_runtime.cpp — context, device buffers, events and error plumbing of libgcslam.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <mutex>
#include <map>
#include <thread>
#include "gc_internal.h"

struct gc_event {
  hipEvent_t ev = nullptr;
};

namespace {
thread_local std::string tl_error;
}

namespace gc {

void set_error(gc_ctx* ctx, const std::string& msg) {
  if (ctx) ctx->err = msg;
  tl_error = msg;
}

hipError_t ensure_dyn_lds(const void* fn, size_t bytes) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, size_t> allowed;  // per (device, kernel)
  int dev = 0;
  if (hipError_t e = hipGetDevice(&dev)) return e;
  std::lock_guard<std::mutex> lock(mu);
  size_t& a = allowed[{dev, fn}];
  if (bytes <= a) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess) a = bytes;
  return e;
}

int ensure_no_static_lds(gc_ctx* ctx, const void* fn) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, bool> checked;
  int dev = 0;
  GC_HIP(ctx, hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(mu);
  auto it = checked.find({dev, fn});
  if (it == checked.end()) {
    hipFuncAttributes a{};
    GC_HIP(ctx, hipFuncGetAttributes(&a, fn));
    it = checked.emplace(std::make_pair(dev, fn), a.sharedSizeBytes == 0).first;
  }
  if (!it->second) {
    set_error(ctx, "internal: a fused bins kernel has static LDS (its exp table is addressed from LDS 0)");
    return GC_ERR_RUNTIME;
  }
  return GC_OK;
}

int scratch(gc_ctx* ctx, size_t bytes, void** out) {
  if (bytes > ctx->scratch_bytes) {
    if (int rc = wait_stream(ctx, ctx->stream, "the stream before growing the scratch")) return rc;
    if (ctx->scratch) GC_HIP(ctx, hipFree(ctx->scratch));
    ctx->scratch = nullptr;
    ctx->scratch_bytes = 0;
    size_t sz = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 4;
    GC_HIP(ctx, hipMalloc(&ctx->scratch, sz));
    ctx->scratch_bytes = sz;
  }
  *out = ctx->scratch;
  return GC_OK;
}

double default_wait_timeout_s() {
  static const double v = [] {
    const char* e = std::getenv("GC_WAIT_TIMEOUT_S");
    const double x = e ? std::atof(e) : 0.0;
    return x > 0.0 ? x : 300.0;
  }();
  return v;
}

namespace {
// The poll loop behind wait_stream / wait_event: query() until hipSuccess, busy for spin_polls polls,
// then in 20 us sleeps; the deadline and the communicator's asynchronous error are checked every 64
// polls. Any other HIP status is returned as the error it is.
template <typename Query>
int bounded_poll(gc_ctx* ctx, const Query& query, const char* what, double* waited_ms, long spin_polls,
                 double limit_s) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  const auto done = [&](int rc) {
    if (waited_ms) *waited_ms = 1e-6 * (double)std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t0).count();
    return rc;
  };
  for (long i = 0;; ++i) {
    const hipError_t q = query();
    if (q == hipSuccess) return done(GC_OK);
    if (q != hipErrorNotReady) {
      set_error(ctx, std::string("HIP error ") + hipGetErrorString(q) + " while waiting for " + what);
      return done(GC_ERR_RUNTIME);
    }
    if ((i & 63) == 0) {
      std::string why;
      if (ctx && ctx->comm && !comm_healthy(ctx->comm, &why)) {
        comm_abort(ctx->comm);
        set_error(ctx, std::string("RCCL communicator failed while waiting for ") + what + ": " + why +
                           " (communicator aborted)");
        return done(GC_ERR_RUNTIME);
      }
      const double el = std::chrono::duration<double>(clk::now() - t0).count();
      if (el >= limit_s) {
        if (ctx && ctx->comm) comm_abort(ctx->comm);
        set_error(ctx, std::string("timed out after ") + std::to_string(el) + " s waiting for " + what +
                           (ctx && ctx->comm ? " (a peer rank may have failed; the RCCL communicator was aborted)"
                                             : " (device work did not complete)"));
        return done(GC_ERR_RUNTIME);
      }
    }
    if (i >= spin_polls) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}
}  // namespace

// gc_test_bounded_wait's entry into the poll loop (no HIP call: the query is the caller's)
template <typename Query>
int bounded_poll_for_test(gc_ctx* ctx, const Query& query, double* waited_ms) {
  return bounded_poll(ctx, query, "a test condition that never completes", waited_ms, 100, ctx->wait_timeout_s);
}

int wait_stream(gc_ctx* ctx, hipStream_t st, const char* what, double* waited_ms, long spin_polls) {
  const double lim = ctx ? ctx->wait_timeout_s : default_wait_timeout_s();
  return bounded_poll(ctx, [&] { return hipStreamQuery(st); }, what, waited_ms, spin_polls, lim);
}

int wait_event(gc_ctx* ctx, hipEvent_t ev, const char* what, double* waited_ms, long spin_polls) {
  const double lim = ctx ? ctx->wait_timeout_s : default_wait_timeout_s();
  return bounded_poll(ctx, [&] { return hipEventQuery(ev); }, what, waited_ms, spin_polls, lim);
}

int join_side(gc_ctx* ctx) {
  if (!ctx || !ctx->side_pending) return GC_OK;
  GC_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->side_ev, 0));
  ctx->side_pending = false;  // only once the wait is enqueued (a failed wait leaves it to the next join)
  return GC_OK;
}

int run_table(gc_ctx* ctx, hipStream_t st, RunTableBuf* T, int64_t rows) {
  uint32_t bits = 8;  // >= 2^kRunLoadShift x rows entries (gc_runs.h); the links: rows <= 2^(bits - shift)
  while (bits < 31 && ((int64_t)1 << bits) < (rows << kRunLoadShift)) ++bits;
  const size_t bytes = ((size_t)8 << bits) + ((size_t)4 << (bits - kRunLoadShift));  // entries + links of 4 B
  if (bits > T->bits) {
    if (int rc = wait_stream(ctx, st, "the stream before growing a run table")) return rc;
    if (T->ptr) GC_HIP(ctx, hipFree(T->ptr));
    T->ptr = nullptr;
    T->bits = 0;
    GC_HIP(ctx, hipMalloc(&T->ptr, bytes));
    T->bits = bits;
    T->dirty = true;
  }
  if (T->dirty) {  // zero: every entry empty, every link none
    GC_HIP(ctx, hipMemsetAsync(T->ptr, 0, ((size_t)8 << T->bits) + ((size_t)4 << (T->bits - kRunLoadShift)), st));
    T->dirty = false;
  }
  return GC_OK;
}

}  // namespace gc

extern "C" {

int32_t gc_version(void) { return 10000; /* 1.0.0 */ }

const char* gc_last_error(const gc_ctx* ctx) {
  if (ctx && !ctx->err.empty()) return ctx->err.c_str();
  return tl_error.c_str();
}

int32_t gc_device_count(int32_t* count) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    gc::set_error(nullptr, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    *count = 0;
    return GC_ERR_RUNTIME;
  }
  *count = n;
  return GC_OK;
}

int32_t gc_ctx_create(int32_t device, gc_ctx** out) {
  GC_CHECK_ARG(nullptr, out != nullptr, "out is NULL");
  int n = 0;
  GC_HIP(nullptr, hipGetDeviceCount(&n));
  GC_CHECK_ARG(nullptr, device >= 0 && device < n, "device index out of range");
  GC_HIP(nullptr, hipSetDevice(device));
  gc_ctx* c = new gc_ctx();
  c->device = device;
  c->wait_timeout_s = gc::default_wait_timeout_s();
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    gc::set_error(nullptr, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    delete c;
    return GC_ERR_RUNTIME;
  }
  e = gc::init_exp_table(c->stream);
  if (e != hipSuccess) {
    gc::set_error(nullptr, std::string("exp table: ") + hipGetErrorString(e));
    (void)hipStreamDestroy(c->stream);
    delete c;
    return GC_ERR_RUNTIME;
  }
  *out = c;
  return GC_OK;
}

int32_t gc_ctx_destroy(gc_ctx* ctx) {
  if (!ctx) return GC_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->comm) gc::comm_detach_ctx(ctx->comm);
  (void)gc::join_side(ctx);
  // bounded: a context whose stream is stuck (a failed peer) is still torn down
  (void)gc::wait_stream(ctx, ctx->stream, "the stream at context destruction");
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->runs.ptr) (void)hipFree(ctx->runs.ptr);
  for (auto& kv : ctx->arena_free) (void)hipFree(kv.second);
  for (auto& kv : ctx->arena_live) (void)hipFree(kv.first);  // buffers not freed before the context
  if (ctx->stage_host) {
    for (hipEvent_t e : ctx->stage_ev)
      if (e) (void)hipEventDestroy(e);
    (void)hipHostFree(ctx->stage_host);
  }
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return GC_OK;
}

int32_t gc_ctx_synchronize(gc_ctx* ctx) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  if (int rc_j = gc::join_side(ctx)) return rc_j;
  GC_HIP(ctx, hipSetDevice(ctx->device));
  return gc::wait_stream(ctx, ctx->stream, "the context's stream (gc_ctx_synchronize)");
}

int32_t gc_ctx_set_wait_timeout(gc_ctx* ctx, double seconds) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  GC_CHECK_ARG(ctx, seconds > 0.0, "the wait timeout must be positive");
  ctx->wait_timeout_s = seconds;
  return GC_OK;
}

int32_t gc_test_bounded_wait(double timeout_s, int64_t ready_after_polls, double* h_waited_ms) {
  GC_CHECK_ARG(nullptr, timeout_s > 0.0 && h_waited_ms, "bad arguments");
  int64_t polls = 0;
  gc_ctx tmp;  // no device, no stream, no communicator: only the timeout bound
  tmp.wait_timeout_s = timeout_s;
  const int rc = gc::bounded_poll_for_test(&tmp, [&] {
    return (ready_after_polls >= 0 && ++polls > ready_after_polls) ? hipSuccess : hipErrorNotReady;
  }, h_waited_ms);
  if (rc != GC_OK) gc::set_error(nullptr, tmp.err);
  return rc;
}

// size class of an arena block: 256-B granules up to 4 KiB, then quarter steps of the power of two
// below (<= 25 % slack), so buffers of one shape always share a class
static size_t arena_class(uint64_t bytes) {
  size_t b = bytes ? (size_t)bytes : 16;
  if (b <= 4096) return (b + 255) & ~(size_t)255;
  size_t p = (size_t)1 << (63 - __builtin_clzll((unsigned long long)b));
  const size_t step = p >> 2;
  return (b + step - 1) / step * step;
}

int32_t gc_buffer_alloc(gc_ctx* ctx, uint64_t bytes, void** d_ptr) {
  GC_CHECK_ARG(nullptr, ctx && d_ptr, "NULL argument");
  const size_t c = arena_class(bytes);
  {
    std::lock_guard<std::mutex> lock(ctx->arena_mu);
    auto it = ctx->arena_free.find(c);
    if (it != ctx->arena_free.end()) {
      *d_ptr = it->second;
      ctx->arena_free.erase(it);
      ctx->arena_cached -= c;
      ctx->arena_live[*d_ptr] = c;
      ctx->arena_live_bytes += c;
      ctx->arena_reuses += 1;
      return GC_OK;
    }
  }
  GC_HIP(ctx, hipSetDevice(ctx->device));
  GC_HIP(ctx, hipMalloc(d_ptr, c));
  std::lock_guard<std::mutex> lock(ctx->arena_mu);
  ctx->arena_live[*d_ptr] = c;
  ctx->arena_live_bytes += c;
  ctx->arena_hip_allocs += 1;
  return GC_OK;
}

int32_t gc_buffer_free(gc_ctx* ctx, void* d_ptr) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  if (int rc_j = gc::join_side(ctx)) return rc_j;
  if (!d_ptr) return GC_OK;
  size_t c = 0;
  {
    std::lock_guard<std::mutex> lock(ctx->arena_mu);
    auto it = ctx->arena_live.find(d_ptr);
    GC_CHECK_ARG(ctx, it != ctx->arena_live.end(), "not a live buffer of this context (gc_buffer_alloc)");
    c = it->second;
    ctx->arena_live.erase(it);
    ctx->arena_live_bytes -= c;
    if (ctx->arena_cached + c <= ctx->arena_cap) {  // cached for the next allocation of its class
      ctx->arena_free.emplace(c, d_ptr);
      ctx->arena_cached += c;
      return GC_OK;
    }
  }
  // over the cap: returned to HIP after the stream's queued work (which may still read it)
  GC_HIP(ctx, hipSetDevice(ctx->device));
  if (int rc = gc::wait_stream(ctx, ctx->stream, "the stream before a buffer free")) return rc;
  GC_HIP(ctx, hipFree(d_ptr));
  std::lock_guard<std::mutex> lock(ctx->arena_mu);
  ctx->arena_hip_frees += 1;
  return GC_OK;
}

int32_t gc_ctx_trim(gc_ctx* ctx) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  if (int rc_j = gc::join_side(ctx)) return rc_j;
  GC_HIP(ctx, hipSetDevice(ctx->device));
  if (int rc = gc::wait_stream(ctx, ctx->stream, "the stream before an arena trim")) return rc;
  std::lock_guard<std::mutex> lock(ctx->arena_mu);
  for (auto& kv : ctx->arena_free) {
    GC_HIP(ctx, hipFree(kv.second));
    ctx->arena_hip_frees += 1;
  }
  ctx->arena_free.clear();
  ctx->arena_cached = 0;
  return GC_OK;
}

int32_t gc_ctx_alloc_stats(gc_ctx* ctx, int64_t* h_out6) {
  GC_CHECK_ARG(nullptr, ctx && h_out6, "NULL argument");
  std::lock_guard<std::mutex> lock(ctx->arena_mu);
  h_out6[0] = ctx->arena_hip_allocs;
  h_out6[1] = ctx->arena_hip_frees;
  h_out6[2] = ctx->arena_reuses;
  h_out6[3] = (int64_t)ctx->arena_live.size();
  h_out6[4] = (int64_t)ctx->arena_live_bytes;
  h_out6[5] = (int64_t)ctx->arena_cached;
  return GC_OK;
}

namespace {
// a pinned staging slot of `bytes` (<= kStageSeg) in ctx's ring (gc_ctx::stage_host)
int stage_slot(gc_ctx* ctx, uint64_t bytes, char** out) {
  if (!ctx->stage_host) {
    void* h = nullptr;
    GC_HIP(ctx, hipHostMalloc(&h, gc_ctx::kStageSegs * gc_ctx::kStageSeg, hipHostMallocDefault));
    for (hipEvent_t& e : ctx->stage_ev) {
      const hipError_t er = hipEventCreateWithFlags(&e, hipEventDisableTiming);
      if (er != hipSuccess) {
        for (hipEvent_t& d : ctx->stage_ev)  // the ones created so far (the ring stays unset: a retry starts over)
          if (d) {
            (void)hipEventDestroy(d);
            d = nullptr;
          }
        (void)hipHostFree(h);
        gc::set_error(ctx, std::string("HIP error ") + hipGetErrorString(er) + " creating the staging events");
        return GC_ERR_RUNTIME;
      }
    }
    ctx->stage_host = (char*)h;
    ctx->stage_seg = 0;
    ctx->stage_off = 0;
  }
  const size_t need = (bytes + 255) & ~(size_t)255;
  if (ctx->stage_off + need > gc_ctx::kStageSeg) {
    // leave the segment: its copies are done once this event has completed
    const int s = ctx->stage_seg;
    GC_HIP(ctx, hipEventRecord(ctx->stage_ev[s], ctx->stream));
    ctx->stage_rec[s] = true;
    const int nx = (s + 1) % gc_ctx::kStageSegs;
    if (ctx->stage_rec[nx]) {  // recorded kStageSegs - 1 segments ago: normally long complete
      if (int rc = gc::wait_event(ctx, ctx->stage_ev[nx], "a staging segment's uploads")) return rc;
      ctx->stage_rec[nx] = false;
    }
    ctx->stage_seg = nx;
    ctx->stage_off = 0;
  }
  *out = ctx->stage_host + (size_t)ctx->stage_seg * gc_ctx::kStageSeg + ctx->stage_off;
  ctx->stage_off += need;
  return GC_OK;
}
}  // namespace

int32_t gc_buffer_upload(gc_ctx* ctx, void* d_dst, const void* h_src, uint64_t bytes) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  if (int rc_j = gc::join_side(ctx)) return rc_j;
  if (bytes == 0) return GC_OK;
  if (bytes <= gc_ctx::kStageSeg) {  // staged: no wait (the pinned copy is the caller's buffer's)
    char* h = nullptr;
    if (int rc = stage_slot(ctx, bytes, &h)) return rc;
    std::memcpy(h, h_src, bytes);
    GC_HIP(ctx, hipMemcpyAsync(d_dst, h, bytes, hipMemcpyHostToDevice, ctx->stream));
    ++ctx->stage_uploads;
    return GC_OK;
  }
  GC_HIP(ctx, hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, ctx->stream));
  return gc::wait_stream(ctx, ctx->stream, "an upload");
}

int32_t gc_buffer_download(gc_ctx* ctx, void* h_dst, const void* d_src, uint64_t bytes) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  if (int rc_j = gc::join_side(ctx)) return rc_j;
  if (bytes == 0) return GC_OK;
  GC_HIP(ctx, hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  return gc::wait_stream(ctx, ctx->stream, "a download");
}

int32_t gc_buffer_copy(gc_ctx* ctx, void* d_dst, const void* d_src, uint64_t bytes) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  if (int rc_j = gc::join_side(ctx)) return rc_j;
  if (bytes == 0) return GC_OK;
  GC_HIP(ctx, hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  return GC_OK;
}

int32_t gc_buffer_memset(gc_ctx* ctx, void* d_dst, int32_t value, uint64_t bytes) {
  GC_CHECK_ARG(nullptr, ctx != nullptr, "ctx is NULL");
  if (int rc_j = gc::join_side(ctx)) return rc_j;
  if (bytes == 0) return GC_OK;
  GC_HIP(ctx, hipMemsetAsync(d_dst, value, bytes, ctx->stream));
  return GC_OK;
}

int32_t gc_event_create(gc_ctx* ctx, gc_event** out) {
  GC_CHECK_ARG(nullptr, ctx && out, "NULL argument");
  gc_event* e = new gc_event();
  hipError_t r = hipEventCreate(&e->ev);
  if (r != hipSuccess) {
    delete e;
    gc::set_error(ctx, std::string("hipEventCreate: ") + hipGetErrorString(r));
    return GC_ERR_RUNTIME;
  }
  *out = e;
  return GC_OK;
}

int32_t gc_event_destroy(gc_event* ev) {
  if (!ev) return GC_OK;
  (void)hipEventDestroy(ev->ev);
  delete ev;
  return GC_OK;
}

int32_t gc_event_record(gc_ctx* ctx, gc_event* ev) {
  GC_CHECK_ARG(nullptr, ctx && ev, "NULL argument");
  if (int rc_j = gc::join_side(ctx)) return rc_j;
  GC_HIP(ctx, hipEventRecord(ev->ev, ctx->stream));
  return GC_OK;
}

int32_t gc_event_elapsed_ms(gc_event* start, gc_event* stop, float* ms) {
  GC_CHECK_ARG(nullptr, start && stop && ms, "NULL argument");
  if (int rc = gc::wait_event(nullptr, stop->ev, "a timing event")) return rc;
  GC_HIP(nullptr, hipEventElapsedTime(ms, start->ev, stop->ev));
  return GC_OK;
}

}  // extern "C"
