// gc_comm.cpp — RCCL communicator for the per-scan hypothesis exchange (one process per GPU).
//
// The path has exactly one real exchange per scan: every rank's fixed-layout partial record
// (weighted information sums, IW statistics, hypothesis-0 map increments; ~17 KB) is
// all-gathered over xGMI and then reduced in rank order on every rank, so the combined belief,
// IW state and map are bit-identical across ranks (deterministic, unlike a ring all-reduce).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <cstring>
#include <string>
#include "gc_internal.h"

struct gc_comm {
  ncclComm_t comm = nullptr;
  int nranks = 1;
  int rank = 0;
  gc_ctx* ctx = nullptr;  // the context it was created on (its waits poll / abort this communicator)
  bool aborted = false;
};

namespace gc {

int comm_size(const gc_comm* c) { return c ? c->nranks : 1; }

bool comm_healthy(gc_comm* c, std::string* why) {
  if (!c) return true;
  if (c->aborted) {  // before the NULL-comm test: an abort clears c->comm
    if (why) *why = "the communicator was aborted by an earlier failure";
    return false;
  }
  if (!c->comm) return true;
  ncclResult_t a = ncclSuccess;
  const ncclResult_t r = ncclCommGetAsyncError(c->comm, &a);
  if (r != ncclSuccess) {
    if (why) *why = std::string("ncclCommGetAsyncError: ") + ncclGetErrorString(r);
    return false;
  }
  if (a != ncclSuccess && a != ncclInProgress) {
    if (why) *why = std::string("asynchronous error: ") + ncclGetErrorString(a);
    return false;
  }
  return true;
}

// ncclCommAbort: the communicator's kernels poll its abort flag and exit, so a stream stuck in an
// all-gather whose peer died drains; the communicator is unusable afterwards (every later exchange
// fails fast with the reason)
void comm_abort(gc_comm* c) {
  if (!c || !c->comm || c->aborted) return;
  c->aborted = true;
  (void)ncclCommAbort(c->comm);
  c->comm = nullptr;
}

void comm_detach_ctx(gc_comm* c) {
  if (c) c->ctx = nullptr;
}

int comm_allgather(gc_comm* c, gc_ctx* ctx, const double* d_send, double* d_recv, int64_t count) {
  std::string why;
  if (!comm_healthy(c, &why)) {  // a failure seen since the last scan: abort before enqueuing more
    comm_abort(c);
    set_error(ctx, "RCCL exchange refused: " + why);
    return GC_ERR_RUNTIME;
  }
  ncclResult_t r = ncclAllGather(d_send, d_recv, (size_t)count, ncclFloat64, c->comm, ctx->stream);
  if (r != ncclSuccess) {
    comm_abort(c);
    set_error(ctx, std::string("ncclAllGather: ") + ncclGetErrorString(r) + " (communicator aborted)");
    return GC_ERR_RUNTIME;
  }
  return GC_OK;
}

}  // namespace gc

extern "C" {

int32_t gc_comm_unique_id(uint8_t* out) {
  GC_CHECK_ARG(nullptr, out != nullptr, "out is NULL");
  static_assert(sizeof(ncclUniqueId) == GC_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    gc::set_error(nullptr, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    return GC_ERR_RUNTIME;
  }
  std::memcpy(out, &id, sizeof(id));
  return GC_OK;
}

int32_t gc_comm_init(gc_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t* id, gc_comm** out) {
  GC_CHECK_ARG(nullptr, ctx && id && out, "NULL argument");
  GC_CHECK_ARG(ctx, nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / nranks");
  GC_HIP(ctx, hipSetDevice(ctx->device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  gc_comm* c = new gc_comm();
  c->nranks = nranks;
  c->rank = rank;
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    gc::set_error(ctx, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    delete c;
    return GC_ERR_RUNTIME;
  }
  c->ctx = ctx;
  ctx->comm = c;  // the context's bounded waits poll and, on a failure, abort this communicator
  *out = c;
  return GC_OK;
}

int32_t gc_comm_destroy(gc_comm* c) {
  if (!c) return GC_OK;
  if (c->ctx && c->ctx->comm == c) c->ctx->comm = nullptr;
  if (c->comm) ncclCommDestroy(c->comm);
  delete c;
  return GC_OK;
}

int32_t gc_comm_abort(gc_comm* c) {
  GC_CHECK_ARG(nullptr, c != nullptr, "NULL communicator");
  gc::comm_abort(c);
  return GC_OK;
}

int32_t gc_comm_healthy(gc_comm* c, int32_t* ok) {
  GC_CHECK_ARG(nullptr, c && ok, "NULL argument");
  std::string why;
  *ok = gc::comm_healthy(c, &why) ? 1 : 0;
  if (!*ok) gc::set_error(c->ctx, why);
  return GC_OK;
}

int32_t gc_comm_allgather_f64(gc_ctx* ctx, gc_comm* c, const double* d_send, double* d_recv, int64_t count) {
  GC_CHECK_ARG(nullptr, ctx && c && d_send && d_recv, "NULL argument");
  GC_CHECK_ARG(ctx, c->comm || c->aborted, "communicator not initialised");
  GC_CHECK_ARG(ctx, count >= 0, "count must be >= 0");
  return gc::comm_allgather(c, ctx, d_send, d_recv, count);
}

}  // extern "C"
