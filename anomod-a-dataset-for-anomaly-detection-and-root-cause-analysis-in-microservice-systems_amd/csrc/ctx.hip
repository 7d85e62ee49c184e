// Context, error, timing and RCCL plumbing of libanomod.
//
// The reference has no comm backend at all (SURVEY.md §5 "Distributed comm
// backend: None"; its only concurrency is the HTTP ThreadPoolExecutor of
// trace_collector.py:519-531).  Here one process drives one GPU and the
// integer edge tables of all ranks are summed with RCCL over xGMI.
#include <chrono>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "common.h"

namespace {
thread_local std::string g_thread_err;
}

namespace anomod {

void set_error(anomod_ctx* ctx, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  g_thread_err = buf;
}

int bind(anomod_ctx* ctx) {
  ANOMOD_HIP(ctx, hipSetDevice(ctx->device));
  return ANOMOD_OK;
}

int stage_begin(anomod_ctx* ctx, Stage s) {
  ANOMOD_HIP(ctx, hipEventRecord(ctx->ev_begin[s], ctx->stream));
  return ANOMOD_OK;
}

int stage_end(anomod_ctx* ctx, Stage s) {
  ANOMOD_HIP(ctx, hipEventRecord(ctx->ev_end[s], ctx->stream));
  ctx->stage_recorded[s] = true;
  return ANOMOD_OK;
}

double host_now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

void host_record(anomod_ctx* ctx, HostSlot s, double ms) {
  ctx->host_ms[s] = ms;
  ++ctx->host_count[s];
}

namespace {
void abort_comm(anomod_ctx* ctx) {
  if (ctx->comm && !ctx->comm_aborted) {
    ncclCommAbort(ctx->comm);
    ctx->comm = nullptr;  // an aborted communicator is not destroyed again
    ctx->comm_aborted = true;
  }
}
}  // namespace

int stream_wait(anomod_ctx* ctx) {
  if (!ctx->comm) {
    ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return ANOMOD_OK;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t spin = 0;; ++spin) {
    const hipError_t q = hipStreamQuery(ctx->stream);
    if (q == hipSuccess) return ANOMOD_OK;
    if (q != hipErrorNotReady) {
      set_error(ctx, "stream failed while waiting on a collective: %s", hipGetErrorString(q));
      abort_comm(ctx);
      return ANOMOD_EHIP;
    }
    ncclResult_t ar = ncclSuccess;
    const ncclResult_t qr = ncclCommGetAsyncError(ctx->comm, &ar);
    if (qr != ncclSuccess || (ar != ncclSuccess && ar != ncclInProgress)) {
      set_error(ctx, "RCCL async error on rank %d of %d: %s; communicator aborted", ctx->rank,
                ctx->nranks, ncclGetErrorString(qr != ncclSuccess ? qr : ar));
      abort_comm(ctx);
      return ANOMOD_ERCCL;
    }
    const double el =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > ctx->comm_timeout_s) {
      set_error(ctx, "collective on rank %d of %d did not finish within %.0f s "
                "(ANOMOD_RCCL_TIMEOUT_S): a peer is gone or stuck; communicator aborted",
                ctx->rank, ctx->nranks, ctx->comm_timeout_s);
      abort_comm(ctx);
      return ANOMOD_ERCCL;
    }
    if (spin > 2000) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

bool comm_attached(const anomod_ctx* ctx) {
  return ctx->comm != nullptr || ctx->host_allreduce != nullptr;
}

int coll_begin(anomod_ctx* ctx) {
  if (ctx->comm) ANOMOD_RCCL(ctx, ncclGroupStart());
  return ANOMOD_OK;
}

int coll_end(anomod_ctx* ctx) {
  if (ctx->comm) ANOMOD_RCCL(ctx, ncclGroupEnd());
  return ANOMOD_OK;
}

namespace {
size_t coll_size(CollType t) { return (t == kCollU64 || t == kCollF64) ? 8 : 4; }
ncclDataType_t nccl_type(CollType t) {
  switch (t) {
    case kCollI32: return ncclInt32;
    case kCollU32: return ncclUint32;
    case kCollU64: return ncclUint64;
    default: return ncclFloat64;
  }
}
ncclRedOp_t nccl_op(CollOp op) { return op == kCollSum ? ncclSum : op == kCollMin ? ncclMin : ncclMax; }

int ensure_coll_stage(anomod_ctx* ctx, size_t bytes) {
  if (ctx->coll_bytes >= bytes) return ANOMOD_OK;
  if (ctx->h_coll) ANOMOD_HIP(ctx, hipHostFree(ctx->h_coll));
  ctx->h_coll = nullptr;
  ctx->coll_bytes = 0;
  ANOMOD_HIP(ctx, hipHostMalloc(&ctx->h_coll, bytes, hipHostMallocDefault));
  ctx->coll_bytes = bytes;
  return ANOMOD_OK;
}

// A host-transport call failed: the transport is dropped like an aborted
// communicator (later calls fail fast instead of entering a collective
// their peers may never join).
int host_coll_failed(anomod_ctx* ctx, const char* what, int rc) {
  set_error(ctx, "host collective %s failed on rank %d of %d (callback returned %d); "
            "transport detached", what, ctx->rank, ctx->nranks, rc);
  ctx->host_allreduce = nullptr;
  ctx->host_allgather = nullptr;
  ctx->comm_aborted = true;
  return ANOMOD_ERCCL;
}
}  // namespace

int coll_allreduce(anomod_ctx* ctx, void* dbuf, size_t count, CollType t, CollOp op) {
  if (ctx->comm) {
    ANOMOD_RCCL(ctx, ncclAllReduce(dbuf, dbuf, count, nccl_type(t), nccl_op(op), ctx->comm,
                                   ctx->stream));
    return ANOMOD_OK;
  }
  const size_t bytes = count * coll_size(t);
  if (int rc = ensure_coll_stage(ctx, bytes)) return rc;
  ANOMOD_HIP(ctx, hipMemcpyAsync(ctx->h_coll, dbuf, bytes, hipMemcpyDeviceToHost, ctx->stream));
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (int rc = ctx->host_allreduce(ctx->host_user, ctx->h_coll, count, (int)t, (int)op))
    return host_coll_failed(ctx, "all-reduce", rc);
  ANOMOD_HIP(ctx, hipMemcpyAsync(dbuf, ctx->h_coll, bytes, hipMemcpyHostToDevice, ctx->stream));
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));  // the staging is reused
  return ANOMOD_OK;
}

int coll_allgather(anomod_ctx* ctx, void* dbuf, size_t count_per_rank, CollType t) {
  const size_t blk = count_per_rank * coll_size(t);
  char* d = static_cast<char*>(dbuf);
  if (ctx->comm) {
    ANOMOD_RCCL(ctx, ncclAllGather(d + (size_t)ctx->rank * blk, d, count_per_rank, nccl_type(t),
                                   ctx->comm, ctx->stream));
    return ANOMOD_OK;
  }
  const size_t bytes = blk * (size_t)ctx->nranks;
  if (int rc = ensure_coll_stage(ctx, bytes)) return rc;
  char* h = static_cast<char*>(ctx->h_coll);
  ANOMOD_HIP(ctx, hipMemcpyAsync(h + (size_t)ctx->rank * blk, d + (size_t)ctx->rank * blk, blk,
                                 hipMemcpyDeviceToHost, ctx->stream));
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (int rc = ctx->host_allgather(ctx->host_user, h, blk))
    return host_coll_failed(ctx, "all-gather", rc);
  ANOMOD_HIP(ctx, hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, ctx->stream));
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ANOMOD_OK;
}

int comm_agree(anomod_ctx* ctx, int local_rc) {
  if (!comm_attached(ctx)) {
    if (ctx->comm_aborted && local_rc == ANOMOD_OK) {
      set_error(ctx, "the communicator of this context was aborted after an earlier failure");
      return ANOMOD_ERCCL;
    }
    return local_rc;
  }
  const std::string local_msg = ctx->err;
  *ctx->h_status = local_rc;
  ANOMOD_HIP(ctx, hipMemcpyAsync(ctx->d_status, ctx->h_status, sizeof(int),
                                 hipMemcpyHostToDevice, ctx->stream));
  // statuses are <= 0: the minimum is an error whenever any rank has one
  if (int rc = coll_allreduce(ctx, ctx->d_status, 1, kCollI32, kCollMin)) return rc;
  ANOMOD_HIP(ctx, hipMemcpyAsync(ctx->h_status, ctx->d_status, sizeof(int),
                                 hipMemcpyDeviceToHost, ctx->stream));
  if (int rc = stream_wait(ctx)) return rc;
  const int agreed = *ctx->h_status;
  if (local_rc != ANOMOD_OK) {
    ctx->err = local_msg;  // this rank's own reason
    return local_rc;
  }
  if (agreed != ANOMOD_OK) {
    set_error(ctx, "another rank failed before the collective (status %d); "
              "this rank skipped it too", agreed);
    return agreed;
  }
  return ANOMOD_OK;
}

uint64_t max_launch_spans() {  // read per call: tests lower it at run time
  // A workgroup's LDS counters are u32, so a launch covers < 2^32 spans (the
  // dynamic tail may hand one workgroup any share of it).  r03: up from 2^31,
  // so a 2^27-trace TrainTicket set (3.1e9 spans) is one launch, not two.
  constexpr uint64_t kMax = (1ull << 32) - 1;
  const char* e = getenv("ANOMOD_MAX_LAUNCH_SPANS");
  const unsigned long long x = e ? strtoull(e, nullptr, 10) : 0ull;
  return x > 0 && x < kMax ? (uint64_t)x : kMax;
}

int span_launch_cuts(anomod_ctx* ctx, const anomod_spans* s, uint64_t max_spans,
                     std::vector<uint64_t>& cuts) {
  cuts.assign(1, 0);
  if (s->n_spans <= max_spans) {
    cuts.push_back(s->n_traces);
    return ANOMOD_OK;
  }
  // Binary searches over the device trace_ptr, one u64 read back per probe
  // (only sets of >= 2^32 - 1 spans get here).
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  auto at = [&](uint64_t t, uint64_t* v) -> int {
    ANOMOD_HIP(ctx, hipMemcpy(v, s->trace_ptr + t, 8, hipMemcpyDeviceToHost));
    return ANOMOD_OK;
  };
  uint64_t cur = 0, pcur = 0;
  while (cur < s->n_traces) {
    uint64_t lo = cur + 1, hi = s->n_traces;  // largest t in [lo, hi] with ptr[t] - pcur <= max
    uint64_t v = 0;
    if (int rc = at(lo, &v)) return rc;
    if (v - pcur > max_spans) {  // one trace alone exceeds the bound
      ANOMOD_REQUIRE(ctx, v - pcur < (1ull << 32), "trace %llu holds %llu >= 2^32 spans",
                     (unsigned long long)cur, (unsigned long long)(v - pcur));
      hi = lo;
    } else {
      while (lo < hi) {
        const uint64_t mid = lo + (hi - lo + 1) / 2;
        if (int rc = at(mid, &v)) return rc;
        if (v - pcur <= max_spans) lo = mid; else hi = mid - 1;
      }
    }
    cuts.push_back(hi);
    if (int rc = at(hi, &pcur)) return rc;
    cur = hi;
  }
  return ANOMOD_OK;
}

int ensure_table(anomod_ctx* ctx, size_t bytes) {
  if (ctx->table_bytes >= bytes) return ANOMOD_OK;
  if (ctx->d_table) {
    ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
    ANOMOD_HIP(ctx, hipFree(ctx->d_table));
    ctx->d_table = nullptr;
    ctx->table_bytes = 0;
  }
  if (hipMalloc(&ctx->d_table, bytes) != hipSuccess) {
    set_error(ctx, "hipMalloc(%zu) for the edge table failed", bytes);
    ctx->d_table = nullptr;
    return ANOMOD_ENOMEM;
  }
  ctx->table_bytes = bytes;
  return ANOMOD_OK;
}

size_t release_scratch(anomod_ctx* ctx, unsigned keep) {
  size_t freed = 0;
  for (int i = 0; i < kNumScratch; ++i) {
    if (((keep >> i) & 1u) || !ctx->scratch[i]) continue;
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->scratch[i]);
    freed += ctx->scratch_bytes[i];
    ctx->scratch[i] = nullptr;
    ctx->scratch_bytes[i] = 0;
  }
  return freed;
}

hipError_t dev_malloc(anomod_ctx* ctx, void** p, size_t bytes) {
  hipError_t e = hipMalloc(p, bytes);
  if (e == hipSuccess) return e;
  (void)hipGetLastError();  // clear the sticky-free error state of the failed call
  if (!release_scratch(ctx)) return e;
  return hipMalloc(p, bytes);
}

int ensure_scratch(anomod_ctx* ctx, ScratchSlot slot, size_t bytes, void** out, unsigned keep) {
  *out = nullptr;
  if (ctx->scratch[slot] && ctx->scratch_bytes[slot] >= bytes) {
    *out = ctx->scratch[slot];
    return ANOMOD_OK;
  }
  if (ctx->scratch[slot]) {
    ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
    ANOMOD_HIP(ctx, hipFree(ctx->scratch[slot]));
    ctx->scratch[slot] = nullptr;
    ctx->scratch_bytes[slot] = 0;
  }
  const size_t want = bytes ? bytes : 256;
  void* p = nullptr;
  if (hipMalloc(&p, want) != hipSuccess) {
    (void)hipGetLastError();
    if (!release_scratch(ctx, keep | (1u << slot)) || hipMalloc(&p, want) != hipSuccess) {
      set_error(ctx, "hipMalloc(%zu) for a scratch workspace failed", want);
      return ANOMOD_ENOMEM;
    }
  }
  ctx->scratch[slot] = p;
  ctx->scratch_bytes[slot] = want;
  *out = p;
  return ANOMOD_OK;
}

int ensure_host_stage(anomod_ctx* ctx, size_t bytes) {
  if (ctx->stage_bytes >= bytes) return ANOMOD_OK;
  if (ctx->h_stage) {
    ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
    ANOMOD_HIP(ctx, hipHostFree(ctx->h_stage));
    ctx->h_stage = nullptr;
    ctx->stage_bytes = 0;
  }
  if (hipHostMalloc(&ctx->h_stage, bytes, hipHostMallocDefault) != hipSuccess) {
    set_error(ctx, "hipHostMalloc(%zu) for the edge-table staging failed", bytes);
    ctx->h_stage = nullptr;
    return ANOMOD_ENOMEM;
  }
  ctx->stage_bytes = bytes;
  return ANOMOD_OK;
}

}  // namespace anomod

extern "C" {

int anomod_abi_version(void) { return ANOMOD_ABI_VERSION; }

const char* anomod_last_error(const anomod_ctx* ctx) {
  if (ctx && !ctx->err.empty()) return ctx->err.c_str();
  return g_thread_err.c_str();
}

int anomod_device_count(int* out) {
  ANOMOD_REQUIRE(nullptr, out != nullptr, "anomod_device_count: out is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *out = 0;
    anomod::set_error(nullptr, "hipGetDeviceCount failed: %s", hipGetErrorString(e));
    return ANOMOD_EHIP;
  }
  *out = n;
  return ANOMOD_OK;
}

int anomod_ctx_create(int device, anomod_ctx** out) {
  ANOMOD_REQUIRE(nullptr, out != nullptr, "anomod_ctx_create: out is NULL");
  *out = nullptr;
  int n = 0;
  ANOMOD_HIP(nullptr, hipGetDeviceCount(&n));
  ANOMOD_REQUIRE(nullptr, device >= 0 && device < n,
                 "anomod_ctx_create: device %d out of range (%d devices)", device, n);
  ANOMOD_HIP(nullptr, hipSetDevice(device));
  hipDeviceProp_t prop;
  ANOMOD_HIP(nullptr, hipGetDeviceProperties(&prop, device));
  auto* ctx = new anomod_ctx();
  ctx->device = device;
  ctx->num_cus = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    anomod::set_error(nullptr, "hipStreamCreate failed");
    return ANOMOD_EHIP;
  }
  for (int s = 0; s < anomod::kNumStages; ++s) {
    if (hipEventCreate(&ctx->ev_begin[s]) != hipSuccess ||
        hipEventCreate(&ctx->ev_end[s]) != hipSuccess) {
      anomod_ctx_destroy(ctx);
      anomod::set_error(nullptr, "hipEventCreate failed");
      return ANOMOD_EHIP;
    }
  }
  *out = ctx;
  return ANOMOD_OK;
}

int anomod_ctx_destroy(anomod_ctx* ctx) {
  if (!ctx) return ANOMOD_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  anomod::free_group_ws(ctx);
  anomod::free_uploader(ctx);
  if (ctx->host_set) anomod::free_spans(ctx->host_set);
  if (ctx->d_status) (void)hipFree(ctx->d_status);
  if (ctx->h_status) (void)hipHostFree(ctx->h_status);
  if (ctx->d_table) (void)hipFree(ctx->d_table);
  anomod::release_scratch(ctx);
  if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
  if (ctx->h_coll) (void)hipHostFree(ctx->h_coll);
  for (int s = 0; s < anomod::kNumStages; ++s) {
    if (ctx->ev_begin[s]) (void)hipEventDestroy(ctx->ev_begin[s]);
    if (ctx->ev_end[s]) (void)hipEventDestroy(ctx->ev_end[s]);
  }
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return ANOMOD_OK;
}

int anomod_ctx_synchronize(anomod_ctx* ctx) {
  ANOMOD_REQUIRE(nullptr, ctx != nullptr, "anomod_ctx_synchronize: ctx is NULL");
  if (int rc = anomod::bind(ctx)) return rc;
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ANOMOD_OK;
}

int anomod_ctx_stage_ms(const anomod_ctx* cctx, int stage, double* ms) {
  auto* ctx = const_cast<anomod_ctx*>(cctx);
  ANOMOD_REQUIRE(nullptr, ctx != nullptr && ms != nullptr, "anomod_ctx_stage_ms: NULL argument");
  ANOMOD_REQUIRE(ctx, stage >= 0 && stage < anomod::kNumStages, "unknown stage %d", stage);
  if (!ctx->stage_recorded[stage]) {
    *ms = -1.0;
    return ANOMOD_OK;
  }
  if (int rc = anomod::bind(ctx)) return rc;
  ANOMOD_HIP(ctx, hipEventSynchronize(ctx->ev_end[stage]));
  float f = 0.f;
  ANOMOD_HIP(ctx, hipEventElapsedTime(&f, ctx->ev_begin[stage], ctx->ev_end[stage]));
  *ms = (double)f;
  return ANOMOD_OK;
}

int anomod_ctx_host_ms(const anomod_ctx* ctx, int slot, double* ms, uint64_t* count) {
  ANOMOD_REQUIRE(nullptr, ctx != nullptr && ms != nullptr, "anomod_ctx_host_ms: NULL argument");
  ANOMOD_REQUIRE(nullptr, slot >= 0 && slot < anomod::kNumHostSlots, "unknown host slot %d", slot);
  *ms = ctx->host_ms[slot];
  if (count) *count = ctx->host_count[slot];
  return ANOMOD_OK;
}

uint32_t anomod_hist_bin(uint32_t v) { return anomod::hist_bin(v); }

int anomod_hist_bin_bounds(uint32_t bin, uint32_t* lo, uint32_t* hi) {
  ANOMOD_REQUIRE(nullptr, lo && hi, "anomod_hist_bin_bounds: NULL output");
  ANOMOD_REQUIRE(nullptr, bin < ANOMOD_HIST_BINS, "bin %u out of range", bin);
  anomod::hist_bounds(bin, lo, hi);
  return ANOMOD_OK;
}

int anomod_comm_unique_id(uint8_t* out) {
  ANOMOD_REQUIRE(nullptr, out != nullptr, "anomod_comm_unique_id: out is NULL");
  static_assert(sizeof(ncclUniqueId) == ANOMOD_UNIQUE_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  ANOMOD_RCCL(nullptr, ncclGetUniqueId(&id));
  memcpy(out, &id, sizeof(id));
  return ANOMOD_OK;
}

int anomod_ctx_attach_comm(anomod_ctx* ctx, const uint8_t* unique_id, int nranks, int rank) {
  ANOMOD_REQUIRE(nullptr, ctx && unique_id, "anomod_ctx_attach_comm: NULL argument");
  ANOMOD_REQUIRE(ctx, nranks >= 1 && rank >= 0 && rank < nranks, "bad rank %d of %d", rank,
                 nranks);
  ANOMOD_REQUIRE(ctx, !anomod::comm_attached(ctx) && !ctx->comm_aborted,
                 "ctx already has (or had) a communicator");
  if (int rc = anomod::bind(ctx)) return rc;
  if (!ctx->d_status) ANOMOD_HIP(ctx, hipMalloc(&ctx->d_status, sizeof(int)));
  if (!ctx->h_status)
    ANOMOD_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->h_status), sizeof(int),
                                  hipHostMallocDefault));
  if (const char* t = getenv("ANOMOD_RCCL_TIMEOUT_S")) {
    const double v = atof(t);
    if (v > 0) ctx->comm_timeout_s = v;
  }
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  // into a local: a refused init (e.g. two ranks on one device) leaves the
  // ctx without a communicator, so the caller may attach the host transport
  ncclComm_t comm = nullptr;
  ANOMOD_RCCL(ctx, ncclCommInitRank(&comm, nranks, id, rank));
  ctx->comm = comm;
  ctx->nranks = nranks;
  ctx->rank = rank;
  return ANOMOD_OK;
}

int anomod_ctx_attach_host_comm(anomod_ctx* ctx, int nranks, int rank,
                                anomod_host_allreduce_fn allreduce,
                                anomod_host_allgather_fn allgather, void* user) {
  ANOMOD_REQUIRE(nullptr, ctx && allreduce && allgather,
                 "anomod_ctx_attach_host_comm: NULL argument");
  ANOMOD_REQUIRE(ctx, nranks >= 1 && rank >= 0 && rank < nranks, "bad rank %d of %d", rank,
                 nranks);
  ANOMOD_REQUIRE(ctx, !anomod::comm_attached(ctx) && !ctx->comm_aborted,
                 "ctx already has (or had) a communicator");
  if (int rc = anomod::bind(ctx)) return rc;
  if (!ctx->d_status) ANOMOD_HIP(ctx, hipMalloc(&ctx->d_status, sizeof(int)));
  if (!ctx->h_status)
    ANOMOD_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->h_status), sizeof(int),
                                  hipHostMallocDefault));
  ctx->host_allreduce = allreduce;
  ctx->host_allgather = allgather;
  ctx->host_user = user;
  ctx->nranks = nranks;
  ctx->rank = rank;
  return ANOMOD_OK;
}

int anomod_ctx_comm_info(const anomod_ctx* ctx, int* nranks, int* rank) {
  ANOMOD_REQUIRE(nullptr, ctx && nranks && rank, "anomod_ctx_comm_info: NULL argument");
  *nranks = ctx->nranks;
  *rank = ctx->rank;
  return ANOMOD_OK;
}

}  // extern "C"
