// Context, error, timing and RCCL plumbing of libanomod.
//
// The reference has no comm backend at all (SURVEY.md §5 "Distributed comm
// backend: None"; its only concurrency is the HTTP ThreadPoolExecutor of
// trace_collector.py:519-531).  Here one process drives one GPU and the
// integer edge tables of all ranks are summed with RCCL over xGMI.
#include <cstdarg>
#include <cstring>

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
  if (ctx->d_table) (void)hipFree(ctx->d_table);
  if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
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
  ANOMOD_REQUIRE(ctx, ctx->comm == nullptr, "ctx already has a communicator");
  if (int rc = anomod::bind(ctx)) return rc;
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  ANOMOD_RCCL(ctx, ncclCommInitRank(&ctx->comm, nranks, id, rank));
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
