// Internal shared definitions of libanomod (not part of the public ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/anomod.h"

namespace anomod {

// Error plumbing: a per-thread message for ctx-less failures, a per-ctx one
// otherwise (anomod_last_error).
void set_error(anomod_ctx* ctx, const char* fmt, ...);

struct GroupWs;   // group.hip
struct Uploader;  // upload.hip

// One host -> device copy of the upload pipeline (upload.hip): kind 0 copies
// n bytes from a; kind 1 packs n elements of svc (u16, a) | flags (u16, b) << 16
// into u32 words.
struct UpItem {
  void* dst;
  const void* a;
  const void* b;
  uint64_t n;
  int kind;
};

enum Stage { kStageEdgeAgg = 0, kStageEdgeFinal = 1, kStageEdgeReduce = 2, kStageEwma = 3,
             kStagePagerank = 4, kStageTraceStruct = 5, kStageSegments = 6, kStageSummary = 7,
             kStageGroup = 8, kNumStages = 9 };

// Host wall-clock slots (anomod_ctx_host_ms): the last occurrence of each
// one-off setup step, or of a call phase the stage events cannot see.
enum HostSlot { kHostGroupAlloc = ANOMOD_HOST_GROUP_ALLOC, kHostGroupPinned = ANOMOD_HOST_GROUP_PINNED,
                kHostGroupWall = ANOMOD_HOST_GROUP_WALL, kHostUploadSetup = ANOMOD_HOST_UPLOAD_SETUP,
                kHostSetAlloc = ANOMOD_HOST_SET_ALLOC, kNumHostSlots = ANOMOD_HOST_SLOTS };

}  // namespace anomod

struct anomod_ctx {
  int device = 0;
  int num_cus = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev_begin[anomod::kNumStages] = {};
  hipEvent_t ev_end[anomod::kNumStages] = {};
  bool stage_recorded[anomod::kNumStages] = {};
  double host_ms[anomod::kNumHostSlots] = {};        // anomod_ctx_host_ms
  uint64_t host_count[anomod::kNumHostSlots] = {};
  std::string err;
  // RCCL communicator (one process per GPU) ...
  ncclComm_t comm = nullptr;
  // ... or a host transport (anomod_ctx_attach_host_comm: ranks sharing a
  // device, or a host-side library such as gloo)
  anomod_host_allreduce_fn host_allreduce = nullptr;
  anomod_host_allgather_fn host_allgather = nullptr;
  void* host_user = nullptr;
  void* h_coll = nullptr;      // pinned staging of host-transport collectives
  size_t coll_bytes = 0;
  int nranks = 1;
  int rank = 0;
  bool comm_aborted = false;   // set once the communicator was aborted
  double comm_timeout_s = 300; // ANOMOD_RCCL_TIMEOUT_S
  int* d_status = nullptr;     // device word of the status agreement
  int* h_status = nullptr;     // pinned host twin
  // Trace-grouping workspace (segmented radix sort of ungrouped span sets).
  anomod::GroupWs* group_ws = nullptr;
  int group_path = 0, group_levels = 0, group_bits = 0;  // anomod_ctx_group_info
  // Grow-only device scratch of the calls that need a large one-call
  // workspace (anomod::ScratchSlot).  Freeing a block of tens of GB costs the
  // driver's wipe of it (~30 ms/GB, in hipFree or in a later allocation:
  // scripts/r06/time_cold2.py), so a call reuses its slot instead of
  // allocating and freeing; released with the ctx, or when an allocation
  // would otherwise fail (release_scratch).
  void* scratch[4] = {};
  size_t scratch_bytes[4] = {};
  // Cached device workspace for the edge table.
  void* d_table = nullptr;
  size_t table_bytes = 0;
  // Pinned host staging for the edge table's small per-edge vectors (one D2H).
  void* h_stage = nullptr;
  size_t stage_bytes = 0;
  // Upload pipeline (worker threads, their streams and pinned buffers) and
  // the grow-only device span set anomod_edge_aggregate_host fills.
  anomod::Uploader* uploader = nullptr;
  anomod_spans* host_set = nullptr;
  uint64_t host_set_spans = 0, host_set_traces = 0;  // its capacity
};

struct anomod_spans {
  int device = 0;
  uint64_t n_spans = 0;
  uint64_t n_traces = 0;
  uint32_t max_svc = 0;      // largest service index present (host-validated)
  // longest trace in spans when known (upload, synthetic generation);
  // UINT64_MAX = unknown.  Lets a call skip the long-trace pass when no
  // trace outgrows a wave chunk.
  uint64_t max_trace_len = ~0ull;
  // Histogram form of the SN / TrainTicket-width edge kernels: 0 = pair (8 Ki
  // slots, right for sets that touch a few thousand (edge, bin) keys per
  // workgroup), 1 = compact (16 Ki packed slots), -1 = not known yet — the
  // aggregation then starts in the pair form and any workgroup whose table
  // saturates hands its remaining traces to a compact-form resume launch
  // (edge_agg.hip); the outcome is kept here for the set's next aggregation.
  mutable int8_t hist_form = -1;
  // Span ids are unique within every trace (declared by the producer: the
  // synthetic generator by construction, anomod_spans_set_unique_ids for
  // decoded / uploaded sets).  Lets the parent lookups scan from both ends
  // (any match is the first match).  false = unknown: forward scan only.
  bool unique_ids = false;
  // Parent-scan order hint for unique-id sets: 1 = collector order (most
  // child spans right after their parent: the bidirectional scan), 0 = not
  // (spans shuffled inside their traces: the forward scan), -1 = unknown —
  // probed on the device at the first aggregation (edge_agg.hip probe_order).
  mutable int8_t order = -1;
  bool grouped = true;       // false: spans in arrival order, trace_ptr = NULL
                             // (anomod_spans_upload_ungrouped; group first)
  uint64_t* trace_hash = nullptr;
  uint64_t* span_id = nullptr;
  uint64_t* parent_span_id = nullptr;
  uint32_t* svc_flags = nullptr;  // svc | flags << 16 (one 4-B load per span)
  uint32_t* dur_us = nullptr;
  uint64_t* trace_ptr = nullptr;  // [n_traces + 1]
};

#define ANOMOD_HIP(ctx, expr)                                                               \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess) {                                                                 \
      anomod::set_error((ctx), "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),      \
                        __FILE__, __LINE__);                                                \
      return ANOMOD_EHIP;                                                                   \
    }                                                                                       \
  } while (0)

#define ANOMOD_RCCL(ctx, expr)                                                              \
  do {                                                                                      \
    ncclResult_t _r = (expr);                                                               \
    if (_r != ncclSuccess) {                                                                \
      anomod::set_error((ctx), "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(_r),     \
                        __FILE__, __LINE__);                                                \
      return ANOMOD_ERCCL;                                                                  \
    }                                                                                       \
  } while (0)

#define ANOMOD_REQUIRE(ctx, cond, ...)                                                      \
  do {                                                                                      \
    if (!(cond)) {                                                                          \
      anomod::set_error((ctx), __VA_ARGS__);                                                \
      return ANOMOD_EINVAL;                                                                 \
    }                                                                                       \
  } while (0)

// ANOMOD_REQUIRE for the checks before a collective: instead of returning,
// record the first failure in `local` (passed to comm_agree afterwards, so
// the other ranks learn of it instead of waiting in the collective).
#define ANOMOD_CHECK_LOCAL(ctx, local, cond, ...)                                           \
  do {                                                                                      \
    if ((local) == ANOMOD_OK && !(cond)) {                                                  \
      anomod::set_error((ctx), __VA_ARGS__);                                                \
      (local) = ANOMOD_EINVAL;                                                              \
    }                                                                                       \
  } while (0)

namespace anomod {

// Make ctx's device current on this host thread.
int bind(anomod_ctx* ctx);
// hipEvent bracketing of a stage on the ctx stream.
int stage_begin(anomod_ctx* ctx, Stage s);
int stage_end(anomod_ctx* ctx, Stage s);
// Host wall clock (ms since an arbitrary origin) and the record of a slot.
double host_now_ms();
void host_record(anomod_ctx* ctx, HostSlot s, double ms);
// Wait for the ctx stream.  With a communicator attached, RCCL's async
// error state is polled while waiting and the communicator is aborted on an
// error or after ctx->comm_timeout_s (a dead peer must not hang the rank).
int stream_wait(anomod_ctx* ctx);
// Status agreement before a collective: every rank passes its local status
// (ANOMOD_OK or an error it would otherwise return early with) and gets back
// ANOMOD_OK only when every rank is OK — so either all ranks enter the data
// collective or none does.  A no-op returning local_rc without a communicator.
int comm_agree(anomod_ctx* ctx, int local_rc);
// Collectives on the ctx stream over whichever transport is attached (RCCL,
// or the host callbacks: staged through pinned memory, synchronous).
// comm_attached: a live transport of any kind.  coll_begin / coll_end bracket
// the calls RCCL should issue as one group.
enum CollType { kCollI32 = ANOMOD_DTYPE_I32, kCollU32 = ANOMOD_DTYPE_U32,
                kCollU64 = ANOMOD_DTYPE_U64, kCollF64 = ANOMOD_DTYPE_F64 };
enum CollOp { kCollSum = ANOMOD_OP_SUM, kCollMin = ANOMOD_OP_MIN, kCollMax = ANOMOD_OP_MAX };
bool comm_attached(const anomod_ctx* ctx);
int coll_begin(anomod_ctx* ctx);
int coll_end(anomod_ctx* ctx);
int coll_allreduce(anomod_ctx* ctx, void* dbuf, size_t count, CollType t, CollOp op);
// in place: this rank's block of count_per_rank elements sits at rank * count_per_rank
int coll_allgather(anomod_ctx* ctx, void* dbuf, size_t count_per_rank, CollType t);
// Trace cut points 0 = c_0 < ... < c_k = n_traces of a span set such that
// every range [c_i, c_{i+1}) holds at most max_spans spans or is a single
// trace (kernels with per-workgroup u32 counters launch once per range).
// 2^32 - 1, or ANOMOD_MAX_LAUNCH_SPANS (tests: forces the multi-launch path).
uint64_t max_launch_spans();
int span_launch_cuts(anomod_ctx* ctx, const anomod_spans* s, uint64_t max_spans,
                     std::vector<uint64_t>& cuts);
// Span-set storage (synth.hip): every array of a set of n_spans spans /
// n_traces traces (trace_hash optional), and its release.
int alloc_spans(anomod_ctx* ctx, uint64_t n_spans, uint64_t n_traces, bool with_hash,
                anomod_spans** out);
void free_spans(anomod_spans* s);
// Trace-grouping workspace (group.hip), released with the ctx.
void free_group_ws(anomod_ctx* ctx);
// Host -> device copies through the pinned staging pipeline (upload.hip);
// *max_svc = the largest service index a kind-1 item packed.  Returns after
// every copy landed.  free_uploader releases the pipeline with the ctx.
int upload_items(anomod_ctx* ctx, const UpItem* items, int n_items, uint32_t* max_svc);
void free_uploader(anomod_ctx* ctx);
// Edge table of n per-span edge records (the fused ungrouped aggregation:
// (parent row * S + service) << 33 | error << 32 | duration, csrc/bucket.hip)
// into `out`, merged over an attached communicator; *hist_form is the set's
// histogram-form hint (read, and updated with what the run learned).
int edge_aggregate_records(anomod_ctx* ctx, const uint64_t* rec, uint64_t n, uint32_t S,
                           int8_t* hist_form, anomod_edge_table* out);
// Grow-only device workspace owned by the ctx.
int ensure_table(anomod_ctx* ctx, size_t bytes);
enum ScratchSlot { kScratchQuantiles = 0, kScratchTraceStruct = 1, kScratchTsLong = 2,
                   kScratchUpload = 3, kNumScratch = 4 };
// *out = the slot's block of at least `bytes` (grown when smaller; on
// failure the slots outside `keep` (a mask; this slot is always kept) are
// released and the allocation retried once).
int ensure_scratch(anomod_ctx* ctx, ScratchSlot slot, size_t bytes, void** out,
                   unsigned keep = 0u);
// Frees every scratch slot whose bit is clear in `keep`.  Returns the bytes freed.
size_t release_scratch(anomod_ctx* ctx, unsigned keep = 0u);
// hipMalloc with one retry after the ctx's scratch was released.
hipError_t dev_malloc(anomod_ctx* ctx, void** p, size_t bytes);
int ensure_host_stage(anomod_ctx* ctx, size_t bytes);

// ---- integer latency histogram (ANOMOD_HIST_*) --------------------------
__host__ __device__ inline uint32_t hist_bin(uint32_t v) {
  if (v < 64u) return v;
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lg = 31u - (uint32_t)__clz((int)v);
#else
  const uint32_t lg = 31u - (uint32_t)__builtin_clz(v);
#endif
  const uint32_t e = lg - ANOMOD_HIST_SUB_BITS;
  return (e << ANOMOD_HIST_SUB_BITS) + (v >> e);
}

__host__ __device__ inline void hist_bounds(uint32_t bin, uint32_t* lo, uint32_t* hi) {
  if (bin < 64u) {
    *lo = bin;
    *hi = bin;
    return;
  }
  const uint32_t e = (bin >> ANOMOD_HIST_SUB_BITS) - 1u;
  const uint64_t m = (uint64_t)(bin & ((1u << ANOMOD_HIST_SUB_BITS) - 1u)) +
                     (1u << ANOMOD_HIST_SUB_BITS);
  *lo = (uint32_t)(m << e);
  *hi = (uint32_t)(((m + 1) << e) - 1);
}

}  // namespace anomod
