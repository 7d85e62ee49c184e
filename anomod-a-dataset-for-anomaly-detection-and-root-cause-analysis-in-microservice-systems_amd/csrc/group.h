// Trace grouping (group.hip, bucket.hip): types shared by the two paths.
// Internal header (not part of the ABI).
#pragma once

#include "common.h"

namespace anomod {

// One span as a 32-B record inside the grouping passes: (hash, span_id,
// parent) then svc|flags and dur — two 16-B halves.
struct __attribute__((aligned(16))) GRec {
  uint64_t h, sid, pid;
  uint32_t sf, dur;
};
static_assert(sizeof(GRec) == 32, "32-B records");

struct SoaIn {
  const uint64_t* __restrict__ h;
  const uint64_t* __restrict__ sid;
  const uint64_t* __restrict__ pid;
  const uint32_t* __restrict__ sf;
  const uint32_t* __restrict__ dur;
};

struct SoaOut {
  uint64_t* __restrict__ h;
  uint64_t* __restrict__ sid;
  uint64_t* __restrict__ pid;
  uint32_t* __restrict__ sf;
  uint32_t* __restrict__ dur;
};

// Order key of a trace: the SplitMix64 finaliser of its hash (a bijection, so
// any hash distribution gives even buckets).
__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Workspace of both grouping paths (one allocation, grow-only; released
// with the ctx).  Sized for the larger need of the two.
struct GroupWs {
  uint64_t cap = 0;                   // spans the buffers hold
  GRec* aos[2] = {nullptr, nullptr};  // ping-pong records; the other one holds the SoA output
  uint64_t* tptr = nullptr;           // [cap + 1]
  // LSD path (group.hip)
  uint64_t* state = nullptr;          // look-back words
  uint64_t state_words = 0;
  unsigned long long* misc = nullptr; // counters
  unsigned long long* list = nullptr; // key changes inside buckets
  unsigned long long* owned = nullptr;  // mixed buckets sorted into scratch (start << 11 | size)
  uint32_t* tcnt = nullptr;           // per-tile digit counts, then run starts (both paths)
  uint32_t* bsum = nullptr;           // block sums of tcnt (both paths)
  uint8_t* dig = nullptr;             // next-pass digits (LSD path)
  uint64_t* pairs[2] = {nullptr, nullptr};  // bucket path: level-A / level-B pairs [cap]
  uint64_t list_cap = 0;
  uint32_t epoch = 0;
  // bucket path (bucket.hip)
  uint32_t* bstart = nullptr;         // [2^T + 1] bucket starts
  uint32_t* bsA = nullptr;            // [2^DA + 1] level-A bucket starts
  uint32_t* btile = nullptr;          // [2^DA + 1] level-B tile starts per level-A bucket
  uint32_t* tmap = nullptr;           // level-B tile -> level-A bucket
  uint32_t* dcnt = nullptr;           // [2^T] traces per bucket, then their exclusive scan
  uint32_t* over = nullptr;           // buckets too large for the per-bucket kernel
  uint32_t* part = nullptr;           // partial sums of the dcnt scan
  uint64_t bucket_cap = 0;            // 2^T the arrays above hold
  uint64_t tile_cap = 0;              // level-B tiles tmap holds
  uint64_t tcnt_words = 0;            // u32 words of tcnt (tile x digit counts)
  unsigned long long* h_misc = nullptr;  // pinned read-back of the counters
  void* block = nullptr;  // one allocation the device buffers are carved from
  void* aos1_block = nullptr;  // aos[1]: allocated when a path writes it
};

// misc layout (u64 words)
constexpr int kMiscTicket = 0;                        // [2] tiles of the two scans
constexpr int kMiscListCnt = kMiscTicket + 2;         // key changes inside buckets
constexpr int kMiscOver = kMiscListCnt + 1;           // oversized mixed buckets
constexpr int kMiscTraces = kMiscOver + 1;            // n_traces
constexpr int kMiscErr = kMiscTraces + 1;             // look-back timeout
constexpr int kMiscBigN = kMiscErr + 1;               // bucket path: buckets over the small cap
constexpr int kMiscTooBig = kMiscBigN + 1;            // bucket path: buckets over the large cap
constexpr int kMiscWords = kMiscTooBig + 1;
constexpr int kMiscRead = kMiscListCnt;               // [kMiscRead, kMiscWords) read back

// The grouped view of the workspace after a run.
struct GroupResult {
  SoaOut cols;
  uint64_t n_traces = 0;
  uint64_t* tptr = nullptr;
  int passes = 0;   // LSD: radix passes; bucket path: scatter levels
  int bits = 0;     // key bits the passes / levels sorted on
  bool bucket = false;
  bool join = false;  // fused aggregation: the per-bucket hash join ran (else the sorting kernels)
};

// Bucket path geometry for n spans (bucket.hip).
struct BucketGeom {
  int T = 0, DA = 0, DB = 0;  // bucket bits = DA + DB (DB = 0: one scatter level)
  uint64_t tilesA = 0, tilesB = 0;  // tilesB: upper bound of the level-B grid
};
BucketGeom bucket_geom(uint64_t n);
// ANOMOD_JOIN_RECB=1 (r06 A/B): level B moves the 32-B records beside the
// pairs (into the second record buffer) and the join reads them
// contiguously; the edge records then go to the trace_ptr buffer.
bool join_records_through_b();
// Runs the bucket path over `in` (ws sized by ensure_group_ws).  *fallback =
// true when a bucket outgrew the large per-bucket kernel: the caller groups
// with the LSD path instead (results are identical; only speed differs).
// With erec (the fused ungrouped aggregation): no grouped columns; every
// span's edge record (parent service row * S + service) << 33 | error << 32 |
// duration goes to erec[grouped position] instead (*fallback also when a
// bucket of long traces needs the unfused path).  want_h = false: the
// grouped trace_hash column is not written (res->cols.h = NULL; an edge
// aggregation of the grouped view reads no trace_hash).
int bucket_group_run(anomod_ctx* ctx, const anomod_spans* in, GroupResult* res, bool* fallback,
                     uint64_t* erec = nullptr, uint32_t S = 0, bool want_h = true);

}  // namespace anomod
