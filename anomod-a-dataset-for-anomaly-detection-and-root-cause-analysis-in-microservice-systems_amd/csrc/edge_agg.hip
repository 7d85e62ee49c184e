// Call-graph edge aggregation — the hot path.
//
// Replaces the per-span Python loops of
//   SN_collection-scripts/Dataset/trace_data/jaeger_to_csv.py:21-90
//     (parent = spanID of the first CHILD_OF reference, :34-38; service
//      resolved through processID, :45-46; duration_us, :83)
//   TT_collection-scripts/T-Dataset/trace_collector.py:401-481
//     (_build_span_records: trace-local parent resolution; roots = spans
//      whose parent is not in the trace, :443)
//   TT_collection-scripts/T-Dataset/enhanced_trace_collector.py:216-296
//     (per-service counts / error counts / latency stats)
// and adds what the reference never computed: a (parent service -> child
// service) edge table with an integer log-linear latency histogram per edge
// and p50/p99 taken with the reference's nearest-rank index convention
// (monitor_http_responses.py:180-190, rank = (n*q)//100).
//
// Design (MI355X):
//  * one pass over the span SoA in HBM: 8 B span_id + 8 B parent_span_id +
//    4 B svc|flags + 4 B dur_us per span + 8 B trace_ptr per trace, read
//    with buffer loads (one scalar descriptor per column and chunk, 32-bit
//    lane offsets, out-of-chunk lanes read 0 — no per-lane address math);
//  * persistent grid, one 1024-thread workgroup per CU; every wave owns a
//    contiguous range of traces and walks it in chunks of <= 256 spans /
//    <= 64 traces, so parent resolution is trace-local in that wave's LDS
//    staging area (no inter-wave synchronisation inside the loop);
//  * parent lookup: ordered scan of the trace's staged ids (first match, the
//    reference rule), 10 ids per 5 x ds_read2_b64 step (a per-wave LDS hash
//    with ds_cmpst inserts measured 1.7x slower, and scanning a lane's 4
//    slots in lockstep 1.1-1.4x slower: register pressure);
//  * the E x 896 histogram does not fit LDS, so each workgroup privatises it
//    in an 8 Ki-slot LDS hash table (2048 buckets x 4 u32 keys, one
//    ds_read_b128 per lookup; u32 counts in a parallel array), flushed once
//    with u64 atomics;
//  * per-edge error/sum/min/max live in LDS (E <= 512) and are flushed once;
//  * all merges are integer adds / min / max: results are bit-exact and
//    independent of geometry, scheduling and shard count.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>


#include "chunk.h"
#include "common.h"
#include "radix.h"

namespace anomod {
namespace {

using namespace chunk;
#ifndef ANOMOD_WAVES
#define ANOMOD_WAVES 16
#endif
constexpr int kWavesPerWG = ANOMOD_WAVES;
constexpr int kThreads = kWave * kWavesPerWG;
// LDS histogram table, two forms in the same 64 KiB (see ht_* below).
enum HistForm { kHtHbm = 0, kHtPair = 1, kHtCompact = 2,
                kHtKeys = 3 };  // exact-quantile mode: write (edge << 32 | dur) per span
constexpr int kPairBucketLog2 = 11;  // pair: 2048 buckets of 4 slots, keys | counts
constexpr uint32_t kPairSlots = 4u << kPairBucketLog2;
constexpr int kPairMaxProbe = 48;
constexpr int kCmpBucketLog2 = 12;   // compact: 4096 buckets of 4 (key | count << kb) slots
constexpr uint32_t kCmpSlots = 4u << kCmpBucketLog2;
constexpr int kHtBytes = 65536;
static_assert(kPairSlots * 8 == kHtBytes && kCmpSlots * 4 == kHtBytes, "64 KiB table");
#ifndef ANOMOD_LDS_EDGES
#define ANOMOD_LDS_EDGES 512
#endif
constexpr uint32_t kLdsEdges = ANOMOD_LDS_EDGES;
constexpr uint32_t kBins = ANOMOD_HIST_BINS;
// Experiment-only ablations (never set in the shipped build): 1 = no stats,
// 2 = no histogram, 4 = no parent lookup, 16 = stream the columns only,
// 32 = compact histogram adds without the wrap check (non-returning), 64 =
// compact-form spans whose two buckets are full are dropped (not counted).
#ifndef ANOMOD_ABL
#define ANOMOD_ABL 0
#endif
#ifndef ANOMOD_LOAD16
#define ANOMOD_LOAD16 0
#endif
static_assert(!ANOMOD_LOAD16 || (ANOMOD_ABL & 16), "16-B loads: stream-only timing builds");

// LDS carve (bytes, every offset a multiple of 16).
constexpr int kOffHt = 0;                      // u32 keys (pair) | u32 slots (compact); 0 = empty
constexpr int kOffHc = kOffHt + (int)kPairSlots * 4;  // u32 counts (pair form)
#ifndef ANOMOD_SUM_REPS
#define ANOMOD_SUM_REPS 8
#endif
constexpr uint32_t kSumReps = ANOMOD_SUM_REPS;           // u64 sum replicas per edge
constexpr int kOffSum = kOffHt + kHtBytes;               // u64 [kLdsEdges][kSumReps]
// Per-edge stats in LDS, two forms.  Direct (E <= kLdsEdges: every SN-width
// table): (min, max) pairs and error counts indexed by edge.  Slot-hashed
// (wider tables, e.g. TrainTicket: E = 48 * 46 = 2208): kSlotEdges 16-B
// entries {edge + 1, min, max, errors} found by hashing the edge (linear
// probing, ds_cmpst inserts), the sum replicas indexed by slot — a trace set
// touches far fewer edges than E.
constexpr uint32_t kSlotEdges = 512;
// the slot form's sums reuse the direct form's replica area
constexpr uint32_t kSlotSumReps = (kLdsEdges * kSumReps) / kSlotEdges;
static_assert(kSlotSumReps >= 1 && (kSlotSumReps & (kSlotSumReps - 1)) == 0, "slot sum replicas");
constexpr int kOffMm = kOffSum + (int)(kLdsEdges * kSumReps) * 8;  // u32 (min, max) pairs | slots
constexpr int kOffErr = kOffMm + (int)kLdsEdges * 8;     // u32 error counts (direct form)
// Wide direct form (kLdsEdges < E <= kWideEdges, e.g. TrainTicket: E = 48 *
// 46 = 2208): one 16-B entry {u64 sum, u32 min, u32 max} per edge + u32
// error counts, indexed by edge (no slot hashing, no sum replicas).
#ifndef ANOMOD_WIDE_EDGES
#define ANOMOD_WIDE_EDGES 2304
#endif
constexpr uint32_t kWideEdges = ANOMOD_WIDE_EDGES;
constexpr int kOffWideErr = kOffSum + (int)kWideEdges * 16;
constexpr int kStatsEnd = std::max({kOffMm + (int)(kLdsEdges * 12),   // direct
                                    kOffMm + (int)(kSlotEdges * 16),  // slot
                                    kOffWideErr + (int)kWideEdges * 4});  // wide
// u32 control words: [0] pair-form inserts that found their probe chain full
// (counted in HBM; added to tab.ovf once per workgroup at the flush)
constexpr int kOffCtl = (kStatsEnd + 15) & ~15;
constexpr int kOffWave = kOffCtl + 16;
// A workgroup of a first (form-unknown) aggregation whose pair table turned
// away this many inserts stops: its waves hand their remaining traces to the
// compact-form resume launch (edge_agg_kernel, kModeAuto / kModeResume).
constexpr uint32_t kSatFails = 64;
// kModeWideScan: kModeNormal with the wide parent scan (process_chunk)
enum LaunchMode : uint32_t { kModeNormal = 0, kModeAuto = 1, kModeResume = 2, kModeWideScan = 3 };
enum StatsForm { kStHbm = 0, kStDirect = 1, kStSlot = 2, kStWide = 3 };
constexpr int kWSid = 0;                          // u64 span ids [kStage + kScanSlack] (scan slack)
constexpr int kWSvc = kWSid + (kStage + chunk::kScanSlack) * 8;  // u16 services [kStage + 8]
constexpr int kWFlag = kWSvc + (kStage + 8) * 2;  // u8 trace-start flags [kStage]
constexpr int kWAuto = kWFlag + kStage;           // u64: kModeAuto, first trace of the chunk
constexpr int kWBytes = kWAuto + 16;
constexpr int kLdsBytes = kOffWave + kWavesPerWG * kWBytes;
static_assert(kWBytes % 16 == 0, "wave staging must stay 16-B aligned");
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

struct Table {
  unsigned long long* hist;  // [E * kBins]
  unsigned long long* err;   // [E]
  unsigned long long* sum;   // [E]
  unsigned int* mn;          // [E]
  unsigned int* mx;          // [E]
  unsigned long long* ctr;   // trace-segment counter of the dynamic tail (zeroed per launch)
  uint32_t kb;               // key bits of a histogram slot (count in the 32 - kb above)
  unsigned long long* keys;  // kHtKeys: [n_spans] edge << 32 | dur, by span position
  unsigned long long* big;       // long traces: [0] listed, [1] / [2] tickets of the
                                 // resolve / record kernels
  unsigned long long* big_list;  // long traces: trace indices
  uint16_t* bpar;            // long traces: every listed span's parent row (S root, S + 1 orphan)
  uint64_t t_base;           // trace index of this launch's first trace
  unsigned long long* ovf;   // [0] spans whose pair-form probe chain was full (counted in
                             // HBM), [1] workgroups that stopped at a saturated pair table
  unsigned long long* left;  // kModeAuto: [2 j], [2 j + 1] = trace range j a stopped wave left
  unsigned long long* nleft; // [0] ranges left, [1] resume ticket
  uint32_t mode;             // LaunchMode
  uint32_t occupancy;        // compact form: report the fullest workgroup's used slots
                             // (tab.ovf[1], atomic max) at the flush
};

struct Cols {
  const uint64_t* __restrict__ span_id;
  const uint64_t* __restrict__ parent;
  const uint32_t* __restrict__ svcfl;  // svc | flags << 16
  const uint32_t* __restrict__ dur;
};

// Histogram increment of key = edge*kBins + bin + 1 in the workgroup's LDS.
//
// Pair form (E <= kLdsEdges, SN width): 2048 buckets of 4 slots, keys and u32
// counts in separate arrays, so one ds_read_b128 fetches a key's home
// bucket; a resident key costs that read + one fire-and-forget ds_add_u32 (0
// for lanes that miss, so no branch around it).  With the SN mix a
// workgroup holds ~3.6 k keys in 8 Ki slots and 0.02 % of spans miss their
// home bucket.  A launch covers < 2^32 spans, so u32 counts do not wrap.
//
// Compact form (wider tables: TrainTicket E = 2208, ~21 k keys per
// workgroup): 16 Ki u32 slots = key | count << kb (kb = the key's bit width,
// 21 for TrainTicket) in 4096 buckets; a key lives in its home bucket or the
// next one, both fetched by two ds_read_b128 in one round trip (95 % / 3.3 %
// of TrainTicket spans, simulated).  The add returns the old slot: a count
// field that was all ones wrapped, and that lane moves 2^(32-kb) counts to
// HBM (exact: one lane per wrap).  When both buckets are full of other keys
// the span counts in HBM at once (1.7 %), so no lane walks a probe chain.
//
// New keys take the first empty slot in probe order from the bucket start
// (ds_cmpst; a key never moves).
__device__ __forceinline__ uint32_t ht_hash(uint32_t key) { return key * 0x9E3779B1u; }

__device__ __attribute__((noinline)) void ht_insert_pair(uint32_t* hk, uint32_t* hc, uint32_t key,
                                                         uint32_t s,
                                                         unsigned long long* __restrict__ ghist,
                                                         uint32_t* ctl) {
  for (int probe = 0; probe < kPairMaxProbe; ++probe) {
    uint32_t cur = __hip_atomic_load(&hk[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == 0u) {
      const uint32_t prev = atomicCAS(&hk[s], 0u, key);
      cur = prev == 0u ? key : prev;
    }
    if (cur == key) {
      atomicAdd(&hc[s], 1u);
      return;
    }
    s = (s + 1u) & (kPairSlots - 1u);
  }
  atomicAdd(&ghist[key - 1u], 1ull);
  // counted per workgroup in LDS (one HBM add at the flush: a device-wide
  // counter bumped per span was itself a contended hot spot); a first
  // aggregation stops the workgroup at kSatFails, and the host switches the
  // set to the compact form
  atomicAdd(&ctl[0], 1u);
}

__device__ __forceinline__ void ht_wrap(uint32_t old, uint32_t key, uint32_t kb,
                                        unsigned long long* __restrict__ ghist) {
  if ((old >> kb) == (0xFFFFFFFFu >> kb)) atomicAdd(&ghist[key - 1u], 1ull << (32u - kb));
}

// Compact form, key not in its two buckets but one of them had room: claim
// the first empty slot of the 8 (or count where another lane just put it).
__device__ __attribute__((noinline)) void ht_insert_cmp(uint32_t* hk, uint32_t key, uint32_t b0,
                                                        uint32_t b1, uint32_t kb,
                                                        unsigned long long* __restrict__ ghist) {
  const uint32_t kmask = 0xFFFFFFFFu >> (32u - kb);
  for (int q = 0; q < 8; ++q) {
    const uint32_t s = (q < 4 ? b0 : b1) + (uint32_t)(q & 3);
    uint32_t cur = __hip_atomic_load(&hk[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == 0u) {
      const uint32_t prev = atomicCAS(&hk[s], 0u, key | (1u << kb));
      if (prev == 0u) return;  // new slot, count 1
      cur = prev;
    }
    if ((cur & kmask) == key) {
      ht_wrap(atomicAdd(&hk[s], 1u << kb), key, kb, ghist);
      return;
    }
  }
  atomicAdd(&ghist[key - 1u], 1ull);
}

using u32x2 = uint32_t __attribute__((ext_vector_type(2)));
using u32x4 = uint32_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t slot_home(uint32_t edge) {
  return (edge * 0x9E3779B1u) >> (32 - 9);  // kSlotEdges = 512
}

// The slot of `key` = edge + 1 past its home (linear probing; inserted on
// first sight); UINT32_MAX when kSlotProbe slots are taken by other edges
// (that span's stats then go to HBM).
constexpr int kSlotProbe = 32;
__device__ __attribute__((noinline)) uint32_t slot_find(uint32_t* st4, uint32_t key) {
  uint32_t s = slot_home(key - 1u) & ~3u;  // the home bucket first
  for (int probe = 0; probe < kSlotProbe; ++probe) {
    uint32_t cur = __hip_atomic_load(&st4[4u * s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == 0u) {
      const uint32_t prev = atomicCAS(&st4[4u * s], 0u, key);
      cur = prev == 0u ? key : prev;
    }
    if (cur == key) return s;
    s = (s + 1u) & (kSlotEdges - 1u);
  }
  return 0xFFFFFFFFu;
}

// The edge's stats position and current (min, max) in LDS, read before the
// span's histogram update so this read and the bucket read share one LDS
// round trip.  slot: the edge itself (direct), its table slot (slot form;
// UINT32_MAX = not at home, resolved by slot_find after the bucket read).
struct StatPeek {
  u32x2 mm;
  uint32_t slot;
};

template <int ST>
__device__ __forceinline__ StatPeek stat_peek(const unsigned char* smem, uint32_t edge) {
  if constexpr (ST == kStDirect && !(ANOMOD_ABL & 1)) {
    return {*reinterpret_cast<const u32x2*>(smem + kOffMm + 8u * edge), edge};
  } else if constexpr (ST == kStWide && !(ANOMOD_ABL & 1)) {
    return {*reinterpret_cast<const u32x2*>(smem + kOffSum + 16u * edge + 8u), edge};
  } else if constexpr (ST == kStSlot && !(ANOMOD_ABL & 1)) {
    // the home bucket of 4 entries (64 B, one round trip): simulated on the
    // TrainTicket mix, ~0 % of spans find their edge elsewhere (2.1 % with
    // 2-entry buckets, and a row with one such lane waits for its probe)
    const uint32_t s = slot_home(edge) & ~3u;
    const u32x4* ent = reinterpret_cast<const u32x4*>(smem + kOffMm + 16u * s);
    const u32x4 e0 = ent[0], e1 = ent[1], e2 = ent[2], e3 = ent[3];
    const uint32_t k = edge + 1u;
    const uint32_t j = e0.x == k ? 0u : e1.x == k ? 1u : e2.x == k ? 2u : e3.x == k ? 3u : 4u;
    const u32x4 e = j == 0u ? e0 : j == 1u ? e1 : j == 2u ? e2 : e3;
    return {u32x2{e.y, e.z}, j < 4u ? s + j : 0xFFFFFFFFu};
  } else {
    return {u32x2{0u, 0u}, edge};
  }
}

template <int ST>
__device__ __forceinline__ void stat_add(unsigned char* smem, uint32_t edge, uint32_t d,
                                         uint32_t fl, const Table& tab, StatPeek pk) {
  if constexpr (ANOMOD_ABL & 1) return;
  auto* lsum = reinterpret_cast<unsigned long long*>(smem + kOffSum);
  if constexpr (ST == kStDirect) {
    // Lanes of one wave-instruction share few edges, and same-address LDS
    // atomics serialise: the sum is spread over kSumReps replicas by lane,
    // and min / max (`mm`, read by stat_peek: a broadcast read) are only
    // updated when the span beats them — after warm-up almost never.  A stale
    // read only costs a redundant atomic.
    auto* lmm = reinterpret_cast<uint32_t*>(smem + kOffMm);
    auto* lerr = reinterpret_cast<uint32_t*>(smem + kOffErr);
    atomicAdd(&lsum[edge * kSumReps + (__lane_id() & (kSumReps - 1u))], (unsigned long long)d);
    if (d < pk.mm.x) atomicMin(&lmm[2u * edge], d);
    if (d > pk.mm.y) atomicMax(&lmm[2u * edge + 1u], d);
    if (fl & ANOMOD_FLAG_ERROR) atomicAdd(&lerr[edge], 1u);
    return;
  }
  if constexpr (ST == kStWide) {
    unsigned char* ent = smem + kOffSum + 16u * edge;
    atomicAdd(reinterpret_cast<unsigned long long*>(ent), (unsigned long long)d);
    if (d < pk.mm.x) atomicMin(reinterpret_cast<uint32_t*>(ent + 8), d);
    if (d > pk.mm.y) atomicMax(reinterpret_cast<uint32_t*>(ent + 12), d);
    if (fl & ANOMOD_FLAG_ERROR) atomicAdd(reinterpret_cast<uint32_t*>(smem + kOffWideErr) + edge, 1u);
    return;
  }
  if constexpr (ST == kStSlot) {
    uint32_t s = pk.slot;
    u32x2 mm = pk.mm;
    auto* st4 = reinterpret_cast<uint32_t*>(smem + kOffMm);
    if (s == 0xFFFFFFFFu) {
      s = slot_find(st4, edge + 1u);
      mm = u32x2{0xFFFFFFFFu, 0u};  // unknown: the atomics below decide
    }
    if (s != 0xFFFFFFFFu) {
      atomicAdd(&lsum[s * kSlotSumReps + (__lane_id() & (kSlotSumReps - 1u))],
                (unsigned long long)d);
      if (d < mm.x) atomicMin(&st4[4u * s + 1u], d);
      if (d > mm.y) atomicMax(&st4[4u * s + 2u], d);
      if (fl & ANOMOD_FLAG_ERROR) atomicAdd(&st4[4u * s + 3u], 1u);
      return;
    }
  }
  atomicAdd(&tab.sum[edge], (unsigned long long)d);
  atomicMin(&tab.mn[edge], d);
  atomicMax(&tab.mx[edge], d);
  if (fl & ANOMOD_FLAG_ERROR) atomicAdd(&tab.err[edge], 1ull);
}

// One span.
template <int HT, int ST>
__device__ __forceinline__ void record(unsigned char* smem, uint32_t edge, uint32_t d, uint32_t fl,
                                       const Table& tab) {
  const StatPeek pk = stat_peek<ST>(smem, edge);
  const uint32_t key = edge * kBins + hist_bin(d) + 1u;
  if constexpr ((ANOMOD_ABL & 2) || HT == kHtHbm) {
    if constexpr (!(ANOMOD_ABL & 2)) atomicAdd(&tab.hist[key - 1u], 1ull);
    stat_add<ST>(smem, edge, d, fl, tab, pk);
  } else if constexpr (HT == kHtPair) {
    // plain 16-B read (other waves insert concurrently; a stale empty slot
    // only sends the lane down the insert path, which re-reads)
    auto* hk = reinterpret_cast<uint32_t*>(smem + kOffHt);
    auto* hc = reinterpret_cast<uint32_t*>(smem + kOffHc);
    const uint32_t s0 = (ht_hash(key) >> (32 - kPairBucketLog2)) * 4u;
    const u32x4 bk = *reinterpret_cast<const u32x4*>(hk + s0);
    const uint32_t j = bk.x == key ? 0u : bk.y == key ? 1u : bk.z == key ? 2u : 3u;
    const bool hit = (j < 3u) | (bk.w == key);
    atomicAdd(&hc[s0 + j], hit ? 1u : 0u);
    stat_add<ST>(smem, edge, d, fl, tab, pk);
    if (!hit) ht_insert_pair(hk, hc, key, s0, tab.hist, reinterpret_cast<uint32_t*>(smem + kOffCtl));
  } else {  // kHtCompact
    auto* hk = reinterpret_cast<uint32_t*>(smem + kOffHt);
    const uint32_t kmask = 0xFFFFFFFFu >> (32u - tab.kb);
    const uint32_t b = ht_hash(key) >> (32 - kCmpBucketLog2);
    const uint32_t s0 = b * 4u, s1 = ((b + 1u) & ((1u << kCmpBucketLog2) - 1u)) * 4u;
    const u32x4 x = *reinterpret_cast<const u32x4*>(hk + s0);
    const u32x4 y = *reinterpret_cast<const u32x4*>(hk + s1);
    const uint32_t j = (x.x & kmask) == key   ? s0
                       : (x.y & kmask) == key ? s0 + 1u
                       : (x.z & kmask) == key ? s0 + 2u
                       : (x.w & kmask) == key ? s0 + 3u
                       : (y.x & kmask) == key ? s1
                       : (y.y & kmask) == key ? s1 + 1u
                       : (y.z & kmask) == key ? s1 + 2u
                       : (y.w & kmask) == key ? s1 + 3u
                                              : 0xFFFFFFFFu;
    const bool hit = j != 0xFFFFFFFFu;
    const uint32_t old = atomicAdd(&hk[hit ? j : s0], hit ? (1u << tab.kb) : 0u);
    const bool room = (x.x == 0u) | (x.y == 0u) | (x.z == 0u) | (x.w == 0u) | (y.x == 0u) |
                      (y.y == 0u) | (y.z == 0u) | (y.w == 0u);
    stat_add<ST>(smem, edge, d, fl, tab, pk);
    if (hit) {
      if (!(ANOMOD_ABL & 32)) ht_wrap(old, key, tab.kb, tab.hist);
    } else if (room) {
      ht_insert_cmp(hk, key, s0, s1, tab.kb, tab.hist);
    } else if (!(ANOMOD_ABL & 64)) {
      atomicAdd(&tab.hist[key - 1u], 1ull);
    }
  }
}

// Span columns of a chunk held in registers while the previous chunk is
// processed (software pipeline, one chunk ahead).
struct Regs {
  uint64_t sid[kPer], pid[kPer];
  uint32_t dur[kPer], sf[kPer];  // sf = svc | flags << 16
};

__device__ __forceinline__ void load_regs(const Cols& col, const Chunk& c, int lane, Regs& R) {
  const uint32_t n = c.k ? c.n : 0u;  // a big trace is read by edge_big_kernel
  const auto rsid = rsrc(col.span_id + c.base, n * 8u);
  const auto rpid = rsrc(col.parent + c.base, n * 8u);
  const auto rsf = rsrc(col.svcfl + c.base, n * 4u);
  const auto rdur = rsrc(col.dur + c.base, n * 4u);
#if ANOMOD_LOAD16  // timing experiment (stream-only builds): 16 B per lane and load
  static_assert(kPer == 4, "16-B loads: 4 rows");
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint32_t i = (uint32_t)(j * 128 + 2 * lane);
    const auto a = __builtin_amdgcn_raw_buffer_load_b128(rsid, (int)(i * 8u), 0, ANOMOD_LOAD_AUX);
    const auto b = __builtin_amdgcn_raw_buffer_load_b128(rpid, (int)(i * 8u), 0, ANOMOD_LOAD_AUX);
    R.sid[2 * j] = ((uint64_t)a[1] << 32) | a[0];
    R.sid[2 * j + 1] = ((uint64_t)a[3] << 32) | a[2];
    R.pid[2 * j] = ((uint64_t)b[1] << 32) | b[0];
    R.pid[2 * j + 1] = ((uint64_t)b[3] << 32) | b[2];
  }
  {
    const auto c = __builtin_amdgcn_raw_buffer_load_b128(rsf, (int)(lane * 16u), 0, ANOMOD_LOAD_AUX);
    const auto d = __builtin_amdgcn_raw_buffer_load_b128(rdur, (int)(lane * 16u), 0, ANOMOD_LOAD_AUX);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      R.sf[r] = c[r];
      R.dur[r] = d[r];
    }
  }
#else
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const uint32_t i = (uint32_t)lane + (uint32_t)(r * kWave);
    R.sid[r] = bload64(rsid, i * 8u);
    R.pid[r] = bload64(rpid, i * 8u);
    R.sf[r] = bload32(rsf, i * 4u);
    R.dur[r] = bload32(rdur, i * 4u);
  }
#endif
}

// First span of [a, b) whose id equals pid: kScan ids per step (ds_read2_b64
// from the trace start itself), matches folded into a bit mask.  First match
// in trace order (the reference rule: jaeger_to_csv.py:34-38 /
// trace_collector.py:424-443).
#ifndef ANOMOD_SCAN_IDS
#define ANOMOD_SCAN_IDS 10
#endif
constexpr uint32_t kScan = ANOMOD_SCAN_IDS;  // ids compared per step (kScan / 2 x ds_read2_b64)
// Per-lane scan steps before a row's remaining lookups go to the whole wave
// (coop_parent); 0 = every lane scans to the end.
#ifndef ANOMOD_COOP_STEPS
#define ANOMOD_COOP_STEPS 0
#endif
constexpr int kCoopSteps = ANOMOD_COOP_STEPS;
static_assert(kScan % 2 == 0 && kScan <= 16, "scan step");

template <int MAXS = 0>  // > 0: -2 after that many steps (completed cooperatively)
__device__ __forceinline__ int find_parent(const uint64_t* lsid, uint32_t a, uint32_t b,
                                           uint64_t pid) {
  int steps = 0;
  for (uint32_t q0 = a; q0 < b; q0 += kScan) {
    if (MAXS > 0 && steps++ >= MAXS) return -2;
    uint64_t v[kScan];
#pragma unroll
    for (uint32_t j = 0; j < kScan; ++j) v[j] = lsid[q0 + j];
    uint32_t m = 0;
#pragma unroll
    for (uint32_t j = 0; j < kScan; ++j) m |= (v[j] == pid ? 1u : 0u) << j;
    const uint32_t hi = (b - q0) < kScan ? (b - q0) : kScan;  // >= 1
    m &= (1u << hi) - 1u;
    if (m) return (int)(q0 + __ffs(m) - 1u);
  }
  return -1;
}

// Scan widths of the bidirectional parent scan: (kFwd, kBwd) = (6, 4) for
// collector-ordered traces of tens of spans (SN / TrainTicket: 8 / 8 measured
// 2-10 % slower there), (8, 8) for sets holding traces longer than a chunk
// (LONG: random ancestors in 128- and 256-span traces, 7.52 vs 8.09 ms).
// r05: the TrainTicket-width and long-trace instantiations take the
// select-built scan (one LDS round trip per step): TT 2^27 17.8-18.4 vs
// 18.5-18.7 ms, LONG 2^23 7.24-7.29 vs 7.60-7.69; the SN pair form gains
// nothing measurable and keeps the mask form (profiles/r05_experiments/
// parent_scan_sel_widths.log).  Then both take the split-word form
// (chunk.h find_parent_split: ids staged as u32 planes, low words compared,
// the candidate confirmed on its high word), whose cheaper steps pay for
// wider ones: TT 12 / 4 16.3-16.7 ms, LONG 12 / 4 6.96-7.04
// (split_scan_*.log); the SN pair form again gains nothing.
#ifndef ANOMOD_SEL_SN
#define ANOMOD_SEL_SN 0
#endif
#ifndef ANOMOD_SEL_WIDE
#define ANOMOD_SEL_WIDE 1
#endif
#ifndef ANOMOD_SEL_LONG
#define ANOMOD_SEL_LONG 1
#endif
#ifndef ANOMOD_SPLIT_LONG
#define ANOMOD_SPLIT_LONG 1
#endif
#ifndef ANOMOD_SPLIT_WIDE
#define ANOMOD_SPLIT_WIDE 1
#endif
#ifndef ANOMOD_SPLIT_SN
#define ANOMOD_SPLIT_SN 0
#endif
#ifndef ANOMOD_LFWD
#define ANOMOD_LFWD 12
#endif
#ifndef ANOMOD_LBWD
#define ANOMOD_LBWD 4
#endif
constexpr uint32_t kLFwd = ANOMOD_LFWD, kLBwd = ANOMOD_LBWD;  // the long-trace sets' widths
#ifndef ANOMOD_WFWD
#define ANOMOD_WFWD 12
#endif
#ifndef ANOMOD_WBWD
#define ANOMOD_WBWD 4
#endif
constexpr uint32_t kWFwd = ANOMOD_WFWD, kWBwd = ANOMOD_WBWD;  // TrainTicket width, split scan
template <int HT, int ST, bool UNI, bool WIDE = false>
__device__ __forceinline__ void process_chunk(unsigned char* smem, unsigned char* wsm, int lane,
                                              const Chunk& c, const Regs& R, uint32_t S,
                                              const Table& tab) {
  auto* lsid = reinterpret_cast<uint64_t*>(wsm + kWSid);
  auto* lsvc = reinterpret_cast<uint16_t*>(wsm + kWSvc);
  auto* lflag = reinterpret_cast<uint8_t*>(wsm + kWFlag);
  // select-built scan (chunk.h find_parent_bidir SEL) per table form
  constexpr bool kSel = WIDE ? ANOMOD_SEL_LONG != 0
                             : (ST == kStWide ? ANOMOD_SEL_WIDE != 0 : ANOMOD_SEL_SN != 0);
  // TrainTicket-width and long-trace sets with unique ids: ids staged as u32
  // planes, low words scanned (chunk.h find_parent_split; it takes precedence
  // over kSel)
  constexpr bool kSplit =
      UNI && kCoopSteps == 0 &&
      (WIDE ? ANOMOD_SPLIT_LONG != 0 : (ST == kStWide ? ANOMOD_SPLIT_WIDE != 0 : ANOMOD_SPLIT_SN != 0));
  auto* llo = reinterpret_cast<uint32_t*>(wsm + kWSid);
  uint32_t* lhi = llo + (kStage + chunk::kScanSlack);
  if constexpr (ANOMOD_ABL & 16) {  // stream only: keep the loads, do nothing
    uint64_t x = 0;
#pragma unroll
    for (int r = 0; r < kPer; ++r) x ^= R.sid[r] ^ R.pid[r] ^ R.sf[r] ^ ((uint64_t)R.dur[r] << 7);
    if (x == 0x0123456789ABCDEFull) tab.err[0] = x;
    return;
  }
  // Stage ids / services (lanes past n hold zeros from the buffer loads);
  // mark trace starts.
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const uint32_t i = lane + r * kWave;
    if constexpr (kSplit) {
      llo[i] = (uint32_t)R.sid[r];
      lhi[i] = (uint32_t)(R.sid[r] >> 32);
    } else {
      lsid[i] = R.sid[r];
    }
    lsvc[i] = (uint16_t)R.sf[r];
  }
  uint64_t Sm[kPer];
  start_masks(lflag, c, lane, Sm);
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const uint32_t i = lane + r * kWave;
    uint32_t p = S;  // ROOT
    if constexpr (kCoopSteps > 0 && !(ANOMOD_ABL & 4)) {
      // kCoopSteps scan steps per lane, then the row's remaining lookups by
      // the whole wave (coop_parent)
      const bool has = i < c.n && R.pid[r] != 0ull;
      uint32_t a, b;
      trace_bounds(Sm, r, lane, c.n, a, b);
      int q = -1;
      if (has) {
        q = UNI ? (WIDE ? find_parent_bidir<kLFwd, kLBwd, kCoopSteps, kSel>(lsid, a, b, i, R.pid[r])
                        : find_parent_bidir<kFwd, kBwd, kCoopSteps, kSel>(lsid, a, b, i, R.pid[r]))
                : find_parent<kCoopSteps>(lsid, a, b, R.pid[r]);
      }
      coop_parent(lsid, __ballot(q == -2), lane, R.pid[r], a, b, q);
      if (has) p = q >= 0 ? lsvc[q] : S + 1u;  // ORPHAN unless found in the trace
    } else if (i < c.n && R.pid[r] != 0ull) {
      p = S + 1u;  // ORPHAN unless found in the trace
      if constexpr (!(ANOMOD_ABL & 4)) {
        uint32_t a, b;
        trace_bounds(Sm, r, lane, c.n, a, b);
        int q;
        if constexpr (kSplit && WIDE)
          q = find_parent_split<kLFwd, kLBwd>(llo, lhi, a, b, i, R.pid[r]);
        else if constexpr (kSplit && ST == kStWide)
          q = find_parent_split<kWFwd, kWBwd>(llo, lhi, a, b, i, R.pid[r]);
        else if constexpr (kSplit)
          q = find_parent_split<kFwd, kBwd>(llo, lhi, a, b, i, R.pid[r]);
        else
          q = UNI ? (WIDE ? find_parent_bidir<kLFwd, kLBwd, 0, kSel>(lsid, a, b, i, R.pid[r])
                          : find_parent_bidir<kFwd, kBwd, 0, kSel>(lsid, a, b, i, R.pid[r]))
                  : find_parent(lsid, a, b, R.pid[r]);
        if (q >= 0) p = lsvc[q];
      } else {  // ablation: a parent-like edge without the lookup (keeps key diversity)
        p = ((R.sf[r] & 0xFFFFu) + 1u + (uint32_t)(R.pid[r] & 1u)) % S;
      }
    }
    if constexpr (HT == kHtKeys) {
      if (i < c.n)
        tab.keys[c.base + i] = ((unsigned long long)(p * S + (R.sf[r] & 0xFFFFu)) << 32) | R.dur[r];
    } else {
      if (i < c.n) record<HT, ST>(smem, p * S + (R.sf[r] & 0xFFFFu), R.dur[r], R.sf[r] >> 16, tab);
    }
  }
  wave_sync();
}

// The workgroup's private LDS tables (histogram + per-edge stats), shared by
// the chunk walk and the long-trace pass: zeroed at the start, merged into
// the device table with integer atomics (order-free) at the end.
template <int HT, int ST>
__device__ __forceinline__ void tables_init(unsigned char* smem, uint32_t E, int tid) {
  if (tid < 4) reinterpret_cast<uint32_t*>(smem + kOffCtl)[tid] = 0u;
  if constexpr (HT == kHtPair || HT == kHtCompact) {
    auto* hk = reinterpret_cast<uint32_t*>(smem + kOffHt);  // both forms: 64 KiB of zeros
    for (uint32_t s = tid; s < (uint32_t)kHtBytes / 4u; s += kThreads) hk[s] = 0u;
  }
  if constexpr (ST == kStDirect) {
    auto* lsum = reinterpret_cast<unsigned long long*>(smem + kOffSum);
    auto* lmm = reinterpret_cast<uint32_t*>(smem + kOffMm);
    auto* lerr = reinterpret_cast<uint32_t*>(smem + kOffErr);
    for (uint32_t e = tid; e < E * kSumReps; e += kThreads) lsum[e] = 0ull;
    for (uint32_t e = tid; e < E; e += kThreads) {
      lerr[e] = 0u;
      lmm[2u * e] = 0xFFFFFFFFu;
      lmm[2u * e + 1u] = 0u;
    }
  }
  if constexpr (ST == kStWide) {
    auto* ent = reinterpret_cast<uint32_t*>(smem + kOffSum);
    auto* lerr = reinterpret_cast<uint32_t*>(smem + kOffWideErr);
    for (uint32_t e = tid; e < E; e += kThreads) {
      ent[4u * e] = 0u;
      ent[4u * e + 1u] = 0u;
      ent[4u * e + 2u] = 0xFFFFFFFFu;
      ent[4u * e + 3u] = 0u;
      lerr[e] = 0u;
    }
  }
  if constexpr (ST == kStSlot) {
    auto* lsum = reinterpret_cast<unsigned long long*>(smem + kOffSum);
    auto* st4 = reinterpret_cast<uint32_t*>(smem + kOffMm);
    for (uint32_t e = tid; e < kSlotEdges * kSlotSumReps; e += kThreads) lsum[e] = 0ull;
    for (uint32_t e = tid; e < kSlotEdges; e += kThreads) {
      st4[4u * e] = 0u;
      st4[4u * e + 1u] = 0xFFFFFFFFu;
      st4[4u * e + 2u] = 0u;
      st4[4u * e + 3u] = 0u;
    }
  }
}

template <int HT, int ST>
__device__ __forceinline__ void tables_flush(unsigned char* smem, uint32_t E, const Table& tab,
                                             int tid) {
  if constexpr (HT == kHtPair) {
    auto* hk = reinterpret_cast<uint32_t*>(smem + kOffHt);
    auto* hc = reinterpret_cast<uint32_t*>(smem + kOffHc);
    for (uint32_t s = tid; s < kPairSlots; s += kThreads) {
      const uint32_t cnt = hc[s];
      if (cnt) atomicAdd(&tab.hist[hk[s] - 1u], (unsigned long long)cnt);
    }
    if (tid == 0) {
      const uint32_t fails = reinterpret_cast<const uint32_t*>(smem + kOffCtl)[0];
      if (fails) atomicAdd(&tab.ovf[0], (unsigned long long)fails);
      if (tab.mode == kModeAuto && fails >= kSatFails) atomicAdd(&tab.ovf[1], 1ull);
    }
  }
  if constexpr (HT == kHtCompact) {
    auto* hk = reinterpret_cast<uint32_t*>(smem + kOffHt);
    const uint32_t kmask = 0xFFFFFFFFu >> (32u - tab.kb);
    uint32_t used = 0;
    for (uint32_t s = tid; s < kCmpSlots; s += kThreads) {
      const uint32_t w = hk[s];
      used += w ? 1u : 0u;
      if (w >> tab.kb) atomicAdd(&tab.hist[(w & kmask) - 1u], (unsigned long long)(w >> tab.kb));
    }
    if (tab.occupancy) {  // the workgroup's used slots -> tab.ovf[1] (max over workgroups)
      auto* ctl = reinterpret_cast<uint32_t*>(smem + kOffCtl);
      for (int o = 32; o > 0; o >>= 1) used += __shfl_xor(used, o);
      if ((tid & (kWave - 1)) == 0) atomicAdd(&ctl[1], used);
      __syncthreads();
      if (tid == 0) atomicMax(&tab.ovf[1], (unsigned long long)ctl[1]);
    }
  }
  if constexpr (ST == kStSlot) {
    auto* lsum = reinterpret_cast<unsigned long long*>(smem + kOffSum);
    auto* st4 = reinterpret_cast<uint32_t*>(smem + kOffMm);
    for (uint32_t s = tid; s < kSlotEdges; s += kThreads) {
      const uint32_t key = st4[4u * s];
      if (key) {
        const uint32_t e = key - 1u;
        unsigned long long sum = 0;
        for (uint32_t k = 0; k < kSlotSumReps; ++k) sum += lsum[s * kSlotSumReps + k];
        atomicAdd(&tab.sum[e], sum);
        if (st4[4u * s + 3u]) atomicAdd(&tab.err[e], (unsigned long long)st4[4u * s + 3u]);
        atomicMin(&tab.mn[e], st4[4u * s + 1u]);
        atomicMax(&tab.mx[e], st4[4u * s + 2u]);
      }
    }
  }
  if constexpr (ST == kStWide) {
    auto* ent = reinterpret_cast<uint32_t*>(smem + kOffSum);
    auto* lerr = reinterpret_cast<uint32_t*>(smem + kOffWideErr);
    for (uint32_t e = tid; e < E; e += kThreads) {
      const uint32_t mn = ent[4u * e + 2u], mx = ent[4u * e + 3u];
      if (mn != 0xFFFFFFFFu || mx != 0u) {
        atomicAdd(&tab.sum[e], *reinterpret_cast<const unsigned long long*>(ent + 4u * e));
        if (lerr[e]) atomicAdd(&tab.err[e], (unsigned long long)lerr[e]);
        atomicMin(&tab.mn[e], mn);
        atomicMax(&tab.mx[e], mx);
      }
    }
  }
  if constexpr (ST == kStDirect) {
    auto* lsum = reinterpret_cast<unsigned long long*>(smem + kOffSum);
    auto* lerr = reinterpret_cast<uint32_t*>(smem + kOffErr);
    auto* lmm = reinterpret_cast<uint32_t*>(smem + kOffMm);
    for (uint32_t e = tid; e < E; e += kThreads) {
      if (lmm[2u * e] != 0xFFFFFFFFu || lmm[2u * e + 1u] != 0u) {
        unsigned long long sum = 0;
        for (uint32_t k = 0; k < kSumReps; ++k) sum += lsum[e * kSumReps + k];
        atomicAdd(&tab.sum[e], sum);
        if (lerr[e]) atomicAdd(&tab.err[e], (unsigned long long)lerr[e]);
        atomicMin(&tab.mn[e], lmm[2u * e]);
        atomicMax(&tab.mx[e], lmm[2u * e + 1u]);
      }
    }
  }
}

// Traces longer than kStage do not fit a wave's staging area: the chunk walk
// only lists them (big_list[j] = trace index, big[0] = count), and
// edge_big_kernel resolves them afterwards, one workgroup per trace.  Its LDS
// holds the same private histogram / per-edge stats tables as the chunk walk
// (flushed once at the end) and, in the wave-staging area's place, a hash
// table of kBigWin span ids at a time (id -> first position in the window,
// atomicMin); the trace's spans are looked up kBigPer per thread against the
// windows in trace order, so the first window holding a span's parent
// reference gives the first match (the reference rule).
// O(L * ceil(L / kBigWin)) work, O(L) for L <= kBigWin.
constexpr int kBigThreads = kThreads;  // the tables' init / flush loops assume it
#ifndef ANOMOD_BIG_MIN
#define ANOMOD_BIG_MIN 256
#endif
// resolve kernel: minimum waves per SIMD the compiler must fit (registers)
#ifndef ANOMOD_RES_MINB
#define ANOMOD_RES_MINB 2
#endif
// 1 = the r02 single-kernel long-trace pass (experiment builds, A/B)
#ifndef ANOMOD_BIG_ONEPASS
#define ANOMOD_BIG_ONEPASS 0
#endif
// traces longer than this take the long-trace pass (<= kStage)
constexpr uint32_t kBigMin = ANOMOD_BIG_MIN;
constexpr uint32_t kBigWin = 2048;    // ids per table window
constexpr uint32_t kBigSlots = 4096;  // table slots (load <= 0.5)
#ifndef ANOMOD_BIG_PER
#define ANOMOD_BIG_PER 8
#endif
constexpr int kBigPer = ANOMOD_BIG_PER;  // spans per thread per lookup block
constexpr int kOffBigKey = kOffWave;                          // u64 [kBigSlots], 0 = empty
constexpr int kOffBigPos = kOffBigKey + (int)kBigSlots * 8;   // u32 [kBigSlots]
static_assert(kBigWin % kBigThreads == 0 && kBigWin <= 65536, "window: whole rows, position << 16 | svc");
constexpr int kBigLdsBytes = kOffBigPos + (int)kBigSlots * 4;
static_assert(kBigLdsBytes <= 160 * 1024, "long-trace pass LDS budget");

__device__ __forceinline__ uint32_t big_slot(uint64_t id) {
  return (uint32_t)((id * 0x9E3779B97F4A7C15ull) >> (64 - 12)) & (kBigSlots - 1u);
}

// One trace longer than kBigWin spans: blocks of kBigThreads * kBigPer
// spans, each looked up against the trace's id windows in order (the first
// window holding a parent reference gives its first match).
template <int HT, int ST>
__device__ void big_one(unsigned char* smem, const uint64_t* __restrict__ span_id,
                        const uint64_t* __restrict__ parent, const uint32_t* __restrict__ svcfl,
                        const uint32_t* __restrict__ dur, uint64_t lo, uint64_t L, uint32_t S,
                        const Table& tab) {
  auto* bkey = reinterpret_cast<unsigned long long*>(smem + kOffBigKey);
  auto* bval = reinterpret_cast<uint32_t*>(smem + kOffBigPos);
  const int tid = threadIdx.x;
  for (uint64_t b0 = 0; b0 < L; b0 += (uint64_t)kBigThreads * kBigPer) {
    uint64_t pid[kBigPer];
    uint32_t sf[kBigPer], dr[kBigPer], psv[kBigPer];  // psv: parent's service (~0: none yet)
    bool need = false;
#pragma unroll
    for (int r = 0; r < kBigPer; ++r) {
      const uint64_t i = b0 + (uint64_t)r * kBigThreads + tid;
      pid[r] = i < L ? parent[lo + i] : 0ull;
      sf[r] = i < L ? svcfl[lo + i] : 0u;
      dr[r] = i < L ? dur[lo + i] : 0u;
      psv[r] = 0xFFFFFFFFu;
      need |= pid[r] != 0ull;
    }
    for (uint64_t w0 = 0; w0 < L; w0 += kBigWin) {
      if (!__syncthreads_or(need)) break;  // also orders the previous clear
      constexpr int kIns = kBigWin / kBigThreads;
      uint64_t id[kIns];
      uint32_t sv[kIns];
#pragma unroll
      for (int u = 0; u < kIns; ++u) {
        const uint32_t k = (uint32_t)(u * kBigThreads + tid);
        id[u] = w0 + k < L ? span_id[lo + w0 + k] : 0ull;
        sv[u] = w0 + k < L ? svcfl[lo + w0 + k] & 0xFFFFu : 0u;
      }
#pragma unroll
      for (int u = 0; u < kIns; ++u) {
        if (id[u] == 0ull) continue;
        const uint32_t k = (uint32_t)(u * kBigThreads + tid);
        for (uint32_t sl = big_slot(id[u]);; sl = (sl + 1u) & (kBigSlots - 1u)) {
          const unsigned long long prev = atomicCAS(&bkey[sl], 0ull, (unsigned long long)id[u]);
          if (prev == 0ull || prev == id[u]) {
            atomicMin(&bval[sl], (k << 16) | sv[u]);  // the first position wins, with its service
            break;
          }
        }
      }
      __syncthreads();
      need = false;
#pragma unroll
      for (int r = 0; r < kBigPer; ++r) {
        if (pid[r] == 0ull || psv[r] != 0xFFFFFFFFu) continue;
        for (uint32_t sl = big_slot(pid[r]);; sl = (sl + 1u) & (kBigSlots - 1u)) {
          const unsigned long long key = bkey[sl];
          if (key == pid[r]) {
            psv[r] = bval[sl] & 0xFFFFu;
            break;
          }
          if (key == 0ull) break;
        }
        need |= psv[r] == 0xFFFFFFFFu;
      }
      __syncthreads();
      for (uint32_t k = tid; k < kBigSlots; k += kBigThreads) {
        bkey[k] = 0ull;
        bval[k] = 0xFFFFFFFFu;
      }
    }
#pragma unroll
    for (int r = 0; r < kBigPer; ++r) {
      const uint64_t i = b0 + (uint64_t)r * kBigThreads + tid;
      if (i >= L) continue;
      const uint32_t p = pid[r] == 0ull ? S : psv[r] == 0xFFFFFFFFu ? S + 1u : psv[r];
      const uint32_t edge = p * S + (sf[r] & 0xFFFFu);
      if constexpr (HT == kHtKeys) {
        tab.keys[lo + i] = ((unsigned long long)edge << 32) | dr[r];
      } else {
        record<HT, ST>(smem, edge, dr[r], sf[r] >> 16, tab);
      }
    }
  }
  __syncthreads();  // the last window's clear before the next user of the table
}

// Up to kGroup listed traces of <= kBigWin spans packed into ONE table window
// (r03): trace i owns table slots [2 off_i, 2 off_i + 2 L_i) (load 1/2;
// range reduction by multiply-shift, linear probing inside the region), so
// ids of different traces never meet, and a workgroup pays the
// load / insert / lookup round trips once per batch instead of once per
// trace.  <= 2 spans per thread (sum L_i <= kBigWin = 2 x kBigThreads).
#ifndef ANOMOD_BIG_GROUP
#define ANOMOD_BIG_GROUP 4
#endif
constexpr int kGroup = ANOMOD_BIG_GROUP;  // traces per ticket (one atomic, their entries and bounds loaded together)
static_assert(kBigWin == 2 * kBigThreads, "a packed batch is two spans per thread");

__device__ __forceinline__ uint32_t big_region_slot(uint64_t id, uint32_t size) {
  return __umulhi((uint32_t)((id * 0x9E3779B97F4A7C15ull) >> 32), size);
}

// bm: the group entries (bits) packed into this window, consecutive
template <int HT, int ST>
__device__ void big_batch(unsigned char* smem, const uint64_t* __restrict__ span_id,
                          const uint64_t* __restrict__ parent, const uint32_t* __restrict__ svcfl,
                          const uint32_t* __restrict__ dur, const uint64_t (&lo)[kGroup],
                          const uint64_t (&L)[kGroup], uint32_t bm, uint32_t S, const Table& tab) {
  auto* bkey = reinterpret_cast<unsigned long long*>(smem + kOffBigKey);
  auto* bval = reinterpret_cast<uint32_t*>(smem + kOffBigPos);
  const int tid = threadIdx.x;
  uint32_t off[kGroup + 1];  // non-members have length 0
  off[0] = 0;
#pragma unroll
  for (int i = 0; i < kGroup; ++i) off[i + 1] = off[i] + (((bm >> i) & 1u) ? (uint32_t)L[i] : 0u);
  const uint32_t tot = off[kGroup];
  uint64_t id[2], pid[2], g[2];
  uint32_t sf[2], dr[2], rb[2], rs[2], pos[2], psv[2];
  bool v[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const uint32_t q = (uint32_t)(u * kBigThreads + tid);
    v[u] = q < tot;
    // the member holding batch position q: the last entry whose start <= q
    // (entries before the batch start at 0 with length 0, entries after it
    // at tot)
    uint32_t a0 = 0, a1 = off[1];
    uint64_t tl = lo[0];
#pragma unroll
    for (int i = 1; i < kGroup; ++i)
      if (q >= off[i] && ((bm >> i) & 1u)) {
        a0 = off[i];
        a1 = off[i + 1];
        tl = lo[i];
      }
    pos[u] = q - a0;
    rb[u] = 2u * a0;  // the trace's table region
    rs[u] = 2u * (a1 - a0);
    g[u] = tl + pos[u];
    id[u] = v[u] ? span_id[g[u]] : 0ull;
    pid[u] = v[u] ? parent[g[u]] : 0ull;
    sf[u] = v[u] ? svcfl[g[u]] : 0u;
    dr[u] = v[u] ? dur[g[u]] : 0u;
    psv[u] = 0xFFFFFFFFu;
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (!v[u] || id[u] == 0ull) continue;
    uint32_t r = big_region_slot(id[u], rs[u]);
    while (true) {
      const uint32_t sl = rb[u] + r;
      const unsigned long long prev = atomicCAS(&bkey[sl], 0ull, (unsigned long long)id[u]);
      if (prev == 0ull || prev == id[u]) {
        atomicMin(&bval[sl], (pos[u] << 16) | (sf[u] & 0xFFFFu));  // the first position wins
        break;
      }
      r = r + 1u == rs[u] ? 0u : r + 1u;
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (!v[u] || pid[u] == 0ull) continue;
    uint32_t r = big_region_slot(pid[u], rs[u]);
    for (uint32_t probe = 0; probe < rs[u]; ++probe) {
      const unsigned long long key = bkey[rb[u] + r];
      if (key == pid[u]) {
        psv[u] = bval[rb[u] + r] & 0xFFFFu;
        break;
      }
      if (key == 0ull) break;
      r = r + 1u == rs[u] ? 0u : r + 1u;
    }
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (!v[u]) continue;
    const uint32_t p = pid[u] == 0ull ? S : psv[u] == 0xFFFFFFFFu ? S + 1u : psv[u];
    const uint32_t edge = p * S + (sf[u] & 0xFFFFu);
    if constexpr (HT == kHtKeys) {
      tab.keys[g[u]] = ((unsigned long long)edge << 32) | dr[u];
    } else {
      record<HT, ST>(smem, edge, dr[u], sf[u] >> 16, tab);
    }
  }
  __syncthreads();  // every lookup done before the clear
  for (uint32_t k = tid; k < 2u * tot; k += kBigThreads) {
    bkey[k] = 0ull;
    bval[k] = 0xFFFFFFFFu;
  }
  __syncthreads();
}

template <int HT, int ST>
__global__ __launch_bounds__(kBigThreads) void edge_big_kernel(
    const uint64_t* __restrict__ span_id, const uint64_t* __restrict__ parent,
    const uint32_t* __restrict__ svcfl, const uint32_t* __restrict__ dur,
    const uint64_t* __restrict__ trace_ptr, uint32_t S, uint32_t E, Table tab) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[kBigLdsBytes];
  __shared__ unsigned long long s_g[kGroup][2];  // the current group: first span, length (0: none)
  auto* bkey = reinterpret_cast<unsigned long long*>(smem + kOffBigKey);  // 0 = empty (id 0 is never a parent ref)
  auto* bval = reinterpret_cast<uint32_t*>(smem + kOffBigPos);  // (first position) << 16 | svc
  const int tid = threadIdx.x;
  const uint64_t nbig = tab.big[0];
  if (nbig == 0) return;
  tables_init<HT, ST>(smem, E, tid);
  for (uint32_t k = tid; k < kBigSlots; k += kBigThreads) {
    bkey[k] = 0ull;
    bval[k] = 0xFFFFFFFFu;
  }
  // Wave 0 keeps the NEXT group of kGroup traces in flight (one ticket, the
  // list entries and bounds loaded by lanes 0..kGroup-1 together) while the
  // workgroup works on the current one.
  unsigned long long nlo = 0, nL = 0;
  auto fetch = [&]() {
    unsigned long long j = 0;
    if (tid == 0) j = atomicAdd(&tab.big[1], (unsigned long long)kGroup);
    j = __shfl(j, 0);
    nlo = nL = 0;
    if (tid < kGroup && j + tid < nbig) {
      const uint64_t t = tab.big_list[j + tid];
      nlo = trace_ptr[t];
      nL = trace_ptr[t + 1] - nlo;
    }
  };
  if (tid < kWave) fetch();
  while (true) {
    __syncthreads();  // the previous group is done with s_g
    if (tid < kGroup) {
      s_g[tid][0] = nlo;
      s_g[tid][1] = nL;
    }
    __syncthreads();
    uint64_t glo[kGroup], gL[kGroup];
    bool any = false;
#pragma unroll
    for (int k = 0; k < kGroup; ++k) {
      glo[k] = s_g[k][0];
      gL[k] = s_g[k][1];
      any |= gL[k] != 0;
    }
    if (!any) break;  // tickets exhausted (listed traces are never empty)
    if (tid < kWave) fetch();  // next group, overlapping this one's work
    // greedy in order: a trace longer than a window alone, else as many
    // consecutive ones as one window holds (group entries addressed by
    // compile-time indices only: the arrays stay in registers)
    uint32_t left = 0;
#pragma unroll
    for (int q = 0; q < kGroup; ++q) left |= (gL[q] != 0 ? 1u : 0u) << q;
    while (left) {
      const int k = __ffs(left) - 1;
      uint64_t lk = 0, Lk = 0;
#pragma unroll
      for (int q = 0; q < kGroup; ++q)
        if (q == k) {
          lk = glo[q];
          Lk = gL[q];
        }
      if (Lk > kBigWin) {
        big_one<HT, ST>(smem, span_id, parent, svcfl, dur, lk, Lk, S, tab);
        left &= ~(1u << k);
        continue;
      }
      uint32_t bm = 0;
      uint64_t tot = 0;
#pragma unroll
      for (int q = 0; q < kGroup; ++q) {
        const bool chain = q == k || (q > 0 && ((bm >> (q - 1)) & 1u));
        if (q >= k && chain && ((left >> q) & 1u) && gL[q] <= kBigWin && tot + gL[q] <= kBigWin) {
          bm |= 1u << q;
          tot += gL[q];
        }
      }
      big_batch<HT, ST>(smem, span_id, parent, svcfl, dur, glo, gL, bm, S, tab);
      left &= ~bm;
    }
  }
  __syncthreads();
  tables_flush<HT, ST>(smem, E, tab, tid);
}

// ---- long-trace pass, r03: resolve, then record ----------------------------
// The pass above holds the histogram / stats tables AND the id table in one
// workgroup's LDS, so a CU runs one workgroup and every batch's column loads,
// inserts, lookups and records follow each other with nothing to hide their
// latency (LONG at 2^23 traces: 3.74 ms for 1.3e8 listed spans).  Split:
// edge_big_resolve_kernel keeps only the id table (48 KiB: three 512-thread
// workgroups per CU) and writes every listed span's parent row — or, in the
// exact-quantile mode, its key — and edge_big_record_kernel streams the
// listed spans (16 traces per ticket, one load round trip per ticket) into
// the chunk walk's tables.  Same first-match rule, same table forms.
#ifndef ANOMOD_RES_THREADS
#define ANOMOD_RES_THREADS 512
#endif
constexpr int kResThreads = ANOMOD_RES_THREADS;
#ifndef ANOMOD_RES_WIN
#define ANOMOD_RES_WIN 2048
#endif
constexpr uint32_t kResWin = ANOMOD_RES_WIN;       // ids per table window
constexpr uint32_t kResSlots = 2 * kResWin;        // load <= 1/2
static_assert((kResSlots & (kResSlots - 1)) == 0, "power-of-two table");
__device__ __forceinline__ uint32_t res_slot(uint64_t id) {
  return (uint32_t)((id * 0x9E3779B97F4A7C15ull) >> 32) & (kResSlots - 1u);
}
constexpr int kResPer = (int)kResWin / kResThreads;  // spans per thread in a packed window
static_assert(kResWin % kResThreads == 0 && kResWin <= 65536, "window: whole rows, pos << 16 | svc");

__device__ __forceinline__ void res_out(const Table& tab, uint64_t g, uint32_t p, uint32_t sf,
                                        uint32_t dr, uint32_t S) {
  if (tab.keys)
    tab.keys[g] = ((unsigned long long)(p * S + (sf & 0xFFFFu)) << 32) | dr;
  else
    tab.bpar[g] = (uint16_t)p;
}

// One trace longer than a window: blocks of kResThreads * kBigPer spans,
// each looked up against the trace's id windows in order.
__device__ void res_one(unsigned long long* bkey, uint32_t* bval,
                        const uint64_t* __restrict__ span_id, const uint64_t* __restrict__ parent,
                        const uint32_t* __restrict__ svcfl, const uint32_t* __restrict__ dur,
                        uint64_t lo, uint64_t L, uint32_t S, const Table& tab) {
  const int tid = threadIdx.x;
  for (uint64_t b0 = 0; b0 < L; b0 += (uint64_t)kResThreads * kBigPer) {
    uint64_t pid[kBigPer];
    uint32_t psv[kBigPer];  // ~0: not found yet
    bool need = false;
#pragma unroll
    for (int r = 0; r < kBigPer; ++r) {
      const uint64_t i = b0 + (uint64_t)r * kResThreads + tid;
      pid[r] = i < L ? parent[lo + i] : 0ull;
      psv[r] = 0xFFFFFFFFu;
      need |= pid[r] != 0ull;
    }
    for (uint64_t w0 = 0; w0 < L; w0 += kResWin) {
      if (!__syncthreads_or(need)) break;  // also orders the previous clear
#pragma unroll
      for (int u = 0; u < kResPer; ++u) {
        const uint32_t k = (uint32_t)(u * kResThreads + tid);
        const uint64_t id = w0 + k < L ? span_id[lo + w0 + k] : 0ull;
        if (id == 0ull) continue;
        const uint32_t sv = svcfl[lo + w0 + k] & 0xFFFFu;
        for (uint32_t sl = res_slot(id);; sl = (sl + 1u) & (kResSlots - 1u)) {
          const unsigned long long prev = atomicCAS(&bkey[sl], 0ull, (unsigned long long)id);
          if (prev == 0ull || prev == id) {
            atomicMin(&bval[sl], (k << 16) | sv);  // the first position wins, with its service
            break;
          }
        }
      }
      __syncthreads();
      need = false;
#pragma unroll
      for (int r = 0; r < kBigPer; ++r) {
        if (pid[r] == 0ull || psv[r] != 0xFFFFFFFFu) continue;
        for (uint32_t sl = res_slot(pid[r]);; sl = (sl + 1u) & (kResSlots - 1u)) {
          const unsigned long long key = bkey[sl];
          if (key == pid[r]) {
            psv[r] = bval[sl] & 0xFFFFu;
            break;
          }
          if (key == 0ull) break;
        }
        need |= psv[r] == 0xFFFFFFFFu;
      }
      __syncthreads();
      for (uint32_t k = tid; k < kResSlots; k += kResThreads) {
        bkey[k] = 0ull;
        bval[k] = 0xFFFFFFFFu;
      }
    }
#pragma unroll
    for (int r = 0; r < kBigPer; ++r) {
      const uint64_t i = b0 + (uint64_t)r * kResThreads + tid;
      if (i >= L) continue;
      const uint32_t p = pid[r] == 0ull ? S : psv[r] == 0xFFFFFFFFu ? S + 1u : psv[r];
      res_out(tab, lo + i, p, tab.keys ? svcfl[lo + i] : 0u, tab.keys ? dur[lo + i] : 0u, S);
    }
  }
  __syncthreads();  // the last window's clear before the next user of the table
}

// Up to kGroup traces (bm) packed into one window, each in a private table
// region [2 off_i, 2 off_i + 2 L_i), as big_batch.
__device__ void res_batch(unsigned long long* bkey, uint32_t* bval,
                          const uint64_t* __restrict__ span_id, const uint64_t* __restrict__ parent,
                          const uint32_t* __restrict__ svcfl, const uint32_t* __restrict__ dur,
                          const uint64_t (&lo)[kGroup], const uint64_t (&L)[kGroup], uint32_t bm,
                          uint32_t S, const Table& tab) {
  const int tid = threadIdx.x;
  uint32_t off[kGroup + 1];
  off[0] = 0;
#pragma unroll
  for (int i = 0; i < kGroup; ++i) off[i + 1] = off[i] + (((bm >> i) & 1u) ? (uint32_t)L[i] : 0u);
  const uint32_t tot = off[kGroup];
  uint64_t id[kResPer], pid[kResPer], g[kResPer];
  uint32_t sv[kResPer], rb[kResPer], rs[kResPer], pos[kResPer];
  bool v[kResPer];
#pragma unroll
  for (int u = 0; u < kResPer; ++u) {
    const uint32_t q = (uint32_t)(u * kResThreads + tid);
    v[u] = q < tot;
    uint32_t a0 = 0, a1 = off[1];
    uint64_t tl = lo[0];
#pragma unroll
    for (int i = 1; i < kGroup; ++i)
      if (q >= off[i] && ((bm >> i) & 1u)) {
        a0 = off[i];
        a1 = off[i + 1];
        tl = lo[i];
      }
    pos[u] = q - a0;
    rb[u] = 2u * a0;
    rs[u] = 2u * (a1 - a0);
    g[u] = tl + pos[u];
    id[u] = v[u] ? span_id[g[u]] : 0ull;
    pid[u] = v[u] ? parent[g[u]] : 0ull;
    sv[u] = v[u] ? svcfl[g[u]] & 0xFFFFu : 0u;
  }
#pragma unroll
  for (int u = 0; u < kResPer; ++u) {
    if (!v[u] || id[u] == 0ull) continue;
    uint32_t r = big_region_slot(id[u], rs[u]);
    while (true) {
      const uint32_t sl = rb[u] + r;
      const unsigned long long prev = atomicCAS(&bkey[sl], 0ull, (unsigned long long)id[u]);
      if (prev == 0ull || prev == id[u]) {
        atomicMin(&bval[sl], (pos[u] << 16) | sv[u]);  // the first position wins
        break;
      }
      r = r + 1u == rs[u] ? 0u : r + 1u;
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kResPer; ++u) {
    if (!v[u]) continue;
    uint32_t psv = 0xFFFFFFFFu;
    if (pid[u] != 0ull) {
      uint32_t r = big_region_slot(pid[u], rs[u]);
      for (uint32_t probe = 0; probe < rs[u]; ++probe) {
        const unsigned long long key = bkey[rb[u] + r];
        if (key == pid[u]) {
          psv = bval[rb[u] + r] & 0xFFFFu;
          break;
        }
        if (key == 0ull) break;
        r = r + 1u == rs[u] ? 0u : r + 1u;
      }
    }
    const uint32_t p = pid[u] == 0ull ? S : psv == 0xFFFFFFFFu ? S + 1u : psv;
    res_out(tab, g[u], p, tab.keys ? svcfl[g[u]] : 0u, tab.keys ? dur[g[u]] : 0u, S);
  }
  __syncthreads();  // every lookup done before the clear
  for (uint32_t k = tid; k < 2u * tot; k += kResThreads) {
    bkey[k] = 0ull;
    bval[k] = 0xFFFFFFFFu;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kResThreads, ANOMOD_RES_MINB) void edge_big_resolve_kernel(
    const uint64_t* __restrict__ span_id, const uint64_t* __restrict__ parent,
    const uint32_t* __restrict__ svcfl, const uint32_t* __restrict__ dur,
    const uint64_t* __restrict__ trace_ptr, uint32_t S, Table tab) {
  __shared__ unsigned long long bkey[kResSlots];  // 0 = empty (id 0 is never a parent ref)
  __shared__ uint32_t bval[kResSlots];            // (first position) << 16 | svc
  __shared__ unsigned long long s_g[kGroup][2];
  const int tid = threadIdx.x;
  const uint64_t nbig = tab.big[0];
  if (nbig == 0) return;
  for (uint32_t k = tid; k < kResSlots; k += kResThreads) {
    bkey[k] = 0ull;
    bval[k] = 0xFFFFFFFFu;
  }
  unsigned long long nlo = 0, nL = 0;
  auto fetch = [&]() {
    unsigned long long j = 0;
    if (tid == 0) j = atomicAdd(&tab.big[1], (unsigned long long)kGroup);
    j = __shfl(j, 0);
    nlo = nL = 0;
    if (tid < kGroup && j + tid < nbig) {
      const uint64_t t = tab.big_list[j + tid];
      nlo = trace_ptr[t];
      nL = trace_ptr[t + 1] - nlo;
    }
  };
  if (tid < kWave) fetch();
  while (true) {
    __syncthreads();
    if (tid < kGroup) {
      s_g[tid][0] = nlo;
      s_g[tid][1] = nL;
    }
    __syncthreads();
    uint64_t glo[kGroup], gL[kGroup];
    bool any = false;
#pragma unroll
    for (int k = 0; k < kGroup; ++k) {
      glo[k] = s_g[k][0];
      gL[k] = s_g[k][1];
      any |= gL[k] != 0;
    }
    if (!any) break;
    if (tid < kWave) fetch();
    uint32_t left = 0;
#pragma unroll
    for (int q = 0; q < kGroup; ++q) left |= (gL[q] != 0 ? 1u : 0u) << q;
    while (left) {
      const int k = __ffs(left) - 1;
      uint64_t lk = 0, Lk = 0;
#pragma unroll
      for (int q = 0; q < kGroup; ++q)
        if (q == k) {
          lk = glo[q];
          Lk = gL[q];
        }
      if (Lk > kResWin) {
        res_one(bkey, bval, span_id, parent, svcfl, dur, lk, Lk, S, tab);
        left &= ~(1u << k);
        continue;
      }
      uint32_t bm = 0;
      uint64_t tot = 0;
#pragma unroll
      for (int q = 0; q < kGroup; ++q) {
        const bool chain = q == k || (q > 0 && ((bm >> (q - 1)) & 1u));
        if (q >= k && chain && ((left >> q) & 1u) && gL[q] <= kResWin && tot + gL[q] <= kResWin) {
          bm |= 1u << q;
          tot += gL[q];
        }
      }
      res_batch(bkey, bval, span_id, parent, svcfl, dur, glo, gL, bm, S, tab);
      left &= ~bm;
    }
  }
}

// The listed spans into the tables, kRecGroup traces per ticket (wave 0 keeps
// the next ticket's entries and bounds in flight).
constexpr int kRecGroup = 16;
#ifndef ANOMOD_REC_PER
#define ANOMOD_REC_PER 4
#endif
constexpr int kRecPer = ANOMOD_REC_PER;  // listed spans per thread loaded together
template <int HT, int ST>
__global__ __launch_bounds__(kBigThreads) void edge_big_record_kernel(
    const uint32_t* __restrict__ svcfl, const uint32_t* __restrict__ dur,
    const uint64_t* __restrict__ trace_ptr, uint32_t S, uint32_t E, Table tab) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[kOffWave];
  __shared__ unsigned long long s_lo[kRecGroup];
  __shared__ uint32_t s_off[kRecGroup + 1];
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const uint64_t nbig = tab.big[0];
  if (nbig == 0) return;
  tables_init<HT, ST>(smem, E, tid);
  unsigned long long nlo = 0;
  uint32_t nL = 0;
  auto fetch = [&]() {
    unsigned long long j = 0;
    if (lane == 0) j = atomicAdd(&tab.big[2], (unsigned long long)kRecGroup);
    j = __shfl(j, 0);
    nlo = 0;
    nL = 0;
    if (lane < kRecGroup && j + lane < nbig) {
      const uint64_t t = tab.big_list[j + lane];
      nlo = trace_ptr[t];
      nL = (uint32_t)(trace_ptr[t + 1] - nlo);
    }
  };
  if (tid < kWave) fetch();
  while (true) {
    __syncthreads();  // the previous ticket is done with s_lo / s_off
    if (tid < kWave) {
      uint32_t inc = nL;  // inclusive scan over the ticket's traces
#pragma unroll
      for (int o = 1; o < kRecGroup; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
      }
      if (lane < kRecGroup) {
        s_lo[lane] = nlo;
        s_off[lane + 1] = inc;
      }
      if (lane == 0) s_off[0] = 0;
      fetch();  // the next ticket, overlapping this one's work
    }
    __syncthreads();
    const uint32_t tot = s_off[kRecGroup];
    if (tot == 0) break;  // tickets exhausted (listed traces are never empty)
    // the ticket's trace offsets in scalar registers (uniform; read once, not
    // per span)
    uint32_t off[kRecGroup];
#pragma unroll
    for (int i = 0; i < kRecGroup; ++i) off[i] = __builtin_amdgcn_readfirstlane(s_off[i]);
    // kRecPer spans per thread loaded together, then recorded (the records'
    // LDS / HBM atomics would otherwise keep the next loads behind them)
    for (uint32_t q0 = tid; q0 < tot; q0 += kRecPer * kBigThreads) {
      uint32_t sf[kRecPer], dr[kRecPer], pr[kRecPer];
#pragma unroll
      for (int j = 0; j < kRecPer; ++j) {
        const uint32_t q = q0 + (uint32_t)j * kBigThreads;
        int t = 0;
        uint32_t base = 0;
#pragma unroll
        for (int i = 1; i < kRecGroup; ++i) {
          const bool in = q >= off[i];
          t = in ? i : t;
          base = in ? off[i] : base;
        }
        const uint64_t g = s_lo[t] + (q - base);
        const bool v = q < tot;
        sf[j] = v ? svcfl[g] : 0u;
        dr[j] = v ? dur[g] : 0u;
        pr[j] = v ? tab.bpar[g] : 0xFFFFu;
      }
#pragma unroll
      for (int j = 0; j < kRecPer; ++j)
        if (pr[j] != 0xFFFFu) record<HT, ST>(smem, pr[j] * S + (sf[j] & 0xFFFFu), dr[j], sf[j] >> 16, tab);
    }
  }
  __syncthreads();
  tables_flush<HT, ST>(smem, E, tab, tid);
}

template <int HT, int ST, bool UNI, int MODE = kModeNormal>
__global__ __launch_bounds__(kThreads) void edge_agg_kernel(
    const uint64_t* __restrict__ span_id, const uint64_t* __restrict__ parent,
    const uint32_t* __restrict__ svcfl, const uint32_t* __restrict__ dur,
    const uint64_t* __restrict__ trace_ptr, uint64_t n_traces, uint32_t S, uint32_t E, Table tab) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[kLdsBytes];
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wid = tid / kWave;
  const Cols col{span_id, parent, svcfl, dur};
#ifndef ANOMOD_DYN
#define ANOMOD_DYN 4
#endif
  // Static share: the first n_static traces split evenly over the waves; with
  // ANOMOD_DYN = d > 0 the last 1/d of the traces are handed out in segments
  // of kDynSeg from a global counter, so waves that finish early take the tail.
#ifndef ANOMOD_DYN_SEG
#define ANOMOD_DYN_SEG 512
#endif
  constexpr uint64_t kDynSeg = ANOMOD_DYN_SEG;
  const uint64_t n_static = ANOMOD_DYN ? n_traces - n_traces / (ANOMOD_DYN ? ANOMOD_DYN : 1) : n_traces;
  // Resume launch (compact form) after a kModeAuto launch: the trace ranges
  // its stopped waves left, then the rest of the dynamic tail.  Nothing left
  // (no workgroup saturated): return before touching LDS.
  constexpr bool resume = MODE == kModeResume;
  const uint64_t n_left = resume ? tab.nleft[0] : 0;
  if (resume && n_left == 0 && n_static + *tab.ctr >= n_traces) return;

  tables_init<HT, ST>(smem, E, tid);
  __syncthreads();

  unsigned char* wsm = smem + kOffWave + wid * kWBytes;
  const uint64_t gw = (uint64_t)blockIdx.x * kWavesPerWG + wid;
  const uint64_t nw = (uint64_t)gridDim.x * kWavesPerWG;
  uint64_t t_begin = uniform64(n_static * gw / nw);
  uint64_t t_end = uniform64(n_static * (gw + 1) / nw);
  bool from_left = resume;
  auto next_left = [&]() {  // the next range a stopped wave left (false: none)
    unsigned long long j = 0;
    if (lane == 0) j = atomicAdd(&tab.nleft[1], 1ull);
    j = uniform64(__shfl(j, 0));
    if (j >= n_left) return false;
    t_begin = uniform64(tab.left[2 * j]);
    t_end = uniform64(tab.left[2 * j + 1]);
    return true;
  };
  if (resume && !next_left()) {
    from_left = false;
    t_begin = t_end = 0;
  }
  bool stopped = false;
  uint32_t* ctl = reinterpret_cast<uint32_t*>(smem + kOffCtl);

  while (true) {
  if (t_begin < t_end) {
    // Pipeline: the bounds of chunk c+2 and the span columns of chunk c+1 are
    // in flight while chunk c is resolved and recorded.
    uint64_t lo, hi;
    load_bounds(trace_ptr, t_begin, t_end, lane, lo, hi);
    Chunk cur = make_chunk(t_begin, t_end, lane, lo, hi, kBigMin);
    Regs R;
    load_regs(col, cur, lane, R);
    // kModeAuto: the first trace of the current chunk lives in the wave's LDS
    // word, not a register (a register more spilled the auto form's loop: 16 /
    // 48 B per lane, 12 % / 40 % slower than the pair form on SN / shuffled SN)
    uint64_t* wt_cur = reinterpret_cast<uint64_t*>(wsm + kWAuto);
    if (MODE == kModeAuto && lane == 0) *wt_cur = t_begin;
    uint64_t t_cur = t_begin;  // (other modes: a register)
    uint64_t t_next = t_begin + (cur.k ? cur.k : 1u);
    load_bounds(trace_ptr, t_next, t_end, lane, lo, hi);
    while (true) {
      // A first aggregation (kModeAuto) whose pair table saturated: leave
      // [first trace of the chunk, t_end) to the compact-form resume launch
      // and stop.
      if (MODE == kModeAuto &&
          (uint32_t)__builtin_amdgcn_readfirstlane(
              __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) >=
              kSatFails) {
        if (lane == 0) {
          const unsigned long long j = atomicAdd(&tab.nleft[0], 1ull);
          tab.left[2 * j] = *wt_cur;
          tab.left[2 * j + 1] = t_end;
        }
        stopped = true;
        break;
      }
      const bool has_next = t_next < t_end;
      const uint64_t t_nxt = t_next;
      if (MODE == kModeAuto && lane == 0 && has_next) wt_cur[1] = t_next;  // the next chunk's
      Chunk nxt{};
      Regs Rn;
      if (has_next) {
        nxt = make_chunk(t_next, t_end, lane, lo, hi, kBigMin);
        load_regs(col, nxt, lane, Rn);
        t_next += nxt.k ? nxt.k : 1u;
        load_bounds(trace_ptr, t_next, t_end, lane, lo, hi);
      }
      if (cur.k == 0) {  // a trace longer than kStage: listed for edge_big_kernel
        if (lane == 0)
          tab.big_list[atomicAdd(&tab.big[0], 1ull)] =
              tab.t_base + (MODE == kModeAuto ? *wt_cur : t_cur);
      } else {
        process_chunk<HT, ST, UNI, MODE == kModeWideScan>(smem, wsm, lane, cur, R, S, tab);
      }
      if (!has_next) break;
      cur = nxt;
      if (MODE == kModeAuto) {
        if (lane == 0) wt_cur[0] = wt_cur[1];
      } else {
        t_cur = t_nxt;
      }
      R = Rn;
    }
  }
  if (stopped) break;
  if (from_left) {
    if (next_left()) continue;
    from_left = false;
  }
  if (!ANOMOD_DYN || n_static == n_traces) break;
  unsigned long long g = 0;
  if (lane == 0) g = atomicAdd(tab.ctr, (unsigned long long)kDynSeg);
  g = __shfl(g, 0);
  t_begin = uniform64(n_static + g);
  if (t_begin >= n_traces) break;
  t_end = uniform64(t_begin + kDynSeg < n_traces ? t_begin + kDynSeg : n_traces);
  }
  __syncthreads();

  tables_flush<HT, ST>(smem, E, tab, tid);
}

// Edge records (the fused ungrouped aggregation, bucket.hip): one 8-B record
// per span — (parent row * S + service) << 33 | error << 32 | duration — into
// the chunk walk's LDS table forms.  A plain stream: 8 records per thread
// loaded together, then recorded.  The compact form also reports its largest
// workgroup occupancy (tab.ovf[1], atomic max), so a set learns whether the
// pair table would hold it.
constexpr int kRecLoad = 8;
template <int HT, int ST>
__global__ __launch_bounds__(kThreads) void edge_rec_kernel(const uint64_t* __restrict__ rec,
                                                            uint64_t n, uint32_t E, Table tab) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[kOffWave];
  const int tid = threadIdx.x;
  tables_init<HT, ST>(smem, E, tid);
  __syncthreads();
  constexpr uint64_t kPerBlock = (uint64_t)kThreads * kRecLoad;
  for (uint64_t b0 = (uint64_t)blockIdx.x * kPerBlock; b0 < n; b0 += (uint64_t)gridDim.x * kPerBlock) {
    uint64_t x[kRecLoad];
#pragma unroll
    for (int j = 0; j < kRecLoad; ++j) {
      const uint64_t i = b0 + (uint64_t)(j * kThreads + tid);
      x[j] = i < n ? rec[i] : ~0ull;
    }
#pragma unroll
    for (int j = 0; j < kRecLoad; ++j)
      if (x[j] != ~0ull)
        record<HT, ST>(smem, (uint32_t)(x[j] >> 33), (uint32_t)x[j],
                       ((x[j] >> 32) & 1ull) ? ANOMOD_FLAG_ERROR : 0u, tab);
  }
  __syncthreads();
  tables_flush<HT, ST>(smem, E, tab, tid);  // (the caller sets tab.occupancy)
}

// Count + nearest-rank quantiles per edge from the merged histogram: one
// wave per edge, 14 contiguous bins per lane, wave prefix sum.
constexpr int kBinsPerLane = (kBins + kWave - 1) / kWave;

__device__ __forceinline__ double quantile_from(uint64_t r, uint64_t excl, uint64_t incl,
                                                const uint64_t* v, int lane) {
  // Called only by the lane whose [excl, incl) contains r.
  uint64_t c = excl;
  for (int j = 0; j < kBinsPerLane; ++j) {
    c += v[j];
    if (r < c) {
      uint32_t lo, hi;
      hist_bounds((uint32_t)(lane * kBinsPerLane + j), &lo, &hi);
      return 0.5 * ((double)lo + (double)hi);
    }
  }
  return 0.0;
}

// Clears the table before a launch: words [0, nz) to zero (hist | err | sum |
// mx | ctr | big) and the E minima to all ones.  One launch in place of two
// memsets, which the runtime splits into several fill kernels (~40 us of
// launches per aggregation, against ~4 us for this).
__global__ __launch_bounds__(256) void edge_table_init_kernel(unsigned long long* __restrict__ z,
                                                              uint64_t nz,
                                                              unsigned int* __restrict__ mn,
                                                              uint32_t E) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint4* z4 = reinterpret_cast<uint4*>(z);  // the table base is 256-B aligned
  for (uint64_t i = i0; i < nz / 2; i += stride) z4[i] = make_uint4(0u, 0u, 0u, 0u);
  if ((nz & 1u) && i0 == 0) z[nz - 1] = 0ull;
  for (uint64_t i = i0; i < E; i += stride) mn[i] = 0xFFFFFFFFu;
}

__global__ __launch_bounds__(kWave) void edge_finalize_kernel(Table tab,
                                                              unsigned long long* count,
                                                              double* p50, double* p99) {
  const uint32_t e = blockIdx.x;
  const int lane = threadIdx.x;
  const unsigned long long* h = tab.hist + (uint64_t)e * kBins;
  uint64_t v[kBinsPerLane];
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < kBinsPerLane; ++j) {
    const int b = lane * kBinsPerLane + j;
    v[j] = (b < (int)kBins) ? h[b] : 0ull;
    s += v[j];
  }
  uint64_t incl = s;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const uint64_t y = __shfl_up(incl, off);
    if (lane >= off) incl += y;
  }
  const uint64_t total = __shfl(incl, kWave - 1);
  const uint64_t excl = incl - s;
  if (lane == 0) {
    count[e] = total;
    if (total == 0) {
      p50[e] = NAN;
      p99[e] = NAN;
    }
  }
  if (total == 0) return;
  const uint64_t r50 = total * 50ull / 100ull;
  const uint64_t r99 = total * 99ull / 100ull;
  if (r50 >= excl && r50 < incl) p50[e] = quantile_from(r50, excl, incl, v, lane);
  if (r99 >= excl && r99 < incl) p99[e] = quantile_from(r99, excl, incl, v, lane);
}

// Exact nearest-rank picks from the per-span keys sorted by (edge, dur): one
// thread per edge finds its segment by binary search and reads
// x[(c * q) // 100] (the reference's sorted(x)[int(c*q)],
// monitor_http_responses.py:180-190).
__global__ __launch_bounds__(256) void exact_pick_kernel(const unsigned long long* __restrict__ sk,
                                                         uint64_t n, uint32_t E,
                                                         const uint32_t* __restrict__ q_pct,
                                                         uint32_t nq, double* __restrict__ out,
                                                         unsigned long long* __restrict__ count) {
  const uint32_t e = blockIdx.x * 256u + threadIdx.x;
  if (e >= E) return;
  auto lower = [&](unsigned long long key) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) / 2;
      if (sk[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
  };
  const uint64_t a = lower((unsigned long long)e << 32);
  const uint64_t b = lower((unsigned long long)(e + 1u) << 32);
  const uint64_t c = b - a;
  if (count) count[e] = c;
  // the reference's int(c * q) with q = q_pct / 100 as a double (the same
  // double as the literal 0.95, ...: IEEE division rounds correctly), the
  // product truncated as Python's int() does (monitor_http_responses.py:
  // 188-189; x[len // 2] at :186 is the same index for q = 50)
  for (uint32_t k = 0; k < nq; ++k)
    out[(uint64_t)e * nq + k] =
        c ? (double)(uint32_t)sk[a + (uint64_t)((double)c * ((double)q_pct[k] / 100.0))]
          : (double)NAN;
}

using KernelFn = void (*)(const uint64_t*, const uint64_t*, const uint32_t*, const uint32_t*,
                          const uint64_t*, uint64_t, uint32_t, uint32_t, Table);
using KernelFn1 = void (*)(const uint64_t*, uint64_t, uint32_t, Table);

// The histogram form a set asks for: 0 pair, 1 compact, -1 unknown (pair with
// the saturation hand-off to a compact resume launch) — its hint, or
// ANOMOD_HIST_FORM = pair / compact / auto (tests force each).
// ANOMOD_HIST_FORM=auto: a form-unknown set takes the r04 auto form (pair
// table, saturated workgroups resumed compact) instead of the probe.
bool auto_forced() {
  const char* f = getenv("ANOMOD_HIST_FORM");
  return f && !strcmp(f, "auto");
}

// The form probe of a first aggregation: spans it covers, workgroups it runs.
constexpr uint64_t kFormProbeSpans = 1ull << 19;
constexpr uint64_t kFormProbeGroups = 16;

int hist_form_of(const anomod_spans* s) {
  const char* f = getenv("ANOMOD_HIST_FORM");
  if (f && !strcmp(f, "compact")) return 1;
  if (f && !strcmp(f, "pair")) return 0;
  if (f && !strcmp(f, "auto")) return -1;
  return s->hist_form;
}

// Collector-order probe of a unique-id set: over its first kProbeSpans spans,
// the share of child spans whose parent is the span right before them
// (0.60-0.75 on the generators in collector order, 0.02-0.11 shuffled inside
// the traces; a pair across a trace boundary matches only by id collision).
constexpr uint64_t kProbeSpans = 1u << 20;
__global__ __launch_bounds__(256) void order_probe_kernel(const uint64_t* __restrict__ sid,
                                                          const uint64_t* __restrict__ pid,
                                                          uint64_t n,
                                                          unsigned long long* __restrict__ cnt) {
  uint32_t ch = 0, adj = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x + 1; i < n;
       i += (uint64_t)gridDim.x * 256) {
    const uint64_t p = pid[i];
    ch += p != 0ull ? 1u : 0u;
    adj += (p != 0ull && p == sid[i - 1]) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) {
    ch += __shfl_xor(ch, o);
    adj += __shfl_xor(adj, o);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&cnt[0], (unsigned long long)ch);
    atomicAdd(&cnt[1], (unsigned long long)adj);
  }
}

// The set's order probe when its order hint is unknown (the first
// aggregation of a unique-id set): the counts go to h[0..1] (pinned) once the
// caller waits; probe_order_take sets the hint from them.
bool need_order_probe(const anomod_spans* s) { return s->unique_ids && s->order < 0; }

int probe_order_launch(anomod_ctx* ctx, const anomod_spans* s, unsigned long long* d_cnt,
                       unsigned long long* h) {
  h[0] = h[1] = 0ull;
  const uint64_t n = std::min<uint64_t>(s->n_spans, kProbeSpans);
  if (n > 1) {
    ANOMOD_HIP(ctx, hipMemsetAsync(d_cnt, 0, 16, ctx->stream));
    hipLaunchKernelGGL(order_probe_kernel, dim3((unsigned)std::min<uint64_t>((n + 255) / 256, 256)),
                       dim3(256), 0, ctx->stream, s->span_id, s->parent_span_id, n, d_cnt);
    ANOMOD_HIP(ctx, hipGetLastError());
    ANOMOD_HIP(ctx, hipMemcpyAsync(h, d_cnt, 16, hipMemcpyDeviceToHost, ctx->stream));
  }
  return ANOMOD_OK;
}

void probe_order_take(const anomod_spans* s, const unsigned long long* h) {
  s->order = 4ull * h[1] >= h[0] ? 1 : 0;
}

// Sets the set's order hint when unknown (one small kernel and one host
// wait, the first aggregation of the set only).
int probe_order(anomod_ctx* ctx, const anomod_spans* s, unsigned long long* d_cnt) {
  if (!need_order_probe(s)) return ANOMOD_OK;
  // the pinned read-back (a ctx's first call may be this one: the exact
  // quantiles allocate no staging of their own)
  if (int rc = ensure_host_stage(ctx, 32)) return rc;
  unsigned long long* h = static_cast<unsigned long long*>(ctx->h_stage);
  if (int rc = probe_order_launch(ctx, s, d_cnt, h)) return rc;
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  probe_order_take(s, h);
  return ANOMOD_OK;
}

// Whether the bidirectional parent scan is used: a unique-id set in collector
// order (ANOMOD_UNIQUE_SCAN=0 forces the forward scan, =1 the bidirectional
// one whatever the order: tests, A/B).  Every other set takes the
// first-match forward scan, correct for any set.
bool use_unique(const anomod_spans* s) {
  const char* f = getenv("ANOMOD_UNIQUE_SCAN");
  if (f && !strcmp(f, "0")) return false;
  if (f && !strcmp(f, "1")) return s->unique_ids;
  return s->unique_ids && s->order == 1;
}

struct Pick {
  KernelFn fn;
  int ht, st;
  const char* name;
};

// mode: kModeAuto only for the pair forms, kModeResume only for the compact
// forms of the SN / TrainTicket widths (the instantiations that exist).
Pick pick_kernel(uint32_t E, bool compact, bool uni, int mode = kModeNormal, bool long_set = false) {
  const uint64_t keys = (uint64_t)E * kBins + 1;  // largest stored key
  const bool lds_hist = keys < (1ull << 31);  // >= 1 count bit above the key
#define ANOMOD_PICK(H, S_, NAME)                                                               \
  return Pick{uni ? edge_agg_kernel<H, S_, true> : edge_agg_kernel<H, S_, false>, H, S_, NAME}
#define ANOMOD_PICK_M(H, S_, M, NAME)                                                          \
  return Pick{uni ? edge_agg_kernel<H, S_, true, M> : edge_agg_kernel<H, S_, false, M>, H, S_, NAME}
  if (lds_hist && E <= kLdsEdges && mode == kModeResume)
    ANOMOD_PICK_M(kHtCompact, kStDirect, kModeResume, "edge_agg_kernel<lds_compact_hist,lds_stats,resume>");
  if (lds_hist && E <= kLdsEdges && !compact && mode == kModeAuto)
    ANOMOD_PICK_M(kHtPair, kStDirect, kModeAuto, "edge_agg_kernel<lds_hist,lds_stats,auto>");
  if (lds_hist && E > kLdsEdges && E <= kWideEdges && mode == kModeResume)
    ANOMOD_PICK_M(kHtCompact, kStWide, kModeResume, "edge_agg_kernel<lds_compact_hist,wide_stats,resume>");
  if (lds_hist && E > kLdsEdges && E <= kWideEdges && !compact && mode == kModeAuto)
    ANOMOD_PICK_M(kHtPair, kStWide, kModeAuto, "edge_agg_kernel<lds_hist,wide_stats,auto>");
  if (lds_hist && E <= kLdsEdges && compact && uni && long_set && mode == kModeNormal)
    return Pick{edge_agg_kernel<kHtCompact, kStDirect, true, kModeWideScan>, kHtCompact, kStDirect,
                "edge_agg_kernel<lds_compact_hist,lds_stats,wide_scan>"};
  if (lds_hist && E <= kLdsEdges && compact)  // a set that overflowed the pair table
    ANOMOD_PICK(kHtCompact, kStDirect, "edge_agg_kernel<lds_compact_hist,lds_stats>");
  if (lds_hist && E <= kLdsEdges) ANOMOD_PICK(kHtPair, kStDirect, "edge_agg_kernel<lds_hist,lds_stats>");
  // TrainTicket width: the pair form while the set's keys fit it (whole-ms
  // SkyWalking latencies give a few thousand (edge, bin) keys per
  // workgroup), the compact form once it overflowed
  if (lds_hist && E <= kWideEdges && !compact)
    ANOMOD_PICK(kHtPair, kStWide, "edge_agg_kernel<lds_hist,wide_stats>");
  if (lds_hist && E <= kWideEdges)
    ANOMOD_PICK(kHtCompact, kStWide, "edge_agg_kernel<lds_compact_hist,wide_stats>");
  if (lds_hist) ANOMOD_PICK(kHtCompact, kStSlot, "edge_agg_kernel<lds_compact_hist,slot_stats>");
  ANOMOD_PICK(kHtHbm, kStHbm, "edge_agg_kernel<hbm_hist,hbm_stats>");
#undef ANOMOD_PICK
#undef ANOMOD_PICK_M
}

// Device table layout inside ctx->d_table: hist | err | sum (u64, one sum
// all-reduce) | mx (u32, zero-initialised with them: one memset) | pad |
// ctr (u64) | big counters (u64 x 3) + probe scratch (u64 x 2) | pair-table
// overflows + stopped workgroups (u64 x 2) | ranges left + resume ticket
// (u64 x 2; all zeroed with them) | count | p50 | p99 | mn | long-trace list |
// ranges left by stopped waves (u64 pairs) | long-trace parent rows (u16 per
// span).  [off_err, end_small) is copied to the host in one D2H.
struct Layout {
  uint64_t E;
  size_t off_hist, off_err, off_sum, off_mx, off_ctr, off_big, off_ovf, off_nleft, off_count,
      off_p50, off_p99, off_mn, end_small, off_left, bytes;
  size_t off_bpar = 0;
  Layout(uint64_t e, uint64_t big_cap, uint64_t n_spans = 0, uint64_t left_cap = 0) : E(e) {
    off_hist = 0;
    off_err = off_hist + E * kBins * 8;
    off_sum = off_err + E * 8;
    off_mx = off_sum + E * 8;
    off_ctr = (off_mx + E * 4 + 7) & ~size_t(7);
    off_big = off_ctr + 8;
    off_ovf = off_big + 40;  // listed, two tickets, two words of order-probe scratch
    off_nleft = off_ovf + 16;
    off_count = off_nleft + 16;
    off_p50 = off_count + E * 8;
    off_p99 = off_p50 + E * 8;
    off_mn = off_p99 + E * 8;
    end_small = off_mn + E * 4;
    off_left = ((end_small + 7) & ~size_t(7)) + big_cap * 8;
    bytes = off_left + left_cap * 16;
    off_bpar = bytes;                           // u16 parent rows, by span position
    if (big_cap) bytes += (n_spans * 2 + 7) & ~size_t(7);
  }
  size_t off_list() const { return (end_small + 7) & ~size_t(7); }
};

// Long traces (> kBigMin spans) a span set can hold: 0 when its longest trace
// is known to fit a chunk.
uint64_t big_capacity(const anomod_spans* s) {
  if (s->max_trace_len <= (uint64_t)kBigMin) return 0;
  const uint64_t by_spans = s->n_spans / (uint64_t)(kBigMin + 1);
  return by_spans < s->n_traces ? by_spans : s->n_traces;
}

// The long-trace pass after the chunk walk (no-op when nothing was listed),
// with the chunk walk's table forms.
template <int HT, int ST>
hipError_t launch_big(anomod_ctx* ctx, const anomod_spans* spans, uint32_t S, uint32_t E,
                      const Table& tab) {
  if (ANOMOD_BIG_ONEPASS) {  // the r02 single-kernel pass (A/B)
    hipLaunchKernelGGL((edge_big_kernel<HT, ST>), dim3((unsigned)ctx->num_cus), dim3(kBigThreads),
                       0, ctx->stream, spans->span_id, spans->parent_span_id, spans->svc_flags,
                       spans->dur_us, spans->trace_ptr, S, E, tab);
    return hipGetLastError();
  }
  int per_cu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per_cu, reinterpret_cast<const void*>(edge_big_resolve_kernel), kResThreads, 0);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(edge_big_resolve_kernel, dim3((unsigned)(ctx->num_cus * std::max(per_cu, 1))),
                     dim3(kResThreads), 0, ctx->stream, spans->span_id, spans->parent_span_id,
                     spans->svc_flags, spans->dur_us, spans->trace_ptr, S, tab);
  if ((e = hipGetLastError()) != hipSuccess || HT == kHtKeys) return e;
  hipLaunchKernelGGL((edge_big_record_kernel<HT, ST>), dim3((unsigned)ctx->num_cus),
                     dim3(kBigThreads), 0, ctx->stream, spans->svc_flags, spans->dur_us,
                     spans->trace_ptr, S, E, tab);
  return hipGetLastError();
}

hipError_t launch_big_for(anomod_ctx* ctx, const anomod_spans* spans, uint32_t S, uint32_t E,
                          const Table& tab) {
  // the LDS tables' u32 counters hold < 2^32 records per workgroup: a set
  // whose listed traces could exceed a launch's bound records to HBM
  if (spans->n_spans >= max_launch_spans()) return launch_big<kHtHbm, kStHbm>(ctx, spans, S, E, tab);
  // the pair form only for a set known to fit it (a form-unknown set records
  // its long traces in the compact form, which has no probe chain)
  const Pick pk = pick_kernel(E, hist_form_of(spans) != 0, false);
  if (pk.ht == kHtPair && pk.st == kStDirect)
    return launch_big<kHtPair, kStDirect>(ctx, spans, S, E, tab);
  if (pk.ht == kHtCompact && pk.st == kStDirect)
    return launch_big<kHtCompact, kStDirect>(ctx, spans, S, E, tab);
  if (pk.ht == kHtPair && pk.st == kStWide)
    return launch_big<kHtPair, kStWide>(ctx, spans, S, E, tab);
  if (pk.ht == kHtCompact && pk.st == kStWide)
    return launch_big<kHtCompact, kStWide>(ctx, spans, S, E, tab);
  if (pk.ht == kHtCompact && pk.st == kStSlot)
    return launch_big<kHtCompact, kStSlot>(ctx, spans, S, E, tab);
  return launch_big<kHtHbm, kStHbm>(ctx, spans, S, E, tab);
}

// Pointers of every section of the device table for layout L.
Table table_at(anomod_ctx* ctx, const Layout& L, uint32_t E) {
  char* base = static_cast<char*>(ctx->d_table);
  Table tab{};  // keys = nullptr: the table forms, not the exact-quantile keys
  tab.hist = reinterpret_cast<unsigned long long*>(base + L.off_hist);
  tab.err = reinterpret_cast<unsigned long long*>(base + L.off_err);
  tab.sum = reinterpret_cast<unsigned long long*>(base + L.off_sum);
  tab.mn = reinterpret_cast<unsigned int*>(base + L.off_mn);
  tab.mx = reinterpret_cast<unsigned int*>(base + L.off_mx);
  tab.ctr = reinterpret_cast<unsigned long long*>(base + L.off_ctr);
  tab.big = reinterpret_cast<unsigned long long*>(base + L.off_big);
  tab.big_list = reinterpret_cast<unsigned long long*>(base + L.off_list());
  tab.bpar = reinterpret_cast<uint16_t*>(base + L.off_bpar);
  tab.ovf = reinterpret_cast<unsigned long long*>(base + L.off_ovf);
  tab.nleft = reinterpret_cast<unsigned long long*>(base + L.off_nleft);
  tab.left = reinterpret_cast<unsigned long long*>(base + L.off_left);
  tab.mode = kModeNormal;
  tab.occupancy = 0;
  tab.kb = 1;
  while (((uint64_t)E * kBins + 1) >> tab.kb) ++tab.kb;  // bits of the largest key
  return tab;
}

// hist | err | sum | mx | counters to zero, mn to all ones (one launch).
int table_clear(anomod_ctx* ctx, const Layout& L, const Table& tab, uint32_t E) {
  const uint64_t nz = L.off_count / 8;  // hist|err|sum|mx|ctr|big|ovf|nleft
  const uint64_t blocks = std::min<uint64_t>((nz / 2 + 255) / 256 + 1, 4ull * ctx->num_cus);
  hipLaunchKernelGGL(edge_table_init_kernel, dim3((unsigned)blocks), dim3(256), 0, ctx->stream,
                     static_cast<unsigned long long*>(ctx->d_table), nz, tab.mn, E);
  ANOMOD_HIP(ctx, hipGetLastError());
  return ANOMOD_OK;
}

// After the aggregation kernels: the merge over an attached communicator, the
// quantiles, and the table to the caller's arrays; ovf[0..1] = the table's
// two overflow words.
int table_finish(anomod_ctx* ctx, const Layout& L, const Table& tab, uint32_t E,
                 anomod_edge_table* out, unsigned long long* ovf) {
  char* base = static_cast<char*>(ctx->d_table);
  auto* count = reinterpret_cast<unsigned long long*>(base + L.off_count);
  auto* p50 = reinterpret_cast<double*>(base + L.off_p50);
  auto* p99 = reinterpret_cast<double*>(base + L.off_p99);
  // Any attached communicator merges, a 1-rank one included (an identity
  // reduce, so the RCCL call sequence is exercised on a single-GPU box too).
  if (comm_attached(ctx)) {
    if (int rc = stage_begin(ctx, kStageEdgeReduce)) return rc;
    if (int rc = coll_begin(ctx)) return rc;
    // hist | err | sum are contiguous u64: one sum all-reduce.
    if (int rc = coll_allreduce(ctx, base, (size_t)E * kBins + 2ull * E, kCollU64, kCollSum))
      return rc;
    if (int rc = coll_allreduce(ctx, tab.mn, E, kCollU32, kCollMin)) return rc;
    if (int rc = coll_allreduce(ctx, tab.mx, E, kCollU32, kCollMax)) return rc;
    if (int rc = coll_end(ctx)) return rc;
    if (int rc = stage_end(ctx, kStageEdgeReduce)) return rc;
  }

  if (int rc = stage_begin(ctx, kStageEdgeFinal)) return rc;
  hipLaunchKernelGGL(edge_finalize_kernel, dim3(E), dim3(kWave), 0, ctx->stream, tab, count, p50,
                     p99);
  ANOMOD_HIP(ctx, hipGetLastError());
  if (int rc = stage_end(ctx, kStageEdgeFinal)) return rc;

  // The per-edge vectors come back in one D2H into pinned staging, then
  // fan out on the host; the histogram (when asked for) goes straight.
  const size_t small = L.end_small - L.off_err;
  ANOMOD_HIP(ctx, hipMemcpyAsync(ctx->h_stage, base + L.off_err, small, hipMemcpyDeviceToHost,
                                 ctx->stream));
  if (out->hist)
    ANOMOD_HIP(ctx, hipMemcpyAsync(out->hist, tab.hist, (size_t)E * kBins * 8ull,
                                   hipMemcpyDeviceToHost, ctx->stream));
  if (int rc = stream_wait(ctx)) return rc;
  const char* hs = static_cast<const char*>(ctx->h_stage);
  auto fan = [&](void* dst, size_t off, size_t bytes) {  // off: device layout offset
    if (dst) memcpy(dst, hs + (off - L.off_err), bytes);
  };
  fan(out->count, L.off_count, E * 8ull);
  fan(out->errors, L.off_err, E * 8ull);
  fan(out->sum_us, L.off_sum, E * 8ull);
  fan(out->min_us, L.off_mn, E * 4ull);
  fan(out->max_us, L.off_mx, E * 4ull);
  fan(out->p50_us, L.off_p50, E * 8ull);
  fan(out->p99_us, L.off_p99, E * 8ull);
  memcpy(ovf, hs + (L.off_ovf - L.off_err), 16);
  return ANOMOD_OK;
}

}  // namespace

int edge_aggregate_records(anomod_ctx* ctx, const uint64_t* rec, uint64_t n, uint32_t S,
                           int8_t* hist_form, anomod_edge_table* out) {
  int local = ANOMOD_OK;
  ANOMOD_CHECK_LOCAL(ctx, local, S >= 1 && S <= 4096, "n_services=%u out of range [1, 4096]", S);
  ANOMOD_CHECK_LOCAL(ctx, local, out->n_services == S, "out->n_services=%u != n_services=%u",
                     out->n_services, S);
  ANOMOD_CHECK_LOCAL(ctx, local, out->n_bins == kBins, "out->n_bins=%u != ANOMOD_HIST_BINS=%u",
                     out->n_bins, kBins);
  ANOMOD_CHECK_LOCAL(ctx, local, n < max_launch_spans(),
                     "%llu edge records: at most 2^32 - 2 per call", (unsigned long long)n);
  const uint32_t E = (S + ANOMOD_ROOT_ROWS) * S;
  const Layout L(E, 0);
  if (local == ANOMOD_OK) local = bind(ctx);
  if (local == ANOMOD_OK) local = ensure_table(ctx, L.bytes);
  if (local == ANOMOD_OK) local = ensure_host_stage(ctx, L.end_small - L.off_err);
  if (int rc = comm_agree(ctx, local)) return rc;
  const Table tab = table_at(ctx, L, E);
  if (int rc = table_clear(ctx, L, tab, E)) return rc;
  // the pair form for a set known to fit it, else the compact form (no probe
  // chain: nothing to saturate), which measures whether the pair form would do
  int form = *hist_form;
  if (const char* f = getenv("ANOMOD_HIST_FORM")) form = !strcmp(f, "pair") ? 0 : 1;
  const uint64_t keys = (uint64_t)E * kBins + 1;
  const bool lds_hist = keys < (1ull << 31);
  KernelFn1 fn = nullptr;
  int ht = kHtCompact;
#define ANOMOD_REC(H, S_) fn = edge_rec_kernel<H, S_>, ht = H
  if (!lds_hist) ANOMOD_REC(kHtHbm, kStHbm);
  else if (E <= kLdsEdges && form == 0) ANOMOD_REC(kHtPair, kStDirect);
  else if (E <= kLdsEdges) ANOMOD_REC(kHtCompact, kStDirect);
  else if (E <= kWideEdges && form == 0) ANOMOD_REC(kHtPair, kStWide);
  else if (E <= kWideEdges) ANOMOD_REC(kHtCompact, kStWide);
  else ANOMOD_REC(kHtCompact, kStSlot);
#undef ANOMOD_REC
  if (int rc = stage_begin(ctx, kStageEdgeAgg)) return rc;
  if (n > 0) {
    int per_cu = 0;
    ANOMOD_HIP(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(
                        &per_cu, reinterpret_cast<const void*>(fn), kThreads, 0));
    const uint64_t want = (n + (uint64_t)kThreads * kRecLoad - 1) / ((uint64_t)kThreads * kRecLoad);
    const uint64_t grid = std::min<uint64_t>((uint64_t)ctx->num_cus * (per_cu > 0 ? per_cu : 1), want);
    Table tr = tab;
    tr.occupancy = ht == kHtCompact;
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(kThreads), 0, ctx->stream, rec, n, E, tr);
    ANOMOD_HIP(ctx, hipGetLastError());
  }
  if (int rc = stage_end(ctx, kStageEdgeAgg)) return rc;
  unsigned long long ovf[2] = {0ull, 0ull};
  if (int rc = table_finish(ctx, L, tab, E, out, ovf)) return rc;
  // what was learned: a compact run whose fullest workgroup used at most half
  // the pair table's slots says pair; a pair run that overflowed, compact
  if (n > 0 && lds_hist) {
    if (ht == kHtCompact && *hist_form < 0) *hist_form = ovf[1] <= kPairSlots / 2 ? 0 : 1;
    if (ht == kHtPair && ovf[0] * 64ull > n) *hist_form = 1;
  }
  return ANOMOD_OK;
}

}  // namespace anomod

using namespace anomod;

extern "C" {

int anomod_edge_aggregate_spans(anomod_ctx* ctx, const anomod_spans* spans, uint32_t S,
                                anomod_edge_table* out) {
  ANOMOD_REQUIRE(nullptr, ctx && spans && out, "anomod_edge_aggregate_spans: NULL argument");
  // Every check that can fail on one rank only (a shard's data, memory)
  // feeds the status agreement instead of returning early: with a
  // communicator attached the other ranks would otherwise wait in the
  // all-reduce below forever.
  int local = ANOMOD_OK;
  ANOMOD_CHECK_LOCAL(ctx, local, S >= 1 && S <= 4096, "n_services=%u out of range [1, 4096]", S);
  ANOMOD_CHECK_LOCAL(ctx, local, out->n_services == S, "out->n_services=%u != n_services=%u",
                     out->n_services, S);
  ANOMOD_CHECK_LOCAL(ctx, local, out->n_bins == kBins, "out->n_bins=%u != ANOMOD_HIST_BINS=%u",
                     out->n_bins, kBins);
  ANOMOD_CHECK_LOCAL(ctx, local, spans->device == ctx->device, "span set lives on another device");
  ANOMOD_CHECK_LOCAL(ctx, local, spans->grouped, "span set is not grouped by trace: "
                     "anomod_spans_group first (or anomod_edge_aggregate_ungrouped)");
  ANOMOD_CHECK_LOCAL(ctx, local, spans->n_spans == 0 || spans->max_svc < S,
                     "span service index %u >= n_services %u", spans->max_svc, S);
  const uint32_t E = (S + ANOMOD_ROOT_ROWS) * S;
  const uint64_t big_cap = big_capacity(spans);
  // Histogram form: a set known to fit the pair table takes it, a set that
  // overflowed it the compact form.  A set not aggregated before (form -1)
  // is probed: its first ~2^19 spans (kFormProbeSpans) run in the compact
  // form — no probe chain, nothing to saturate — on 16 workgroups (each then
  // sees ~32 k spans, near a full-size workgroup's key diversity) that
  // report their largest slot occupancy; at most half the pair table's
  // slots says pair.  The rest of the set runs in that form as an ordinary
  // launch: the probe's counts are part of the table.  A set of at most
  // 4 x 2^19 spans runs whole in the compact form and learns the same way.
  // The order probe of a unique-id set (probe_order_launch) runs beside it:
  // one host wait for both.  (r04 started form-unknown sets in a pair form
  // that stopped saturated workgroups and resumed them compact: its loop
  // spilled 16 / 48 B per lane, so a first call cost 12 % / 40 % more than
  // the pair form on SN / in-trace-shuffled SN; ANOMOD_HIST_FORM=auto keeps
  // it for tests.)
  int form = hist_form_of(spans);
  bool uni = use_unique(spans);  // (re-decided after an order probe)
  const bool pair_ok = pick_kernel(E, false, uni).ht == kHtPair;
  const bool autof = form < 0 && pair_ok && auto_forced();
  // (a set with traces longer than a chunk: LONG-like, the wide parent scan)
  const bool long_set = spans->max_trace_len != ~0ull && spans->max_trace_len > (uint64_t)kBigMin;
  // A unique-id collector-order set with long traces takes the wide parent
  // scan, which only the compact form has: nothing to probe for (r06: its
  // first call paid ~0.9 ms for a 16-workgroup probe over 2^19 LONG spans
  // whose answer was compact anyway, 1.16-1.20 x the warm call).
  if (form < 0 && pair_ok && !autof && long_set && uni) {
    form = 1;
    spans->hist_form = 1;
  }
  const bool probe = form < 0 && pair_ok && !autof && spans->n_traces > 0;
  // the probe's compact form (the forward scan when the order is still unknown)
  const Pick pc = pick_kernel(E, true, uni, kModeNormal, long_set);
  Pick pk = pick_kernel(E, form == 1, uni, autof ? kModeAuto : kModeNormal, long_set);
  const Pick pr = autof ? pick_kernel(E, true, uni, kModeResume) : pk;  // the resume launch's form
  // As many workgroups as are resident at once (LDS / registers decide).
  int per_cu = 0, per_cu_r = 0;
  if (local == ANOMOD_OK) local = bind(ctx);
  if (local == ANOMOD_OK &&
      (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(pk.fn),
                                                    kThreads, 0) != hipSuccess ||
       hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_r, reinterpret_cast<const void*>(pr.fn),
                                                    kThreads, 0) != hipSuccess)) {
    set_error(ctx, "occupancy query of %s failed", pk.name);
    local = ANOMOD_EHIP;
  }
  const uint64_t grid = (uint64_t)ctx->num_cus * (uint64_t)(per_cu > 0 ? per_cu : 1);
  const uint64_t grid_r = (uint64_t)ctx->num_cus * (uint64_t)(per_cu_r > 0 ? per_cu_r : 1);
  const Layout L(E, big_cap, spans->n_spans, autof ? grid * kWavesPerWG : 0);
  if (local == ANOMOD_OK) local = ensure_table(ctx, L.bytes);
  if (local == ANOMOD_OK) local = ensure_host_stage(ctx, L.end_small - L.off_err);
  if (int rc = comm_agree(ctx, local)) return rc;
  const Table tab = table_at(ctx, L, E);
  if (int rc = table_clear(ctx, L, tab, E)) return rc;

  // A first aggregation's probes (order, histogram form) run back to back
  // and are read back with one host wait.
  const bool oprobe = spans->n_traces > 0 && need_order_probe(spans);
  auto* hst = static_cast<unsigned long long*>(ctx->h_stage);  // [0..1] order, [2] occupancy
  if (oprobe)  // scratch: the big counters' 4th and 5th words
    if (int rc = probe_order_launch(ctx, spans, tab.big + 3, hst)) return rc;
  if (!probe && oprobe) {
    ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
    probe_order_take(spans, hst);
    uni = use_unique(spans);
    pk = pick_kernel(E, form == 1, uni, autof ? kModeAuto : kModeNormal, long_set);
  }
  if (int rc = stage_begin(ctx, kStageEdgeAgg)) return rc;
  if (spans->n_traces > 0) {
    // A workgroup's LDS counters (histogram slots, errors) are u32 and the
    // dynamic tail may hand one workgroup any share of a launch, so a launch
    // covers < 2^32 spans: larger sets run as several launches over whole
    // trace ranges (split on the device trace_ptr).
    std::vector<uint64_t> cuts;
    if (int rc = span_launch_cuts(ctx, spans, max_launch_spans(), cuts)) return rc;
    if (probe) {
      const bool whole = spans->n_spans <= 4 * kFormProbeSpans;
      uint64_t P = cuts[1];
      unsigned pgrid = (unsigned)grid;
      if (!whole) {
        const uint64_t want = (kFormProbeSpans * spans->n_traces + spans->n_spans - 1) / spans->n_spans;
        P = std::min<uint64_t>(std::max<uint64_t>(want, 1), cuts[1]);
        pgrid = (unsigned)std::min<uint64_t>(grid, kFormProbeGroups);
      }
      Table tp = tab;
      tp.t_base = 0;
      tp.occupancy = 1;
      hipLaunchKernelGGL(pc.fn, dim3(pgrid), dim3(kThreads), 0, ctx->stream, spans->span_id,
                         spans->parent_span_id, spans->svc_flags, spans->dur_us, spans->trace_ptr,
                         P, S, E, tp);
      ANOMOD_HIP(ctx, hipGetLastError());
      ANOMOD_HIP(ctx, hipMemcpyAsync(hst + 2, tab.ovf + 1, 8, hipMemcpyDeviceToHost,
                                     ctx->stream));
      ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
      if (oprobe) {
        probe_order_take(spans, hst);
        uni = use_unique(spans);
      }
      form = hst[2] <= kPairSlots / 2 ? 0 : 1;
      spans->hist_form = (int8_t)form;
      pk = pick_kernel(E, form == 1, uni, kModeNormal, long_set);
      // the rest from P on (ovf[1] back to 0: after the run it counts
      // pair-table overflows again)
      ANOMOD_HIP(ctx, hipMemsetAsync(tab.ctr, 0, 8, ctx->stream));
      ANOMOD_HIP(ctx, hipMemsetAsync(tab.ovf + 1, 0, 8, ctx->stream));
      cuts[0] = P;
    }
    if (const char* lg = getenv("ANOMOD_LOG_KERNEL"); lg && lg[0] == '1')  // (tests)
      fprintf(stderr, "anomod: edge aggregation kernel %s\n", pk.name);
    for (size_t k = 0; k + 1 < cuts.size(); ++k) {
      if (cuts[k] >= cuts[k + 1]) continue;
      if (k > 0) {
        ANOMOD_HIP(ctx, hipMemsetAsync(tab.ctr, 0, 8, ctx->stream));
        if (autof) ANOMOD_HIP(ctx, hipMemsetAsync(tab.nleft, 0, 16, ctx->stream));
      }
      Table tk = tab;
      tk.t_base = cuts[k];
      tk.mode = autof ? kModeAuto : kModeNormal;
      hipLaunchKernelGGL(pk.fn, dim3((unsigned)grid), dim3(kThreads), 0, ctx->stream,
                         spans->span_id, spans->parent_span_id, spans->svc_flags, spans->dur_us,
                         spans->trace_ptr + cuts[k], cuts[k + 1] - cuts[k], S, E, tk);
      ANOMOD_HIP(ctx, hipGetLastError());
      if (autof) {  // returns at once when no workgroup stopped
        tk.mode = kModeResume;
        hipLaunchKernelGGL(pr.fn, dim3((unsigned)grid_r), dim3(kThreads), 0, ctx->stream,
                           spans->span_id, spans->parent_span_id, spans->svc_flags, spans->dur_us,
                           spans->trace_ptr + cuts[k], cuts[k + 1] - cuts[k], S, E, tk);
        ANOMOD_HIP(ctx, hipGetLastError());
      }
    }
    if (big_cap) ANOMOD_HIP(ctx, launch_big_for(ctx, spans, S, E, tab));
  }
  if (int rc = stage_end(ctx, kStageEdgeAgg)) return rc;
  unsigned long long ovf[2] = {0ull, 0ull};
  if (int rc = table_finish(ctx, L, tab, E, out, ovf)) return rc;
  // The set's form from here on: compact when a workgroup of a first
  // aggregation stopped at a saturated pair table, or when more than 1/64 of
  // the spans were counted in HBM past a full one (the set touches more (edge,
  // bin) keys than 8 Ki slots hold, e.g. random call trees over every service
  // pair); else pair.  Same results either way.
  if (pk.ht == kHtPair) {
    if (ovf[1] > 0 || ovf[0] * 64ull > spans->n_spans) spans->hist_form = 1;
    else if (spans->hist_form < 0) spans->hist_form = 0;
  }
  return ANOMOD_OK;
}

int anomod_edge_quantiles_exact(anomod_ctx* ctx, const anomod_spans* spans, uint32_t S,
                                const uint32_t* q_pct, uint32_t nq, double* out,
                                uint64_t* count) {
  ANOMOD_REQUIRE(nullptr, ctx && spans && q_pct && out,
                 "anomod_edge_quantiles_exact: NULL argument");
  ANOMOD_REQUIRE(ctx, S >= 1 && S <= 4096, "n_services=%u out of range [1, 4096]", S);
  ANOMOD_REQUIRE(ctx, nq >= 1 && nq <= 16, "nq=%u outside [1, 16]", nq);
  for (uint32_t k = 0; k < nq; ++k)
    ANOMOD_REQUIRE(ctx, q_pct[k] <= 99, "q_pct[%u]=%u outside [0, 99]", k, q_pct[k]);
  ANOMOD_REQUIRE(ctx, spans->device == ctx->device, "span set lives on another device");
  ANOMOD_REQUIRE(ctx, spans->grouped, "span set is not grouped by trace: anomod_spans_group first");
  ANOMOD_REQUIRE(ctx, spans->n_spans == 0 || spans->max_svc < S,
                 "span service index %u >= n_services %u", spans->max_svc, S);
  // one radix sort over every span's key (u32 tile offsets inside)
  ANOMOD_REQUIRE(ctx, spans->n_spans <= kMaxSortKeys,
                 "exact edge quantiles: %llu spans, at most 2^32 - 4097 per call",
                 (unsigned long long)spans->n_spans);
  if (int rc = bind(ctx)) return rc;
  const uint32_t E = (S + ANOMOD_ROOT_ROWS) * S;
  const uint64_t n = spans->n_spans;
  int kbits = 1;
  while ((uint64_t)E >> kbits) ++kbits;
  // One workspace: keys | sorted keys | sort temp | q | out | count | ctr +
  // long-trace counters | long-trace list
  const uint64_t big_cap = big_capacity(spans);
  const size_t sort_tmp = n ? radix_temp_bytes(n) : 0;
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t b_keys = al(n * 8), b_tmp = al(sort_tmp), b_q = al(nq * 4), b_out = al(E * nq * 8ull),
               b_cnt = al(E * 8ull);
  // (the ctx's scratch slot: reused by the next call instead of freed)
  char* w = nullptr;
  if (int rc = ensure_scratch(ctx, kScratchQuantiles,
                              2 * b_keys + b_tmp + b_q + b_out + b_cnt + 256 + big_cap * 8,
                              reinterpret_cast<void**>(&w)))
    return rc;
  auto* keys = reinterpret_cast<unsigned long long*>(w);
  auto* sorted = reinterpret_cast<unsigned long long*>(w + b_keys);
  void* tmp = w + 2 * b_keys;
  auto* d_q = reinterpret_cast<uint32_t*>(w + 2 * b_keys + b_tmp);
  auto* d_out = reinterpret_cast<double*>(w + 2 * b_keys + b_tmp + b_q);
  auto* d_cnt = reinterpret_cast<unsigned long long*>(w + 2 * b_keys + b_tmp + b_q + b_out);
  auto* d_ctr = reinterpret_cast<unsigned long long*>(w + 2 * b_keys + b_tmp + b_q + b_out + b_cnt);
  int rc = ANOMOD_OK;
  hipError_t e = hipMemcpyAsync(d_q, q_pct, nq * 4, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess && n && spans->n_traces) {
    // per-span (edge, latency) keys from the aggregation kernel's own walk and
    // parent rule, then one radix sort over edge|dur
    Table tab{};
    tab.keys = keys;
    tab.ctr = d_ctr;
    tab.big = d_ctr + 1;
    tab.big_list = d_ctr + 32;
    rc = probe_order(ctx, spans, d_ctr + 4);
    KernelFn fn = use_unique(spans) ? edge_agg_kernel<kHtKeys, kStHbm, true>
                                    : edge_agg_kernel<kHtKeys, kStHbm, false>;
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(fn),
                                                     kThreads, 0);
    const uint64_t grid = (uint64_t)ctx->num_cus * (uint64_t)(per_cu > 0 ? per_cu : 1);
    std::vector<uint64_t> cuts;
    if (e == hipSuccess && rc == ANOMOD_OK) rc = span_launch_cuts(ctx, spans, max_launch_spans(), cuts);
    if (e == hipSuccess) e = hipMemsetAsync(d_ctr, 0, 32, ctx->stream);  // ctr + big counters
    for (size_t k = 0; e == hipSuccess && rc == ANOMOD_OK && k + 1 < cuts.size(); ++k) {
      if (k > 0) e = hipMemsetAsync(d_ctr, 0, 8, ctx->stream);
      if (e != hipSuccess) break;
      Table tk = tab;
      tk.t_base = cuts[k];
      hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(kThreads), 0, ctx->stream, spans->span_id,
                         spans->parent_span_id, spans->svc_flags, spans->dur_us,
                         spans->trace_ptr + cuts[k], cuts[k + 1] - cuts[k], S, E, tk);
      e = hipGetLastError();
    }
    if (e == hipSuccess && rc == ANOMOD_OK && big_cap)
      e = launch_big<kHtKeys, kStHbm>(ctx, spans, S, E, tab);
    if (e == hipSuccess && rc == ANOMOD_OK)
      e = radix_sort_u64(reinterpret_cast<const uint64_t*>(keys),
                         reinterpret_cast<uint64_t*>(sorted), n, 0, 32 + kbits, tmp, sort_tmp,
                         ctx->stream);
  }
  if (e == hipSuccess && rc == ANOMOD_OK) {
    hipLaunchKernelGGL(exact_pick_kernel, dim3((E + 255) / 256), dim3(256), 0, ctx->stream,
                       sorted, spans->n_traces ? n : 0, E, d_q, nq, d_out, d_cnt);
    e = hipGetLastError();
  }
  if (e == hipSuccess && rc == ANOMOD_OK)
    e = hipMemcpyAsync(out, d_out, E * nq * 8ull, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess && rc == ANOMOD_OK && count)
    e = hipMemcpyAsync(count, d_cnt, E * 8ull, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (rc != ANOMOD_OK) return rc;
  if (e != hipSuccess) {
    set_error(ctx, "exact edge quantiles failed: %s", hipGetErrorString(e));
    return ANOMOD_EHIP;
  }
  return ANOMOD_OK;
}

int anomod_edge_aggregate(anomod_ctx* ctx, const anomod_span_soa* soa, uint64_t n_spans,
                          const uint64_t* trace_ptr, uint64_t n_traces, anomod_edge_table* out) {
  ANOMOD_REQUIRE(nullptr, ctx && soa && out, "anomod_edge_aggregate: NULL argument");
  anomod_spans* s = nullptr;
  if (int rc = anomod_spans_upload(ctx, soa, n_spans, trace_ptr, n_traces, &s)) return rc;
  const int rc = anomod_edge_aggregate_spans(ctx, s, out->n_services, out);
  anomod_spans_free(s);
  return rc;
}

}  // extern "C"
