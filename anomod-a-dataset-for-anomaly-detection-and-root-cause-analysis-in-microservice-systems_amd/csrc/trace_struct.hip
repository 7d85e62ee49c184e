// Trace-structure features: per span the parent's
// position in its trace, the BFS depth and the child count; per trace the
// number of roots and the set of services involved.
//
// Restates on the GPU what TT_collection-scripts/T-Dataset/trace_collector.py
// computes per trace, one Python dict at a time, in _build_span_records
// (:401-481) and collect_traces (:536-547).  Spans are nodes keyed by their
// id (node_id = segmentId:spanId, :414); with duplicated ids the reference's
// dicts keep the LAST span's parent (parents[node_id] = ..., :437) while every
// span appends itself to its own parent's child list (:438-439):
//   parent_pos  position of the node's parent: the first span of the trace
//               whose id equals the parent reference of the LAST span with
//               this node's id; ANOMOD_NO_PARENT when that reference is 0 or
//               names no span of the trace (:427-437)
//   depth       the BFS of :441-449 over the child lists: it enqueues a node
//               once per child-list entry and keeps the LAST (= deepest)
//               visit, i.e. the longest path from a root along the edges
//               "first span of my own parent reference -> my node".  0 when
//               no root reaches the node (:477 default) or when a cycle the
//               BFS reaches feeds it (the reference never terminates there).
//               Without duplicated ids this is the walk up the node parents.
//   n_children  spans whose own parent reference names this node (:438-439),
//               shared by every span carrying the node's id (:476)
//   span_flags  ANOMOD_SPAN_ROOT (node parent not in the trace, :443) |
//               ANOMOD_SPAN_FIRST (first span of the trace with this id)
//   n_roots     distinct root nodes of the trace (len(root_span_node_ids))
//   svc_mask    services_involved (:536) as a bit set of service indices
//
// GPU form: the chunk walk of the edge kernel (chunk.h) with its software
// pipeline — whole traces in a wave's LDS, one fused ordered scan (8 ids per
// step) for the three id questions of a span, parent pointer-jumping in
// LDS for the depth (<= 8 rounds for a 256-span chunk) when the chunk has no
// duplicated id, else longest-path relaxation in LDS (rounds until nothing
// changes, bounded by 2L + 2 so a reached cycle is recognised by its depth
// outgrowing L); per-trace counters in LDS.  A trace longer than 256 spans is
// resolved by the whole wave against HBM (O(L^2 / 64) compares plus
// relaxation rounds over a scratch edge list; rare).
#include <cstdlib>
#include <cstring>

#include "chunk.h"
#include "common.h"

#ifndef ANOMOD_SEL_TS
#define ANOMOD_SEL_TS 0  // select-built parent scan (chunk.h find_parent_bidir SEL)
#endif
#ifndef ANOMOD_SPLIT_TS
#define ANOMOD_SPLIT_TS 0  // unique-id sets: split-word scan (chunk.h find_parent_split)
#endif
#ifndef ANOMOD_TS_FWD
#define ANOMOD_TS_FWD 12
#endif
#ifndef ANOMOD_TS_BWD
#define ANOMOD_TS_BWD 4
#endif

namespace anomod {
namespace {

using namespace chunk;

constexpr int kTsWaves = 8;
// Experiment-only ablations (never set in the shipped build): 1 = no per-trace
// pass, 2 = no pointer jumping.
#ifndef ANOMOD_TS_ABL
#define ANOMOD_TS_ABL 0
#endif
constexpr int kTsThreads = kTsWaves * kWave;
constexpr uint32_t kDone = 0x80000000u;  // pointer-jumping: chain reached a root

// Per-wave LDS carve (bytes; 16-B aligned offsets).
constexpr int kTSid = 0;                          // u64 span ids   [kStage + kScanSlack] (scan slack)
constexpr int kTPid = kTSid + (kStage + chunk::kScanSlack) * 8;  // u64 parent refs [kStage]
constexpr int kTNxt = kTPid + kStage * 8;         // u32 jump target | kDone [kStage]
constexpr int kTDst = kTNxt + kStage * 4;         // u32 distance to the target [kStage]
constexpr int kTCnt = kTDst + kStage * 4;         // u32 child counts [kStage]
constexpr int kTPfl = kTCnt + kStage * 4;         // u32 (own parent pos + 1) | trace len << 16
constexpr int kTSvc = kTPfl + kStage * 4;         // u16 services [kStage]
constexpr int kTRf = kTSvc + kStage * 2;          // u8 root-node flag of first spans [kStage]
constexpr int kTFlag = kTRf + kStage;             // u8 trace-start flags [kStage]
constexpr int kTTm = kTFlag + kStage;             // u64 per-trace service bits [kWave]
constexpr int kTTr = kTTm + kWave * 8;            // u32 per-trace root-node counts [kWave]
constexpr int kTBytes = kTTr + kWave * 4;
static_assert(kTBytes % 16 == 0, "wave area must stay 16-B aligned");
static_assert(kTBytes * kTsWaves <= 80 * 1024, "LDS budget: two workgroups per CU");

struct TsOut {
  uint32_t* parent_pos;
  uint32_t* depth;
  uint32_t* n_children;
  uint8_t* flags;
  uint32_t* n_roots;
  unsigned long long* svc_mask;  // [n_traces * words]
  uint32_t words;                // ceil(S / 64)
  unsigned long long* ctr;       // trace-segment counter of the dynamic tail (zeroed per launch)
  // Traces longer than kStage, listed by the chunk walk for ts_big_kernel:
  // big[0] listed, big[1] their spans, big[2] ticket, big[3] error flag;
  // big_list[2j] = trace index, big_list[2j + 1] = its offset in the scratch.
  unsigned long long* big;
  unsigned long long* big_list;
  uint32_t* scr;                 // ts_big_kernel: 4 u32 per listed span (4 arrays of big[1])
  uint64_t scr_n;                // big[1]
};

// One ordered pass over [a, b), kTsScan ids per step (ds_read2_b64 from the
// trace start itself), answering the three per-span id questions together:
// f / l = first / last position whose id equals x (the span's own id: the
// whole range is scanned for l), pf = first position whose id equals y (the
// span's parent reference; -1 when y == 0).  -1 when none.
#ifndef ANOMOD_TS_SCAN_IDS
#define ANOMOD_TS_SCAN_IDS 10
#endif
constexpr uint32_t kTsScan = ANOMOD_TS_SCAN_IDS;  // ids per step (kTsScan / 2 x ds_read2_b64)

__device__ __forceinline__ void scan_ids(const uint64_t* lsid, uint32_t a, uint32_t b, uint64_t x,
                                         uint64_t y, int& f, int& l, int& pf) {
  f = l = pf = -1;
  for (uint32_t q0 = a; q0 < b; q0 += kTsScan) {
    uint64_t v[kTsScan];
#pragma unroll
    for (uint32_t j = 0; j < kTsScan; ++j) v[j] = lsid[q0 + j];
    uint32_t mx = 0, my = 0;
#pragma unroll
    for (uint32_t j = 0; j < kTsScan; ++j) {
      mx |= (v[j] == x ? 1u : 0u) << j;
      my |= (v[j] == y ? 1u : 0u) << j;
    }
    const uint32_t hi = (b - q0) < kTsScan ? (b - q0) : kTsScan;  // >= 1
    const uint32_t rm = (1u << hi) - 1u;
    mx &= rm;
    my &= rm;
    if (mx) {
      if (f < 0) f = (int)(q0 + __ffs(mx) - 1u);
      l = (int)(q0 + 31u - __clz(mx));
    }
    if (my && pf < 0) pf = (int)(q0 + __ffs(my) - 1u);
  }
  if (y == 0ull) pf = -1;
}

// First position in [a, b) whose id equals x (-1 when none or x == 0).
__device__ __forceinline__ int first_of(const uint64_t* lsid, uint32_t a, uint32_t b, uint64_t x) {
  if (x == 0ull) return -1;
  for (uint32_t q = a; q < b; ++q)
    if (lsid[q] == x) return (int)q;
  return -1;
}

template <bool UNI>
__device__ void ts_chunk(unsigned char* wsm, int lane, const Chunk& c, uint64_t t0,
                         const uint64_t (&sid)[kPer], const uint64_t (&pid)[kPer],
                         const uint32_t (&svc)[kPer], const TsOut& o) {
  auto* lsid = reinterpret_cast<uint64_t*>(wsm + kTSid);
  constexpr bool kSplit = UNI && ANOMOD_SPLIT_TS != 0;
  auto* llo = reinterpret_cast<uint32_t*>(wsm + kTSid);  // kSplit: u32 planes in the same area
  uint32_t* lhi = llo + (kStage + chunk::kScanSlack);
  auto* lpid = reinterpret_cast<uint64_t*>(wsm + kTPid);
  auto* lnxt = reinterpret_cast<uint32_t*>(wsm + kTNxt);
  auto* ldst = reinterpret_cast<uint32_t*>(wsm + kTDst);
  auto* lcnt = reinterpret_cast<uint32_t*>(wsm + kTCnt);
  auto* lpfl = reinterpret_cast<uint32_t*>(wsm + kTPfl);
  auto* lsvc = reinterpret_cast<uint16_t*>(wsm + kTSvc);
  auto* lrf = reinterpret_cast<uint8_t*>(wsm + kTRf);
  auto* lflag = reinterpret_cast<uint8_t*>(wsm + kTFlag);
  auto* ltm = reinterpret_cast<unsigned long long*>(wsm + kTTm);
  auto* ltr = reinterpret_cast<uint32_t*>(wsm + kTTr);
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const uint32_t i = lane + r * kWave;
    if constexpr (kSplit) {
      llo[i] = (uint32_t)sid[r];
      lhi[i] = (uint32_t)(sid[r] >> 32);
    } else {
      lsid[i] = sid[r];
    }
    lpid[i] = pid[r];
    lcnt[i] = 0u;
    lsvc[i] = (uint16_t)svc[r];
  }
  ltm[lane] = 0ull;
  ltr[lane] = 0u;
  uint64_t Sm[kPer];
  start_masks(lflag, c, lane, Sm);
  // Trace t (lane t < k) spans chunk positions [s, e).  Empty traces share a
  // start position, so only without them is a span's trace the rank of its
  // start among the start flags (trace_in_chunk).
  const uint32_t next_start = (uint32_t)__shfl((int)c.start, (lane + 1) & (kWave - 1));
  const uint32_t t_e = (lane + 1 < (int)c.k) ? next_start : c.n;
  const bool span_par = __ballot((uint32_t)lane < c.k && t_e == c.start) == 0ull;

  int f[kPer], np[kPer];
  uint32_t a[kPer], nxt[kPer], dst[kPer];
  bool dup = false;
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const uint32_t i = lane + r * kWave;
    f[r] = np[r] = -1;
    a[r] = 0;
    uint32_t pfl = 0;
    if (i < c.n) {
      uint32_t b;
      trace_bounds(Sm, r, lane, c.n, a[r], b);
      int l, pf;  // pf: own parent (child lists)
      if constexpr (UNI) {
        // ids unique in the trace: the span is its node's only span (f = l =
        // i), and the parent reference has at most one match, found from
        // either end (chunk.h find_parent_bidir); no own-id scan
        f[r] = l = (int)i;
        if constexpr (kSplit)
          pf = pid[r] != 0ull
                   ? find_parent_split<ANOMOD_TS_FWD, ANOMOD_TS_BWD>(llo, lhi, a[r], b, i, pid[r])
                   : -1;
        else
          pf = pid[r] != 0ull
                   ? find_parent_bidir<kFwd, kBwd, 0, ANOMOD_SEL_TS != 0>(lsid, a[r], b, i, pid[r])
                   : -1;
        np[r] = pf;
      } else {
        scan_ids(lsid, a[r], b, sid[r], pid[r], f[r], l, pf);
        np[r] = (l == (int)i) ? pf : first_of(lsid, a[r], b, lpid[l]);  // node parent
      }
      if (pf >= 0) atomicAdd(&lcnt[pf], 1u);
      if constexpr (!UNI) dup |= f[r] != (int)i;
      pfl = (uint32_t)(pf + 1) | (b - a[r]) << 16;
    }
    lpfl[i] = pfl;
    const bool rf = i < c.n && np[r] < 0 && f[r] == (int)i;
    lrf[i] = (uint8_t)rf;
    // Per-trace services involved / root nodes: every span adds itself to
    // its trace's LDS words (no-return atomics) instead of one lane per trace
    // walking the trace.
    if (span_par && i < c.n && !(ANOMOD_TS_ABL & 1)) {
      const uint32_t ti = trace_in_chunk(Sm, r, lane);
      const uint32_t sv = svc[r];
      if (o.words == 1u) atomicOr(&ltm[ti], 1ull << sv);
      else atomicOr(&o.svc_mask[(t0 + ti) * o.words + (sv >> 6)], 1ull << (sv & 63u));
      if (rf) atomicAdd(&ltr[ti], 1u);
    }
    nxt[r] = np[r] >= 0 ? (uint32_t)np[r] : (i | kDone);
    dst[r] = np[r] >= 0 ? 1u : 0u;
    lnxt[i] = nxt[r];
    ldst[i] = dst[r];
  }
  wave_sync();
  if (__ballot(dup) != 0ull) {
    // Duplicated ids: a node may have several parents (one per span carrying
    // its id), and the BFS keeps its deepest visit.  Longest-path relaxation
    // of the edges pf -> f over the node depths in LDS (reusing the jump
    // array), from the roots (depth 0); -1 = not reached.
    auto* ld = reinterpret_cast<int*>(lnxt);
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const uint32_t i = lane + r * kWave;
      ld[i] = lrf[i] ? 0 : -1;
    }
    wave_sync();
    for (uint32_t round = 0; round < 2u * c.n + 2u; ++round) {
      bool changed = false;
#pragma unroll
      for (int r = 0; r < kPer; ++r) {
        const int pf = (int)(lpfl[lane + r * kWave] & 0xFFFFu) - 1;
        if (pf >= 0) {
          const int dp = ld[pf];
          if (dp >= 0 && dp + 1 > ld[f[r]]) {
            atomicMax(&ld[f[r]], dp + 1);
            changed = true;
          }
        }
      }
      wave_sync();
      if (__ballot(changed) == 0ull) break;
    }
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int d = f[r] >= 0 ? ld[f[r]] : -1;
      nxt[r] = kDone;  // the output below reads dst as the depth
      dst[r] = (d >= 0 && d < (int)(lpfl[lane + r * kWave] >> 16)) ? (uint32_t)d : 0u;
    }
  }
  // Pointer jumping: after round k every span points 2^k ancestors up (or at
  // its root, flagged kDone) and knows the distance; 8 rounds cover 256.
  for (int round = 0; round < ((ANOMOD_TS_ABL & 2) ? 0 : 8); ++round) {
    bool live = false;
#pragma unroll
    for (int r = 0; r < kPer; ++r) live |= !(nxt[r] & kDone);
    if (__ballot(live) == 0ull) break;
    uint32_t nn[kPer], nd[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      nn[r] = nxt[r];
      nd[r] = 0u;
      if (!(nxt[r] & kDone)) {
        nn[r] = lnxt[nxt[r]];
        nd[r] = ldst[nxt[r]];
      }
    }
    wave_sync();
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      if (!(nxt[r] & kDone)) {
        const uint32_t i = lane + r * kWave;
        dst[r] += nd[r];
        nxt[r] = nn[r];  // the target's target; a root target carries kDone
        lnxt[i] = nxt[r];
        ldst[i] = dst[r];
      }
    }
    wave_sync();
  }
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const uint32_t i = lane + r * kWave;
    if (i < c.n) {
      const uint64_t g = c.base + i;
      st_out(&o.parent_pos[g], np[r] >= 0 ? (uint32_t)np[r] - a[r] : ANOMOD_NO_PARENT);
      st_out(&o.depth[g], (nxt[r] & kDone) ? dst[r] : 0u);
      st_out(&o.n_children[g], (uint32_t)lcnt[f[r]]);
      st_out(&o.flags[g], (uint8_t)((np[r] < 0 ? ANOMOD_SPAN_ROOT : 0u) |
                                    (f[r] == (int)i ? ANOMOD_SPAN_FIRST : 0u)));
    }
  }
  // Per trace: lane l < k owns trace t0 + l.  Span-parallel words (complete:
  // the wave_syncs above order every span's atomics before these reads), or,
  // when the chunk holds an empty trace, a walk over the trace's positions.
  if ((uint32_t)lane < c.k && !(ANOMOD_TS_ABL & 1)) {
    const uint64_t t = t0 + lane;
    if (span_par) {
      o.n_roots[t] = ltr[lane];
      if (o.words == 1u) o.svc_mask[t] = ltm[lane];
    } else {
      uint32_t roots = 0;
      unsigned long long mask = 0;
      for (uint32_t q = c.start; q < t_e; ++q) {
        roots += lrf[q];
        const uint32_t sv = lsvc[q];
        if (o.words == 1u) mask |= 1ull << sv;
        else
          atomicOr(&o.svc_mask[t * o.words + (sv >> 6)], 1ull << (sv & 63u));
      }
      o.n_roots[t] = roots;
      if (o.words == 1u) o.svc_mask[t] = mask;
    }
  }
  wave_sync();
}

// Traces longer than kStage: one workgroup per trace (ts_big_kernel), after
// the chunk walk.  The span-id questions are answered through an LDS hash
// table of kBigWin ids at a time (id -> first / last position in the window):
// every span probes each window in trace order, so the first window holding
// an id gives its first occurrence and the last one its last occurrence —
// O(L * ceil(L / kBigWin)) work.  Depth: parent pointer jumping over the
// trace in global scratch (log L rounds) without duplicated ids, else the
// longest-path relaxation of ts_chunk over the whole workgroup.
constexpr int kBigThreads = 1024;
constexpr uint32_t kBigWin = 4096;    // ids per table window
constexpr uint32_t kBigSlots = 8192;  // table slots (load <= 0.5)
constexpr int kBigPer = 4;            // spans per thread per lookup block
constexpr uint32_t kNone = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t big_slot(uint64_t id) {
  return (uint32_t)((id * 0x9E3779B97F4A7C15ull) >> (64 - 13)) & (kBigSlots - 1u);
}

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kBigThreads) void ts_big_kernel(
    const uint64_t* __restrict__ span_id, const uint64_t* __restrict__ parent,
    const uint32_t* __restrict__ svcfl, const uint64_t* __restrict__ trace_ptr, TsOut o) {
  __shared__ unsigned long long bkey[kBigSlots];  // 0 = empty; id 0 goes to zmin / zmax
  __shared__ uint32_t bmin[kBigSlots], bmax[kBigSlots];
  __shared__ uint32_t zmin, zmax, s_roots;
  __shared__ unsigned long long s_j, s_mask;
  const int tid = threadIdx.x;
  const uint64_t nbig = o.big[0];
  uint32_t* const s0 = o.scr;  // f, then jump target (even rounds)
  uint32_t* const s1 = o.scr + o.scr_n;      // pf, then distance (even rounds)
  uint32_t* const s2 = o.scr + 2 * o.scr_n;  // l, then jump target (odd rounds)
  uint32_t* const s3 = o.scr + 3 * o.scr_n;  // node parent, then distance (odd rounds)
  for (uint32_t k = tid; k < kBigSlots; k += kBigThreads) {
    bkey[k] = 0ull;
    bmin[k] = kNone;
    bmax[k] = 0u;
  }
  while (true) {
    __syncthreads();
    if (tid == 0) {
      s_j = atomicAdd(&o.big[2], 1ull);
      zmin = kNone;
      zmax = 0u;
      s_roots = 0u;
      s_mask = 0ull;
    }
    __syncthreads();
    const uint64_t j = s_j;
    if (j >= nbig) break;
    const uint64_t t = o.big_list[2 * j], off = o.big_list[2 * j + 1];
    const uint64_t lo = trace_ptr[t];
    const uint64_t L64 = trace_ptr[t + 1] - lo;
    if (L64 >= (uint64_t)kDone) {  // positions are u32 with a flag bit
      if (tid == 0) atomicOr(&o.big[3], 1ull);
      continue;
    }
    const uint32_t L = (uint32_t)L64;
    // ---- phase 1: f / l (own id), pf (own parent reference) per span
    for (uint32_t b0 = 0; b0 < L; b0 += kBigThreads * kBigPer) {
      uint64_t sid[kBigPer], pid[kBigPer];
      uint32_t f[kBigPer], l[kBigPer], pf[kBigPer];
#pragma unroll
      for (int r = 0; r < kBigPer; ++r) {
        const uint32_t i = b0 + (uint32_t)r * kBigThreads + tid;
        sid[r] = i < L ? span_id[lo + i] : 0ull;
        pid[r] = i < L ? parent[lo + i] : 0ull;
        f[r] = l[r] = pf[r] = kNone;
      }
      for (uint32_t w0 = 0; w0 < L; w0 += kBigWin) {
        for (uint32_t k = tid; k < kBigWin && w0 + k < L; k += kBigThreads) {
          const uint64_t id = span_id[lo + w0 + k];
          if (id == 0ull) {
            atomicMin(&zmin, k);
            atomicMax(&zmax, k);
            continue;
          }
          for (uint32_t sl = big_slot(id);; sl = (sl + 1u) & (kBigSlots - 1u)) {
            const unsigned long long prev = atomicCAS(&bkey[sl], 0ull, (unsigned long long)id);
            if (prev == 0ull || prev == id) {
              atomicMin(&bmin[sl], k);
              atomicMax(&bmax[sl], k);
              break;
            }
          }
        }
        __syncthreads();
        auto probe = [&](uint64_t x, uint32_t& mn, uint32_t& mx) {
          if (x == 0ull) {
            mn = zmin;
            mx = zmax;
            return mn != kNone;
          }
          for (uint32_t sl = big_slot(x);; sl = (sl + 1u) & (kBigSlots - 1u)) {
            const unsigned long long key = bkey[sl];
            if (key == x) {
              mn = bmin[sl];
              mx = bmax[sl];
              return true;
            }
            if (key == 0ull) return false;
          }
        };
#pragma unroll
        for (int r = 0; r < kBigPer; ++r) {
          const uint32_t i = b0 + (uint32_t)r * kBigThreads + tid;
          if (i >= L) continue;
          uint32_t mn, mx;
          if (probe(sid[r], mn, mx)) {
            if (f[r] == kNone) f[r] = w0 + mn;
            l[r] = w0 + mx;
          }
          if (pid[r] != 0ull && pf[r] == kNone && probe(pid[r], mn, mx)) pf[r] = w0 + mn;
        }
        __syncthreads();
        for (uint32_t k = tid; k < kBigSlots; k += kBigThreads) {
          bkey[k] = 0ull;
          bmin[k] = kNone;
          bmax[k] = 0u;
        }
        if (tid == 0) {
          zmin = kNone;
          zmax = 0u;
        }
        __syncthreads();
      }
#pragma unroll
      for (int r = 0; r < kBigPer; ++r) {
        const uint32_t i = b0 + (uint32_t)r * kBigThreads + tid;
        if (i >= L) continue;
        s0[off + i] = f[r];
        s1[off + i] = pf[r];
        s2[off + i] = l[r];
      }
    }
    __syncthreads();
    // ---- phase 2: node parent (the LAST span's reference, resolved = that
    // span's pf), child counts, flags, roots, services
    bool dup = false;
    uint32_t roots = 0;
    unsigned long long mask = 0;
    for (uint32_t i = tid; i < L; i += kBigThreads) {
      const uint32_t f = s0[off + i], pf = s1[off + i], l = s2[off + i];
      const uint32_t np = (l == i) ? pf : s1[off + l];
      if (pf != kNone) atomicAdd(&o.n_children[lo + pf], 1u);
      o.parent_pos[lo + i] = np != kNone ? np : ANOMOD_NO_PARENT;
      o.flags[lo + i] = (uint8_t)((np == kNone ? ANOMOD_SPAN_ROOT : 0u) |
                                  (f == i ? ANOMOD_SPAN_FIRST : 0u));
      if (np == kNone && f == i) ++roots;
      dup |= f != i;
      s3[off + i] = np;
      const uint32_t sv = svcfl[lo + i] & 0xFFFFu;
      if (o.words == 1u) mask |= 1ull << sv;
      else atomicOr(&o.svc_mask[t * o.words + (sv >> 6)], 1ull << (sv & 63u));
    }
    if (roots) atomicAdd(&s_roots, roots);
    if (mask) atomicOr(&s_mask, mask);
    if (!__syncthreads_or(dup)) {
      // ---- phase 3: pointer jumping (every node is its own first span)
      for (uint32_t i = tid; i < L; i += kBigThreads) {
        const uint32_t np = s3[off + i];
        s0[off + i] = np != kNone ? np : (i | kDone);
        s1[off + i] = np != kNone ? 1u : 0u;
      }
      uint32_t rounds = 1;
      while ((1ull << rounds) < (uint64_t)L) ++rounds;
      uint32_t *na = s0, *da = s1, *nb = s2, *db = s3;
      for (uint32_t round = 0; round <= rounds; ++round) {
        bool live = false;
        __syncthreads();
        for (uint32_t i = tid; i < L; i += kBigThreads) {
          const uint32_t nx = na[off + i], d = da[off + i];
          if (nx & kDone) {
            nb[off + i] = nx;
            db[off + i] = d;
          } else {
            nb[off + i] = na[off + nx];
            db[off + i] = d + da[off + nx];
            live = true;
          }
        }
        uint32_t* tn = na; na = nb; nb = tn;
        uint32_t* td = da; da = db; db = td;
        if (!__syncthreads_or(live)) break;
      }
      __syncthreads();
      for (uint32_t i = tid; i < L; i += kBigThreads) {
        const uint32_t nx = na[off + i];
        o.depth[lo + i] = (nx & kDone) ? da[off + i] : 0u;
      }
    } else {
      // ---- phase 3 (duplicated ids): longest path from the roots along the
      // edges pf -> f over node depths (in the depth output, -1 = not
      // reached); a depth outgrowing L marks a reached cycle -> 0
      int* D = reinterpret_cast<int*>(o.depth + lo);
      for (uint32_t i = tid; i < L; i += kBigThreads) {
        const uint32_t f = s0[off + i];
        D[i] = (f == i && s3[off + i] == kNone) ? 0 : -1;
      }
      for (uint64_t round = 0; round < 2ull * L + 2ull; ++round) {
        __syncthreads();
        bool changed = false;
        for (uint32_t i = tid; i < L; i += kBigThreads) {
          const uint32_t pf = s1[off + i];
          if (pf == kNone) continue;
          const uint32_t f = s0[off + i];
          const int dp = (int)ld_agent(reinterpret_cast<uint32_t*>(D) + pf);
          if (dp >= 0 && dp + 1 > (int)ld_agent(reinterpret_cast<uint32_t*>(D) + f)) {
            atomicMax(&D[f], dp + 1);
            changed = true;
          }
        }
        if (!__syncthreads_or(changed)) break;
      }
      __syncthreads();
      for (uint32_t i = tid; i < L; i += kBigThreads) {
        const int d = (int)ld_agent(reinterpret_cast<uint32_t*>(D) + s0[off + i]);
        s2[off + i] = (d >= 0 && d < (int)L) ? (uint32_t)d : 0u;
      }
      __syncthreads();
      for (uint32_t i = tid; i < L; i += kBigThreads) o.depth[lo + i] = s2[off + i];
    }
    // a duplicated id's child count is its node's (first span's)
    for (uint32_t i = tid; i < L; i += kBigThreads) {
      const uint32_t f = s0[off + i];
      if (dup && f != i) o.n_children[lo + i] = ld_agent(&o.n_children[lo + f]);
    }
    if (tid == 0) {
      o.n_roots[t] = s_roots;
      if (o.words == 1u) o.svc_mask[t] = s_mask;
    }
  }
}

template <bool UNI>
__global__ __launch_bounds__(kTsThreads) __attribute__((amdgpu_waves_per_eu(4))) void trace_struct_kernel(
    const uint64_t* __restrict__ span_id, const uint64_t* __restrict__ parent,
    const uint32_t* __restrict__ svcfl, const uint64_t* __restrict__ trace_ptr, uint64_t n_traces,
    TsOut o) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[kTBytes * kTsWaves];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  unsigned char* wsm = smem + wid * kTBytes;
  const uint64_t gw = (uint64_t)blockIdx.x * kTsWaves + wid;
  const uint64_t nw = (uint64_t)gridDim.x * kTsWaves;
  auto run = [&](const uint64_t t_begin, const uint64_t t_end) __attribute__((always_inline)) {
  // Software pipeline (as the edge kernel): the bounds of chunk c+2 and the
  // span columns of chunk c+1 are in flight while chunk c is resolved.
  auto load_cols = [&](const Chunk& c, uint64_t (&sid)[kPer], uint64_t (&pid)[kPer],
                       uint32_t (&svc)[kPer]) {
    const uint32_t n = c.k ? c.n : 0u;  // a big trace is read by ts_big_kernel
    const auto rsid = rsrc(span_id + c.base, n * 8u);
    const auto rpid = rsrc(parent + c.base, n * 8u);
    const auto rsf = rsrc(svcfl + c.base, n * 4u);
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const uint32_t i = (uint32_t)lane + (uint32_t)(r * kWave);
      sid[r] = bload64(rsid, i * 8u);
      pid[r] = bload64(rpid, i * 8u);
      svc[r] = bload32(rsf, i * 4u) & 0xFFFFu;
    }
  };
  uint64_t lo, hi;
  load_bounds(trace_ptr, t_begin, t_end, lane, lo, hi);
  Chunk cur = make_chunk(t_begin, t_end, lane, lo, hi);
  uint64_t t_cur = t_begin;
  uint64_t sid[kPer], pid[kPer];
  uint32_t svc[kPer];
  load_cols(cur, sid, pid, svc);
  uint64_t t_next = t_begin + (cur.k ? cur.k : 1u);
  load_bounds(trace_ptr, t_next, t_end, lane, lo, hi);
  while (true) {
    const bool has_next = t_next < t_end;
    Chunk nxt{};
    uint64_t sid_n[kPer], pid_n[kPer];
    uint32_t svc_n[kPer];
    const uint64_t t_nxt = t_next;
    if (has_next) {
      nxt = make_chunk(t_next, t_end, lane, lo, hi);
      load_cols(nxt, sid_n, pid_n, svc_n);
      t_next += nxt.k ? nxt.k : 1u;
      load_bounds(trace_ptr, t_next, t_end, lane, lo, hi);
    }
    if (cur.k == 0) {  // longer than kStage: listed for ts_big_kernel
      if (lane == 0) {
        const unsigned long long j = atomicAdd(&o.big[0], 1ull);
        o.big_list[2 * j] = t_cur;
        o.big_list[2 * j + 1] = atomicAdd(&o.big[1], (unsigned long long)cur.n);
      }
    } else {
      ts_chunk<UNI>(wsm, lane, cur, t_cur, sid, pid, svc, o);
    }
    if (!has_next) break;
    cur = nxt;
    t_cur = t_nxt;
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      sid[r] = sid_n[r];
      pid[r] = pid_n[r];
      svc[r] = svc_n[r];
    }
  }
  };
#ifndef ANOMOD_TS_DYN
#define ANOMOD_TS_DYN 2
#endif
#ifndef ANOMOD_TS_DYN_SEG
#define ANOMOD_TS_DYN_SEG 512
#endif
  // As the edge kernel: a static share per wave, then the last 1/ANOMOD_TS_DYN
  // of the traces in segments of kDynSeg from a global counter.
  constexpr uint64_t kDynSeg = ANOMOD_TS_DYN_SEG;
  const uint64_t n_static =
      ANOMOD_TS_DYN ? n_traces - n_traces / (ANOMOD_TS_DYN ? ANOMOD_TS_DYN : 1) : n_traces;
  uint64_t t_begin = uniform64(n_static * gw / nw);
  uint64_t t_end = uniform64(n_static * (gw + 1) / nw);
  while (true) {
    if (t_begin < t_end) run(t_begin, t_end);
    if (!ANOMOD_TS_DYN || n_static == n_traces) break;
    unsigned long long g = 0;
    if (lane == 0) g = atomicAdd(o.ctr, (unsigned long long)kDynSeg);
    g = __shfl(g, 0);
    t_begin = uniform64(n_static + g);
    if (t_begin >= n_traces) break;
    t_end = uniform64(t_begin + kDynSeg < n_traces ? t_begin + kDynSeg : n_traces);
  }
}

}  // namespace
}  // namespace anomod

using namespace anomod;

extern "C" {

int anomod_trace_structure_spans(anomod_ctx* ctx, const anomod_spans* spans,
                                 anomod_trace_struct_out* out) {
  ANOMOD_REQUIRE(nullptr, ctx && spans && out, "anomod_trace_structure_spans: NULL argument");
  ANOMOD_REQUIRE(ctx, out->n_services >= 1 && out->n_services <= 4096,
                 "n_services=%u out of range [1, 4096]", out->n_services);
  ANOMOD_REQUIRE(ctx, spans->device == ctx->device, "span set lives on another device");
  ANOMOD_REQUIRE(ctx, spans->grouped, "span set is not grouped by trace: anomod_spans_group first");
  ANOMOD_REQUIRE(ctx, spans->n_spans == 0 || spans->max_svc < out->n_services,
                 "span service index %u >= n_services %u", spans->max_svc, out->n_services);
  if (int rc = bind(ctx)) return rc;
  const uint64_t n = spans->n_spans, nt = spans->n_traces;
  const uint32_t words = (out->n_services + 63u) / 64u;
  // device outputs: parent_pos | depth | n_children (u32 x n), flags (u8 x n),
  // n_roots (u32 x nt), svc_mask (u64 x nt x words)
  const size_t off_depth = n * 4, off_cnt = 2 * n * 4, off_flags = 3 * n * 4;
  const size_t off_roots = (off_flags + n + 7) & ~(size_t)7;
  const size_t off_mask = (off_roots + nt * 4 + 7) & ~(size_t)7;
  // + the long-trace counters and list (traces > kStage spans: at most
  // n / (kStage + 1) of them; none when the longest trace is known to fit)
  const uint64_t big_cap = spans->max_trace_len <= (uint64_t)kStage
                               ? 0
                               : std::min<uint64_t>(nt, n / (uint64_t)(kStage + 1));
  const size_t off_big = (off_mask + nt * words * 8 + 15) & ~(size_t)15;
  const size_t off_ctr = off_big + 32;
  const size_t off_list = off_ctr + 8;
  const size_t bytes = off_list + big_cap * 16;
  // the ctx's scratch slots (reused by the next call instead of freed)
  char* d = nullptr;
  if (int rc = ensure_scratch(ctx, kScratchTraceStruct, bytes, reinterpret_cast<void**>(&d)))
    return rc;
  uint32_t* scr = nullptr;
  auto fail = [&](hipError_t e, const char* what) {
    set_error(ctx, "%s failed: %s", what, hipGetErrorString(e));
    return ANOMOD_EHIP;
  };
  hipError_t e = hipMemsetAsync(d + off_cnt, 0, n * 4, ctx->stream);
  if (e == hipSuccess) e = hipMemsetAsync(d + off_mask, 0, nt * words * 8, ctx->stream);
  if (e == hipSuccess) e = hipMemsetAsync(d + off_big, 0, 40, ctx->stream);  // big counters + ctr
  if (e != hipSuccess) return fail(e, "hipMemsetAsync");
  TsOut o;
  o.parent_pos = reinterpret_cast<uint32_t*>(d);
  o.depth = reinterpret_cast<uint32_t*>(d + off_depth);
  o.n_children = reinterpret_cast<uint32_t*>(d + off_cnt);
  o.flags = reinterpret_cast<uint8_t*>(d + off_flags);
  o.n_roots = reinterpret_cast<uint32_t*>(d + off_roots);
  o.svc_mask = reinterpret_cast<unsigned long long*>(d + off_mask);
  o.words = words;
  o.ctr = reinterpret_cast<unsigned long long*>(d + off_ctr);
  o.big = reinterpret_cast<unsigned long long*>(d + off_big);
  o.big_list = reinterpret_cast<unsigned long long*>(d + off_list);
  o.scr = nullptr;
  o.scr_n = 0;
  if (int rc = stage_begin(ctx, kStageTraceStruct)) return rc;
  if (nt > 0) {
    // ids unique within every trace (the set's declaration; ANOMOD_UNIQUE_SCAN=0
    // forces the general scan): no own-id scans, no duplicate path
    const char* us = getenv("ANOMOD_UNIQUE_SCAN");
    const bool uni = spans->unique_ids && !(us && !strcmp(us, "0"));
    auto kfn = uni ? trace_struct_kernel<true> : trace_struct_kernel<false>;
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kfn),
                                                     kTsThreads, 0);
    if (e != hipSuccess) return fail(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    const uint64_t grid = (uint64_t)ctx->num_cus * (uint64_t)(per_cu > 0 ? per_cu : 1);
    hipLaunchKernelGGL(kfn, dim3((unsigned)grid), dim3(kTsThreads), 0, ctx->stream,
                       spans->span_id, spans->parent_span_id, spans->svc_flags, spans->trace_ptr,
                       nt, o);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(e, "trace_struct_kernel launch");
  }
  if (big_cap) {
    // the long traces listed by the walk -> scratch sized to their spans
    unsigned long long cnt[2] = {0, 0};
    e = hipMemcpyAsync(cnt, o.big, 16, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return fail(e, "reading the long-trace count");
    if (cnt[0]) {
      if (int rc = ensure_scratch(ctx, kScratchTsLong, cnt[1] * 16, reinterpret_cast<void**>(&scr),
                                  1u << kScratchTraceStruct))
        return rc;
      o.scr = scr;
      o.scr_n = cnt[1];
      hipLaunchKernelGGL(ts_big_kernel, dim3((unsigned)std::min<uint64_t>(cnt[0], ctx->num_cus)),
                         dim3(kBigThreads), 0, ctx->stream, spans->span_id, spans->parent_span_id,
                         spans->svc_flags, spans->trace_ptr, o);
      e = hipGetLastError();
      if (e != hipSuccess) return fail(e, "ts_big_kernel launch");
    }
  }
  if (int rc = stage_end(ctx, kStageTraceStruct)) return rc;
  auto d2h = [&](void* dst, const void* src, size_t nbytes) -> hipError_t {
    if (!dst || nbytes == 0) return hipSuccess;
    return hipMemcpyAsync(dst, src, nbytes, hipMemcpyDeviceToHost, ctx->stream);
  };
  e = d2h(out->parent_pos, o.parent_pos, n * 4);
  if (e == hipSuccess) e = d2h(out->depth, o.depth, n * 4);
  if (e == hipSuccess) e = d2h(out->n_children, o.n_children, n * 4);
  if (e == hipSuccess) e = d2h(out->span_flags, o.flags, n);
  if (e == hipSuccess) e = d2h(out->n_roots, o.n_roots, nt * 4);
  if (e == hipSuccess) e = d2h(out->svc_mask, o.svc_mask, nt * words * 8);
  unsigned long long too_long = 0;
  if (e == hipSuccess && big_cap) e = d2h(&too_long, o.big + 3, 8);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return fail(e, "trace-structure download");
  ANOMOD_REQUIRE(ctx, !too_long, "a trace holds 2^31 spans or more");
  return ANOMOD_OK;
}

int anomod_trace_structure(anomod_ctx* ctx, const anomod_span_soa* soa, uint64_t n_spans,
                           const uint64_t* trace_ptr, uint64_t n_traces,
                           anomod_trace_struct_out* out) {
  ANOMOD_REQUIRE(nullptr, ctx && soa && out, "anomod_trace_structure: NULL argument");
  anomod_spans* s = nullptr;
  if (int rc = anomod_spans_upload(ctx, soa, n_spans, trace_ptr, n_traces, &s)) return rc;
  const int rc = anomod_trace_structure_spans(ctx, s, out);
  anomod_spans_free(s);
  return rc;
}

}  // extern "C"
