// Ungrouped span sets -> grouped by trace: the segmented radix sort of
// BASELINE.json north_star (2) ("segmented radix sort by (traceId, ...)").
//
// Every span kernel of this library reads spans grouped by trace (the
// order jaeger_to_csv.py:21-32 and trace_collector.py:539-546 emit).  Spans
// that arrive interleaved across traces — the Elasticsearch path pulls
// sw_segment-* hits sorted by start_time over all traces
// (TT_collection-scripts/T-Dataset/enhanced_trace_collector.py:80-90,
// 109-110) — are grouped here first.  Trace membership is the trace_hash
// (equal hash = same trace).  Output order: traces by k = mix64(trace_hash)
// ascending (mix64 = the SplitMix64 finaliser, a bijection, so any hash
// distribution gives even buckets), spans of a trace in arrival order (the
// sort is stable), so parent resolution sees the trace's spans in the order
// the reference would (first match, trace_collector.py:424-443).
//
// Design (MI355X):
//  * P LSD passes over 8-bit digits of the top 8P bits of k.  Per pass: the
//    digit counts of every 4096-record tile (a read of trace_hash for the
//    first pass, of the 1-B digits the previous pass wrote beside its
//    records for the others), an exclusive scan of those counts over tiles
//    (reduce-then-scan: no chained look-back, no per-tile ticket), then ONE
//    scatter kernel: a tile is ranked stably with wave ballots (8 ballots
//    give each lane its same-digit peers; rank = popc of the lower peers; a
//    per-wave LDS counter per digit carries the running count down the
//    wave's 4 rows), staged in LDS in digit order and written as coalesced
//    digit runs — 32-B records (hash, span_id, parent, svc|flags, dur), the
//    last pass the grouped SoA columns themselves;
//  * with P = ceil(log2(n) / 8) the top 8P bits nearly always separate
//    traces; a scan over the grouped hashes lists every key change inside a
//    bucket of equal top bits; one wave per such bucket sorts it by (k,
//    arrival) — rank = #{smaller k} + #{equal k earlier} — into a scratch
//    copy that is then written back; a list overflow or a mixed bucket larger
//    than the wave's LDS reruns the sort with P + 1 (at P = 8 no bucket is
//    mixed), so the output never depends on P;
//  * trace_ptr: one pass over the grouped hashes, trace starts compacted
//    with ballot ranks and a decoupled look-back over 4096-span tiles.
// Bytes per span: 8 + 2 (P - 1) (tile counts) + 64 per radix pass + 8 (bucket
// list) + 8 (trace_ptr) + 8 per trace.
#include <algorithm>
#include <cmath>

#include <cstdlib>

#include "chunk.h"
#include "group.h"

namespace anomod {

namespace {

using chunk::wave_sync;
// Experiment-only ablation (never set in the shipped build; timing only,
// wrong output): 1 = every pass writes its staged tile to the tile's own rows.
#ifndef ANOMOD_GRP_ABL
#define ANOMOD_GRP_ABL 0
#endif
constexpr int kWv = 64;
constexpr int kSThreads = 1024;              // scatter workgroup
constexpr int kSWaves = kSThreads / kWv;
constexpr int kSPer = 4;                     // records per thread
constexpr int kSTile = kSThreads * kSPer;    // 4096 records per tile
constexpr int kRowsPerWave = kSTile / kSWaves / kWv;  // 4
constexpr int kDig = 256;
constexpr int kMaxPasses = 8;
constexpr int kTThreads = 1024;              // scan workgroup (bucket list / trace_ptr)
constexpr int kTPer = 16;
constexpr int kTTile = kTThreads * kTPer;    // 16384 spans: fewer tiles, fewer tickets
constexpr int kFixCap = 1024;                // records of a mixed bucket one wave sorts
constexpr int kFixWaves = 4;
constexpr uint64_t kValMask = (1ull << 54) - 1;
constexpr uint32_t kSpinLimit = 1u << 26;

__device__ inline uint64_t pack_state(uint32_t epoch, uint32_t flag, uint64_t v) {
  return ((uint64_t)epoch << 56) | ((uint64_t)flag << 54) | (v & kValMask);
}

__device__ inline void publish(uint64_t* w, uint64_t v) {
  __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sum of the predecessors' totals of one look-back lane (state words
// strided by `stride` per tile): aggregates (flag 1) are added and the walk
// continues, an inclusive prefix (flag 2) ends it.  A bounded spin: a
// predecessor that never publishes sets the error word instead of hanging.
__device__ uint64_t look_back(uint64_t* state, uint64_t stride, uint64_t tile, uint32_t lane,
                              uint32_t epoch, unsigned long long* err) {
  uint64_t excl = 0;
  int64_t j = (int64_t)tile - 1;
  uint32_t spins = 0;
  while (j >= 0) {
    const uint64_t w = __hip_atomic_load(&state[(uint64_t)j * stride + lane], __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t ep = (uint32_t)(w >> 56), fl = (uint32_t)(w >> 54) & 3u;
    if (ep != epoch || fl == 0u) {
      if (++spins > kSpinLimit) {
        atomicAdd(err, 1ull);
        return excl;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    excl += w & kValMask;
    if (fl == 2u) break;
    --j;
  }
  return excl;
}

// ---- per-tile digit counts and their exclusive scan over tiles -------------
// Reduce-then-scan instead of a decoupled look-back: a chained look-back over
// ~n/4096 tiles waits on predecessors' L2 round trips (measured: 36 % of the
// grouping time at 2^25 traces), while counting a tile's digits costs one
// more read of 1 B/span (8 B/span from trace_hash for the first pass): the
// previous pass writes every record's next digit beside it.
template <bool FROM_H>
__global__ __launch_bounds__(256) void group_tcount_kernel(const uint64_t* __restrict__ h,
                                                           const uint8_t* __restrict__ dig,
                                                           uint64_t n, int shift,
                                                           uint32_t* __restrict__ tcnt) {
  __shared__ uint32_t lh[kDig];
  const int tid = threadIdx.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * kSTile;
  lh[tid] = 0u;
  __syncthreads();
  if constexpr (FROM_H) {
#pragma unroll
    for (int j = 0; j < kSTile / 256; ++j) {
      const uint64_t p = t0 + (uint64_t)(j * 256 + tid);
      if (p < n) atomicAdd(&lh[(uint32_t)(mix64(h[p]) >> shift) & 255u], 1u);
    }
  } else {
    // 16 consecutive digits per thread (one 16-B load), 4096 per tile
    const uint64_t p0 = t0 + (uint64_t)tid * 16u;
    if (p0 + 16u <= n) {
      const uint4 v = *reinterpret_cast<const uint4*>(dig + p0);
      const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 16; ++q) atomicAdd(&lh[(wv[q >> 2] >> (8 * (q & 3))) & 255u], 1u);
    } else {
      for (uint64_t p = p0; p < n && p < p0 + 16u; ++p) atomicAdd(&lh[dig[p]], 1u);
    }
  }
  __syncthreads();
  tcnt[(uint64_t)blockIdx.x * kDig + tid] = lh[tid];
}

constexpr int kTScanRows = 256;  // tiles per block of the tile-count scan

// column sums of kTScanRows tiles (one thread per digit)
__global__ __launch_bounds__(kDig) void group_tscan_up_kernel(const uint32_t* __restrict__ tcnt,
                                                              uint64_t tiles,
                                                              uint32_t* __restrict__ bsum) {
  const uint64_t a = (uint64_t)blockIdx.x * kTScanRows;
  const uint64_t b = a + kTScanRows < tiles ? a + kTScanRows : tiles;
  uint32_t s = 0;
#pragma unroll 8
  for (uint64_t t = a; t < b; ++t) s += tcnt[t * kDig + threadIdx.x];
  bsum[(uint64_t)blockIdx.x * kDig + threadIdx.x] = s;
}

// one block: exclusive scan of the block sums down every digit, digit starts
// (exclusive scan of the digit totals) added in
__global__ __launch_bounds__(kDig) void group_tscan_top_kernel(uint32_t* __restrict__ bsum,
                                                               uint64_t nb) {
  __shared__ uint32_t wsum[kDig / kWv];
  const int d = threadIdx.x, lane = d & (kWv - 1), w = d / kWv;
  uint32_t run = 0;
  for (uint64_t b = 0; b < nb; ++b) {
    const uint32_t x = bsum[b * kDig + d];
    bsum[b * kDig + d] = run;
    run += x;
  }
  uint32_t inc = run;
#pragma unroll
  for (int o = 1; o < kWv; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == kWv - 1) wsum[w] = inc;
  __syncthreads();
  uint32_t start = inc - run;
  for (int ww = 0; ww < w; ++ww) start += wsum[ww];
  for (uint64_t b = 0; b < nb; ++b) bsum[b * kDig + d] += start;
}

// every tile's count replaced by the global start of its digit run
__global__ __launch_bounds__(kDig) void group_tscan_down_kernel(uint32_t* __restrict__ tcnt,
                                                                uint64_t tiles,
                                                                const uint32_t* __restrict__ bsum) {
  const uint64_t a = (uint64_t)blockIdx.x * kTScanRows;
  const uint64_t b = a + kTScanRows < tiles ? a + kTScanRows : tiles;
  uint32_t run = bsum[(uint64_t)blockIdx.x * kDig + threadIdx.x];
#pragma unroll 8
  for (uint64_t t = a; t < b; ++t) {
    const uint32_t x = tcnt[t * kDig + threadIdx.x];
    tcnt[t * kDig + threadIdx.x] = run;
    run += x;
  }
}

// ---- one stable LSD pass ----------------------------------------------------
// Tile = 4096 records (1024 threads x 4), ranked stably with wave ballots (8
// ballots give each lane its same-digit peers; rank = popc of the lower
// peers; a per-wave LDS counter per digit carries the count down the wave's
// 4 rows), staged in LDS in digit order and written as digit runs from the
// global run starts of the tile-count scan.  The last pass writes the grouped
// SoA columns; the others 32-B records plus the next pass's digit.
template <bool SOA_IN, bool SOA_OUT>
__global__ __launch_bounds__(kSThreads) void group_scatter_kernel(
    SoaIn sin, const GRec* __restrict__ ain, GRec* __restrict__ aout, SoaOut sout, uint64_t n,
    int shift, const uint32_t* __restrict__ toff, uint8_t* __restrict__ dnext) {
  __shared__ GRec stage[kSTile];                 // 128 KiB
  __shared__ uint16_t wcnt[kSWaves][kDig];       // per-wave digit counts, then wave offsets
  __shared__ uint8_t sdig[kSTile];
  __shared__ uint32_t tstart[kDig];              // tile-local start of each digit
  __shared__ uint32_t gbase[kDig];               // global start of each digit's run
  __shared__ uint32_t wsum_t[kDig / kWv];
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;

  // a record as two 16-B halves: (h, sid) and (pid, sf | dur << 32)
  const uint64_t tile = blockIdx.x;
  const uint64_t base = tile * kSTile;
  uint4 ra[kSPer], rb[kSPer];
#pragma unroll
  for (int k = 0; k < kSPer; ++k) {
    const uint64_t i = base + (uint64_t)(w * (kRowsPerWave * kWv) + k * kWv + lane);
    ra[k] = make_uint4(0, 0, 0, 0);
    rb[k] = make_uint4(0, 0, 0, 0);
    if (i < n) {
      if constexpr (SOA_IN) {
        const uint64_t h = sin.h[i], sid = sin.sid[i], pid = sin.pid[i];
        ra[k] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)sid, (uint32_t)(sid >> 32));
        rb[k] = make_uint4((uint32_t)pid, (uint32_t)(pid >> 32), sin.sf[i], sin.dur[i]);
      } else {
        const uint4* q = reinterpret_cast<const uint4*>(ain + i);
        ra[k] = q[0];
        rb[k] = q[1];
      }
    }
  }
  for (int i = tid; i < kSWaves * kDig / 2; i += kSThreads)
    reinterpret_cast<uint32_t*>(&wcnt[0][0])[i] = 0u;
  if (tid < kDig) gbase[tid] = toff[tile * kDig + tid];
  __syncthreads();
  uint32_t d[kSPer];
  bool v[kSPer];
#pragma unroll
  for (int k = 0; k < kSPer; ++k) {
    v[k] = base + (uint64_t)(w * (kRowsPerWave * kWv) + k * kWv + lane) < n;
    d[k] = (uint32_t)(mix64(((uint64_t)ra[k].y << 32) | ra[k].x) >> shift) & 255u;
  }

  // Wave multisplit, rows in order: peers = lanes of the row with the same
  // digit (8 ballots); rank = lower peers + the wave's running digit count.
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  uint32_t off[kSPer];
#pragma unroll
  for (int k = 0; k < kSPer; ++k) {
    uint64_t peers = __ballot(v[k]);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d[k] >> b) & 1u;
      const uint64_t bb = __ballot(v[k] && bit);
      peers &= bit ? bb : ~bb;
    }
    off[k] = 0;
    if (v[k]) {
      const uint64_t lower = peers & lt_mask;
      const uint32_t b0 = wcnt[w][d[k]];
      off[k] = b0 + (uint32_t)__popcll(lower);
      if (lower == 0ull) wcnt[w][d[k]] = (uint16_t)(b0 + (uint32_t)__popcll(peers));
    }
    wave_sync();
  }
  __syncthreads();

  // Per digit (threads 0..255): wave offsets + tile total, then the tile's
  // digit starts (block scan).
  if (tid < kDig) {
    uint32_t run = 0;
    for (int ww = 0; ww < kSWaves; ++ww) {
      const uint32_t c = wcnt[ww][tid];
      wcnt[ww][tid] = (uint16_t)run;
      run += c;
    }
    const uint32_t total = run;
    uint32_t inc = total;
#pragma unroll
    for (int o = 1; o < kWv; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o);
      if (lane >= o) inc += y;
    }
    tstart[tid] = inc - total;
    if (lane == kWv - 1) wsum_t[w] = inc;
  }
  __syncthreads();
  if (tid < kDig)
    for (int ww = 0; ww < w; ++ww) tstart[tid] += wsum_t[ww];
  __syncthreads();

  // Stage the tile in digit order.
#pragma unroll
  for (int k = 0; k < kSPer; ++k) {
    if (v[k]) {
      const uint32_t lp = tstart[d[k]] + wcnt[w][d[k]] + off[k];
      uint4* q = reinterpret_cast<uint4*>(&stage[lp]);
      q[0] = ra[k];
      q[1] = rb[k];
      sdig[lp] = (uint8_t)d[k];
    }
  }
  __syncthreads();
  const uint64_t nvalid = n - base < (uint64_t)kSTile ? n - base : (uint64_t)kSTile;
#pragma unroll
  for (int k = 0; k < kSPer; ++k) {
    const uint32_t p = (uint32_t)(tid + k * kSThreads);
    if (p < nvalid) {
      const uint32_t dd = sdig[p];
      const uint4* q = reinterpret_cast<const uint4*>(&stage[p]);
      const uint64_t g = (uint64_t)gbase[dd] + (p - tstart[dd]);
      const uint4 x0 = q[0], x1 = q[1];
      if (dnext)
        dnext[g] = (uint8_t)(mix64(((uint64_t)x0.y << 32) | x0.x) >> (shift + 8));
      if constexpr (SOA_OUT) {  // the last pass writes the grouped columns
        sout.h[g] = ((uint64_t)x0.y << 32) | x0.x;
        sout.sid[g] = ((uint64_t)x0.w << 32) | x0.z;
        sout.pid[g] = ((uint64_t)x1.y << 32) | x1.x;
        sout.sf[g] = x1.z;
        sout.dur[g] = x1.w;
      } else {
        uint4* o = reinterpret_cast<uint4*>(aout + g);
        o[0] = x0;
        o[1] = x1;
      }
    }
  }
}

// ---- key changes inside buckets (LIST) / trace_ptr (!LIST) ----------------
// One pass over the grouped hashes in 4096-span tiles (tile ids from a
// ticket, so a tile only waits on running predecessors): row j of a tile is
// 256 consecutive spans, one per thread (coalesced loads; the predecessor of
// a lane's span from its neighbour lane, across waves through LDS).  Events:
// LIST — a key that differs from its predecessor's while their top bits
// agree (a bucket holding several traces, sorted by group_fix_kernel);
// !LIST — a trace start.  Events are compacted in position order (ballot
// ranks, a scan over the tile's 64 (row, wave) counts, decoupled look-back
// over tiles; no same-address atomics) into `out` (list / trace_ptr); the
// total lands in *total (and closes trace_ptr).
template <bool LIST>
__global__ __launch_bounds__(kTThreads) void group_scan_kernel(
    const uint64_t* __restrict__ h, uint64_t n, int top_shift, uint64_t* __restrict__ out,
    uint64_t out_cap, uint64_t* __restrict__ state, uint32_t epoch,
    unsigned long long* __restrict__ ticket, unsigned long long* __restrict__ total,
    unsigned long long* __restrict__ err) {
  constexpr int kW = kTThreads / kWv;  // waves per block
  __shared__ uint64_t s_last[kTPer][kW];
  __shared__ uint32_t s_cnt[kTPer * kW];
  __shared__ unsigned long long s_tile, s_excl;
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  if (tid == 0) s_tile = atomicAdd(ticket, 1ull);
  __syncthreads();
  const uint64_t tile = s_tile;
  const uint64_t ntiles = (n + kTTile - 1) / kTTile;
  const uint64_t t0 = tile * kTTile;
  uint64_t x[kTPer];
#pragma unroll
  for (int j = 0; j < kTPer; ++j) {
    const uint64_t p = t0 + (uint64_t)(j * kTThreads + tid);
    x[j] = p < n ? h[p] : 0ull;
  }
  const uint64_t before = (tid == 0 && t0 > 0) ? h[t0 - 1] : ~0ull;
  if (lane == kWv - 1) {
#pragma unroll
    for (int j = 0; j < kTPer; ++j) s_last[j][w] = x[j];
  }
  __syncthreads();
  uint32_t ev = 0, below[kTPer];
#pragma unroll
  for (int j = 0; j < kTPer; ++j) {
    const uint64_t p = t0 + (uint64_t)(j * kTThreads + tid);
    uint64_t prev = __shfl_up(x[j], 1);
    if (lane == 0) prev = w > 0 ? s_last[j][w - 1] : (j > 0 ? s_last[j - 1][kW - 1] : before);
    bool e = false;
    if (p < n) {
      if constexpr (LIST)
        e = p > 0 && x[j] != prev && (mix64(x[j]) >> top_shift) == (mix64(prev) >> top_shift);
      else
        e = p == 0 || x[j] != prev;
    }
    const uint64_t b = __ballot(e);
    below[j] = __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                         __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
    ev |= (e ? 1u : 0u) << j;
    if (lane == 0) s_cnt[j * kW + w] = (uint32_t)__popcll(b);
  }
  __syncthreads();
  if (w == 0) {  // exclusive scan of the (row, wave) counts in position order
    constexpr int kE = kTPer * kW / kWv;  // entries per lane
    uint32_t c[kE], sum = 0;
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      c[e] = s_cnt[lane * kE + e];
      sum += c[e];
    }
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < kWv; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o);
      if (lane >= o) inc += y;
    }
    uint32_t run = inc - sum;
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      s_cnt[lane * kE + e] = run;
      run += c[e];
    }
    if (lane == kWv - 1) {
      const uint64_t tot = inc;
      uint64_t* st = state + tile;
      uint64_t excl = 0;
      if (tile == 0) {
        publish(st, pack_state(epoch, 2u, tot));
      } else {
        publish(st, pack_state(epoch, 1u, tot));
        excl = look_back(state, 1, tile, 0u, epoch, err);
        publish(st, pack_state(epoch, 2u, excl + tot));
      }
      s_excl = excl;
      if (tile == ntiles - 1) {
        *total = excl + tot;
        if (!LIST) out[excl + tot] = n;  // closes trace_ptr
      }
    }
  }
  __syncthreads();
  const uint64_t ex = s_excl;
#pragma unroll
  for (int j = 0; j < kTPer; ++j)
    if ((ev >> j) & 1u) {
      const uint64_t idx = ex + s_cnt[j * kW + w] + below[j];
      if (!LIST || idx < out_cap) out[idx] = t0 + (uint64_t)(j * kTThreads + tid);
    }
}

// ---- one wave per mixed bucket: sort it by (k, arrival) ------------------
// Reads the grouped columns (not written here) and writes the bucket's
// records in (k, arrival) order to the same rows of a scratch SoA, listing
// the bucket as owned[e] = start << 11 | size for group_fixback_kernel
// (0: entry e is not its bucket's first key change; its owner sorts it).
__global__ __launch_bounds__(kFixWaves * kWv) void group_fix_kernel(
    SoaOut a, uint64_t n, int top_shift, SoaOut out, const unsigned long long* __restrict__ list,
    uint64_t list_cap, const unsigned long long* __restrict__ cnt,
    unsigned long long* __restrict__ over, unsigned long long* __restrict__ owned) {
  __shared__ uint64_t lk[kFixWaves][kFixCap];
  const int lane = threadIdx.x & (kWv - 1), w = threadIdx.x / kWv;
  uint64_t m_list = *cnt;
  if (m_list > list_cap) m_list = list_cap;  // overflow: the host reruns with more passes
  uint64_t* keys = lk[w];
  for (uint64_t e = (uint64_t)blockIdx.x * kFixWaves + w; e < m_list;
       e += (uint64_t)gridDim.x * kFixWaves) {
    const uint64_t i = list[e];
    if (lane == 0) owned[e] = 0ull;  // set below when this entry owns its bucket
    const uint64_t ki = mix64(a.h[i]), kprev = mix64(a.h[i - 1]);
    const uint64_t top = ki >> top_shift;
    // bucket start: walk back from i - 1; this entry owns the bucket only if
    // it is the bucket's first key change (everything before it = kprev)
    uint64_t bs = 0;
    bool owner = true;
    for (uint64_t s0 = 0;; s0 += kWv) {
      const uint64_t off = s0 + lane + 1;  // position i - off
      const bool valid = off <= i;
      const uint64_t kj = valid ? mix64(a.h[i - off]) : 0;
      const bool same_top = valid && (kj >> top_shift) == top;
      const uint64_t end_m = __ballot(!same_top);
      const uint64_t bad_m = __ballot(same_top && kj != kprev);
      if (end_m) {
        const int f = __ffsll((long long)end_m) - 1;  // first lane past the bucket
        if (bad_m & ((1ull << f) - 1ull)) owner = false;
        bs = i - (s0 + (uint64_t)f);
        break;
      }
      if (bad_m) {
        owner = false;
        break;
      }
    }
    if (!owner) continue;
    uint64_t be = n;
    for (uint64_t j0 = i + 1; j0 < n; j0 += kWv) {
      const uint64_t j = j0 + lane;
      const bool same_top = j < n && (mix64(a.h[j]) >> top_shift) == top;
      const uint64_t end_m = __ballot(!same_top);
      if (end_m) {
        be = j0 + (uint64_t)(__ffsll((long long)end_m) - 1);
        break;
      }
    }
    const uint64_t m = be - bs;
    if (m > (uint64_t)kFixCap) {
      if (lane == 0) atomicAdd(over, 1ull);
      continue;
    }
    for (uint32_t q = lane; q < m; q += kWv) keys[q] = mix64(a.h[bs + q]);
    wave_sync();
    for (uint32_t q0 = 0; q0 < m; q0 += kWv) {
      const uint32_t q = q0 + lane;
      const bool act = q < m;
      const uint64_t kq = act ? keys[q] : 0;
      uint32_t rank = 0;
      for (uint32_t t = 0; t < m; ++t) {
        const uint64_t kt = keys[t];
        rank += (kt < kq || (kt == kq && t < q)) ? 1u : 0u;
      }
      if (act) {
        const uint64_t src = bs + q, p = bs + rank;
        out.h[p] = a.h[src];
        out.sid[p] = a.sid[src];
        out.pid[p] = a.pid[src];
        out.sf[p] = a.sf[src];
        out.dur[p] = a.dur[src];
      }
    }
    if (lane == 0) owned[e] = (bs << 11) | m;
    wave_sync();
  }
}

// ---- sorted mixed buckets back into the grouped columns --------------------
__global__ __launch_bounds__(256) void group_fixback_kernel(
    SoaOut cols, SoaOut sorted, const unsigned long long* __restrict__ owned, uint64_t list_cap,
    const unsigned long long* __restrict__ cnt) {
  const int lane = threadIdx.x & (kWv - 1);
  const uint64_t nb = *cnt < list_cap ? *cnt : list_cap;
  for (uint64_t e = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / kWv; e < nb;
       e += (uint64_t)gridDim.x * 256 / kWv) {
    const uint64_t bs = owned[e] >> 11, m = owned[e] & 2047u;  // m = 0: not an owner
    for (uint64_t q = lane; q < m; q += kWv) {
      const uint64_t p = bs + q;
      cols.h[p] = sorted.h[p];
      cols.sid[p] = sorted.sid[p];
      cols.pid[p] = sorted.pid[p];
      cols.sf[p] = sorted.sf[p];
      cols.dur[p] = sorted.dur[p];
    }
  }
}

// ---- synthetic arrival orders (bench / tests; not a product path) --------
// Keyed bijection of [0, m) (4-round Feistel over the next power of 4,
// cycle-walking back into range).
__device__ inline uint64_t feistel_perm(uint64_t x, uint64_t m, uint64_t key) {
  if (m <= 1) return 0;
  int bits = 64 - __clzll((long long)(m - 1));
  if (bits & 1) ++bits;
  const int half = bits / 2;
  const uint64_t mask = (1ull << half) - 1ull;
  do {
    uint64_t l = x >> half, r = x & mask;
    for (int round = 0; round < 4; ++round) {
      const uint64_t f = mix64(r ^ (key + 0x9E3779B97F4A7C15ull * (round + 1))) & mask;
      const uint64_t nl = r;
      r = l ^ f;
      l = nl;
    }
    x = (l << half) | r;
  } while (x >= m);
  return x;
}

// Window w (traces [w*W, (w+1)*W)) gathers its span range in a random order.
__global__ __launch_bounds__(256) void shuffle_window_kernel(SoaIn in, SoaOut out,
                                                             const uint64_t* __restrict__ tptr,
                                                             uint64_t n_traces, uint64_t W,
                                                             uint64_t seed) {
  const uint64_t nwin = (n_traces + W - 1) / W;
  for (uint64_t win = blockIdx.x; win < nwin; win += gridDim.x) {
    const uint64_t a = tptr[win * W];
    const uint64_t b = tptr[(win + 1) * W < n_traces ? (win + 1) * W : n_traces];
    const uint64_t m = b - a, key = mix64(seed ^ (win * 0xD1B54A32D192ED03ull));
    for (uint64_t q = threadIdx.x; q < m; q += 256) {
      const uint64_t src = a + feistel_perm(q, m, key);
      out.h[a + q] = in.h[src];
      out.sid[a + q] = in.sid[src];
      out.pid[a + q] = in.pid[src];
      out.sf[a + q] = in.sf[src];
      out.dur[a + q] = in.dur[src];
    }
  }
}

// One thread per trace: its spans in a random order (stays grouped).
__global__ __launch_bounds__(256) void shuffle_in_trace_kernel(SoaIn in, SoaOut out,
                                                               const uint64_t* __restrict__ tptr,
                                                               uint64_t n_traces, uint64_t seed) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < n_traces; t += stride) {
    const uint64_t a = tptr[t], m = tptr[t + 1] - a, key = mix64(seed ^ (t * 0xA24BAED4963EE407ull));
    for (uint64_t q = 0; q < m; ++q) {
      const uint64_t src = a + feistel_perm(q, m, key);
      if (out.h) out.h[a + q] = in.h[src];
      out.sid[a + q] = in.sid[src];
      out.pid[a + q] = in.pid[src];
      out.sf[a + q] = in.sf[src];
      out.dur[a + q] = in.dur[src];
    }
  }
}

// The second record buffer (aos[1]): the LSD passes' ping-pong and the
// sorting bucket kernels' grouped columns.  The ungrouped aggregation's join
// needs none of it (its edge records go to the trace_ptr buffer), so it is
// its own allocation, made only when a path that writes it runs.
int ensure_group_aos1(anomod_ctx* ctx) {
  GroupWs* ws = ctx->group_ws;
  if (ws->aos1_block) return ANOMOD_OK;
  const double t0 = host_now_ms();
  const bool ok = dev_malloc(ctx, &ws->aos1_block, ws->cap * sizeof(GRec)) == hipSuccess;
  host_record(ctx, kHostGroupAlloc, host_now_ms() - t0);
  if (!ok) {
    ws->aos1_block = nullptr;
    set_error(ctx, "hipMalloc failed for the trace-grouping record buffer of %llu spans",
              (unsigned long long)ws->cap);
    return ANOMOD_ENOMEM;
  }
  ws->aos[1] = static_cast<GRec*>(ws->aos1_block);
  return ANOMOD_OK;
}

int ensure_group_ws(anomod_ctx* ctx, uint64_t n, bool both_records) {
  GroupWs* ws = ctx->group_ws;
  if (ws && ws->cap >= n) return both_records ? ensure_group_aos1(ctx) : ANOMOD_OK;
  free_group_ws(ctx);
  ws = new GroupWs();
  ctx->group_ws = ws;
  const uint64_t cap = n ? n : 1;
  const uint64_t tiles = (cap + kSTile - 1) / kSTile;
  ws->cap = cap;
  ws->state_words = (cap + kTTile - 1) / kTTile;  // look-back words of the scans
  ws->list_cap = cap / 8 + 65536;
  // Bucket path: any geometry bucket_geom picks for n <= cap (digits of up
  // to 11 bits per level, 2^T buckets with T at most that of a 64-span mean,
  // or a level of 11 bits more).
  int tmax = 1;
  while (tmax < 22 && (cap >> tmax) > 64u) ++tmax;
  ws->bucket_cap = 1ull << std::min(22, tmax + 11);  // + a retry with 11-bit level B
  ws->tile_cap = tiles + 2048;
  const size_t tcnt_words = std::max<size_t>(tiles * kDig, ws->tile_cap * 2048);
  ws->tcnt_words = tcnt_words;
  const size_t bsum_words = (tiles / kTScanRows + 2) * 2048;
  // Bytes per span: 32 (the level-A record buffer) + 16 (two pair buffers;
  // the LSD path's 2-B digits live in the second, which only the bucket path
  // uses) + 8 (trace_ptr, or the join's edge records) + ~2 (tile counts,
  // lists) ~= 58 B, plus 32 for the second record buffer when a grouping
  // path needs it (ensure_group_aos1), plus the input set's 32 B: 1.15e9
  // spans take ~67 (+ 37) + 37 GB of the 288 GB, and n is bounded by the u32
  // positions (< 2^32) before HBM runs out.
  static_assert(8 >= 2 + 1, "the digits fit a pair buffer");
  const size_t sizes[] = {cap * sizeof(GRec), (cap + 1) * 8,
                          ws->state_words * 8, kMiscWords * 8, ws->list_cap * 8,
                          ws->list_cap * 8, tcnt_words * 4, bsum_words * 4,
                          (ws->bucket_cap + 1) * 4, 2049 * 4, 2049 * 4, ws->tile_cap * 4,
                          (ws->bucket_cap + 1) * 4, ws->bucket_cap * 4,
                          (ws->bucket_cap / 4096 + 2) * 4, cap * 8, cap * 8 + 32};
  void** ptrs[] = {(void**)&ws->aos[0], (void**)&ws->tptr,
                   (void**)&ws->state, (void**)&ws->misc, (void**)&ws->list,
                   (void**)&ws->owned, (void**)&ws->tcnt, (void**)&ws->bsum,
                   (void**)&ws->bstart, (void**)&ws->bsA, (void**)&ws->btile, (void**)&ws->tmap,
                   (void**)&ws->dcnt, (void**)&ws->over, (void**)&ws->part,
                   (void**)&ws->pairs[0], (void**)&ws->pairs[1]};
  constexpr int kBufs = sizeof(sizes) / sizeof(sizes[0]);
  static_assert(kBufs == sizeof(ptrs) / sizeof(ptrs[0]), "one pointer per size");
  // Carved 2-MiB aligned from one allocation (the radix passes' time varies by
  // process either way: 98.8-113.4 ms at 2^27 traces over 12 processes of
  // this form, 100.0-112.6 over 8 with one hipMalloc per buffer).
  constexpr size_t kAlign = size_t(2) << 20;
  size_t total = 0;
  for (size_t z : sizes) total += (z + kAlign - 1) / kAlign * kAlign;
  double t0 = host_now_ms();
  bool ok = dev_malloc(ctx, &ws->block, total) == hipSuccess;
  host_record(ctx, kHostGroupAlloc, host_now_ms() - t0);
  if (ok) {
    size_t off = 0;
    for (int i = 0; i < kBufs; ++i) {
      *ptrs[i] = static_cast<char*>(ws->block) + off;
      off += (sizes[i] + kAlign - 1) / kAlign * kAlign;
    }
    // the LSD path's next-pass digits (2 B per span + slack) share the
    // level-B pair buffer: the two paths never hold both at once (the LSD
    // path runs alone, or after the bucket path handed the set back)
    ws->dig = reinterpret_cast<uint8_t*>(ws->pairs[1]);
  } else {
    ws->block = nullptr;
  }
  t0 = host_now_ms();
  ok = ok && hipHostMalloc(reinterpret_cast<void**>(&ws->h_misc), kMiscWords * 8,
                           hipHostMallocDefault) == hipSuccess;
  host_record(ctx, kHostGroupPinned, host_now_ms() - t0);
  if (!ok) {
    free_group_ws(ctx);
    set_error(ctx, "hipMalloc failed for the trace-grouping workspace of %llu spans "
              "(~%llu GB)", (unsigned long long)n, (unsigned long long)(total >> 30));
    return ANOMOD_ENOMEM;
  }
  ANOMOD_HIP(ctx, hipMemsetAsync(ws->state, 0, ws->state_words * 8, ctx->stream));
  ws->epoch = 0;
  return both_records ? ensure_group_aos1(ctx) : ANOMOD_OK;
}

uint32_t next_epoch(anomod_ctx* ctx) {
  GroupWs* ws = ctx->group_ws;
  if (ws->epoch >= 255u) {  // the 8-bit tag wraps: clear the look-back words once
    (void)hipMemsetAsync(ws->state, 0, ws->state_words * 8, ctx->stream);
    ws->epoch = 0;
  }
  return ++ws->epoch;
}

// ANOMOD_GROUP_PATH=lsd: the LSD path even where the bucket path applies
// (A/B timing, tests).
bool force_lsd() {
  const char* e = std::getenv("ANOMOD_GROUP_PATH");
  return e && e[0] == 'l';
}

int group_run(anomod_ctx* ctx, const anomod_spans* in, GroupResult* res, bool want_h = true) {
  const uint64_t n = in->n_spans;
  if (n > 0xFFFFFFFFull - kSTile) {  // u32 run starts (the workspace alone would be > 300 GB)
    set_error(ctx, "trace grouping of %llu spans: at most 2^32 - %d per call",
              (unsigned long long)n, kSTile);
    return ANOMOD_EINVAL;
  }
  if (int rc = ensure_group_ws(ctx, n, true)) return rc;
  GroupWs* ws = ctx->group_ws;
  if (n > 0 && !force_lsd()) {
    bool fallback = false;
    if (int rc = bucket_group_run(ctx, in, res, &fallback, nullptr, 0, want_h)) return rc;
    if (!fallback) {
      ctx->group_path = 1;
      ctx->group_levels = res->passes;
      ctx->group_bits = res->bits;
      return ANOMOD_OK;
    }
  }
  int P = 1;
  while (P < kMaxPasses && (1ull << (8 * P)) < n) ++P;  // 2^(8P) >= n
  const SoaIn sin{in->trace_hash, in->span_id, in->parent_span_id, in->svc_flags, in->dur_us};
  const uint64_t tiles = (n + kSTile - 1) / kSTile;
  for (;; ++P) {
    ANOMOD_HIP(ctx, hipMemsetAsync(ws->misc, 0, kMiscWords * 8, ctx->stream));
    const int shift0 = 64 - 8 * P;
    // The last pass writes the grouped SoA columns into the buffer it would
    // have written records to; the other buffer (the last pass's input) is
    // the scratch group_fix_kernel sorts mixed buckets into.
    const uint64_t cap = ws->cap;
    auto soa_of = [cap](GRec* buf) {
      char* ob = reinterpret_cast<char*>(buf);
      return SoaOut{reinterpret_cast<uint64_t*>(ob), reinterpret_cast<uint64_t*>(ob + 8 * cap),
                    reinterpret_cast<uint64_t*>(ob + 16 * cap),
                    reinterpret_cast<uint32_t*>(ob + 24 * cap),
                    reinterpret_cast<uint32_t*>(ob + 28 * cap)};
    };
    const SoaOut cols = soa_of(ws->aos[(P - 1) & 1]);
    const SoaOut scratch = soa_of(ws->aos[P & 1]);
    if (n > 0) {
      const uint64_t nb = (tiles + kTScanRows - 1) / kTScanRows;
      const GRec* src = nullptr;
      for (int p = 0; p < P; ++p) {
        GRec* dst = ws->aos[p & 1];
        const int shift = shift0 + 8 * p;
        if (p == 0)
          hipLaunchKernelGGL(group_tcount_kernel<true>, dim3((unsigned)tiles), dim3(256), 0,
                             ctx->stream, in->trace_hash, nullptr, n, shift, ws->tcnt);
        else
          hipLaunchKernelGGL(group_tcount_kernel<false>, dim3((unsigned)tiles), dim3(256), 0,
                             ctx->stream, nullptr, ws->dig, n, shift, ws->tcnt);
        hipLaunchKernelGGL(group_tscan_up_kernel, dim3((unsigned)nb), dim3(kDig), 0, ctx->stream,
                           ws->tcnt, tiles, ws->bsum);
        hipLaunchKernelGGL(group_tscan_top_kernel, dim3(1), dim3(kDig), 0, ctx->stream, ws->bsum,
                           nb);
        hipLaunchKernelGGL(group_tscan_down_kernel, dim3((unsigned)nb), dim3(kDig), 0,
                           ctx->stream, ws->tcnt, tiles, ws->bsum);
        auto fn = p == 0 ? (p == P - 1 ? group_scatter_kernel<true, true>
                                       : group_scatter_kernel<true, false>)
                         : (p == P - 1 ? group_scatter_kernel<false, true>
                                       : group_scatter_kernel<false, false>);
        hipLaunchKernelGGL(fn, dim3((unsigned)tiles), dim3(kSThreads), 0, ctx->stream, sin, src,
                           dst, cols, n, shift, ws->tcnt, p == P - 1 ? nullptr : ws->dig);
        ANOMOD_HIP(ctx, hipGetLastError());
        src = dst;
      }
      const int top_shift = 64 - 8 * P;  // 0 at P = 8: every bucket is one key
      const unsigned scan_grid = (unsigned)((n + kTTile - 1) / kTTile);
      uint32_t ep = next_epoch(ctx);
      hipLaunchKernelGGL(group_scan_kernel<true>, dim3(scan_grid), dim3(kTThreads), 0,
                         ctx->stream, cols.h, n, top_shift, reinterpret_cast<uint64_t*>(ws->list),
                         ws->list_cap, ws->state, ep, ws->misc + kMiscTicket,
                         ws->misc + kMiscListCnt, ws->misc + kMiscErr);
      ANOMOD_HIP(ctx, hipGetLastError());
      hipLaunchKernelGGL(group_fix_kernel, dim3(ctx->num_cus * 4), dim3(kFixWaves * kWv), 0,
                         ctx->stream, cols, n, top_shift, scratch, ws->list, ws->list_cap,
                         ws->misc + kMiscListCnt, ws->misc + kMiscOver, ws->owned);
      ANOMOD_HIP(ctx, hipGetLastError());
      hipLaunchKernelGGL(group_fixback_kernel, dim3(ctx->num_cus * 4), dim3(256), 0, ctx->stream,
                         cols, scratch, ws->owned, ws->list_cap, ws->misc + kMiscListCnt);
      ANOMOD_HIP(ctx, hipGetLastError());
      ep = next_epoch(ctx);
      hipLaunchKernelGGL(group_scan_kernel<false>, dim3(scan_grid), dim3(kTThreads), 0,
                         ctx->stream, cols.h, n, top_shift, ws->tptr, n + 1, ws->state, ep,
                         ws->misc + kMiscTicket + 1, ws->misc + kMiscTraces, ws->misc + kMiscErr);
      ANOMOD_HIP(ctx, hipGetLastError());
    } else {
      ANOMOD_HIP(ctx, hipMemsetAsync(ws->tptr, 0, 8, ctx->stream));
    }
    ANOMOD_HIP(ctx, hipMemcpyAsync(ws->h_misc + kMiscRead, ws->misc + kMiscRead,
                                   (kMiscWords - kMiscRead) * 8, hipMemcpyDeviceToHost,
                                   ctx->stream));
    ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const unsigned long long* hm = ws->h_misc;
    if (hm[kMiscErr]) {
      set_error(ctx, "trace grouping: a look-back wait timed out (%llu lanes)", hm[kMiscErr]);
      return ANOMOD_EHIP;
    }
    if (n > 0 && P < kMaxPasses && (hm[kMiscListCnt] > ws->list_cap || hm[kMiscOver] > 0))
      continue;  // too many traces share their top 8P bits: one more pass
    res->cols = cols;
    res->n_traces = n > 0 ? hm[kMiscTraces] : 0;
    res->tptr = ws->tptr;
    res->passes = P;
    res->bits = 8 * P;
    ctx->group_path = 0;
    ctx->group_levels = P;
    ctx->group_bits = 8 * P;
    return ANOMOD_OK;
  }
}

anomod_spans view_of(const anomod_spans* in, const GroupResult& g) {
  anomod_spans v;
  v.device = in->device;
  v.n_spans = in->n_spans;
  v.n_traces = g.n_traces;
  v.max_svc = in->max_svc;
  v.grouped = true;
  v.unique_ids = in->unique_ids;  // grouping permutes spans, ids stay per trace
  v.max_trace_len = in->max_trace_len;  // and traces keep their spans (long-trace pass sizing)
  v.trace_hash = g.cols.h;
  v.span_id = g.cols.sid;
  v.parent_span_id = g.cols.pid;
  v.svc_flags = g.cols.sf;
  v.dur_us = g.cols.dur;
  v.trace_ptr = g.tptr;
  return v;
}

}  // namespace

void free_group_ws(anomod_ctx* ctx) {
  GroupWs* ws = ctx->group_ws;
  if (!ws) return;
  (void)hipStreamSynchronize(ctx->stream);
  if (ws->block) (void)hipFree(ws->block);
  if (ws->aos1_block) (void)hipFree(ws->aos1_block);
  if (ws->h_misc) (void)hipHostFree(ws->h_misc);
  delete ws;
  ctx->group_ws = nullptr;
}

}  // namespace anomod

using namespace anomod;

extern "C" {

int anomod_spans_upload_ungrouped(anomod_ctx* ctx, const anomod_span_soa* soa, uint64_t n_spans,
                                  anomod_spans** out) {
  ANOMOD_REQUIRE(nullptr, ctx && soa && out, "anomod_spans_upload_ungrouped: NULL argument");
  ANOMOD_REQUIRE(ctx, n_spans == 0 || soa->trace_hash,
                 "an ungrouped span set needs trace_hash (it defines the traces)");
  if (int rc = anomod_spans_upload(ctx, soa, n_spans, nullptr, 0, out)) return rc;
  (*out)->grouped = false;
  return ANOMOD_OK;
}

int anomod_ctx_reserve_grouping(anomod_ctx* ctx, uint64_t n_spans, int both_records) {
  ANOMOD_REQUIRE(nullptr, ctx, "anomod_ctx_reserve_grouping: NULL ctx");
  ANOMOD_REQUIRE(ctx, n_spans <= 0xFFFFFFFFull - kSTile,
                 "trace grouping of %llu spans: at most 2^32 - %d per call",
                 (unsigned long long)n_spans, kSTile);
  if (int rc = bind(ctx)) return rc;
  return ensure_group_ws(ctx, n_spans, both_records != 0);
}

int anomod_ctx_group_info(const anomod_ctx* ctx, int* path, int* levels, int* bits) {
  ANOMOD_REQUIRE(nullptr, ctx && path && levels && bits, "anomod_ctx_group_info: NULL argument");
  *path = ctx->group_path;
  *levels = ctx->group_levels;
  *bits = ctx->group_bits;
  return ANOMOD_OK;
}

int anomod_spans_grouped(const anomod_spans* spans, int* grouped) {
  ANOMOD_REQUIRE(nullptr, spans && grouped, "anomod_spans_grouped: NULL argument");
  *grouped = spans->grouped ? 1 : 0;
  return ANOMOD_OK;
}

int anomod_spans_group(anomod_ctx* ctx, const anomod_spans* in, anomod_spans** out) {
  ANOMOD_REQUIRE(nullptr, ctx && in && out, "anomod_spans_group: NULL argument");
  *out = nullptr;
  ANOMOD_REQUIRE(ctx, in->device == ctx->device, "span set lives on another device");
  ANOMOD_REQUIRE(ctx, in->n_spans == 0 || in->trace_hash, "span set has no trace_hash");
  if (int rc = bind(ctx)) return rc;
  if (int rc = stage_begin(ctx, kStageGroup)) return rc;
  GroupResult g;
  if (int rc = group_run(ctx, in, &g)) return rc;
  if (int rc = stage_end(ctx, kStageGroup)) return rc;
  anomod_spans* s = nullptr;
  if (int rc = alloc_spans(ctx, in->n_spans, g.n_traces, true, &s)) return rc;
  s->max_svc = in->max_svc;
  s->unique_ids = in->unique_ids;
  const uint64_t n = in->n_spans;
  hipError_t e = hipSuccess;
  auto cp = [&](void* d, const void* src, size_t bytes) {
    if (e == hipSuccess && bytes)
      e = hipMemcpyAsync(d, src, bytes, hipMemcpyDeviceToDevice, ctx->stream);
  };
  cp(s->trace_hash, g.cols.h, n * 8);
  cp(s->span_id, g.cols.sid, n * 8);
  cp(s->parent_span_id, g.cols.pid, n * 8);
  cp(s->svc_flags, g.cols.sf, n * 4);
  cp(s->dur_us, g.cols.dur, n * 4);
  cp(s->trace_ptr, g.tptr, (g.n_traces + 1) * 8);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    free_spans(s);
    set_error(ctx, "copying the grouped span set failed: %s", hipGetErrorString(e));
    return ANOMOD_EHIP;
  }
  *out = s;
  return ANOMOD_OK;
}

int anomod_edge_aggregate_ungrouped(anomod_ctx* ctx, const anomod_spans* spans,
                                    uint32_t n_services, anomod_edge_table* out) {
  ANOMOD_REQUIRE(nullptr, ctx && spans && out, "anomod_edge_aggregate_ungrouped: NULL argument");
  if (spans->grouped) return anomod_edge_aggregate_spans(ctx, spans, n_services, out);
  int rc = ANOMOD_OK;
  if (spans->device != ctx->device) {
    set_error(ctx, "span set lives on another device");
    rc = ANOMOD_EINVAL;
  } else if (spans->n_spans && !spans->trace_hash) {
    set_error(ctx, "span set has no trace_hash");
    rc = ANOMOD_EINVAL;
  }
  GroupResult g;
  if (rc == ANOMOD_OK) rc = bind(ctx);
  // Fused path (bucket grouping only; the default, ANOMOD_UNGROUPED_FUSED=0
  // turns it off): the buckets write one 8-B edge record per span instead of
  // the grouped columns, and the edge table is taken from those records — no
  // grouped columns, no trace_ptr, no walk over them.  Each bucket finds the
  // parents by an LDS hash join (bk_bucket_join_kernel, no sort): 52.6 + 2.1
  // vs 57.8 + 5.7 ms unfused at 2^27 SN traces (gpurun_out/r4u_ab.log; with
  // the sorting bucket kernel's in-trace scan, ANOMOD_FUSED_JOIN=0, it was
  // 71.0 + 2.1).  A set whose buckets hold traces of thousands of spans side
  // by side takes the unfused path below.
  const char* fz = std::getenv("ANOMOD_UNGROUPED_FUSED");
  const uint64_t n = spans->n_spans;
  if (rc == ANOMOD_OK && n > 0 && !force_lsd() && !(fz && fz[0] == '0') && n_services >= 1 &&
      n_services <= 4096 && spans->max_svc < n_services && n <= 0xFFFFFFFFull - 4096) {
    // (the sorting bucket kernels' edge form, ANOMOD_FUSED_JOIN=0, and the
    // records-through-level-B join write the second record buffer)
    const char* fj = std::getenv("ANOMOD_FUSED_JOIN");
    rc = ensure_group_ws(ctx, n, join_records_through_b() || (fj && fj[0] == '0'));
    bool fallback = true;
    if (rc == ANOMOD_OK) rc = stage_begin(ctx, kStageGroup);
    if (rc == ANOMOD_OK) {
      const double t0 = host_now_ms();
      // edge records (8 B per span) in trace_ptr's buffer, which the join
      // path leaves unused
      uint64_t* erec = ctx->group_ws->tptr;
      rc = bucket_group_run(ctx, spans, &g, &fallback, erec, n_services);
      host_record(ctx, kHostGroupWall, host_now_ms() - t0);
      if (rc == ANOMOD_OK) rc = stage_end(ctx, kStageGroup);
      if (rc == ANOMOD_OK && !fallback) {
        ctx->group_path = g.join ? 2 : 3;  // join / fused-sort
        ctx->group_levels = g.passes;
        ctx->group_bits = g.bits;
        return edge_aggregate_records(ctx, erec, n, n_services, &spans->hist_form, out);
      }
    }
    if (rc != ANOMOD_OK) return comm_agree(ctx, rc);
  }
  if (rc == ANOMOD_OK) rc = stage_begin(ctx, kStageGroup);
  if (rc == ANOMOD_OK) rc = group_run(ctx, spans, &g, /*want_h=*/false);
  if (rc == ANOMOD_OK) rc = stage_end(ctx, kStageGroup);
  if (rc != ANOMOD_OK) return comm_agree(ctx, rc);  // peers learn of it before their reduce
  anomod_spans view = view_of(spans, g);
  view.hist_form = spans->hist_form;  // the set's hints: learned once, kept on the set
  view.order = spans->order;
  const int rc2 = anomod_edge_aggregate_spans(ctx, &view, n_services, out);
  spans->hist_form = view.hist_form;
  spans->order = view.order;
  return rc2;
}

int anomod_spans_shuffle(anomod_ctx* ctx, const anomod_spans* in, uint64_t seed,
                         uint64_t window_traces, anomod_spans** out) {
  ANOMOD_REQUIRE(nullptr, ctx && in && out, "anomod_spans_shuffle: NULL argument");
  *out = nullptr;
  ANOMOD_REQUIRE(ctx, in->grouped, "anomod_spans_shuffle needs a grouped span set");
  ANOMOD_REQUIRE(ctx, window_traces == 0 || in->n_spans == 0 || in->trace_hash,
                 "interleaving traces needs trace_hash");
  ANOMOD_REQUIRE(ctx, in->device == ctx->device, "span set lives on another device");
  if (int rc = bind(ctx)) return rc;
  const bool keep = window_traces == 0;  // in-trace shuffle: stays grouped
  anomod_spans* s = nullptr;
  if (int rc = alloc_spans(ctx, in->n_spans, keep ? in->n_traces : 0, in->trace_hash != nullptr,
                           &s))
    return rc;
  s->max_svc = in->max_svc;
  s->max_trace_len = in->max_trace_len;  // traces keep their spans either way
  s->unique_ids = in->unique_ids;
  s->grouped = keep;
  const SoaIn sin{in->trace_hash, in->span_id, in->parent_span_id, in->svc_flags, in->dur_us};
  const SoaOut sout{s->trace_hash, s->span_id, s->parent_span_id, s->svc_flags, s->dur_us};
  hipError_t e = hipSuccess;
  if (keep) {
    e = hipMemcpyAsync(s->trace_ptr, in->trace_ptr, (in->n_traces + 1) * 8,
                       hipMemcpyDeviceToDevice, ctx->stream);
    if (e == hipSuccess && in->trace_hash && in->n_spans)
      e = hipMemcpyAsync(s->trace_hash, in->trace_hash, in->n_spans * 8,
                         hipMemcpyDeviceToDevice, ctx->stream);  // constant within a trace
    if (e == hipSuccess && in->n_traces) {
      SoaOut o = sout;
      o.h = nullptr;
      hipLaunchKernelGGL(shuffle_in_trace_kernel, dim3(ctx->num_cus * 8), dim3(256), 0,
                         ctx->stream, sin, o, in->trace_ptr, in->n_traces, seed);
      e = hipGetLastError();
    }
  } else {
    if (e == hipSuccess) e = hipMemsetAsync(s->trace_ptr, 0, 8, ctx->stream);
    if (e == hipSuccess && in->n_traces) {
      hipLaunchKernelGGL(shuffle_window_kernel, dim3(ctx->num_cus * 16), dim3(256), 0, ctx->stream,
                         sin, sout, in->trace_ptr, in->n_traces, window_traces, seed);
      e = hipGetLastError();
    }
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    free_spans(s);
    set_error(ctx, "span shuffle failed: %s", hipGetErrorString(e));
    return ANOMOD_EHIP;
  }
  *out = s;
  return ANOMOD_OK;
}

}  // extern "C"
