// Trace grouping, bucket path: a stable MSD scatter of the 32-B records over
// the top DA bits of k = mix64(trace_hash), a second level over 8-B PAIRS
// (the next 32 key bits << 32 | the record's position), then one workgroup
// per bucket of ~1000 spans that sorts the bucket's pairs in LDS, gathers
// each record by its position from the level-A output and writes the grouped
// SoA columns and the bucket's trace starts.  Same output as the LSD path of
// group.hip (traces by k ascending, spans of a trace in arrival order — the
// order the reference's first-match parent rule sees,
// trace_collector.py:424-443).
//
// Per span (n = 1.15e9: T = 20, DA = 9, DB = 11):
//   level A: 8 (count: trace_hash) + 32 (SoA in) + 32 (records out) + 8 (pairs out)
//   level B: 8 (count: pairs) + 8 + 8 (pairs in, out)
//   buckets: 8 (pairs) + 32 (records gathered: the buckets in flight lie in one
//            ~72 MB level-A bucket, so the gathers hit the Infinity Cache) +
//            32 (SoA columns out) + 24/trace (trace starts, trace_ptr)
// + tile counts (4 B per tile and digit, five touches) ≈ 180 B/span, against
// ~220 B/span when level B moved the 32-B records (r03) and 286 B/span for
// the LSD path.
//
// Pairs sort exactly: a pair's value orders by (key bits, position), and
// positions inside a level-A bucket are arrival order (level A is stable), so
// sorting a bucket's pairs as u64 gives (k, arrival) order — unless two
// traces of a bucket share all T + 32 key bits the pairs see.  The bucket
// kernel checks the gathered records' full keys and re-ranks such a bucket by
// (k, arrival) (rare: ~1e-6 of the buckets at 1.2e8 traces; crafted hashes
// in the tests).
//
// A bucket larger than the small kernel's 2048 spans (a long trace, or the
// tail of the size distribution) goes to a list that a 1024-thread kernel
// works through: up to 8192 spans with its pairs in LDS, beyond that by a
// one-wave walk over the bucket's distinct keys (bucket_huge).  Only a huge
// bucket with more distinct keys than that walk holds (adversarial hashes)
// makes the caller regroup with the LSD path.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "chunk.h"
#include "group.h"

namespace anomod {
namespace {

using chunk::wave_sync;
// Experiment-only builds (never set in the shipped library):
//  2 = level A stores nothing, then the LSD path groups (timing of level A's
//      loads and ranking only);
//  4 = nontemporal record stores in level A;
//  8 = small bucket kernel: no record gathers (records made from the pairs);
// 16 = small bucket kernel: no column / trace-start stores;
// 32 = small bucket kernel: no in-LDS ranking (arrival order kept).
// (8 / 16 / 32 give wrong groupings: timing only.)


#ifndef ANOMOD_BK_ABL
#define ANOMOD_BK_ABL 0
#endif
constexpr int kWv = 64;
constexpr int kBThreads = 1024;                // scatter workgroup
constexpr int kBWaves = kBThreads / kWv;       // 16
// Level-A records per thread: 2 -> 2048-record tiles, 76 KiB of LDS, two
// workgroups per CU (one tile's loads and ranking overlap the other's
// scattered stores): grouping 62.7 -> 58.7 ms at 2^27 SN traces against
// 4096-record tiles at one workgroup per CU (gpurun_out/r4d_aper2.log).
#ifndef ANOMOD_BK_APER
#define ANOMOD_BK_APER 2
#endif
constexpr int kBPer = ANOMOD_BK_APER;          // records per thread
constexpr int kBTile = kBThreads * kBPer;      // 2048 records per level-A tile
constexpr int kPPer = 16;                      // pairs per thread (level B)
constexpr int kPTile = kBThreads * kPPer;      // 16384 pairs per level-B tile (128 KiB)
constexpr int kDMax = 11;                      // digit bits per scatter level
constexpr int kNDMax = 1 << kDMax;
constexpr int kScanRows = 256;                 // tiles per block of the tile scan
constexpr int kScanB = 16;                     // loads in flight per serial scan step
constexpr int kSubBits = 9;                    // per-bucket split before the key compare
constexpr int kSub = 1 << kSubBits;
#ifndef ANOMOD_BK_SPER
#define ANOMOD_BK_SPER 4
#endif
constexpr int kSmallW = 512, kSmallPer = ANOMOD_BK_SPER;  // per-bucket kernel: 2048 spans
constexpr int kBigW = 1024, kBigPer = 8;       // oversized buckets: 8192 spans
#ifndef ANOMOD_BK_RANK
#define ANOMOD_BK_RANK 0  // small bucket kernel: 0 = stable split, 1 = atomic slots + compare rank
#endif
constexpr bool kRankAtomic = ANOMOD_BK_RANK != 0;
constexpr int kDChunk = 4096;                  // entries per partial sum of the trace-count scan

// Exclusive scan of one value per thread across a workgroup of NW waves;
// *tot = the sum.  Every thread must call it (two barriers).
template <int NW>
__device__ inline uint32_t block_excl_scan(uint32_t x, uint32_t* wsum, uint32_t* tot) {
  const int lane = threadIdx.x & (kWv - 1), w = threadIdx.x / kWv;
  uint32_t inc = x;
#pragma unroll
  for (int o = 1; o < kWv; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == kWv - 1) wsum[w] = inc;
  __syncthreads();
  uint32_t pre = 0, all = 0;
#pragma unroll
  for (int ww = 0; ww < NW; ++ww) {
    const uint32_t s = wsum[ww];
    pre += ww < w ? s : 0u;
    all += s;
  }
  __syncthreads();
  *tot = all;
  return pre + inc - x;
}

// ---- level A: per-tile digit counts of the top DA bits -----------------------
__global__ __launch_bounds__(256) void bk_count_a_kernel(const uint64_t* __restrict__ h, uint64_t n,
                                                         int da, uint32_t* __restrict__ tcnt) {
  __shared__ uint32_t lh[kNDMax];
  const int nd = 1 << da, tid = threadIdx.x, sh = 64 - da;
  for (int i = tid; i < nd; i += 256) lh[i] = 0u;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * kBTile;
#pragma unroll 4
  for (int j = 0; j < kBTile / 256; ++j) {
    const uint64_t p = t0 + (uint64_t)(j * 256 + tid);
    if (p < n) atomicAdd(&lh[(uint32_t)(mix64(h[p]) >> sh)], 1u);
  }
  __syncthreads();
  for (int i = tid; i < nd; i += 256) tcnt[(uint64_t)blockIdx.x * nd + i] = lh[i];
}

// ---- level A: exclusive scan of the tile counts over tiles, per digit -------
// column sums of kScanRows tiles; grid (blocks, ceil(nd / 256))
__global__ __launch_bounds__(256) void bk_scan_up_kernel(const uint32_t* __restrict__ tcnt,
                                                         uint64_t tiles, int nd,
                                                         uint32_t* __restrict__ bsum) {
  const int d = blockIdx.y * 256 + threadIdx.x;
  if (d >= nd) return;
  const uint64_t a = (uint64_t)blockIdx.x * kScanRows;
  const uint64_t b = a + kScanRows < tiles ? a + kScanRows : tiles;
  uint32_t s = 0;
#pragma unroll 8
  for (uint64_t t = a; t < b; ++t) s += tcnt[t * nd + d];
  bsum[(uint64_t)blockIdx.x * nd + d] = s;
}

// One block: the block sums scanned down every digit, the digit starts (=
// level-A bucket starts, bsA[nd] = n) added in, and the level-B tile starts of
// every level-A bucket (btile[nd] = level-B tiles in all).
__global__ __launch_bounds__(1024) void bk_scan_top_kernel(uint32_t* __restrict__ bsum,
                                                           uint64_t nbk, int nd, uint64_t n,
                                                           uint32_t* __restrict__ bsA,
                                                           uint32_t* __restrict__ btile,
                                                           uint32_t tile_b) {
  __shared__ uint32_t wsum[16];
  const int tid = threadIdx.x;
  const int dpt = nd > 1024 ? nd / 1024 : 1;  // consecutive digits per thread (nd <= 2048)
  uint32_t tot[2] = {0u, 0u}, til[2] = {0u, 0u};
  for (int i = 0; i < dpt; ++i) {
    const int d = tid * dpt + i;
    if (d >= nd) continue;
    uint32_t run = 0;
    for (uint64_t b = 0; b < nbk; b += kScanB) {
      uint32_t x[kScanB];
#pragma unroll
      for (int j = 0; j < kScanB; ++j) x[j] = b + j < nbk ? bsum[(b + j) * nd + d] : 0u;
#pragma unroll
      for (int j = 0; j < kScanB; ++j)
        if (b + j < nbk) {
          bsum[(b + j) * nd + d] = run;
          run += x[j];
        }
    }
    tot[i] = run;
    til[i] = (run + tile_b - 1) / tile_b;
  }
  uint32_t all, allt;
  const uint32_t pre = block_excl_scan<16>(tot[0] + tot[1], wsum, &all);
  const uint32_t pret = block_excl_scan<16>(til[0] + til[1], wsum, &allt);
  for (int i = 0; i < dpt; ++i) {
    const int d = tid * dpt + i;
    if (d >= nd) continue;
    const uint32_t start = pre + (i ? tot[0] : 0u);
    bsA[d] = start;
    btile[d] = pret + (i ? til[0] : 0u);
    for (uint64_t b = 0; b < nbk; b += kScanB) {
      uint32_t x[kScanB];
#pragma unroll
      for (int j = 0; j < kScanB; ++j) x[j] = b + j < nbk ? bsum[(b + j) * nd + d] : 0u;
#pragma unroll
      for (int j = 0; j < kScanB; ++j)
        if (b + j < nbk) bsum[(b + j) * nd + d] = x[j] + start;
    }
  }
  if (tid == 0) {
    bsA[nd] = (uint32_t)n;
    btile[nd] = allt;
  }
}

__global__ __launch_bounds__(256) void bk_scan_down_kernel(uint32_t* __restrict__ tcnt,
                                                           uint64_t tiles, int nd,
                                                           const uint32_t* __restrict__ bsum) {
  const int d = blockIdx.y * 256 + threadIdx.x;
  if (d >= nd) return;
  const uint64_t a = (uint64_t)blockIdx.x * kScanRows;
  const uint64_t b = a + kScanRows < tiles ? a + kScanRows : tiles;
  uint32_t run = bsum[(uint64_t)blockIdx.x * nd + d];
#pragma unroll 8
  for (uint64_t t = a; t < b; ++t) {
    const uint32_t x = tcnt[t * nd + d];
    tcnt[t * nd + d] = run;
    run += x;
  }
}

// ---- level B: tiles inside level-A buckets -----------------------------------
__global__ __launch_bounds__(256) void bk_tilemap_kernel(const uint32_t* __restrict__ btile,
                                                         uint32_t* __restrict__ tmap) {
  const uint32_t b = blockIdx.x;
  for (uint32_t t = btile[b] + threadIdx.x; t < btile[b + 1]; t += 256) tmap[t] = b;
}

// Level-B tile t (kPTile pairs, never straddling a level-A bucket).
__device__ inline bool seg_tile(uint64_t t, const uint32_t* __restrict__ bsA,
                                const uint32_t* __restrict__ btile,
                                const uint32_t* __restrict__ tmap, int na, uint64_t* base,
                                uint64_t* nvalid) {
  if (t >= btile[na]) return false;
  const uint32_t b = tmap[t];
  const uint64_t a = (uint64_t)bsA[b] + (t - btile[b]) * (uint64_t)kPTile;
  const uint64_t e = a + kPTile < (uint64_t)bsA[b + 1] ? a + kPTile : (uint64_t)bsA[b + 1];
  *base = a;
  *nvalid = e - a;
  return true;
}

// Per level-B tile: counts of the pairs' top db bits (the key bits right
// below level A's).
__global__ __launch_bounds__(256) void bk_count_b_kernel(const uint64_t* __restrict__ pr,
                                                         const uint32_t* __restrict__ bsA,
                                                         const uint32_t* __restrict__ btile,
                                                         const uint32_t* __restrict__ tmap,
                                                         int na, int db,
                                                         uint32_t* __restrict__ tcnt) {
  __shared__ uint32_t lh[kNDMax];
  uint64_t base, nvalid;
  if (!seg_tile(blockIdx.x, bsA, btile, tmap, na, &base, &nvalid)) return;
  const int nd = 1 << db, tid = threadIdx.x, sh = 64 - db;
  for (int i = tid; i < nd; i += 256) lh[i] = 0u;
  __syncthreads();
#pragma unroll 4
  for (uint64_t p = tid; p < nvalid; p += 256) atomicAdd(&lh[(uint32_t)(pr[base + p] >> sh)], 1u);
  __syncthreads();
  for (int i = tid; i < nd; i += 256) tcnt[(uint64_t)blockIdx.x * nd + i] = lh[i];
}

// One block per level-A bucket: its tiles' counts scanned per digit, the
// digit starts inside the bucket added in (= the final bucket starts).
__global__ __launch_bounds__(1024) void bk_scan_seg_kernel(uint32_t* __restrict__ tcnt,
                                                           const uint32_t* __restrict__ bsA,
                                                           const uint32_t* __restrict__ btile,
                                                           int na, int db,
                                                           uint32_t* __restrict__ bstart) {
  __shared__ uint32_t wsum[16];
  const int tid = threadIdx.x, nd = 1 << db;
  const int dpt = nd > 1024 ? nd / 1024 : 1;
  const uint32_t b = blockIdx.x, t0 = btile[b], t1 = btile[b + 1], base = bsA[b];
  // Both walks down the tiles batch kScanB loads ahead of their adds /
  // stores (one HBM round trip per batch, not per tile: 2.8 -> 0.x ms at
  // 2^27 SN traces).
  uint32_t tot[2] = {0u, 0u};
  for (int i = 0; i < dpt; ++i) {
    const int d = tid * dpt + i;
    if (d >= nd) continue;
    uint32_t s = 0;
    for (uint32_t t = t0; t < t1; t += kScanB) {
      uint32_t x[kScanB];
#pragma unroll
      for (int j = 0; j < kScanB; ++j)
        x[j] = t + j < t1 ? tcnt[(uint64_t)(t + j) * nd + d] : 0u;
#pragma unroll
      for (int j = 0; j < kScanB; ++j) s += x[j];
    }
    tot[i] = s;
  }
  uint32_t all;
  const uint32_t pre = block_excl_scan<16>(tot[0] + tot[1], wsum, &all);
  for (int i = 0; i < dpt; ++i) {
    const int d = tid * dpt + i;
    if (d >= nd) continue;
    const uint32_t start = base + pre + (i ? tot[0] : 0u);
    bstart[(uint64_t)b * nd + d] = start;
    uint32_t run = start;
    for (uint32_t t = t0; t < t1; t += kScanB) {
      uint32_t x[kScanB];
#pragma unroll
      for (int j = 0; j < kScanB; ++j)
        x[j] = t + j < t1 ? tcnt[(uint64_t)(t + j) * nd + d] : 0u;
#pragma unroll
      for (int j = 0; j < kScanB; ++j)
        if (t + j < t1) {
          tcnt[(uint64_t)(t + j) * nd + d] = run;
          run += x[j];
        }
    }
  }
  if (b == (uint32_t)na - 1 && tid == 0) bstart[(uint64_t)na * nd] = bsA[na];
}

// ---- level A: one stable scatter of the records ------------------------------
// Tile = kBTile records (1024 threads x kBPer; wave w owns positions
// [64 kBPer w, 64 kBPer (w + 1))), ranked with wave ballots (da ballots give
// each lane its same-digit peers; a per-wave LDS counter per digit carries the
// count down the wave's rows), staged whole in LDS in digit order — over the
// per-wave counters, which are dead by then — and written as 16-B chunks, a
// wave instruction covering 32 consecutive staged records (1 KiB, runs of ~4
// records to one place each at 9 digit bits and 2048-record tiles; the XCD
// tile order below lets neighbouring tiles' runs meet in L2).  Beside every record goes its pair for level B
// and the buckets: the next 32 key bits << 32 | the record's position.
// (Measured at 2^25 SN traces, 9-bit levels: half-record staging with one
// 16-B store per lane and record half 9.2 ms; whole records 6.0; no stores at
// all 1.0 ms — the scattered writes are the cost.)
//
// Workgroups are dispatched to the 8 XCDs round-robin by block index, so
// consecutive blocks would write the two ends of a shared 128-B line from two
// different L2s.  With nx = 8, XCD x takes a contiguous eighth of the tiles
// instead: the tiles one XCD has in flight are neighbours, their runs of one
// digit are neighbours in the output, and their partial lines meet in that
// XCD's L2 before write-back.
__device__ inline uint64_t xcd_tile(uint64_t b, uint64_t g, uint32_t nx) {
  if (nx <= 1u) return b;
  const uint64_t x = b % nx, s = b / nx, q = g / nx, r = g % nx;
  return x * q + (x < r ? x : r) + s;
}

// The pair of a record at position g whose key is k (level A took the top da
// bits): the next 32 key bits << 32 | g.
__device__ inline uint64_t make_pair(uint64_t k, int da, uint64_t g) {
  return (((k << da) >> 32) << 32) | (uint32_t)g;
}

__global__ __launch_bounds__(kBThreads) void bk_scatter_a_kernel(
    SoaIn sin, GRec* __restrict__ aout, uint64_t* __restrict__ pout, uint64_t n, int da,
    const uint32_t* __restrict__ toff, uint32_t nx) {
  constexpr bool kNoStore = (ANOMOD_BK_ABL & 2) != 0;
  static_assert(kBWaves * kNDMax * 2 <= kBTile * 32, "counters fit under the stage");
  union Lds {
    uint4 stage[2 * kBTile];              // 128 KiB: the tile's records in digit order
    uint16_t wcnt[kBWaves][kNDMax];       // per-wave digit counts, then wave offsets
  };
  __shared__ Lds u;
  __shared__ uint16_t tstart[kNDMax];     // tile-local start of each digit (<= kBTile)
  __shared__ uint32_t gbase[kNDMax];      // global start of each digit's run
  __shared__ uint32_t wsum[kBWaves];
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  const int nd = 1 << da, shift = 64 - da;
  const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x, nx);
  const uint64_t base = tile * kBTile;
  const uint64_t nvalid = n - base < (uint64_t)kBTile ? n - base : (uint64_t)kBTile;
  uint4 ra[kBPer], rb[kBPer];
  uint32_t d[kBPer];
  bool v[kBPer];
#pragma unroll
  for (int k = 0; k < kBPer; ++k) {
    const uint32_t loc = (uint32_t)(w * (kBPer * kWv) + k * kWv + lane);
    const uint64_t i = base + loc;
    v[k] = loc < nvalid;
    ra[k] = make_uint4(0, 0, 0, 0);
    rb[k] = make_uint4(0, 0, 0, 0);
    if (v[k]) {
      const uint64_t h = sin.h[i], sid = sin.sid[i], pid = sin.pid[i];
      ra[k] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)sid, (uint32_t)(sid >> 32));
      rb[k] = make_uint4((uint32_t)pid, (uint32_t)(pid >> 32), sin.sf[i], sin.dur[i]);
    }
    d[k] = (uint32_t)(mix64(((uint64_t)ra[k].y << 32) | ra[k].x) >> shift) & (uint32_t)(nd - 1);
  }
  for (int ww = 0; ww < kBWaves; ++ww)
    for (int dd = tid; dd < nd; dd += kBThreads) u.wcnt[ww][dd] = 0;
  for (int dd = tid; dd < nd; dd += kBThreads) gbase[dd] = toff[tile * nd + dd];
  __syncthreads();

  // wave multisplit, rows in order
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  uint32_t off[kBPer];
#pragma unroll
  for (int k = 0; k < kBPer; ++k) {
    uint64_t peers = __ballot(v[k]);
    for (int b = 0; b < da; ++b) {
      const bool bit = (d[k] >> b) & 1u;
      const uint64_t bb = __ballot(v[k] && bit);
      peers &= bit ? bb : ~bb;
    }
    off[k] = 0;
    if (v[k]) {
      const uint64_t lower = peers & lt_mask;
      const uint32_t b0 = u.wcnt[w][d[k]];
      off[k] = b0 + (uint32_t)__popcll(lower);
      if (lower == 0ull) u.wcnt[w][d[k]] = (uint16_t)(b0 + (uint32_t)__popcll(peers));
    }
    wave_sync();
  }
  __syncthreads();

  // per digit: wave offsets and the tile total, then the tile's digit starts
  const int dpt = nd > kBThreads ? nd / kBThreads : 1;
  uint32_t tot[2] = {0u, 0u};
  for (int i = 0; i < dpt; ++i) {
    const int dd = tid * dpt + i;
    if (dd >= nd) continue;
    uint32_t run = 0;
    for (int ww = 0; ww < kBWaves; ++ww) {
      const uint32_t c = u.wcnt[ww][dd];
      u.wcnt[ww][dd] = (uint16_t)run;
      run += c;
    }
    tot[i] = run;
  }
  uint32_t all;
  const uint32_t pre = block_excl_scan<kBWaves>(tot[0] + tot[1], wsum, &all);
  for (int i = 0; i < dpt; ++i) {
    const int dd = tid * dpt + i;
    if (dd < nd) tstart[dd] = (uint16_t)(pre + (i ? tot[0] : 0u));
  }
  __syncthreads();
  uint32_t lp[kBPer];
#pragma unroll
  for (int k = 0; k < kBPer; ++k) lp[k] = v[k] ? tstart[d[k]] + u.wcnt[w][d[k]] + off[k] : 0u;
  __syncthreads();  // the counters are dead: the stage goes over them
#pragma unroll
  for (int k = 0; k < kBPer; ++k) {
    if (v[k]) {
      u.stage[2 * lp[k]] = ra[k];
      u.stage[2 * lp[k] + 1] = rb[k];
    }
  }
  __syncthreads();
  if constexpr (kNoStore) return;
  // 16-B chunks in staged order: chunk c is half (c & 1) of staged record c / 2;
  // the lane holding a record's first half also writes its pair
  const uint64_t nch = 2 * nvalid;
#pragma unroll
  for (int j = 0; j < 2 * kBPer; ++j) {
    const uint32_t c = (uint32_t)(tid + j * kBThreads);
    if (c < nch) {
      const uint32_t p = c >> 1;
      const uint4 x = u.stage[c];
      const uint4 x0 = (c & 1u) ? u.stage[c - 1] : x;  // the record's (h, sid) half
      const uint64_t k = mix64(((uint64_t)x0.y << 32) | x0.x);
      const uint32_t dd = (uint32_t)(k >> shift) & (uint32_t)(nd - 1);
      const uint64_t g = (uint64_t)gbase[dd] + (p - tstart[dd]);
      if constexpr ((ANOMOD_BK_ABL & 4) != 0) {
        using u32x4 = uint32_t __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(u32x4{x.x, x.y, x.z, x.w},
                                    reinterpret_cast<u32x4*>(aout) + 2 * g + (c & 1u));
      } else
        reinterpret_cast<uint4*>(aout)[2 * g + (c & 1u)] = x;
      if (!(c & 1u)) pout[g] = make_pair(k, da, g);
    }
  }
}

// ---- level B: one stable scatter of the pairs inside every level-A bucket ----
// Tile = 16384 pairs (1024 threads x 16, wave w owns positions [1024w, 1024w +
// 1024)) of one level-A bucket, ranked by the top db bits of the pair with
// the same wave multisplit, staged in LDS in digit order (128 KiB) and written
// 8 B per lane in staged order.  An 8-B pair in place of the 32-B record: a
// quarter of the bytes, and a tile of four times as many entries (runs of ~8
// pairs per digit at 11 bits, against ~2 records).
__global__ __launch_bounds__(kBThreads) void bk_scatter_b_kernel(
    const uint64_t* __restrict__ pin, uint64_t* __restrict__ pout, int db,
    const uint32_t* __restrict__ toff, const uint32_t* __restrict__ bsA,
    const uint32_t* __restrict__ btile, const uint32_t* __restrict__ tmap, int na, uint32_t nx) {
  static_assert(kBWaves * kNDMax * 2 <= kPTile * 8, "counters fit under the stage");
  union Lds {
    uint64_t stage[kPTile];               // 128 KiB: the tile's pairs in digit order
    uint16_t wcnt[kBWaves][kNDMax];       // per-wave digit counts, then wave offsets
  };
  __shared__ Lds u;
  __shared__ uint32_t tstart[kNDMax];
  __shared__ uint32_t gbase[kNDMax];
  __shared__ uint32_t wsum[kBWaves];
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  const int nd = 1 << db, shift = 64 - db;
  const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x, nx);
  uint64_t base, nvalid;
  if (!seg_tile(tile, bsA, btile, tmap, na, &base, &nvalid)) return;
  uint64_t x[kPPer];
#pragma unroll
  for (int k = 0; k < kPPer; ++k) {
    const uint32_t loc = (uint32_t)(w * (kPPer * kWv) + k * kWv + lane);
    x[k] = loc < nvalid ? pin[base + loc] : 0ull;
  }
  for (int ww = 0; ww < kBWaves; ++ww)
    for (int dd = tid; dd < nd; dd += kBThreads) u.wcnt[ww][dd] = 0;
  for (int dd = tid; dd < nd; dd += kBThreads) gbase[dd] = toff[tile * nd + dd];
  __syncthreads();

  const uint64_t lt_mask = (1ull << lane) - 1ull;
  uint32_t off[kPPer];
#pragma unroll
  for (int k = 0; k < kPPer; ++k) {
    const bool v = (uint32_t)(w * (kPPer * kWv) + k * kWv + lane) < nvalid;
    const uint32_t d = (uint32_t)(x[k] >> shift);
    uint64_t peers = __ballot(v);
    for (int b = 0; b < db; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bb = __ballot(v && bit);
      peers &= bit ? bb : ~bb;
    }
    off[k] = 0;
    if (v) {
      const uint64_t lower = peers & lt_mask;
      const uint32_t b0 = u.wcnt[w][d];
      off[k] = b0 + (uint32_t)__popcll(lower);
      if (lower == 0ull) u.wcnt[w][d] = (uint16_t)(b0 + (uint32_t)__popcll(peers));
    }
    wave_sync();
  }
  __syncthreads();

  const int dpt = nd > kBThreads ? nd / kBThreads : 1;
  uint32_t tot[2] = {0u, 0u};
  for (int i = 0; i < dpt; ++i) {
    const int dd = tid * dpt + i;
    if (dd >= nd) continue;
    uint32_t run = 0;
    for (int ww = 0; ww < kBWaves; ++ww) {
      const uint32_t c = u.wcnt[ww][dd];
      u.wcnt[ww][dd] = (uint16_t)run;
      run += c;
    }
    tot[i] = run;
  }
  uint32_t all;
  const uint32_t pre = block_excl_scan<kBWaves>(tot[0] + tot[1], wsum, &all);
  for (int i = 0; i < dpt; ++i) {
    const int dd = tid * dpt + i;
    if (dd < nd) tstart[dd] = pre + (i ? tot[0] : 0u);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPPer; ++k) {  // the wave offsets into off[]
    const bool v = (uint32_t)(w * (kPPer * kWv) + k * kWv + lane) < nvalid;
    const uint32_t d = (uint32_t)(x[k] >> shift);
    off[k] = v ? tstart[d] + u.wcnt[w][d] + off[k] : 0xFFFFFFFFu;
  }
  __syncthreads();  // the counters are dead: the stage goes over them
#pragma unroll
  for (int k = 0; k < kPPer; ++k)
    if (off[k] != 0xFFFFFFFFu) u.stage[off[k]] = x[k];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPPer; ++j) {
    const uint32_t c = (uint32_t)(tid + j * kBThreads);
    if (c < nvalid) {
      const uint64_t y = u.stage[c];
      const uint32_t dd = (uint32_t)(y >> shift);
      pout[(uint64_t)gbase[dd] + (c - tstart[dd])] = y;
    }
  }
}

// ---- level B for the join: the same scatter, ranks from LDS atomics -----------
// The ungrouped aggregation's join resolves a repeated (trace, id) by the
// pairs' level-A positions (arrival order: level A is stable), not by the
// order inside a bucket, so level B need not be stable there.  A pair's rank
// inside its digit is one returning LDS add instead of db wave ballots per
// row; the digit totals are the counters themselves (one scan, no per-wave
// counter matrix).  Same tile map, counts and output bucket starts as the
// stable kernel.
__global__ __launch_bounds__(kBThreads) void bk_scatter_b_fast_kernel(
    const uint64_t* __restrict__ pin, uint64_t* __restrict__ pout, int db,
    const uint32_t* __restrict__ toff, const uint32_t* __restrict__ bsA,
    const uint32_t* __restrict__ btile, const uint32_t* __restrict__ tmap, int na, uint32_t nx) {
  __shared__ uint64_t stage[kPTile];      // 128 KiB: the tile's pairs in digit order
  __shared__ uint32_t lcnt[kNDMax];       // digit counts, then the tile's digit starts
  __shared__ uint32_t delta[kNDMax];      // global start - tile start, per digit
  __shared__ uint32_t wsum[kBWaves];
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  const int nd = 1 << db, shift = 64 - db;
  const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x, nx);
  uint64_t base, nvalid;
  if (!seg_tile(tile, bsA, btile, tmap, na, &base, &nvalid)) return;
  uint64_t x[kPPer];
#pragma unroll
  for (int k = 0; k < kPPer; ++k) {
    const uint32_t loc = (uint32_t)(w * (kPPer * kWv) + k * kWv + lane);
    x[k] = loc < nvalid ? pin[base + loc] : 0ull;
  }
  for (int dd = tid; dd < nd; dd += kBThreads) lcnt[dd] = 0u;
  __syncthreads();
  uint32_t off[kPPer];
#pragma unroll
  for (int k = 0; k < kPPer; ++k) {
    const uint32_t loc = (uint32_t)(w * (kPPer * kWv) + k * kWv + lane);
    off[k] = loc < nvalid ? atomicAdd(&lcnt[(uint32_t)(x[k] >> shift)], 1u) : 0xFFFFFFFFu;
  }
  __syncthreads();
  const int dpt = nd > kBThreads ? nd / kBThreads : 1;
  uint32_t c[2] = {0u, 0u};
  for (int i = 0; i < dpt; ++i) {
    const int dd = tid * dpt + i;
    if (dd < nd) c[i] = lcnt[dd];
  }
  uint32_t all;
  const uint32_t pre = block_excl_scan<kBWaves>(c[0] + c[1], wsum, &all);
  for (int i = 0; i < dpt; ++i) {
    const int dd = tid * dpt + i;
    if (dd >= nd) continue;
    const uint32_t ts = pre + (i ? c[0] : 0u);
    lcnt[dd] = ts;
    delta[dd] = toff[tile * nd + dd] - ts;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPPer; ++k)
    if (off[k] != 0xFFFFFFFFu) stage[lcnt[(uint32_t)(x[k] >> shift)] + off[k]] = x[k];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPPer; ++j) {
    const uint32_t cc = (uint32_t)(tid + j * kBThreads);
    if (cc < nvalid) {
      const uint64_t y = stage[cc];
      pout[(uint64_t)(uint32_t)(delta[(uint32_t)(y >> shift)] + cc)] = y;
    }
  }
}

// ---- level B moving the records too (ANOMOD_JOIN_RECB=1, r06 A/B) -------------
// The fast scatter above, plus each pair's 32-B record: read by the pair's
// level-A position (inside the tile's own 16384 records, 512 KiB that one
// workgroup brings into L2 once) and written beside the pair at its level-B
// position, so the join reads its bucket's records contiguously instead of
// gathering one 128-B line per span.  Bytes per span: 8 + 32 in, 8 + 32 out
// (against 8 + 8), for a join that reads 8 + 32 contiguously.
__global__ __launch_bounds__(kBThreads) void bk_scatter_b_rec_kernel(
    const uint64_t* __restrict__ pin, uint64_t* __restrict__ pout, const GRec* __restrict__ rin,
    GRec* __restrict__ rout, int db, const uint32_t* __restrict__ toff,
    const uint32_t* __restrict__ bsA, const uint32_t* __restrict__ btile,
    const uint32_t* __restrict__ tmap, int na, uint32_t nx) {
  __shared__ uint64_t stage[kPTile];
  __shared__ uint32_t lcnt[kNDMax];
  __shared__ uint32_t delta[kNDMax];
  __shared__ uint32_t wsum[kBWaves];
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  const int nd = 1 << db, shift = 64 - db;
  const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x, nx);
  uint64_t base, nvalid;
  if (!seg_tile(tile, bsA, btile, tmap, na, &base, &nvalid)) return;
  uint64_t x[kPPer];
#pragma unroll
  for (int k = 0; k < kPPer; ++k) {
    const uint32_t loc = (uint32_t)(w * (kPPer * kWv) + k * kWv + lane);
    x[k] = loc < nvalid ? pin[base + loc] : 0ull;
  }
  for (int dd = tid; dd < nd; dd += kBThreads) lcnt[dd] = 0u;
  __syncthreads();
  uint32_t off[kPPer];
#pragma unroll
  for (int k = 0; k < kPPer; ++k) {
    const uint32_t loc = (uint32_t)(w * (kPPer * kWv) + k * kWv + lane);
    off[k] = loc < nvalid ? atomicAdd(&lcnt[(uint32_t)(x[k] >> shift)], 1u) : 0xFFFFFFFFu;
  }
  __syncthreads();
  const int dpt = nd > kBThreads ? nd / kBThreads : 1;
  uint32_t c[2] = {0u, 0u};
  for (int i = 0; i < dpt; ++i) {
    const int dd = tid * dpt + i;
    if (dd < nd) c[i] = lcnt[dd];
  }
  uint32_t all;
  const uint32_t pre = block_excl_scan<kBWaves>(c[0] + c[1], wsum, &all);
  for (int i = 0; i < dpt; ++i) {
    const int dd = tid * dpt + i;
    if (dd >= nd) continue;
    const uint32_t ts = pre + (i ? c[0] : 0u);
    lcnt[dd] = ts;
    delta[dd] = toff[tile * nd + dd] - ts;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPPer; ++k)
    if (off[k] != 0xFFFFFFFFu) stage[lcnt[(uint32_t)(x[k] >> shift)] + off[k]] = x[k];
  __syncthreads();
  const uint4* rq = reinterpret_cast<const uint4*>(rin);
  uint4* wq = reinterpret_cast<uint4*>(rout);
#pragma unroll 4
  for (int j = 0; j < kPPer; ++j) {
    const uint32_t cc = (uint32_t)(tid + j * kBThreads);
    if (cc < nvalid) {
      const uint64_t y = stage[cc];
      const uint64_t g = (uint64_t)(uint32_t)(delta[(uint32_t)(y >> shift)] + cc);
      const uint64_t src = (uint32_t)y;  // the record's level-A position
      const uint4 r0 = rq[2 * src], r1 = rq[2 * src + 1];
      pout[g] = y;
      wq[2 * g] = r0;
      wq[2 * g + 1] = r1;
    }
  }
}

// ---- one bucket in (k, arrival) order ---------------------------------------
template <int W, int PER, bool EDGE = false>
struct BucketLds {
  static constexpr int kCap = W * PER, kNW = W / kWv;
  static_assert(kNW * kSub >= kCap, "trace starts fit over the sub-digit counters");
  struct Pre {
    uint64_t skey[kCap];          // pairs in sub-digit order, then full keys by final position
    uint32_t mixed[kSub];         // sub-bucket holds more than one key
    uint32_t tstart[kSub + 1];
    uint16_t sorig[kCap];         // arrival position of every staged pair
    uint16_t wcnt[kNW][kSub];
    uint8_t sflag[kCap];          // trace start at final position f
  };
  union {
    Pre pre;
  } u;
  uint16_t sfinal[kCap];          // final position of every arrival position
  uint16_t ssvc[EDGE ? kCap : 1]; // edge records: services by final position
  uint32_t wsum[kNW];
  uint32_t flag;
};

// Edge-record output of the fused ungrouped aggregation: per span, its
// (parent service row * S + service) edge << 33 | error << 32 | duration,
// the parent found in the span's trace by the first-match rule.
struct EdgeOut {
  uint64_t* rec;  // [n], by grouped position
  uint32_t S;
};

// A bucket beyond the large kernel (a trace of thousands of spans, or two
// such traces side by side): its distinct keys (at most kHugeKeys) counted in
// an LDS hash table and ranked, then ONE wave walks the pairs in arrival
// order (= position order: level B is stable) and sends each record to its
// trace's next row (peers of a row found by ballots over the slot index; a
// per-slot running row in LDS) — stable, and O(m) for any size.  More
// distinct keys than that sends the set to the LSD path.  Uses the large
// kernel's LDS (>= 82 KiB) as raw bytes.
constexpr uint32_t kHugeSlots = 4096;
constexpr uint32_t kHugeKeys = 2048;
constexpr uint64_t kEmptyKey = ~0ull;

__device__ inline int huge_slot(const uint64_t* hkey, uint64_t k) {
  uint32_t s = (uint32_t)k & (kHugeSlots - 1u);
  for (uint32_t probe = 0; probe < kHugeSlots; ++probe) {
    const uint64_t cur = hkey[s];
    if (cur == k) return (int)s;
    if (cur == kEmptyKey) return -1;
    s = (s + 1u) & (kHugeSlots - 1u);
  }
  return -1;
}

template <int W>
__device__ void bucket_huge(unsigned char* lds, uint32_t c, uint32_t a0, uint32_t m,
                            uint64_t* __restrict__ pin, const GRec* __restrict__ rec, SoaOut out,
                            uint32_t* __restrict__ dcnt, unsigned long long* __restrict__ too_big) {
  constexpr int kNW = W / kWv;
  uint64_t* hkey = reinterpret_cast<uint64_t*>(lds);               // [kHugeSlots]
  uint32_t* hcnt = reinterpret_cast<uint32_t*>(lds + 32768);       // count, then next row
  uint32_t* hrank = reinterpret_cast<uint32_t*>(lds + 49152);      // rank of the slot's key
  uint32_t* rrow = reinterpret_cast<uint32_t*>(lds + 65536);       // [kHugeKeys] by rank
  uint32_t* slots = reinterpret_cast<uint32_t*>(lds + 73728);      // [kHugeKeys] occupied
  uint32_t* hm = reinterpret_cast<uint32_t*>(lds + 81920);         // distinct, failed, listed
  uint32_t* wsum = hm + 4;                                          // [kNW]
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  for (uint32_t i = tid; i < kHugeSlots; i += W) {
    hkey[i] = kEmptyKey;
    hcnt[i] = 0u;
  }
  if (tid < 4) hm[tid] = 0u;
  __syncthreads();
  for (uint32_t p = tid; p < m; p += W) {
    const uint64_t k = mix64(rec[(uint32_t)pin[a0 + p]].h);
    bool done = k == kEmptyKey;  // the table's empty mark: LSD path
    if (done) hm[1] = 1u;
    uint32_t s = (uint32_t)k & (kHugeSlots - 1u);
    for (uint32_t probe = 0; !done && probe < kHugeSlots; ++probe) {
      uint64_t cur = hkey[s];
      if (cur == kEmptyKey) {
        const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(&hkey[s]),
                                        (unsigned long long)kEmptyKey, (unsigned long long)k);
        if (prev == kEmptyKey) atomicAdd(&hm[0], 1u);
        cur = prev == kEmptyKey ? k : prev;
      }
      if (cur == k) {
        atomicAdd(&hcnt[s], 1u);
        done = true;
      }
      s = (s + 1u) & (kHugeSlots - 1u);
    }
    if (!done) hm[1] = 1u;
  }
  __syncthreads();
  const uint32_t d = hm[0];
  if (hm[1] || d > kHugeKeys) {
    if (tid == 0) atomicAdd(too_big, 1ull);
    return;
  }
  for (uint32_t i = tid; i < kHugeSlots; i += W)
    if (hkey[i] != kEmptyKey) slots[atomicAdd(&hm[2], 1u)] = i;
  __syncthreads();
  for (uint32_t j = tid; j < d; j += W) {  // rank = keys below (d is small)
    const uint32_t sj = slots[j];
    const uint64_t kj = hkey[sj];
    uint32_t r = 0;
    for (uint32_t i = 0; i < d; ++i) r += hkey[slots[i]] < kj ? 1u : 0u;
    hrank[sj] = r;
    rrow[r] = hcnt[sj];
  }
  __syncthreads();
  const uint32_t x0 = 2u * tid < d ? rrow[2 * tid] : 0u;
  const uint32_t x1 = 2u * tid + 1u < d ? rrow[2 * tid + 1] : 0u;
  uint32_t all;
  const uint32_t pre = block_excl_scan<kNW>(x0 + x1, wsum, &all);
  if (2u * tid < d) rrow[2 * tid] = pre;
  if (2u * tid + 1u < d) rrow[2 * tid + 1] = pre + x0;
  __syncthreads();
  for (uint32_t i = tid; i < kHugeSlots; i += W)
    if (hkey[i] != kEmptyKey) hcnt[i] = rrow[hrank[i]];
  __syncthreads();
  if (w == 0) {
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    for (uint32_t p0 = 0; p0 < m; p0 += kWv) {
      const uint32_t p = p0 + (uint32_t)lane;
      const bool v = p < m;
      uint4 r0 = make_uint4(0, 0, 0, 0), r1 = make_uint4(0, 0, 0, 0);
      if (v) {
        const uint4* q = reinterpret_cast<const uint4*>(rec + (uint32_t)pin[a0 + p]);
        r0 = q[0];
        r1 = q[1];
      }
      const int sl = v ? huge_slot(hkey, mix64(((uint64_t)r0.y << 32) | r0.x)) : 0;
      const uint32_t su = (uint32_t)(sl < 0 ? 0 : sl);
      uint64_t peers = __ballot(v);
      for (int b = 0; b < 12; ++b) {
        const bool bit = (su >> b) & 1u;
        const uint64_t bb = __ballot(v && bit);
        peers &= bit ? bb : ~bb;
      }
      const uint32_t row = v ? hcnt[su] + (uint32_t)__popcll(peers & lt_mask) : 0u;
      wave_sync();
      if (v && (peers >> lane) == 1ull) hcnt[su] += (uint32_t)__popcll(peers);
      wave_sync();
      if (v) {
        if (out.h) out.h[a0 + row] = ((uint64_t)r0.y << 32) | r0.x;
        out.sid[a0 + row] = ((uint64_t)r0.w << 32) | r0.z;
        out.pid[a0 + row] = ((uint64_t)r1.y << 32) | r1.x;
        out.sf[a0 + row] = r1.z;
        out.dur[a0 + row] = r1.w;
      }
    }
  }
  __syncthreads();  // every pair read before the trace starts go over them
  for (uint32_t r = tid; r < d; r += W) pin[a0 + r] = (uint64_t)a0 + rrow[r];
  if (tid == 0) dcnt[c] = d;
}

// The bucket in final order -> one edge record per span (fused ungrouped
// aggregation): span ids and services staged in LDS by final position, each
// trace's bounds from its start flags, the parent found by the first-match
// scan over the trace (the order jaeger_to_csv.py:34-38 /
// trace_collector.py:424-443 see: arrival order inside the trace).
template <int W, int PER, bool EDGE, int R>
__device__ void bucket_edges(BucketLds<W, PER, EDGE>& L, uint32_t a0, uint32_t m,
                             const uint64_t (&k)[PER], const bool (&v)[PER], const uint4 (&ra)[R],
                             const uint4 (&rb)[R], const GRec* __restrict__ rec, EdgeOut eo) {
  constexpr int kNW = W / kWv;
  constexpr bool REG = R == PER;
  auto& P = L.u.pre;
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  uint16_t* tord = P.sorig;            // trace ordinal of every final position
  uint16_t* tsf = &P.wcnt[0][0];       // first final position of every trace
  // ordinals of the trace starts (thread tid: final positions tid * PER + j)
  uint32_t cnt = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t f = (uint32_t)(tid * PER + j);
    cnt += f < m ? P.sflag[f] : 0u;
  }
  uint32_t nt;
  uint32_t ord = block_excl_scan<kNW>(cnt, L.wsum, &nt);  // its barriers order sflag / skey
  uint4 x0[PER], x1[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t p = (uint32_t)(w * (PER * kWv) + j * kWv + lane);
    if constexpr (REG) {
      x0[j] = ra[j];
      x1[j] = rb[j];
    } else {
      const uint4* q = reinterpret_cast<const uint4*>(rec + (uint32_t)k[j]);
      x0[j] = v[j] ? q[0] : make_uint4(0, 0, 0, 0);
      x1[j] = v[j] ? q[1] : make_uint4(0, 0, 0, 0);
    }
    if (v[j]) {
      const uint32_t f = L.sfinal[p];
      P.skey[f] = ((uint64_t)x0[j].w << 32) | x0[j].z;  // span id
      L.ssvc[f] = (uint16_t)x1[j].z;                     // service
    }
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t f = (uint32_t)(tid * PER + j);
    if (f < m) {
      if (P.sflag[f]) tsf[ord++] = (uint16_t)f;
      tord[f] = (uint16_t)(ord - 1u);
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if (!v[j]) continue;
    const uint32_t p = (uint32_t)(w * (PER * kWv) + j * kWv + lane);
    const uint32_t f = L.sfinal[p], t = tord[f];
    const uint32_t a = tsf[t], b = t + 1u < nt ? tsf[t + 1u] : m;
    const uint64_t pid = ((uint64_t)x1[j].y << 32) | x1[j].x;
    uint32_t prow = eo.S;  // ROOT: no parent reference
    if (pid != 0ull) {
      prow = eo.S + 1u;  // ORPHAN unless the trace holds the reference
      for (uint32_t q0 = a; q0 < b; q0 += 4) {  // first match, 4 ids per LDS round trip
        uint64_t id[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) id[u] = P.skey[q0 + u < b ? q0 + u : a];
        int hit = -1;
#pragma unroll
        for (int u = 3; u >= 0; --u)
          if (q0 + u < b && id[u] == pid) hit = u;
        if (hit >= 0) {
          prow = L.ssvc[q0 + hit];
          break;
        }
      }
    }
    const uint32_t svc = x1[j].z & 0xFFFFu, fl = x1[j].z >> 16;
    eo.rec[a0 + f] = ((uint64_t)(prow * eo.S + svc) << 33) |
                     ((uint64_t)((fl & ANOMOD_FLAG_ERROR) ? 1u : 0u) << 32) | x1[j].w;
  }
}

// Two traces of a bucket whose keys agree in every bit the pairs carry: the
// bucket ranked by (full key, arrival) instead (rare: O(m^2) compares by
// every thread).  Every thread calls it (barriers).
template <int W, int PER, bool EDGE>
__device__ void bucket_rerank_exact(BucketLds<W, PER, EDGE>& L, uint32_t m,
                                    const uint64_t (&fk)[PER], const bool (&v)[PER]) {
  auto& P = L.u.pre;
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  (void)tid;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t p = (uint32_t)(w * (PER * kWv) + j * kWv + lane);
    if (v[j]) P.skey[p] = fk[j];  // full keys by arrival position
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t p = (uint32_t)(w * (PER * kWv) + j * kWv + lane);
    if (v[j]) {
      uint32_t rank = 0, first = 1;
      for (uint32_t q = 0; q < m; ++q) {
        const uint64_t kq = P.skey[q];
        rank += (kq < fk[j] || (kq == fk[j] && q < p)) ? 1u : 0u;
        first &= (kq == fk[j] && q < p) ? 0u : 1u;
      }
      L.sfinal[p] = (uint16_t)rank;
      P.sflag[rank] = (uint8_t)first;
    }
  }
  __syncthreads();
}

// The bucket's final order in LDS (sfinal: arrival -> final position; sflag:
// trace starts by final position).
template <int W, int PER, bool EDGE, int R>
__device__ void bucket_rank(BucketLds<W, PER, EDGE>& L, uint32_t a0, uint32_t m,
                            const GRec* __restrict__ rec, int kshift, const uint64_t (&k)[PER],
                            const bool (&v)[PER], const uint4 (&ra)[R], const uint4 (&rb)[R]) {
  constexpr int kCap = W * PER, kNW = W / kWv;
  constexpr bool REG = R == PER;
  auto& P = L.u.pre;
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  (void)kCap;
  (void)a0;
  uint64_t fk[PER];
  uint32_t e[PER], off[PER];
  if constexpr (!REG) {
#pragma unroll
    for (int j = 0; j < PER; ++j) fk[j] = v[j] ? rec[(uint32_t)k[j]].h : 0ull;
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if constexpr (REG) fk[j] = ((uint64_t)ra[j].y << 32) | ra[j].x;
    fk[j] = mix64(fk[j]);
    e[j] = (uint32_t)(k[j] >> kshift) & (kSub - 1);
  }
  for (int i = tid; i < kNW * kSub; i += W) (&P.wcnt[0][0])[i] = 0;
  for (int i = tid; i < kSub; i += W) P.mixed[i] = 0u;
  if (tid == 0) L.flag = 0u;
  __syncthreads();

  const uint64_t lt_mask = (1ull << lane) - 1ull;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    uint64_t peers = __ballot(v[j]);
#pragma unroll
    for (int b = 0; b < kSubBits; ++b) {
      const bool bit = (e[j] >> b) & 1u;
      const uint64_t bb = __ballot(v[j] && bit);
      peers &= bit ? bb : ~bb;
    }
    off[j] = 0;
    if (v[j]) {
      const uint64_t lower = peers & lt_mask;
      const uint32_t b0 = P.wcnt[w][e[j]];
      off[j] = b0 + (uint32_t)__popcll(lower);
      if (lower == 0ull) P.wcnt[w][e[j]] = (uint16_t)(b0 + (uint32_t)__popcll(peers));
    }
    wave_sync();
  }
  __syncthreads();
  uint32_t tot = 0;
  if (tid < kSub) {
    uint32_t run = 0;
    for (int ww = 0; ww < kNW; ++ww) {
      const uint32_t cc = P.wcnt[ww][tid];
      P.wcnt[ww][tid] = (uint16_t)run;
      run += cc;
    }
    tot = run;
  }
  uint32_t all;
  const uint32_t pre = block_excl_scan<kNW>(tot, L.wsum, &all);
  if (tid < kSub) P.tstart[tid] = pre;
  if (tid == 0) P.tstart[kSub] = m;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if (v[j]) {
      const uint32_t sp = P.tstart[e[j]] + P.wcnt[w][e[j]] + off[j];
      P.skey[sp] = k[j];
      P.sorig[sp] = (uint16_t)(w * (PER * kWv) + j * kWv + lane);
    }
  }
  __syncthreads();
  // one key per sub-bucket? (plain stores of 1: any writer will do)
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t sp = (uint32_t)(tid + j * W);
    if (sp < m) {
      const uint64_t kp = P.skey[sp];
      const uint32_t ee = (uint32_t)(kp >> kshift) & (kSub - 1);
      if ((kp >> 32) != (P.skey[P.tstart[ee]] >> 32)) P.mixed[ee] = 1u;
    }
  }
  __syncthreads();

  // final position inside the bucket
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t sp = (uint32_t)(tid + j * W);
    if (sp < m) {
      const uint64_t kp = P.skey[sp];
      const uint32_t ee = (uint32_t)(kp >> kshift) & (kSub - 1);
      const uint32_t a = P.tstart[ee], b = P.tstart[ee + 1];
      uint32_t rank, first;
      if (!P.mixed[ee]) {
        rank = sp - a;
        first = sp == a;
      } else {
        rank = 0;
        first = 1;
        for (uint32_t q0 = a; q0 < b; q0 += 4) {  // 4 pairs per step: one LDS round trip
          uint64_t kq[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) kq[t] = P.skey[q0 + t < b ? q0 + t : a];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const bool in = q0 + t < b;
            const bool below = in && kq[t] < kp;  // pairs are distinct
            rank += below ? 1u : 0u;
            first &= (below && (kq[t] >> 32) == (kp >> 32)) ? 0u : 1u;
          }
        }
      }
      const uint32_t f = a + rank;
      P.sflag[f] = (uint8_t)first;
      L.sfinal[P.sorig[sp]] = (uint16_t)f;
    }
  }
  __syncthreads();

  // Two traces of the bucket whose keys agree in every bit the pairs carry:
  // their spans sit in one run of equal pair keys, in position order.  Seen
  // as a run whose full keys differ; the bucket is then ranked by (full key,
  // arrival) instead (rare: O(m^2) compares by every thread).
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t p = (uint32_t)(w * (PER * kWv) + j * kWv + lane);
    if (v[j]) P.skey[L.sfinal[p]] = fk[j];  // skey is dead: full keys by final position
  }
  __syncthreads();
  bool clash = false;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t f = (uint32_t)(tid + j * W);
    clash |= f > 0 && f < m && !P.sflag[f] && P.skey[f] != P.skey[f - 1];
  }
  if constexpr ((ANOMOD_BK_ABL & 8) != 0) clash = false;  // timing: keys are not the records'
  if (__syncthreads_or(clash)) bucket_rerank_exact<W, PER, EDGE>(L, m, fk, v);

}

// Small-kernel ranking without the stable split (ANOMOD_BK_RANK=1): each span
// takes a slot in its sub-bucket with one LDS atomic (any order), the
// sub-bucket starts come from one block scan, and a span's final position is
// a + #{pairs of its sub-bucket below its own} — pairs are distinct and order
// by (key bits, arrival), so this is the stable order however the slots were
// taken.  The compare loop is O(s) per span, so a bucket holding a sub-bucket
// of more than kLongSub spans (a long trace) returns false and goes to the
// large kernel's stable split.  The full-key check rides along: spans with
// equal pair keys must have equal low 32 bits of k (the bucket and the pair
// fix the other da + 32 >= 33), else the bucket is re-ranked exactly.
constexpr uint32_t kLongSub = 128;
template <int W, int PER, bool EDGE, int R>
__device__ bool bucket_rank_atomic(BucketLds<W, PER, EDGE>& L, uint32_t m, int kshift,
                                   const uint64_t (&k)[PER], const bool (&v)[PER],
                                   const uint4 (&ra)[R]) {
  static_assert(R == PER, "records in registers");
  constexpr int kCap = W * PER, kNW = W / kWv;
  static_assert(kNW * kSub * 2 >= kCap * 4, "low key words fit over the wave counters");
  static_assert(W == kSub, "one thread per sub-digit");
  auto& P = L.u.pre;
  uint32_t* cnt = P.mixed;                                      // [kSub] spans per sub-bucket
  uint32_t* sfk = reinterpret_cast<uint32_t*>(&P.wcnt[0][0]);  // [kCap] low key word, staged
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  uint64_t fk[PER];
  uint32_t e[PER], o[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    fk[j] = mix64(((uint64_t)ra[j].y << 32) | ra[j].x);
    e[j] = (uint32_t)(k[j] >> kshift) & (kSub - 1);
  }
  cnt[tid] = 0u;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j) o[j] = v[j] ? atomicAdd(&cnt[e[j]], 1u) : 0u;
  __syncthreads();
  const uint32_t tot = cnt[tid];
  uint32_t all;
  const uint32_t pre = block_excl_scan<kNW>(tot, L.wsum, &all);
  P.tstart[tid] = pre;
  if (tid == 0) P.tstart[kSub] = m;
  if (__syncthreads_or(tot > kLongSub)) return false;  // (also orders tstart)
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if (v[j]) {
      const uint32_t sp = P.tstart[e[j]] + o[j];
      P.skey[sp] = k[j];
      sfk[sp] = (uint32_t)fk[j];
      P.sorig[sp] = (uint16_t)(w * (PER * kWv) + j * kWv + lane);
    }
  }
  __syncthreads();
  bool clash = false;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t sp = (uint32_t)(tid + j * W);
    if (sp < m) {
      const uint64_t kp = P.skey[sp];
      const uint32_t fp = sfk[sp];
      const uint32_t ee = (uint32_t)(kp >> kshift) & (kSub - 1);
      const uint32_t a = P.tstart[ee], b = P.tstart[ee + 1];
      uint32_t rank = 0, first = 1;
      if (b - a > 1u) {
        for (uint32_t q0 = a; q0 < b; q0 += 4) {  // 4 pairs per step: one LDS round trip
          uint64_t kq[4];
          uint32_t fq[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const uint32_t q = q0 + t < b ? q0 + t : a;
            kq[t] = P.skey[q];
            fq[t] = sfk[q];
          }
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const bool in = q0 + t < b;
            const bool below = in && kq[t] < kp;  // pairs are distinct
            const bool same = in && (kq[t] >> 32) == (kp >> 32);
            rank += below ? 1u : 0u;
            first &= (below && same) ? 0u : 1u;
            clash |= same && fq[t] != fp;
          }
        }
      }
      const uint32_t f = a + rank;
      P.sflag[f] = (uint8_t)first;
      L.sfinal[P.sorig[sp]] = (uint16_t)f;
    }
  }
  if (__syncthreads_or(clash)) bucket_rerank_exact<W, PER, EDGE>(L, m, fk, v);
  return true;
}

// The bucket in final order out: its grouped columns (records by final
// position), its trace starts over the bucket's own pairs (pin[a0 +
// ordinal], read before) and its trace count dcnt[c].
template <int W, int PER, bool EDGE, int R>
__device__ void bucket_emit(BucketLds<W, PER, EDGE>& L, uint32_t c, uint32_t a0, uint32_t m,
                            uint64_t* __restrict__ pin, const GRec* __restrict__ rec, SoaOut out,
                            uint32_t* __restrict__ dcnt, const uint64_t (&k)[PER],
                            const bool (&v)[PER], const uint4 (&ra)[R], const uint4 (&rb)[R]) {
  constexpr int kNW = W / kWv;
  constexpr bool REG = R == PER;
  auto& P = L.u.pre;
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  // trace starts: ordinals in final order (written last: over the bucket's
  // own pairs, read until then)
  uint32_t cnt = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t f = (uint32_t)(tid * PER + j);
    cnt += f < m ? P.sflag[f] : 0u;
  }
  uint32_t nt;
  const uint32_t ord0 = block_excl_scan<kNW>(cnt, L.wsum, &nt);
  uint32_t fl = 0;  // bit j: tid * PER + j is a trace start
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t f = (uint32_t)(tid * PER + j);
    fl |= (f < m && P.sflag[f]) ? (1u << j) : 0u;
  }

  // each record straight to its final row (the bucket's rows of every column
  // are a few KiB: the stores merge in L2)
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t p = (uint32_t)(w * (PER * kWv) + j * kWv + lane);
    if (v[j]) {
      uint4 x0, x1;
      if constexpr (REG) {
        x0 = ra[j];
        x1 = rb[j];
      } else {
        const uint4* q = reinterpret_cast<const uint4*>(rec + (uint32_t)k[j]);
        x0 = q[0];
        x1 = q[1];
      }
      const uint32_t i = L.sfinal[p];
      if constexpr ((ANOMOD_BK_ABL & 16) != 0) {  // timing: no stores
        if (x0.x == 0x12345678u && x1.w == 0x9ABCDEF0u) out.sf[a0 + i] = i;
        continue;
      }
      if (out.h) out.h[a0 + i] = ((uint64_t)x0.y << 32) | x0.x;  // (aggregate-only calls: none)
      out.sid[a0 + i] = ((uint64_t)x0.w << 32) | x0.z;
      out.pid[a0 + i] = ((uint64_t)x1.y << 32) | x1.x;
      out.sf[a0 + i] = x1.z;
      out.dur[a0 + i] = x1.w;
    }
  }
  uint32_t ord = ord0;  // every pair was read into registers before the first barrier
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if ((fl >> j) & 1u) pin[a0 + ord++] = (uint64_t)a0 + (uint32_t)(tid * PER + j);
  if (tid == 0) dcnt[c] = nt;
}

// Bucket c = [a0, a0 + m) of the pairs `pin` (in arrival order inside the
// bucket; every key shares its top T bits), its pairs k / v and — REG, the
// small kernel — its records ra / rb already in registers (the big kernel
// gathers the keys itself).  Split once more by the next 9 key bits (stable);
// a sub-bucket holding one key is already in arrival order, a mixed one ranks
// each pair by compares: rank = #{smaller pair} (a pair orders by (key bits,
// position) and positions are arrival order).  The records come from `rec` by
// position.  Writes the grouped columns of the bucket, its trace starts over
// the bucket's own pairs (pin[a0 + ordinal], read before) and the trace count
// dcnt[c] — or, EDGE, its edge records.
template <int W, int PER, bool EDGE, int R, bool ATOMIC = false>
__device__ bool bucket_body(BucketLds<W, PER, EDGE>& L, uint32_t c, uint32_t a0, uint32_t m,
                            uint64_t* __restrict__ pin, const GRec* __restrict__ rec, SoaOut out,
                            EdgeOut eo, int kshift, uint32_t* __restrict__ dcnt,
                            const uint64_t (&k)[PER], const bool (&v)[PER], const uint4 (&ra)[R],
                            const uint4 (&rb)[R]) {
  static_assert(W >= kSub, "one thread per sub-digit");
  constexpr bool REG = R == PER;
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  (void)tid;
  (void)lane;
  (void)w;
  if constexpr ((ANOMOD_BK_ABL & 32) != 0 && REG) {  // timing: arrival order, every span a trace
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t p = (uint32_t)(w * (PER * kWv) + j * kWv + lane);
      if (v[j]) {
        L.sfinal[p] = (uint16_t)p;
        L.u.pre.sflag[p] = 1;
      }
    }
    __syncthreads();
  } else if constexpr (ATOMIC) {
    if (!bucket_rank_atomic<W, PER, EDGE, R>(L, m, kshift, k, v, ra)) return false;
  } else {
    bucket_rank<W, PER, EDGE, R>(L, a0, m, rec, kshift, k, v, ra, rb);
  }
  if constexpr (EDGE) {
    bucket_edges(L, a0, m, k, v, ra, rb, rec, eo);
    return true;
  }
  bucket_emit<W, PER, EDGE, R>(L, c, a0, m, pin, rec, out, dcnt, k, v, ra, rb);
  return true;
}



// One bucket by one workgroup: the size checks (over-size buckets listed for
// the big kernel, or the huge walk), the pair loads and gathers, the body.
template <int W, int PER, bool EDGE>
__device__ void bucket_sort_one(BucketLds<W, PER, EDGE>& L, uint32_t c, uint64_t* __restrict__ pin,
                                const GRec* __restrict__ rec, SoaOut out, EdgeOut eo,
                                const uint32_t* __restrict__ bstart, int kshift,
                                uint32_t* __restrict__ dcnt, bool small,
                                uint32_t* __restrict__ over, unsigned long long* __restrict__ over_n,
                                uint32_t over_cap, unsigned long long* __restrict__ too_big) {
  constexpr int kCap = W * PER;
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  const uint32_t a0 = bstart[c], m = bstart[c + 1] - a0;
  if (m > (uint32_t)kCap) {
    if (small) {
      if (tid == 0) {
        const unsigned long long i = atomicAdd(over_n, 1ull);
        if (i < over_cap) over[i] = c;
        else atomicAdd(too_big, 1ull);
      }
      return;
    }
    // (the fused aggregation leaves such a bucket — traces of thousands of
    // spans side by side — to the unfused path: too_big)
    if constexpr (!EDGE && sizeof(BucketLds<W, PER, EDGE>) >= 81920 + 16 + 4 * (W / kWv))
      bucket_huge<W>(reinterpret_cast<unsigned char*>(&L), c, a0, m, pin, rec, out, dcnt, too_big);
    else if (tid == 0)
      atomicAdd(too_big, 1ull);
    return;
  }
  if (m == 0) {
    if (tid == 0 && !EDGE) dcnt[c] = 0;
    return;
  }
  // REG (the small kernel): whole records held in registers from the gather
  // on; else only their keys, the records gathered again when written.
  constexpr bool REG = PER <= 4;
  constexpr int R = REG ? PER : 1;
  uint64_t k[PER];
  bool v[PER];
  uint4 ra[R], rb[R];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t p = (uint32_t)(w * (PER * kWv) + j * kWv + lane);
    v[j] = p < m;
    k[j] = v[j] ? pin[a0 + p] : 0ull;
  }
  if constexpr (REG) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {  // the gathers: issued together, after every pair load
      if constexpr ((ANOMOD_BK_ABL & 8) != 0) {
        ra[j] = make_uint4((uint32_t)k[j], (uint32_t)(k[j] >> 32), (uint32_t)k[j], 0u);
        rb[j] = make_uint4((uint32_t)(k[j] >> 32), 0u, 0u, 0u);
        continue;
      }
      const uint4* q = reinterpret_cast<const uint4*>(rec + (uint32_t)k[j]);
      ra[j] = v[j] ? q[0] : make_uint4(0, 0, 0, 0);
      rb[j] = v[j] ? q[1] : make_uint4(0, 0, 0, 0);
    }
  }
  if constexpr (W == kSmallW && kRankAtomic) {
    if (!bucket_body<W, PER, EDGE, R, true>(L, c, a0, m, pin, rec, out, eo, kshift, dcnt, k, v, ra,
                                            rb) &&
        tid == 0) {  // a sub-bucket too long for the compare rank: the large kernel
      const unsigned long long i = atomicAdd(over_n, 1ull);
      if (i < over_cap) over[i] = c;
      else atomicAdd(too_big, 1ull);
    }
  } else {
    bucket_body<W, PER, EDGE, R>(L, c, a0, m, pin, rec, out, eo, kshift, dcnt, k, v, ra, rb);
  }
}

#ifndef ANOMOD_BK_MINW
#define ANOMOD_BK_MINW 1  // waves per SIMD the small bucket kernel's registers must allow
#endif
__global__ __launch_bounds__(kSmallW, ANOMOD_BK_MINW) void bk_bucket_kernel(
    uint64_t* __restrict__ pin, const GRec* __restrict__ rec, SoaOut out,
    const uint32_t* __restrict__ bstart, int kshift, uint32_t* __restrict__ dcnt,
    uint32_t* __restrict__ over, unsigned long long* __restrict__ over_n, uint32_t over_cap,
    unsigned long long* __restrict__ too_big, uint32_t nx) {
  __shared__ BucketLds<kSmallW, kSmallPer> L;
  bucket_sort_one<kSmallW, kSmallPer, false>(L, (uint32_t)xcd_tile(blockIdx.x, gridDim.x, nx), pin,
                                             rec, out, EdgeOut{}, bstart, kshift, dcnt, true, over,
                                             over_n, over_cap, too_big);
}

// Persistent, pipelined form of the small bucket kernel (ANOMOD_BK_PIPE=1): the
// workgroups take buckets b, b + G, b + 2G, ... (so the buckets in flight are
// neighbours: every XCD inside one level-A bucket, whose records the gathers
// then find in the Infinity Cache), and while one sorts bucket c, the records
// of c + G are being gathered and the pairs of c + 2G loaded — the gather
// latency hides behind the sort instead of stalling it.
#ifndef ANOMOD_BK_PIPE_MINB
#define ANOMOD_BK_PIPE_MINB 2  // waves per SIMD the registers must allow
#endif
template <bool EDGE>
__global__ __launch_bounds__(kSmallW, ANOMOD_BK_PIPE_MINB) void bk_bucket_pipe_kernel(
    uint64_t* __restrict__ pin, const GRec* __restrict__ rec, SoaOut out, EdgeOut eo,
    const uint32_t* __restrict__ bstart, uint32_t nbk, int kshift, uint32_t* __restrict__ dcnt,
    uint32_t* __restrict__ over, unsigned long long* __restrict__ over_n, uint32_t over_cap,
    unsigned long long* __restrict__ too_big) {
  __shared__ BucketLds<kSmallW, kSmallPer, EDGE> L;
  constexpr int PER = kSmallPer, kCap = kSmallW * kSmallPer;
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  const uint32_t G = gridDim.x;
  struct Slot {
    uint32_t a0, m;
    uint64_t k[PER];
    bool v[PER];
  };
  auto load = [&](Slot& s, uint32_t c) {
    s.a0 = 0u;
    s.m = 0u;
    if (c < nbk) {
      s.a0 = bstart[c];
      s.m = bstart[c + 1] - s.a0;
    }
    const bool fits = s.m <= (uint32_t)kCap;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t p = (uint32_t)(w * (PER * kWv) + j * kWv + lane);
      s.v[j] = fits && p < s.m;
      s.k[j] = s.v[j] ? pin[s.a0 + p] : 0ull;
    }
  };
  auto gather = [&](const Slot& s, uint4 (&ra)[PER], uint4 (&rb)[PER]) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint4* q = reinterpret_cast<const uint4*>(rec + (uint32_t)s.k[j]);
      ra[j] = s.v[j] ? q[0] : make_uint4(0, 0, 0, 0);
      rb[j] = s.v[j] ? q[1] : make_uint4(0, 0, 0, 0);
    }
  };
  Slot cur, nxt, nx2;
  uint4 ra[PER], rb[PER], ran[PER], rbn[PER];
  uint32_t c = blockIdx.x;
  load(cur, c);
  gather(cur, ra, rb);
  load(nxt, c + G);
  for (; c < nbk; c += G) {
    gather(nxt, ran, rbn);
    load(nx2, c + 2u * G);
    if (cur.m > (uint32_t)kCap) {  // for the big kernel (or, EDGE, the unfused path)
      if (tid == 0) {
        const unsigned long long i = atomicAdd(over_n, 1ull);
        if (i < over_cap) over[i] = c;
        else atomicAdd(too_big, 1ull);
      }
    } else if (cur.m == 0u) {
      if (tid == 0 && !EDGE) dcnt[c] = 0;
    } else {
      bucket_body<kSmallW, PER, EDGE, PER>(L, c, cur.a0, cur.m, pin, rec, out, eo, kshift, dcnt,
                                           cur.k, cur.v, ra, rb);
    }
    __syncthreads();  // the next bucket reuses the LDS
    cur = nxt;
    nxt = nx2;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      ra[j] = ran[j];
      rb[j] = rbn[j];
    }
  }
}

// The fused ungrouped aggregation without the sort (the fused path's default;
// ANOMOD_FUSED_JOIN=0: the sorting kernels below).  A bucket holds every span
// of its traces, so a span's parent is found by an LDS hash join on (trace,
// span id) over the bucket: no ranking, no trace bounds.  A repeated (trace,
// id) resolves to its earliest arrival — the smallest level-A position, since
// level A is stable (level B is not: bk_scatter_b_fast_kernel), read from the
// bucket's pairs — which is the first-match rule (jaeger_to_csv.py:34-38 /
// trace_collector.py:424-443).  Records go out by bucket position (the edge
// table is order-free).
//
// LDS per span: the trace key, the span id and half a u16 table slot (load
// <= 1/2).  PACK (T >= 12 bucket bits: every k of a bucket shares its top 12
// bits, and a service index is < 4096) keeps the service in those 12 bits of
// the key word: 20 B per span, so the 2 048-span kernel takes 40 KiB and four
// workgroups share a CU (the r04 form, 26 B per span, fit three).
constexpr uint64_t kKeyLow = (1ull << 52) - 1ull;  // the k bits a PACK key word compares

template <int W, int PER, bool PACK, bool T16 = true>
struct JoinGeom {
  static constexpr int kCap = W * PER;
  static constexpr uint32_t kSlots = 2u * (uint32_t)kCap;  // load <= 1/2
  static constexpr size_t kTabBytes = T16 ? 4ull * kCap : 8ull * kCap;  // u16 (two per word) / u32
  static constexpr size_t kOffSid = 8ull * kCap, kOffTab = 16ull * kCap;
  static constexpr size_t kOffSvc = kOffTab + kTabBytes;
  static constexpr size_t kBytes = kOffSvc + (PACK ? 0ull : 2ull * kCap);
  static_assert((kSlots & (kSlots - 1u)) == 0u, "join table size");
  static_assert(kCap <= 65535, "u16 slots hold arrival + 1");
};

__device__ __forceinline__ uint32_t join_slot(uint64_t k, uint64_t id, uint32_t slots) {
  return (uint32_t)(mix64(k ^ (id * 0x9E3779B97F4A7C15ull)) >> 32) & (slots - 1u);
}

template <bool T16>
__device__ __forceinline__ uint32_t slot_get(const uint32_t* tab, uint32_t s) {
  if constexpr (!T16) return tab[s];
  return (tab[s >> 1] >> ((s & 1u) * 16u)) & 0xFFFFu;
}

// Compare-and-swap of u16 slot s (a 32-bit CAS on its word, retried while only
// the other half changes): the slot's value before, == expect when swapped.
template <bool T16>
__device__ __forceinline__ uint32_t slot_cas(uint32_t* tab, uint32_t s, uint32_t expect,
                                             uint32_t desired) {
  if constexpr (!T16) return atomicCAS(&tab[s], expect, desired);
  uint32_t* wp = &tab[s >> 1];
  const uint32_t sh = (s & 1u) * 16u, mask = 0xFFFFu << sh;
  uint32_t w = (expect << sh) | (*wp & ~mask);
  while (true) {
    const uint32_t old = atomicCAS(wp, w, (w & ~mask) | (desired << sh));
    if (old == w) return expect;
    const uint32_t cur = (old >> sh) & 0xFFFFu;
    if (cur != expect) return cur;
    w = old;
  }
}

// One bucket [a0, a0 + m) of the level-B pairs `pin` joined in LDS; every
// thread of the workgroup calls it.  The records come from `rec` by the pairs'
// level-A positions.
template <int W, int PER, bool PACK, bool T16 = true, bool CONTIG = false>
__device__ __forceinline__ void join_bucket(unsigned char* lds, uint32_t a0, uint32_t m,
                                            const uint64_t* __restrict__ pin,
                                            const GRec* __restrict__ rec, EdgeOut eo) {
  using G = JoinGeom<W, PER, PACK, T16>;
  constexpr uint32_t kSlots = G::kSlots;
  uint64_t* lkx = reinterpret_cast<uint64_t*>(lds);
  uint64_t* lsid = reinterpret_cast<uint64_t*>(lds + G::kOffSid);
  uint32_t* tab = reinterpret_cast<uint32_t*>(lds + G::kOffTab);
  uint16_t* lsvc = reinterpret_cast<uint16_t*>(lds + G::kOffSvc);  // !PACK only
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  uint32_t p[PER], ap[PER];
  bool v[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    p[j] = (uint32_t)(w * (PER * kWv) + j * kWv + lane);
    v[j] = p[j] < m;
    ap[j] = v[j] ? (uint32_t)pin[a0 + p[j]] : 0u;  // level-A position
  }
  uint4 ra[PER], rb[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {  // the gathers (CONTIG: the bucket's own records) together
    const uint4* q = reinterpret_cast<const uint4*>(rec + (CONTIG ? a0 + p[j] : ap[j]));
    ra[j] = v[j] ? q[0] : make_uint4(0, 0, 0, 0);
    rb[j] = v[j] ? q[1] : make_uint4(0, 0, 0, 0);
  }
  for (uint32_t i = tid; i < (uint32_t)(G::kTabBytes / 16u); i += W)
    reinterpret_cast<uint4*>(tab)[i] = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint64_t k = mix64(((uint64_t)ra[j].y << 32) | ra[j].x);
    if (v[j]) {
      lkx[p[j]] = PACK ? (((uint64_t)(rb[j].z & 0xFFFu) << 52) | (k & kKeyLow)) : k;
      lsid[p[j]] = ((uint64_t)ra[j].w << 32) | ra[j].z;
      if constexpr (!PACK) lsvc[p[j]] = (uint16_t)rb[j].z;
    }
  }
  __syncthreads();
  auto same_trace = [](uint64_t a, uint64_t b) {
    return PACK ? ((a ^ b) & kKeyLow) == 0ull : a == b;
  };
  // inserts: every span's first CAS issued together; a taken slot (another
  // key, or the same (trace, id) again) continues in the probe loop
  // (keys and span ids are read back from LDS: the records' first halves are
  // dead after the staging, which keeps the kernel at four workgroups per CU)
  uint32_t sl[PER], cur[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j)
    sl[j] = v[j] ? join_slot(lkx[p[j]] & (PACK ? kKeyLow : ~0ull), lsid[p[j]], kSlots) : 0u;
#pragma unroll
  for (int j = 0; j < PER; ++j) cur[j] = v[j] ? slot_cas<T16>(tab, sl[j], 0u, p[j] + 1u) : 0u;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if (cur[j] == 0u) continue;
    const uint64_t id = lsid[p[j]], kj = lkx[p[j]];
    uint32_t s = sl[j], c = cur[j];
    while (true) {
      uint32_t q = c - 1u;
      if (same_trace(lkx[q], kj) && lsid[q] == id) {
        // a repeated (trace, id): the smallest level-A position keeps the slot
        const uint32_t mine = (uint32_t)pin[a0 + p[j]];
        while ((uint32_t)pin[a0 + q] > mine) {
          const uint32_t old = slot_cas<T16>(tab, s, q + 1u, p[j] + 1u);
          if (old == q + 1u) break;
          q = old - 1u;  // another copy took it first: compare with that one
        }
        break;
      }
      s = (s + 1u) & (kSlots - 1u);
      c = slot_cas<T16>(tab, s, 0u, p[j] + 1u);
      if (c == 0u) break;
    }
  }
  __syncthreads();
  // lookups: first probes, their candidates' keys, then the services, each
  // round issued for every span together; a miss on an occupied slot probes on
  uint32_t e[PER], prow[PER];
  uint64_t pid[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    pid[j] = ((uint64_t)rb[j].y << 32) | rb[j].x;
    sl[j] = v[j] ? join_slot(lkx[p[j]] & (PACK ? kKeyLow : ~0ull), pid[j], kSlots) : 0u;
    e[j] = v[j] && pid[j] != 0ull ? slot_get<T16>(tab, sl[j]) : 0u;
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    prow[j] = pid[j] == 0ull ? eo.S : eo.S + 1u;  // ROOT / ORPHAN unless the trace holds it
    if (e[j] == 0u) continue;
    const uint32_t q = e[j] - 1u;
    const uint64_t kj = lkx[p[j]];
    if (same_trace(lkx[q], kj) && lsid[q] == pid[j]) continue;  // found: its service below
    uint32_t s = sl[j];
    e[j] = 0u;
    while (true) {
      s = (s + 1u) & (kSlots - 1u);
      const uint32_t c = slot_get<T16>(tab, s);
      if (c == 0u) break;
      if (same_trace(lkx[c - 1u], kj) && lsid[c - 1u] == pid[j]) {
        e[j] = c;
        break;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if (!v[j]) continue;
    if (e[j] != 0u) prow[j] = PACK ? (uint32_t)(lkx[e[j] - 1u] >> 52) : lsvc[e[j] - 1u];
    const uint32_t svc = rb[j].z & 0xFFFFu, fl = rb[j].z >> 16;
    eo.rec[a0 + p[j]] = ((uint64_t)(prow[j] * eo.S + svc) << 33) |
                        ((uint64_t)((fl & ANOMOD_FLAG_ERROR) ? 1u : 0u) << 32) | rb[j].w;
  }
}

constexpr int kJoinW = 512, kJoinPer = 4;           // 2 048 spans per bucket

constexpr int kJoinBigW = 1024;                     // buckets over 2 048 spans
constexpr int join_big_per(bool pack) { return pack ? 8 : 4; }  // 8 192 / 4 096 spans

// One workgroup per bucket; a bucket over 2 048 spans is listed for the big
// kernel (a list overflow: the unfused path).
// MINW: waves per SIMD the registers must allow (6 = three 512-thread
// workgroups per CU; 8 = four, 64 VGPRs with 28 B per lane spilled); T16: u16
// table slots (PACK at 2 048 spans: 40 KiB, else 48).
template <bool PACK, int MINW = 6, bool T16 = !PACK, bool CONTIG = false>
__global__ __launch_bounds__(kJoinW, MINW) void bk_join_kernel(
    const uint64_t* __restrict__ pin, const GRec* __restrict__ rec, EdgeOut eo,
    const uint32_t* __restrict__ bstart, uint32_t* __restrict__ over,
    unsigned long long* __restrict__ over_n, uint32_t over_cap,
    unsigned long long* __restrict__ too_big) {
  using G = JoinGeom<kJoinW, kJoinPer, PACK, T16>;
  __shared__ __attribute__((aligned(16))) unsigned char lds[G::kBytes];
  const uint32_t c = blockIdx.x;
  const uint32_t a0 = bstart[c], m = bstart[c + 1] - a0;
  if (m > (uint32_t)G::kCap) {
    if (threadIdx.x == 0) {
      const unsigned long long i = atomicAdd(over_n, 1ull);
      if (i < over_cap) over[i] = c;
      else atomicAdd(too_big, 1ull);
    }
    return;
  }
  if (m == 0) return;
  join_bucket<kJoinW, kJoinPer, PACK, T16, CONTIG>(lds, a0, m, pin, rec, eo);
}

// The listed buckets, one workgroup each in turn; one over this kernel's
// capacity (traces of thousands of spans side by side) sends the set to the
// unfused path (too_big).
template <bool PACK, bool CONTIG = false>
__global__ __launch_bounds__(kJoinBigW) void bk_join_big_kernel(
    const uint64_t* __restrict__ pin, const GRec* __restrict__ rec, EdgeOut eo,
    const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ over,
    const unsigned long long* __restrict__ over_n, uint32_t over_cap,
    unsigned long long* __restrict__ too_big) {
  constexpr int PER = join_big_per(PACK);
  using G = JoinGeom<kJoinBigW, PER, PACK>;
  __shared__ __attribute__((aligned(16))) unsigned char lds[G::kBytes];
  const uint64_t cnt = *over_n < over_cap ? *over_n : over_cap;
  for (uint64_t i = blockIdx.x; i < cnt; i += gridDim.x) {
    const uint32_t c = over[i];
    const uint32_t a0 = bstart[c], m = bstart[c + 1] - a0;
    if (m > (uint32_t)G::kCap) {
      if (threadIdx.x == 0) atomicAdd(too_big, 1ull);
      continue;
    }
    join_bucket<kJoinBigW, PER, PACK, true, CONTIG>(lds, a0, m, pin, rec, eo);
    __syncthreads();  // the next bucket reuses the LDS
  }
}

// The fused ungrouped aggregation's bucket kernels: the same sort, then
// edge records instead of grouped columns.
__global__ __launch_bounds__(kSmallW) void bk_bucket_edge_kernel(
    uint64_t* __restrict__ pin, const GRec* __restrict__ rec, EdgeOut eo,
    const uint32_t* __restrict__ bstart, int kshift, uint32_t* __restrict__ over,
    unsigned long long* __restrict__ over_n, uint32_t over_cap,
    unsigned long long* __restrict__ too_big) {
  __shared__ BucketLds<kSmallW, kSmallPer, true> L;
  bucket_sort_one<kSmallW, kSmallPer, true>(L, blockIdx.x, pin, rec, SoaOut{}, eo, bstart, kshift,
                                            nullptr, true, over, over_n, over_cap, too_big);
}

__global__ __launch_bounds__(kBigW) void bk_bucket_edge_big_kernel(
    uint64_t* __restrict__ pin, const GRec* __restrict__ rec, EdgeOut eo,
    const uint32_t* __restrict__ bstart, int kshift, const uint32_t* __restrict__ over,
    const unsigned long long* __restrict__ over_n, uint32_t over_cap,
    unsigned long long* __restrict__ too_big) {
  __shared__ BucketLds<kBigW, kBigPer, true> L;
  const uint64_t cnt = *over_n < over_cap ? *over_n : over_cap;
  for (uint64_t i = blockIdx.x; i < cnt; i += gridDim.x) {
    bucket_sort_one<kBigW, kBigPer, true>(L, over[i], pin, rec, SoaOut{}, eo, bstart, kshift,
                                          nullptr, false, nullptr, nullptr, 0, too_big);
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBigW) void bk_bucket_big_kernel(
    uint64_t* __restrict__ pin, const GRec* __restrict__ rec, SoaOut out,
    const uint32_t* __restrict__ bstart, int kshift, uint32_t* __restrict__ dcnt,
    const uint32_t* __restrict__ over, const unsigned long long* __restrict__ over_n,
    uint32_t over_cap, unsigned long long* __restrict__ too_big) {
  __shared__ BucketLds<kBigW, kBigPer> L;
  const uint64_t cnt = *over_n < over_cap ? *over_n : over_cap;
  for (uint64_t i = blockIdx.x; i < cnt; i += gridDim.x) {
    bucket_sort_one<kBigW, kBigPer, false>(L, over[i], pin, rec, out, EdgeOut{}, bstart, kshift,
                                           dcnt, false, nullptr, nullptr, 0, too_big);
    __syncthreads();
  }
}

// Largest bucket -> *mx (the host skips the bucket kernels when one cannot hold it).
__global__ __launch_bounds__(256) void bk_maxsize_kernel(const uint32_t* __restrict__ bstart,
                                                         uint64_t nb,
                                                         unsigned long long* __restrict__ mx) {
  uint32_t m = 0;
  for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < nb; c += (uint64_t)gridDim.x * 256) {
    const uint32_t s = bstart[c + 1] - bstart[c];
    m = s > m ? s : m;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t y = __shfl_xor(m, o);
    m = y > m ? y : m;
  }
  if ((threadIdx.x & (kWv - 1)) == 0) atomicMax(mx, (unsigned long long)m);
}

// ---- trace_ptr from the buckets' trace starts --------------------------------
__global__ __launch_bounds__(256) void bk_dsum_kernel(const uint32_t* __restrict__ dcnt, uint64_t nb,
                                                      uint32_t* __restrict__ part) {
  __shared__ uint32_t wsum[4];
  const uint64_t a = (uint64_t)blockIdx.x * kDChunk;
  uint32_t s = 0;
  for (int j = 0; j < kDChunk / 256; ++j) {
    const uint64_t p = a + (uint64_t)(j * 256 + threadIdx.x);
    s += p < nb ? dcnt[p] : 0u;
  }
  uint32_t all;
  (void)block_excl_scan<4>(s, wsum, &all);
  if (threadIdx.x == 0) part[blockIdx.x] = all;
}

// one block: exclusive scan of the partial sums (<= 1024 of them), the trace
// count to *total, trace_ptr closed
__global__ __launch_bounds__(1024) void bk_dscan_top_kernel(uint32_t* __restrict__ part, uint64_t np,
                                                            unsigned long long* __restrict__ total,
                                                            uint64_t* __restrict__ tptr, uint64_t n) {
  __shared__ uint32_t wsum[16];
  const uint32_t x = threadIdx.x < np ? part[threadIdx.x] : 0u;
  uint32_t all;
  const uint32_t pre = block_excl_scan<16>(x, wsum, &all);
  if (threadIdx.x < np) part[threadIdx.x] = pre;
  if (threadIdx.x == 0) {
    *total = all;
    tptr[all] = n;
  }
}

// dcnt -> its exclusive scan in place, dcnt[nb] = the total
__global__ __launch_bounds__(256) void bk_ddown_kernel(uint32_t* __restrict__ dcnt, uint64_t nb,
                                                       const uint32_t* __restrict__ part) {
  __shared__ uint32_t wsum[4];
  constexpr int kPerT = kDChunk / 256;
  const uint64_t a = (uint64_t)blockIdx.x * kDChunk + (uint64_t)threadIdx.x * kPerT;
  uint32_t x[kPerT], s = 0;
#pragma unroll
  for (int j = 0; j < kPerT; ++j) {
    x[j] = a + j < nb ? dcnt[a + j] : 0u;
    s += x[j];
  }
  uint32_t all;
  uint32_t run = part[blockIdx.x] + block_excl_scan<4>(s, wsum, &all);
#pragma unroll
  for (int j = 0; j < kPerT; ++j) {
    if (a + j < nb) dcnt[a + j] = run;
    run += x[j];
  }
}

// one wave per bucket: its trace starts (over its pairs) to trace_ptr[tbase[c] ...]
__global__ __launch_bounds__(256) void bk_tptr_kernel(const uint64_t* __restrict__ tsp,
                                                      const uint32_t* __restrict__ bstart,
                                                      const uint32_t* __restrict__ tbase,
                                                      uint64_t nb,
                                                      const unsigned long long* __restrict__ total,
                                                      uint64_t* __restrict__ tptr) {
  const uint64_t c = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / kWv;
  const uint32_t lane = threadIdx.x & (kWv - 1);
  if (c >= nb) return;
  const uint32_t t0 = tbase[c];
  const uint32_t t1 = c + 1 < nb ? tbase[c + 1] : (uint32_t)*total;
  const uint64_t src = bstart[c];
  for (uint32_t o = lane; o < t1 - t0; o += kWv) tptr[t0 + o] = tsp[src + o];
}

inline int env_int(const char* name, int dflt) {
  const char* s = std::getenv(name);
  return s && *s ? std::atoi(s) : dflt;
}

}  // namespace

bool join_records_through_b() { return env_int("ANOMOD_JOIN_RECB", 0) != 0; }

BucketGeom bucket_geom(uint64_t n) {
  BucketGeom g;
  // mean bucket size in (avg/2, avg]; the small kernel holds 2048 spans (at
  // a mean of 1400 SN spans that is +3.6 sigma: ~1e-4 of the buckets take
  // the large kernel)
  int avg = env_int("ANOMOD_BUCKET_AVG", 1400);
  avg = std::min(std::max(avg, 64), 2048);
  g.T = 1;
  while (g.T < 2 * kDMax && (n >> g.T) > (uint64_t)avg) ++g.T;
  if (g.T <= kDMax) {
    g.DA = g.T;
    g.DB = 0;
  } else {
    // Level A's writes cost more with more digits (1 KiB wave stores cover
    // shorter runs), level B's less (its writes stay inside one level-A bucket,
    // and smaller buckets stay in the Infinity Cache): level A takes at most 9
    // bits.  (2^27 SN traces, T = 20: A + B 25.5 + 25.1 ms at 9 + 11 bits,
    // 30.4 + 23.8 at 10 + 10, 32.8 + 21.3 at 11 + 9; 2^25, T = 18: 9 + 9 best,
    // 16.0 vs 16.4 / 17.8 ms grouping at 8 + 10 / 7 + 11.)
    g.DA = std::max(g.T - kDMax, std::min((g.T + 1) / 2, 9));
    // experiment knob: level A's share of the bits (the rest, <= kDMax, to level B)
    const int da = env_int("ANOMOD_BUCKET_DA", 0);
    if (da > 0) g.DA = std::min(std::max(da, g.T - kDMax), kDMax);
    g.DB = g.T - g.DA;
  }
  g.tilesA = n ? (n + kBTile - 1) / kBTile : 1;
  g.tilesB = g.DB ? (n + kPTile - 1) / kPTile + (1ull << g.DA) : 0;
  return g;
}

namespace {

// Largest bucket of bstart[0 .. nbk] (one host wait).
int max_bucket(anomod_ctx* ctx, const uint32_t* bstart, uint64_t nbk, uint64_t* mx) {
  GroupWs* ws = ctx->group_ws;
  hipStream_t st = ctx->stream;
  ANOMOD_HIP(ctx, hipMemsetAsync(ws->misc + kMiscTooBig, 0, 8, st));
  hipLaunchKernelGGL(bk_maxsize_kernel, dim3((unsigned)std::min<uint64_t>((nbk + 255) / 256, 1024)),
                     dim3(256), 0, st, bstart, nbk, ws->misc + kMiscTooBig);
  ANOMOD_HIP(ctx, hipMemcpyAsync(ws->h_misc + kMiscTooBig, ws->misc + kMiscTooBig, 8,
                                 hipMemcpyDeviceToHost, st));
  ANOMOD_HIP(ctx, hipStreamSynchronize(st));
  *mx = ws->h_misc[kMiscTooBig];
  return hipMemsetAsync(ws->misc + kMiscTooBig, 0, 8, st) == hipSuccess ? ANOMOD_OK : ANOMOD_EHIP;
}

int bucket_run_geom(anomod_ctx* ctx, const anomod_spans* in, BucketGeom g, GroupResult* res,
                    bool* fallback, bool* escalate, const EdgeOut* eo, bool want_h) {
  *fallback = false;
  *escalate = false;
  GroupWs* ws = ctx->group_ws;
  const uint64_t n = in->n_spans;
  const int na = 1 << g.DA;
  if ((1ull << g.T) > ws->bucket_cap || g.tilesB > ws->tile_cap ||  // sized for the geometry
      g.DA > kDMax || g.DB > kDMax || (g.tilesA << g.DA) > ws->tcnt_words ||
      (g.tilesB << kDMax) > ws->tcnt_words) {
    *fallback = true;
    return ANOMOD_OK;
  }
  const uint64_t cap = ws->cap;
  auto soa_of = [cap](GRec* buf) {
    char* ob = reinterpret_cast<char*>(buf);
    return SoaOut{reinterpret_cast<uint64_t*>(ob), reinterpret_cast<uint64_t*>(ob + 8 * cap),
                  reinterpret_cast<uint64_t*>(ob + 16 * cap),
                  reinterpret_cast<uint32_t*>(ob + 24 * cap),
                  reinterpret_cast<uint32_t*>(ob + 28 * cap)};
  };
  const SoaIn sin{in->trace_hash, in->span_id, in->parent_span_id, in->svc_flags, in->dur_us};
  GRec* recs = ws->aos[0];                    // level-A records (gathered by the buckets)
  SoaOut cols = ws->aos[1] ? soa_of(ws->aos[1]) : SoaOut{};  // the grouped columns
  if (!want_h) cols.h = nullptr;              // an aggregation reads no trace_hash column
  // the fused aggregation's per-bucket hash join (ANOMOD_FUSED_JOIN=0: the
  // sorting bucket kernels' edge form)
  const bool join = eo && env_int("ANOMOD_FUSED_JOIN", 1) != 0;
  // (records through level B: the join reads them contiguously; two levels only)
  const bool recb = join && g.DB > 0 && join_records_through_b();
  uint64_t* pa = ws->pairs[0];                // level-A pairs
  uint64_t* pb = ws->pairs[1];                // level-B pairs
  hipStream_t st = ctx->stream;
  ANOMOD_HIP(ctx, hipMemsetAsync(ws->misc, 0, kMiscWords * 8, st));

  // XCD-contiguous tile order per scatter level (experiment knob
  // ANOMOD_BK_XCD: bit 0 level A, bit 1 level B, bit 2 the bucket kernel —
  // off by default there: buckets in index order keep every XCD inside one
  // level-A bucket, whose records the gathers then find in the Infinity Cache)
  const int xk = env_int("ANOMOD_BK_XCD", 3);
  const uint32_t nxA = (xk & 1) ? 8u : 1u, nxB = (xk & 2) ? 8u : 1u;
  // level A (its bucket starts bsA; btile: level-B tiles per level-A bucket)
  const uint64_t nbA = (g.tilesA + kScanRows - 1) / kScanRows;
  const unsigned dgA = (unsigned)((na + 255) / 256);
  hipLaunchKernelGGL(bk_count_a_kernel, dim3((unsigned)g.tilesA), dim3(256), 0, st,
                     in->trace_hash, n, g.DA, ws->tcnt);
  hipLaunchKernelGGL(bk_scan_up_kernel, dim3((unsigned)nbA, dgA), dim3(256), 0, st, ws->tcnt,
                     g.tilesA, na, ws->bsum);
  hipLaunchKernelGGL(bk_scan_top_kernel, dim3(1), dim3(1024), 0, st, ws->bsum, nbA, na, n,
                     ws->bsA, ws->btile, (uint32_t)kPTile);
  hipLaunchKernelGGL(bk_scan_down_kernel, dim3((unsigned)nbA, dgA), dim3(256), 0, st, ws->tcnt,
                     g.tilesA, na, ws->bsum);
  hipLaunchKernelGGL(bk_scatter_a_kernel, dim3((unsigned)g.tilesA), dim3(kBThreads), 0, st, sin,
                     recs, pa, n, g.DA, ws->tcnt, nxA);
  ANOMOD_HIP(ctx, hipGetLastError());
  if (ANOMOD_BK_ABL & 2) {  // timing of level A only
    *fallback = true;
    return ANOMOD_OK;
  }
  uint64_t* pin;
  const uint32_t* bstart;
  uint64_t mx = 0;
  if (g.DB > 0) {
    hipLaunchKernelGGL(bk_tilemap_kernel, dim3((unsigned)na), dim3(256), 0, st, ws->btile,
                       ws->tmap);
    for (;;) {
      hipLaunchKernelGGL(bk_count_b_kernel, dim3((unsigned)g.tilesB), dim3(256), 0, st, pa,
                         ws->bsA, ws->btile, ws->tmap, na, g.DB, ws->tcnt);
      hipLaunchKernelGGL(bk_scan_seg_kernel, dim3((unsigned)na), dim3(1024), 0, st, ws->tcnt,
                         ws->bsA, ws->btile, na, g.DB, ws->bstart);
      ANOMOD_HIP(ctx, hipGetLastError());
      if (int rc = max_bucket(ctx, ws->bstart, 1ull << g.T, &mx)) return rc;
      if (env_int("ANOMOD_BUCKET_DEBUG", 0))
        std::fprintf(stderr, "bucket path: DA=%d DB=%d max bucket %llu\n", g.DA, g.DB,
                     (unsigned long long)mx);
      if (mx <= (uint64_t)(kBigW * kBigPer) || g.DB == kDMax ||
          (1ull << (g.DA + kDMax)) > ws->bucket_cap)
        break;
      g.DB = kDMax;  // long traces side by side: split finer
      g.T = g.DA + g.DB;
    }
    // the join resolves repeated ids by level-A position: level B need not be
    // stable there (ANOMOD_BK_STABLE_B=1 keeps the stable scatter for A/B);
    // ANOMOD_JOIN_RECB=1: level B moves the records too (r06 A/B)
    if (join && recb)
      hipLaunchKernelGGL(bk_scatter_b_rec_kernel, dim3((unsigned)g.tilesB), dim3(kBThreads), 0, st,
                         pa, pb, recs, ws->aos[1], g.DB, ws->tcnt, ws->bsA, ws->btile, ws->tmap,
                         na, nxB);
    else if (join && !env_int("ANOMOD_BK_STABLE_B", 0))
      hipLaunchKernelGGL(bk_scatter_b_fast_kernel, dim3((unsigned)g.tilesB), dim3(kBThreads), 0, st,
                         pa, pb, g.DB, ws->tcnt, ws->bsA, ws->btile, ws->tmap, na, nxB);
    else
      hipLaunchKernelGGL(bk_scatter_b_kernel, dim3((unsigned)g.tilesB), dim3(kBThreads), 0, st, pa,
                         pb, g.DB, ws->tcnt, ws->bsA, ws->btile, ws->tmap, na, nxB);
    pin = pb;
    bstart = ws->bstart;
  } else {
    ANOMOD_HIP(ctx, hipGetLastError());
    if (int rc = max_bucket(ctx, ws->bsA, 1ull << g.T, &mx)) return rc;
    if (env_int("ANOMOD_BUCKET_DEBUG", 0))
      std::fprintf(stderr, "bucket path: one level, T=%d, max bucket %llu\n", g.T,
                   (unsigned long long)mx);
    if (mx > (uint64_t)(kBigW * kBigPer)) {  // the caller retries with two levels
      *escalate = true;
      return ANOMOD_OK;
    }
    pin = pa;
    bstart = ws->bsA;
  }
  ANOMOD_HIP(ctx, hipGetLastError());
  const uint64_t nbk = 1ull << g.T;

  // buckets: <= 2048 spans in the small kernel, the rest listed for the
  // large one (<= 8192 spans, or any size holding one trace); the sub-split
  // takes the 9 pair bits below the DB bits level B took
  const int kshift = 64 - g.DB - kSubBits;
  // one workgroup per bucket; ANOMOD_BK_PIPE=1: the persistent pipelined
  // bucket kernel, as many workgroups as are resident at once (measured
  // slower: 93 vs 64 ms grouping at 2^27 SN traces, gpurun_out/r4c_pipe_f0.log)
  const bool pipe = env_int("ANOMOD_BK_PIPE", 0) != 0;
  auto pipe_grid = [&](const void* fn) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kSmallW, 0) != hipSuccess)
      per_cu = 1;
    return (unsigned)std::min<uint64_t>(nbk, (uint64_t)std::max(ctx->num_cus, 1) *
                                                 (uint64_t)std::max(per_cu, 1));
  };
  if (eo) {  // the fused ungrouped aggregation: edge records, no columns, no trace_ptr
    if (join) {
      // PACK: the service rides in the 12 key bits every k of a bucket shares
      // (ANOMOD_JOIN_PACK=0 forces the separate service array: tests)
      const bool pack = g.T >= 12 && env_int("ANOMOD_JOIN_PACK", 1) != 0;
      const unsigned big_grid = (unsigned)std::max(ctx->num_cus, 1);
      if (pack) {
        // ANOMOD_JOIN_W6=1: the 3-workgroups-per-CU form (no spills; A/B)
        // u32 slots, three workgroups per CU (48 KiB): 48.0 ms grouping at
        // 2^27 SN traces, against 48.3 with u16 slots (40 KiB) at three and
        // 49.8 at four per CU, which spills (gpurun_out/r5b/ab_w6.log);
        // ANOMOD_JOIN_FORM = 1 / 2 runs those two (A/B)
        const int jv = env_int("ANOMOD_JOIN_FORM", 0);
        auto fn = recb ? bk_join_kernel<true, 6, false, true>
                  : jv == 2 ? bk_join_kernel<true, 8, true>
                  : jv == 1 ? bk_join_kernel<true, 6, true> : bk_join_kernel<true, 6, false>;
        const GRec* jrec = recb ? ws->aos[1] : recs;
        hipLaunchKernelGGL(fn, dim3((unsigned)nbk), dim3(kJoinW), 0, st, pin,
                           jrec, *eo, bstart, ws->over, ws->misc + kMiscBigN, (uint32_t)nbk,
                           ws->misc + kMiscTooBig);
        auto fb = recb ? bk_join_big_kernel<true, true> : bk_join_big_kernel<true>;
        hipLaunchKernelGGL(fb,
                           dim3(big_grid), dim3(kJoinBigW), 0, st, pin,
                           jrec, *eo, bstart, ws->over, ws->misc + kMiscBigN, (uint32_t)nbk,
                           ws->misc + kMiscTooBig);
      } else {
        const GRec* jrec = recb ? ws->aos[1] : recs;
        auto fs = recb ? bk_join_kernel<false, 6, true, true> : bk_join_kernel<false, 6, true>;
        auto fb = recb ? bk_join_big_kernel<false, true> : bk_join_big_kernel<false>;
        hipLaunchKernelGGL(fs,
                           dim3((unsigned)nbk), dim3(kJoinW), 0, st, pin,
                           jrec, *eo, bstart, ws->over, ws->misc + kMiscBigN, (uint32_t)nbk,
                           ws->misc + kMiscTooBig);
        hipLaunchKernelGGL(fb,
                           dim3(big_grid), dim3(kJoinBigW), 0, st, pin,
                           jrec, *eo, bstart, ws->over, ws->misc + kMiscBigN, (uint32_t)nbk,
                           ws->misc + kMiscTooBig);
      }
    } else if (pipe)
      hipLaunchKernelGGL(bk_bucket_pipe_kernel<true>,
                         dim3(pipe_grid(reinterpret_cast<const void*>(bk_bucket_pipe_kernel<true>))),
                         dim3(kSmallW), 0, st, pin, recs, SoaOut{}, *eo, bstart, (uint32_t)nbk,
                         kshift, nullptr, ws->over, ws->misc + kMiscBigN, (uint32_t)nbk,
                         ws->misc + kMiscTooBig);
    else
      hipLaunchKernelGGL(bk_bucket_edge_kernel, dim3((unsigned)nbk), dim3(kSmallW), 0, st, pin,
                         recs, *eo, bstart, kshift, ws->over, ws->misc + kMiscBigN, (uint32_t)nbk,
                         ws->misc + kMiscTooBig);
    if (!join)
      hipLaunchKernelGGL(bk_bucket_edge_big_kernel, dim3((unsigned)std::max(ctx->num_cus, 1)),
                         dim3(kBigW), 0, st, pin, recs, *eo, bstart, kshift, ws->over,
                         ws->misc + kMiscBigN, (uint32_t)nbk, ws->misc + kMiscTooBig);
    ANOMOD_HIP(ctx, hipGetLastError());
    ANOMOD_HIP(ctx, hipMemcpyAsync(ws->h_misc + kMiscRead, ws->misc + kMiscRead,
                                   (kMiscWords - kMiscRead) * 8, hipMemcpyDeviceToHost, st));
    ANOMOD_HIP(ctx, hipStreamSynchronize(st));
    *fallback = ws->h_misc[kMiscTooBig] != 0;
    res->passes = g.DB ? 2 : 1;
    res->bits = g.T;
    res->bucket = true;
    res->join = join;
    return ANOMOD_OK;
  }
  if (pipe)
    hipLaunchKernelGGL(bk_bucket_pipe_kernel<false>,
                       dim3(pipe_grid(reinterpret_cast<const void*>(bk_bucket_pipe_kernel<false>))),
                       dim3(kSmallW), 0, st, pin, recs, cols, EdgeOut{}, bstart, (uint32_t)nbk,
                       kshift, ws->dcnt, ws->over, ws->misc + kMiscBigN, (uint32_t)nbk,
                       ws->misc + kMiscTooBig);
  else
    hipLaunchKernelGGL(bk_bucket_kernel, dim3((unsigned)nbk), dim3(kSmallW), 0, st, pin, recs,
                       cols, bstart, kshift, ws->dcnt, ws->over, ws->misc + kMiscBigN,
                       (uint32_t)nbk, ws->misc + kMiscTooBig, (xk & 4) ? 8u : 1u);
  hipLaunchKernelGGL(bk_bucket_big_kernel, dim3((unsigned)std::max(ctx->num_cus, 1)),
                     dim3(kBigW), 0, st, pin, recs, cols, bstart, kshift, ws->dcnt, ws->over,
                     ws->misc + kMiscBigN, (uint32_t)nbk, ws->misc + kMiscTooBig);
  ANOMOD_HIP(ctx, hipGetLastError());

  // trace_ptr
  const uint64_t np = (nbk + kDChunk - 1) / kDChunk;  // <= 1024 (T <= 22)
  hipLaunchKernelGGL(bk_dsum_kernel, dim3((unsigned)np), dim3(256), 0, st, ws->dcnt, nbk,
                     ws->part);
  hipLaunchKernelGGL(bk_dscan_top_kernel, dim3(1), dim3(1024), 0, st, ws->part, np,
                     ws->misc + kMiscTraces, ws->tptr, n);
  hipLaunchKernelGGL(bk_ddown_kernel, dim3((unsigned)np), dim3(256), 0, st, ws->dcnt, nbk,
                     ws->part);
  hipLaunchKernelGGL(bk_tptr_kernel, dim3((unsigned)((nbk * kWv + 255) / 256)), dim3(256), 0, st,
                     pin, bstart, ws->dcnt, nbk, ws->misc + kMiscTraces, ws->tptr);
  ANOMOD_HIP(ctx, hipGetLastError());
  ANOMOD_HIP(ctx, hipMemcpyAsync(ws->h_misc + kMiscRead, ws->misc + kMiscRead,
                                 (kMiscWords - kMiscRead) * 8, hipMemcpyDeviceToHost, st));
  ANOMOD_HIP(ctx, hipStreamSynchronize(st));
  if (env_int("ANOMOD_BUCKET_DEBUG", 0))
    std::fprintf(stderr, "bucket path: T=%d DA=%d DB=%d max bucket %llu, %llu over 2048, %llu too big\n",
                 g.T, g.DA, g.DB, (unsigned long long)mx, ws->h_misc[kMiscBigN],
                 ws->h_misc[kMiscTooBig]);
  if (ws->h_misc[kMiscTooBig]) {
    *fallback = true;
    return ANOMOD_OK;
  }
  res->cols = cols;
  res->n_traces = ws->h_misc[kMiscTraces];
  res->tptr = ws->tptr;
  res->passes = g.DB ? 2 : 1;
  res->bits = g.T;
  res->bucket = true;
  return ANOMOD_OK;
}

}  // namespace

int bucket_group_run(anomod_ctx* ctx, const anomod_spans* in, GroupResult* res, bool* fallback,
                     uint64_t* erec, uint32_t S, bool want_h) {
  BucketGeom g = bucket_geom(in->n_spans);
  bool escalate = false;
  const EdgeOut eo{erec, S};
  const EdgeOut* pe = erec ? &eo : nullptr;
  if (int rc = bucket_run_geom(ctx, in, g, res, fallback, &escalate, pe, want_h)) return rc;
  if (!escalate) return ANOMOD_OK;
  // one level was not enough for the set's longest traces: two, the second
  // with kDMax bits
  g.DB = kDMax;
  g.T = g.DA + g.DB;
  g.tilesB = (in->n_spans + kPTile - 1) / kPTile + (1ull << g.DA);
  return bucket_run_geom(ctx, in, g, res, fallback, &escalate, pe, want_h);
}

}  // namespace anomod
