// Trace-chunk walking shared by the span kernels (edge aggregation, trace
// structure).  A wave owns a contiguous range of traces and walks it in
// chunks of up to 64 whole traces holding <= kStage spans (or one trace longer
// than kStage), so every per-trace question is answered inside the wave's own
// LDS staging area.  Internal header (not part of the ABI).
#pragma once

#include "common.h"

namespace anomod {
namespace {  // internal linkage: a kernel file may pick its own chunk size
namespace chunk {

#ifndef ANOMOD_STAGE
#define ANOMOD_STAGE 256
#endif
constexpr int kWave = 64;
constexpr int kStage = ANOMOD_STAGE;  // spans staged per wave chunk
constexpr int kPer = kStage / kWave;
static_assert(kStage % kWave == 0 && kStage <= 1024, "chunk size");

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Make a wave-uniform 64-bit value provably uniform (SGPR) for the compiler.
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
}

// Buffer descriptor over [base, base + bytes): loads past the end return 0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                           0x00020000);
}

// Cache policy of the streamed span-column loads (aux bits: 1 = sc0, 2 = nt,
// 16 = sc1); every column is read once per launch.
#ifndef ANOMOD_LOAD_AUX
#define ANOMOD_LOAD_AUX 0
#endif

__device__ __forceinline__ uint64_t bload64(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return (uint64_t)__builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, ANOMOD_LOAD_AUX);
}

__device__ __forceinline__ uint32_t bload32(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, ANOMOD_LOAD_AUX);
}

// Streamed per-span output stores (written once, never re-read by the
// kernel): plain, or nontemporal with ANOMOD_STORE_NT.
#ifndef ANOMOD_STORE_NT
#define ANOMOD_STORE_NT 0
#endif
template <class T>
__device__ __forceinline__ void st_out(T* p, T v) {
  if constexpr (ANOMOD_STORE_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// One wave's chunk: up to 64 consecutive traces holding <= kStage spans, or a
// single trace longer than kStage (k == 0).  base / k / n are wave-uniform.
struct Chunk {
  uint64_t base;   // first span
  uint32_t k;      // traces in the chunk (0 = one big trace)
  uint32_t n;      // spans in the chunk
  uint32_t start;  // this lane's trace start relative to base (lanes < k)
};

// Lane `l` (wave-uniform) of a 64-bit value, through v_readlane (SALU side,
// no LDS-pipe permute).
__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
}

// lo/hi = trace_ptr[t + lane], trace_ptr[t + lane + 1] (see load_bounds).
// A trace longer than big_min (<= kStage) is a chunk of its own (k == 0):
// the kernels hand such traces to their workgroup-per-trace pass.
__device__ __forceinline__ Chunk make_chunk(uint64_t t, uint64_t t_end, int lane, uint64_t lo,
                                            uint64_t hi, uint32_t big_min = kStage) {
  Chunk c;
  const bool valid = t + lane < t_end;
  c.base = readlane64(lo, 0);
  const bool fits = valid && (hi - c.base) <= (uint64_t)kStage;
  c.k = (uint32_t)__popcll(__ballot(fits));  // fits is a prefix of the lanes
  if (big_min < (uint32_t)kStage) {
    const uint64_t lm = __ballot(valid && (hi - lo) > (uint64_t)big_min);
    const uint32_t first = lm ? (uint32_t)__ffsll((unsigned long long)lm) - 1u : 64u;
    c.k = first < c.k ? first : c.k;  // 0 when the first trace is long: a chunk of its own
  }
  c.n = (uint32_t)(readlane64(hi, c.k ? (int)c.k - 1 : 0) - c.base);
  c.start = (uint32_t)(lo - c.base);
  return c;
}

// trace_ptr[t + lane] and trace_ptr[t + lane + 1] for lanes t + lane < t_end
// (0 elsewhere).  t and t_end are wave-uniform.
__device__ __forceinline__ void load_bounds(const uint64_t* __restrict__ trace_ptr, uint64_t t,
                                            uint64_t t_end, int lane, uint64_t& lo, uint64_t& hi) {
  t = uniform64(t);
  const uint64_t avail = t_end > t ? t_end - t : 0;
  const uint32_t bytes = (uint32_t)(avail < (uint64_t)kWave ? avail : (uint64_t)kWave) * 8u;
  lo = bload64(rsrc(trace_ptr + t, bytes), (uint32_t)lane * 8u);
  hi = bload64(rsrc(trace_ptr + t + 1, bytes), (uint32_t)lane * 8u);
}

// Trace-start masks of a chunk: bit l of Sm[r] is set when chunk position
// 64*r + l starts a trace.  lflag is the wave's u8[kStage] LDS scratch.
__device__ __forceinline__ void start_masks(uint8_t* lflag, const Chunk& c, int lane,
                                            uint64_t (&Sm)[kPer]) {
  for (int w = lane; w < kStage / 4; w += kWave) reinterpret_cast<uint32_t*>(lflag)[w] = 0u;
  wave_sync();
  if ((uint32_t)lane < c.k && c.start < c.n) lflag[c.start] = 1;
  wave_sync();
#pragma unroll
  for (int r = 0; r < kPer; ++r) Sm[r] = __ballot(lflag[lane + r * kWave] != 0);
}

// Bounds [a, b) of the trace holding chunk position i = 64*r + lane, from the
// four 64-bit trace-start masks (wave-uniform); branch-free (selects only).
__device__ __forceinline__ void trace_bounds(const uint64_t (&Sm)[kPer], int r, int lane,
                                             uint32_t n, uint32_t& a, uint32_t& b) {
  const uint64_t le = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
  a = 0;
  b = n;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    if (q > r) break;
    const uint64_t m = (q == r) ? (Sm[q] & le) : Sm[q];
    const uint32_t pos = 64u * q + 63u - (uint32_t)__clzll((long long)m);
    a = m ? pos : a;
  }
#pragma unroll
  for (int q = kPer - 1; q >= 0; --q) {
    if (q < r) break;
    const uint64_t m = (q == r) ? (Sm[q] & ~le) : Sm[q];
    const uint32_t pos = 64u * q + (uint32_t)__ffsll((unsigned long long)m) - 1u;
    b = m ? pos : b;
  }
  if (b > n) b = n;
}

// Index of the trace (within the chunk) holding chunk position 64*r + lane.
__device__ __forceinline__ uint32_t trace_in_chunk(const uint64_t (&Sm)[kPer], int r, int lane) {
  uint32_t before = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q)
    if (q < r) before += (uint32_t)__popcll(Sm[q]);
  const uint64_t m = Sm[r];
  const uint32_t below =
      __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  return before + below + (uint32_t)((m >> lane) & 1ull) - 1u;
}

// Span sets whose ids are unique within every trace (declared by their
// producer: the synthetic generator by construction, the decoders after
// checking, anomod_spans_set_unique_ids): at most one span of [a, b) holds
// pid, so the first match is the only match and the scan may run from both
// ends — kFwd ids forward from the trace start and kBwd backward from the
// span's own position per step (same 5 x ds_read2_b64 as the forward scan).
// Parents usually sit right before their children (Jaeger / SkyWalking emit
// a callee's spans after the calling span) or near the trace start (the
// caller's entry span); simulated row-steps per 256-span chunk: TrainTicket
// 18.8 -> 9.2, SocialNetwork 6.5 -> 4.0.
#ifndef ANOMOD_FWD
#define ANOMOD_FWD 6
#endif
#ifndef ANOMOD_BWD
#define ANOMOD_BWD 4
#endif
constexpr uint32_t kFwd = ANOMOD_FWD, kBwd = ANOMOD_BWD;
static_assert(kFwd % 2 == 0 && kBwd % 2 == 0 && kFwd + kBwd <= 16, "bidirectional step");
// Ids are staged with this many entries of slack past the chunk (edge_agg.hip
// kWSid, trace_struct.hip kTSid): a forward block may read that far past the
// trace end, so no forward block is wider.
constexpr uint32_t kScanSlack = 16;

// MAXS > 0: give up after that many steps and return -2 (not found yet; the
// caller completes the lookup cooperatively).
// SEL: the matches found by selects (lowest matching slot of each block, kept
// if inside the block's valid range) with both blocks' loads issued before
// the one branch — otherwise the compiler sinks the backward block's loads
// under the forward block's test, two LDS round trips per step.
template <uint32_t FW = kFwd, uint32_t BW = kBwd, int MAXS = 0, bool SEL = false>
__device__ __forceinline__ int find_parent_bidir(const uint64_t* lsid, uint32_t a, uint32_t b,
                                                 uint32_t i, uint64_t pid) {
  int steps = 0;
  // FW: the staging slack; BW < 32: the mask form shifts 1u by up to BW
  static_assert(FW % 2 == 0 && BW % 2 == 0 && FW <= kScanSlack && BW < 32, "bidirectional step");
  uint32_t f = a;             // next forward block [f, f + FW)
  int32_t g = (int32_t)i - 1;  // backward blocks end at g (inclusive)
  while (true) {
    // backward block [gb, gb + BW) clamped to start at the trace start
    const int32_t gb0 = g - (int32_t)BW + 1;
    const uint32_t gb = gb0 < (int32_t)a ? a : (uint32_t)gb0;
    uint64_t v[FW], w[BW];
#pragma unroll
    for (uint32_t j = 0; j < FW; ++j) v[j] = lsid[f + j];
#pragma unroll
    for (uint32_t j = 0; j < BW; ++j) w[j] = lsid[gb + j];
    if constexpr (SEL) {
    uint32_t qf = FW, qb = BW;
#pragma unroll
    for (int j = (int)FW - 1; j >= 0; --j) qf = v[j] == pid ? (uint32_t)j : qf;
#pragma unroll
    for (int j = (int)BW - 1; j >= 0; --j) qb = w[j] == pid ? (uint32_t)j : qb;
    const uint32_t hi = (b - f) < FW ? (b - f) : FW;  // >= 1 while f < b
    const int32_t nb = g - (int32_t)gb + 1;
    const bool okf = qf < hi, okb = (int32_t)qb < nb;
    if (okf || okb) return (int)(okf ? f + qf : gb + qb);
    } else {
    uint32_t mf = 0, mb = 0;
#pragma unroll
    for (uint32_t j = 0; j < FW; ++j) mf |= (v[j] == pid ? 1u : 0u) << j;
#pragma unroll
    for (uint32_t j = 0; j < BW; ++j) mb |= (w[j] == pid ? 1u : 0u) << j;
    const uint32_t hi = (b - f) < FW ? (b - f) : FW;  // >= 1 while f < b
    mf &= (1u << hi) - 1u;
    // backward lanes past g (the clamp re-reads) or with g < a hold nothing new
    const int32_t nb = g - (int32_t)gb + 1;
    mb &= nb > 0 ? (1u << (uint32_t)nb) - 1u : 0u;
    if (mf) return (int)(f + __ffs(mf) - 1u);
    if (mb) return (int)(gb + 31u - __clz(mb));  // unique ids: any match is the match
    }
    f += FW;
    g -= (int32_t)BW;
    if (f >= b) return -1;
    if (MAXS > 0 && ++steps >= MAXS) return -2;
  }
}

// find_parent_bidir<SEL> over ids staged as two u32 planes (lo[], hi[]): the
// steps compare low words only (half the LDS bytes, 32-bit compares), and a
// low-word candidate is confirmed on its high word; a false candidate (two ids
// of the trace sharing a low word) finishes with an exact forward scan of the
// trace.  Unique ids: any confirmed match is the match.
template <uint32_t FW, uint32_t BW>
__device__ __forceinline__ int find_parent_split(const uint32_t* lo, const uint32_t* hi, uint32_t a,
                                                 uint32_t b, uint32_t i, uint64_t pid) {
  static_assert(FW <= kScanSlack && BW < 32, "split-word step: the staging slack");
  const uint32_t plo = (uint32_t)pid, phi = (uint32_t)(pid >> 32);
  uint32_t f = a;
  int32_t g = (int32_t)i - 1;
  while (true) {
    const int32_t gb0 = g - (int32_t)BW + 1;
    const uint32_t gb = gb0 < (int32_t)a ? a : (uint32_t)gb0;
    uint32_t v[FW], w[BW];
#pragma unroll
    for (uint32_t j = 0; j < FW; ++j) v[j] = lo[f + j];
#pragma unroll
    for (uint32_t j = 0; j < BW; ++j) w[j] = lo[gb + j];
    uint32_t qf = FW, qb = BW;
#pragma unroll
    for (int j = (int)FW - 1; j >= 0; --j) qf = v[j] == plo ? (uint32_t)j : qf;
#pragma unroll
    for (int j = (int)BW - 1; j >= 0; --j) qb = w[j] == plo ? (uint32_t)j : qb;
    const uint32_t hf = (b - f) < FW ? (b - f) : FW;
    const int32_t nb = g - (int32_t)gb + 1;
    const bool okf = qf < hf, okb = (int32_t)qb < nb;
    if (okf || okb) {
      const uint32_t q = okf ? f + qf : gb + qb;
      if (hi[q] == phi) return (int)q;
      for (uint32_t k = a; k < b; ++k)  // a low-word alias: exact scan
        if (lo[k] == plo && hi[k] == phi) return (int)k;
      return -1;
    }
    f += FW;
    g -= (int32_t)BW;
    if (f >= b) return -1;
  }
}

// The first span of [a_j, b_j) whose id is pid_j for each lane j of `pend`
// (wave-uniform mask), the whole wave scanning 64 ids per step with a ballot:
// the lookups the per-lane scans left after their first steps (a row would
// otherwise wait for its slowest lane).  First match in trace order.
__device__ __forceinline__ void coop_parent(const uint64_t* lsid, uint64_t pend, int lane,
                                            uint64_t pid, uint32_t a, uint32_t b, int& q) {
  while (pend) {
    const int j = __ffsll((unsigned long long)pend) - 1;
    const uint64_t pj = readlane64(pid, j);
    const uint32_t aj = (uint32_t)__builtin_amdgcn_readlane((int)a, j);
    const uint32_t bj = (uint32_t)__builtin_amdgcn_readlane((int)b, j);
    int qj = -1;
    for (uint32_t s0 = aj; s0 < bj; s0 += kWave) {
      const uint32_t sp = s0 + (uint32_t)lane;
      const uint64_t hit = __ballot(sp < bj && lsid[sp < bj ? sp : aj] == pj);
      if (hit) {
        qj = (int)(s0 + (uint32_t)__ffsll((unsigned long long)hit) - 1u);
        break;
      }
    }
    if (lane == j) q = qj;
    pend &= pend - 1ull;
  }
}

}  // namespace chunk
}  // namespace
}  // namespace anomod
