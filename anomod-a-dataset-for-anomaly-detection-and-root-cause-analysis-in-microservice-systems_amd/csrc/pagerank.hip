// Personalized PageRank root-cause ranking (build-defined,
// the reference ranks nothing).  Convention = networkx 3.4.2
// pagerank/_pagerank_scipy: row-normalised weights, x0 = 1/N, dangling mass
// redistributed along the personalization vector, L1 stopping rule N*tol.
//
// GPU form: pull SpMV over the in-edge CSR (transpose of the caller ->
// callee graph, weights pre-divided by the caller's out-weight), one lane per
// row with the row's in-edge loads batched 8 at a time (no grid-stride
// passes; every row in flight in one round).  One launch per iteration: each block adds its share of the new
// vector's dangling mass and of |x_new - x_old| (the stopping test) to 64-bit
// fixed-point accumulators with integer atomics (order-free, so the result is
// bit-reproducible), and the next launch reads one scalar.  The
// fixed-iteration loop is captured once into a hipGraph and replayed; a
// tolerance-mode solve whose blocks all fit on the chip at once runs as one
// cooperative launch with a grid barrier per iteration and the stopping test
// on the device.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.h"
#include "synth.h"

struct anomod_graph {
  int device = 0;
  uint32_t N = 0;
  uint64_t nnz = 0;
  uint32_t grid = 0;
  uint32_t* in_ptr = nullptr;  // [N+1]
  uint32_t* in_col = nullptr;  // [nnz]
  float* in_w = nullptr;       // [nnz] w / outweight(src)
  uint8_t* dangling = nullptr; // [N]
  double* p = nullptr;         // [N]
  uint32_t n_dangling = 0;
  double* x[2] = {nullptr, nullptr};
  uint64_t x_cap = 0;          // doubles per x buffer (>= N; row-sharded solves pad)
  // Fixed-point accumulators, kAccSlots-way spread, triple-buffered by
  // iteration (k reads buffer k%3, adds into (k+1)%3, zeroes (k+2)%3):
  // buffers 0..2 dangling mass (2^-62 units), 3..5 L1 change (2^-61 units).
  unsigned long long* acc = nullptr;
  std::vector<unsigned long long> host_acc;
  // batched solves (anomod_graph_pagerank_batch): node-major [N][Kb] vectors
  uint32_t kb = 0;                  // allocated batch width
  double* bp = nullptr;             // [N][kb] personalizations
  double* bx[2] = {nullptr, nullptr};
  unsigned long long* bacc = nullptr;  // [6][kb][kAccSlots]
  std::vector<unsigned long long> host_bacc;
  // persistent solve: [0] barrier arrivals, [1] timeout flag, [2] iterations done
  unsigned int* bar = nullptr;
  int coop_blocks = -1;  // co-resident workgroups of the persistent kernel (-1: not queried)
  int coop_sub = 0;      // its 256-row blocks per workgroup
  int bcoop_blocks = -1; // the same for the persistent batch kernel of width bcoop_kb
  uint32_t bcoop_kb = 0;
  bool bcoop_ring = false;
  uint32_t bcoop_sub = 0;
  uint32_t last_path = 0;   // ANOMOD_PPR_PATH_* of the last single-vector solve
  uint32_t fallbacks = 0;   // persistent solves rerun per launch (barrier timed out)
  double* h_pin = nullptr;  // pinned [N] staging of p in / x out (single-vector solve)
  double* h_bpin = nullptr;  // pinned [N][kb] staging of a batch's P in / X out
  uint64_t h_bpin_n = 0;
  // persistent solve: one fresh vector per iteration (see ppr_persistent_kernel)
  double* ring = nullptr;
  uint64_t ring_bytes = 0;  // bytes the ring holds (single solves and batches share it)
  // cached fixed-iteration graph
  hipGraphExec_t exec = nullptr;
  uint32_t exec_iters = 0;
  double exec_alpha = 0.0;
};

namespace anomod {
namespace {

constexpr int kPprThreads = 256;
constexpr int kRowsPerBlock = kPprThreads;  // one row per lane
#ifndef ANOMOD_PPR_EBATCH
#define ANOMOD_PPR_EBATCH 8
#endif
constexpr int kEdgeBatch = ANOMOD_PPR_EBATCH;  // in-edge loads issued together per lane
constexpr double kDScale = 4611686018427387904.0;  // 2^62: dangling mass <= 1
constexpr double kEScale = 2305843009213693952.0;  // 2^61: L1 change <= 2
constexpr int kAccSlots = 64;  // atomics spread over 64 words: no single-address queue

// Block-wide sum, fixed reduction tree (deterministic); result valid in thread 0.
__device__ __forceinline__ double block_sum(double v, double* red) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  __syncthreads();
  return s;
}

// Two block sums in one pass (two barriers instead of four), each with
// block_sum's reduction tree, so the results are block_sum's bit for bit.
// `red` holds 2 * waves doubles.  Results valid in thread 0.
__device__ __forceinline__ void block_sum2(double a, double b, double* red, double& sa,
                                           double& sb) {
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off);
    b += __shfl_xor(b, off);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (int)(blockDim.x >> 6);
  if (lane == 0) {
    red[wid] = a;
    red[nw + wid] = b;
  }
  __syncthreads();
  sa = 0.0;
  sb = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < nw; ++w) {
      sa += red[w];
      sb += red[nw + w];
    }
  __syncthreads();
}

// The per-row arithmetic, spelled out (explicit fma, no contraction left to
// the compiler) so every kernel — per-launch, persistent, batched — rounds
// identically and their vectors agree bit for bit.
__device__ __forceinline__ double ppr_edge(double acc, double x, float w) {
  return fma(x, (double)w, acc);
}
__device__ __forceinline__ double ppr_row(double alpha, double sum, double dsum, double pr) {
  return fma(alpha, fma(dsum, pr, sum), (1.0 - alpha) * pr);
}

__global__ __launch_bounds__(kPprThreads) void ppr_init_kernel(uint32_t N, double x0,
                                                               double* __restrict__ x) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x)
    x[i] = x0;
}

// x = x0 everywhere and p /= psum in place (the same IEEE division the host
// did before: identical bits); also seeds the accumulator slots (acc[0] =
// acc0, the rest zero) and clears the grid-barrier words, so a solve issues
// no host->device copy or memset besides p itself.
__global__ __launch_bounds__(kPprThreads) void ppr_init_norm_kernel(
    uint32_t N, double x0, double* __restrict__ x, double* __restrict__ p, double psum,
    unsigned long long* __restrict__ acc, uint32_t n_acc, unsigned long long acc0,
    unsigned int* __restrict__ bar, uint32_t n_bar) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t i = gid; i < n_acc; i += gridDim.x * blockDim.x) acc[i] = i == 0 ? acc0 : 0ull;
  for (uint32_t i = gid; i < n_bar; i += gridDim.x * blockDim.x) bar[i] = 0u;
  for (uint32_t i = gid; i < N; i += gridDim.x * blockDim.x) {
    x[i] = x0;
    p[i] = p[i] / psum;
  }
}

// One power iteration x_in -> x_out for the block's rows (the body of both
// the per-launch and the persistent kernel).  One lane per row pulls the
// in-edges.  The block's share of the new vector's dangling mass and of
// |x_out - x_in| is rounded to 64-bit fixed point and added with one integer
// atomic each: integer adds commute, so the next iteration reads a
// bit-reproducible scalar without a reduction kernel or an inter-block
// hand-off.  Block 0 zeroes the slots the iteration after next adds into.
__device__ __forceinline__ void ppr_iter_body(
    uint32_t N, const uint32_t* __restrict__ in_ptr, const uint32_t* __restrict__ in_col,
    const float* __restrict__ in_w, const uint8_t* __restrict__ dangling,
    const double* __restrict__ p, double alpha, const double* __restrict__ x_in,
    double* __restrict__ x_out, const unsigned long long* __restrict__ d_in,
    unsigned long long* d_out, unsigned long long* d_zero, unsigned long long* e_out,
    unsigned long long* e_zero, double* red, double* s_dsum, uint32_t block0 = 0) {
  const uint32_t gb = block0 + blockIdx.x;  // global row block (row shards start at one)
  const uint32_t r = gb * kRowsPerBlock + threadIdx.x;
  // The row's own operands do not depend on the SpMV: issue them first so
  // their latency overlaps the CSR chain (in_ptr -> in_col/in_w -> x gathers).
  double pr = 0.0, xr = 0.0;
  bool dg = false;
  if (r < N) {
    pr = p[r];
    xr = x_in[r];
    dg = dangling[r] != 0;
  }
  double acc = 0.0;
  if (r < N) {
    const uint32_t b = in_ptr[r], e = in_ptr[r + 1];
    // In-degrees are short (uniform callees): one lane per row, kEdgeBatch
    // (col, w) pairs loaded together, then the x gathers together (lanes past
    // the row's end gather their own row's x with weight 0: adds +0.0, the
    // same bits as skipping them; padding with x[0] sent every padded load of
    // the grid to one address).
    for (uint32_t k0 = b; k0 < e; k0 += kEdgeBatch) {
      uint32_t c[kEdgeBatch];
      float wv[kEdgeBatch];
#pragma unroll
      for (int j = 0; j < kEdgeBatch; ++j) {
        const bool ok = k0 + j < e;
        c[j] = ok ? in_col[k0 + j] : r;  // padding: the row's own x (weight 0)
        wv[j] = ok ? in_w[k0 + j] : 0.f;
      }
      double xv[kEdgeBatch];
#pragma unroll
      for (int j = 0; j < kEdgeBatch; ++j) xv[j] = x_in[c[j]];
#pragma unroll
      for (int j = 0; j < kEdgeBatch; ++j)
        if (k0 + j < e) acc = ppr_edge(acc, xv[j], wv[j]);
    }
  }
  // Dangling mass of x_in: wave 0 folds the fixed-point slots (exact).
  if (threadIdx.x < 64) {
    unsigned long long v = d_in[threadIdx.x];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (threadIdx.x == 0) *s_dsum = (double)v * (1.0 / kDScale);
  }
  __syncthreads();
  const double dsum = *s_dsum;
  double dacc = 0.0, eacc = 0.0;
  if (r < N) {
    const double y = ppr_row(alpha, acc, dsum, pr);
    x_out[r] = y;
    if (dg) dacc = y;
    eacc = fabs(y - xr);
  }
  double ds, es;
  block_sum2(dacc, eacc, red, ds, es);
  if (threadIdx.x == 0) {
    const int slot = gb & (kAccSlots - 1);
    atomicAdd(&d_out[slot], __double2ull_rn(ds * kDScale));
    atomicAdd(&e_out[slot], __double2ull_rn(es * kEScale));
  }
  if (blockIdx.x == 0 && threadIdx.x < kAccSlots) {  // the launch's first block
    d_zero[threadIdx.x] = 0ull;
    e_zero[threadIdx.x] = 0ull;
  }
}

__global__ __launch_bounds__(kPprThreads) void ppr_iter_kernel(
    uint32_t N, const uint32_t* __restrict__ in_ptr, const uint32_t* __restrict__ in_col,
    const float* __restrict__ in_w, const uint8_t* __restrict__ dangling,
    const double* __restrict__ p, double alpha, const double* __restrict__ x_in,
    double* __restrict__ x_out, const unsigned long long* __restrict__ d_in,
    unsigned long long* d_out, unsigned long long* d_zero, unsigned long long* e_out,
    unsigned long long* e_zero, uint32_t block0) {
  __shared__ double red[2 * (kPprThreads / 64)];
  __shared__ double s_dsum;
  ppr_iter_body(N, in_ptr, in_col, in_w, dangling, p, alpha, x_in, x_out, d_in, d_out, d_zero,
                e_out, e_zero, red, &s_dsum, block0);
}

// Grid-wide barrier of a cooperative launch.  Two-level arrival so no
// address sees more than ~50 atomics: block b adds to the counter of group
// b % 8 (one 128-B line each); the group's last arriver adds to the top
// counter, which every block polls.  Counters are monotonic (target =
// arrivals x barriers passed).
// Bounded: a wait past ~2^22 polls (ANOMOD_PPR_SPIN overrides: a test knob
// that forces the timeout) raises the flag and every block leaves; the host
// then reruns the solve through the per-launch path.
constexpr uint32_t kSpinLimit = 1u << 22;
#ifndef ANOMOD_PPR_FLATPOLL
#define ANOMOD_PPR_FLATPOLL 0
#endif
constexpr int kBarGroups = 8;  // 16 / 32 groups measured slower
constexpr int kBarStride = 32;  // u32 words between counters (128 B)
// ANOMOD_PPR_REPL copies of the top counter (0: one, bar[0]); block b polls copy
// b mod ANOMOD_PPR_REPL
#ifndef ANOMOD_PPR_REPL
#define ANOMOD_PPR_REPL 8
#endif
#ifndef ANOMOD_PPR_SLEEP
#define ANOMOD_PPR_SLEEP 1
#endif
constexpr int kBarCopies = ANOMOD_PPR_REPL;
static_assert(kBarCopies >= 0 && kBarCopies <= 64, "top-counter copies");
// bar[0] top counter, bar[1] timeout flag, bar[2] iterations done,
// bar[kBarStride * (1 + g)] group counters, bar[kBarStride * (1 + kBarGroups + c)]
// copy c of the top counter
constexpr int kBarWords = kBarStride * (1 + kBarGroups + kBarCopies);

__device__ __forceinline__ bool grid_barrier(unsigned int* bar, uint32_t k, int* s_flag,
                                             uint32_t spin_limit) {
  // Every wave drains its own stores (x written with agent-scope atomic
  // stores, i.e. through to the coherent level) before the workgroup meets;
  // no L2 write-back / invalidate is needed because every cross-block datum
  // (x, accumulator slots, counters) is accessed with agent-scope atomics.
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
#if ANOMOD_PPR_FLATPOLL
  // Flat poll: each block adds to its group counter (no return awaited) and
  // lanes 0..ng-1 of wave 0 poll the ng group counters together — no
  // second (top-counter) atomic round trip on the critical path.
  if (threadIdx.x < 64) {
    const uint32_t lane = threadIdx.x;
    const uint32_t nb = gridDim.x;
    const uint32_t ng = nb < (uint32_t)kBarGroups ? nb : (uint32_t)kBarGroups;
    if (lane == 0)
      __hip_atomic_fetch_add(&bar[kBarStride * (1 + blockIdx.x % ng)], 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t gl = lane < ng ? lane : 0u;
    const uint32_t target = ((nb - gl + ng - 1) / ng) * (k + 1u);  // group gl's arrivals
    uint32_t spins = 0;
    int fail = 0;
    while (true) {
      const uint32_t v = lane < ng ? __hip_atomic_load(&bar[kBarStride * (1 + gl)], __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                                   : 0xFFFFFFFFu;
      if (__ballot(v < target) == 0ull) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > spin_limit) {
        if (lane == 0) atomicOr(&bar[1], 1u);
        fail = 1;
        break;
      }
      if ((spins & 1023u) == 0u &&
          __hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        fail = 1;
        break;
      }
    }
    if (lane == 0) *s_flag = fail;
  }
  __syncthreads();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  return *s_flag == 0;
#endif
  if (threadIdx.x == 0) {
    const uint32_t nb = gridDim.x;
    const uint32_t ng = nb < (uint32_t)kBarGroups ? nb : (uint32_t)kBarGroups;
    const uint32_t g = blockIdx.x % ng;
    const uint32_t gsize = (nb - g + ng - 1) / ng;  // blocks with index = g (mod ng)
    const uint32_t old = __hip_atomic_fetch_add(&bar[kBarStride * (1 + g)], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
#if ANOMOD_PPR_REPL
    // the group's last arriver bumps every copy of the top counter and each
    // block polls one copy: a line takes ~1/kBarCopies of the polls (one
    // polled line: 8.3 vs 7.9 us per iteration at N = 1e5)
    if (old + 1u == gsize * (k + 1u))
      for (uint32_t j = 0; j < (uint32_t)kBarCopies; ++j)
        __hip_atomic_fetch_add(&bar[kBarStride * (1 + kBarGroups + j)], 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    unsigned int* const top = &bar[kBarStride * (1 + kBarGroups + blockIdx.x % kBarCopies)];
#else
    if (old + 1u == gsize * (k + 1u))
      __hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned int* const top = &bar[0];
#endif
    const uint32_t target = ng * (k + 1u);
    uint32_t spins = 0;
    int fail = 0;
    while (__hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (ANOMOD_PPR_SLEEP) __builtin_amdgcn_s_sleep(ANOMOD_PPR_SLEEP);
      if (++spins > spin_limit) {
        atomicOr(&bar[1], 1u);
        fail = 1;
        break;
      }
      if ((spins & 1023u) == 0u &&
          __hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        fail = 1;
        break;
      }
    }
    *s_flag = fail;
  }
  __syncthreads();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  return *s_flag == 0;
}

// All iterations in one cooperative launch (every block resident).  The
// block's in-edges (col, w) are staged in LDS once (up to kLdsEdges; the
// rest stay in HBM), row bounds / p / dangling / the row's previous value stay
// in registers, so an iteration's only global reads are the x gathers and the
// 64 accumulator slots.  Per row and per block the arithmetic, the edge order,
// the block partition and the fixed-point slots are those of
// ppr_iter_kernel, so the vector is bit-identical to the per-launch path; in
// tolerance mode every block reads the same L1 slots after the barrier and
// stops at the same iteration.  bar[2] receives the iterations done.
// A workgroup holds SUB consecutive 256-row blocks (SUB * 256 threads): the
// rows, the edge order, the 256-row fixed-point partials and their slots are
// the per-launch kernel's whatever SUB, only the number of workgroups meeting
// at the grid barrier shrinks (391 -> 98 at N = 10^5 with SUB = 4).
constexpr uint32_t kLdsEdgeBytes = 128 * 1024;  // (col, w) staging per workgroup
constexpr uint64_t kRingBytes = 4ull << 30;       // most HBM the per-iteration vectors take
// (4 GiB of 288: K = 16 at N = 10^5 takes 12.8 MB per iteration, 1.28 GB per
// 100-iteration solve; at 1 GiB it ran the two-buffer form, agent-scope loads)
#ifndef ANOMOD_PPR_GATHER
#define ANOMOD_PPR_GATHER 4
#endif
constexpr int kPBatch = ANOMOD_PPR_GATHER;  // x gathers in flight per lane (persistent kernel)
// Timing-only ablations of the persistent kernel (never set in the shipped
// library): 1 = no x gathers (the SpMV sum is 0), 2 = no grid barrier (a
// workgroup barrier only; wrong results), 3 = both.
#ifndef ANOMOD_PPR_ABL
#define ANOMOD_PPR_ABL 0
#endif

// RING: iteration `it` writes its vector to a slot of `ring` no load of this
// launch has touched before (slot it; iteration 0 reads x0, which an earlier
// launch wrote) and reads the previous one, so the x gathers can be PLAIN
// loads: a line of a fresh slot cannot be stale in any L1 or L2 (it was never
// cached there), the first gather of it misses to the coherent memory side,
// and later gathers of that line on the same XCD hit its L2 — against one
// agent-scope (sc1) load per gather that goes to the memory side every time.
// The owner's stores stay agent-scope and are drained before the grid
// barrier, as without the ring.
template <int SUB, bool RING>
__global__ __launch_bounds__(kPprThreads * SUB) void ppr_persistent_kernel(
    uint32_t N, const uint32_t* __restrict__ in_ptr, const uint32_t* __restrict__ in_col,
    const float* __restrict__ in_w, const uint8_t* __restrict__ dangling,
    const double* __restrict__ p, double alpha, double x0v, double* x0, double* x1,
    unsigned long long* acc, uint32_t iters, double ntol, unsigned int* bar, uint32_t spin_limit,
    double* ring, uint64_t slot) {
  constexpr uint32_t kLdsE = SUB == 1 ? 6144u : kLdsEdgeBytes / 8u;  // SUB 1: 48 KB, 3 per CU
  __shared__ uint32_t lcol[kLdsE];
  __shared__ float lw[kLdsE];
  __shared__ double red[2 * SUB * (kPprThreads / 64)];
  __shared__ double s_dsum;
  __shared__ int s_flag;
  __shared__ int s_stop;
  constexpr int S = kAccSlots;
  const uint32_t sub = threadIdx.x / kPprThreads, lt = threadIdx.x % kPprThreads;
  const uint32_t gb = blockIdx.x * SUB + sub;  // the 256-row block of this thread
  const uint32_t r = gb * kRowsPerBlock + lt;
  const uint32_t r0 = blockIdx.x * SUB * kRowsPerBlock;
  const uint32_t r0e = r0 < N ? r0 : N;
  const uint32_t r1 = r0 + SUB * kRowsPerBlock < N ? r0 + SUB * kRowsPerBlock : N;
  const uint32_t e0 = in_ptr[r0e], e1 = in_ptr[r1];
  const uint32_t nc = e1 - e0 < kLdsE ? e1 - e0 : kLdsE;
  for (uint32_t i = threadIdx.x; i < nc; i += kPprThreads * SUB) {
    lcol[i] = in_col[e0 + i];
    lw[i] = in_w[e0 + i];
  }
  uint32_t rb = 0, re = 0;
  double pr = 0.0, xr = x0v;
  bool dg = false;
  if (r < N) {
    rb = in_ptr[r];
    re = in_ptr[r + 1];
    pr = p[r];
    dg = dangling[r] != 0;
  }
  __syncthreads();
  uint32_t done = iters;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (uint32_t it = 0; it < iters; ++it) {
    const bool odd = it & 1u;
    const double* x_in = RING ? (it == 0 ? x0 : ring + (uint64_t)(it - 1u) * slot) : odd ? x1 : x0;
    double* x_out = RING ? ring + (uint64_t)it * slot : odd ? x0 : x1;
    const int rr = it % 3, w = (it + 1) % 3, z = (it + 2) % 3;
    // wave 0 first issues the reads of the previous iteration's slots — its
    // dangling mass and (tolerance mode) its L1 change, whose stopping test
    // is taken here rather than after the barrier — so they overlap the
    // gathers
    unsigned long long dv = 0, ev = 0;
    const bool check = ntol > 0.0 && it > 0;
    if (threadIdx.x < 64) {
      dv = __hip_atomic_load(&acc[rr * S + threadIdx.x], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      if (check)
        ev = __hip_atomic_load(&acc[(3 + rr) * S + threadIdx.x], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    double sum = 0.0;
    if (!(ANOMOD_PPR_ABL & 1) && r < N) {
      // kPBatch gathers in flight per lane (in-degrees ~ Poisson(7) here: one
      // round for nearly every row); lanes past the row's end gather their own
      // row's x with weight 0 (adds +0.0: the same bits as skipping them)
      for (uint32_t k0 = rb; k0 < re; k0 += kPBatch) {
        uint32_t c[kPBatch];
        float wv[kPBatch];
#pragma unroll
        for (int j = 0; j < kPBatch; ++j) {
          const uint32_t k = k0 + j, li = k - e0;
          const bool ok = k < re;
          c[j] = !ok ? r : li < nc ? lcol[li] : in_col[k];
          wv[j] = !ok ? 0.f : li < nc ? lw[li] : in_w[k];
        }
        double xv[kPBatch];
#pragma unroll
        for (int j = 0; j < kPBatch; ++j)
          xv[j] = RING ? x_in[c[j]]
                       : __hip_atomic_load(&x_in[c[j]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int j = 0; j < kPBatch; ++j)
          if (k0 + j < re) sum = ppr_edge(sum, xv[j], wv[j]);
      }
    }
    if (threadIdx.x < 64) {
      for (int off = 32; off > 0; off >>= 1) {
        dv += __shfl_xor(dv, off);
        ev += __shfl_xor(ev, off);
      }
      if (threadIdx.x == 0) {
        s_dsum = (double)dv * (1.0 / kDScale);
        s_stop = check && (double)ev * (1.0 / kEScale) < ntol;
      }
    }
    __syncthreads();
    if (s_stop) {  // iteration it-1 converged: x after `it` iterations stands
      done = it;
      break;
    }
    const double dsum = s_dsum;
    double dacc = 0.0, eacc = 0.0;
    if (r < N) {
      const double y = ppr_row(alpha, sum, dsum, pr);
      __hip_atomic_store(&x_out[r], y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (dg) dacc = y;
      eacc = fabs(y - xr);
      xr = y;
    }
    // per 256-row block: block_sum2's reduction tree (wave xor, then the
    // block's 4 wave partials in order)
    for (int off = 32; off > 0; off >>= 1) {
      dacc += __shfl_xor(dacc, off);
      eacc += __shfl_xor(eacc, off);
    }
    constexpr int nw = kPprThreads / 64;
    if (lane == 0) {
      red[2 * nw * sub + (wid % nw)] = dacc;
      red[2 * nw * sub + nw + (wid % nw)] = eacc;
    }
    __syncthreads();
    if (lt == 0) {
      double ds = 0.0, es = 0.0;
      for (int k = 0; k < nw; ++k) {
        ds += red[2 * nw * sub + k];
        es += red[2 * nw * sub + nw + k];
      }
      const int slot = gb & (kAccSlots - 1);
      atomicAdd(&acc[w * S + slot], __double2ull_rn(ds * kDScale));
      atomicAdd(&acc[(3 + w) * S + slot], __double2ull_rn(es * kEScale));
    }
    if (blockIdx.x == 0 && threadIdx.x < kAccSlots) {
      __hip_atomic_store(&acc[z * S + threadIdx.x], 0ull, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&acc[(3 + z) * S + threadIdx.x], 0ull, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr ((ANOMOD_PPR_ABL & 2) != 0) {
      __syncthreads();
    } else if (!grid_barrier(bar, it, &s_flag, spin_limit)) {
      done = it;
      break;
    }
  }
  // Every row's final value (xr: the last vector this block computed, or x0
  // when none) lands in x0, so the host copies one buffer without first
  // reading `done` back.  Safe: every block leaves the loop at the same
  // iteration, and a block still gathering for an abandoned iteration
  // discards what it reads.
  if (r < N) __hip_atomic_store(&x0[r], xr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (blockIdx.x == 0 && threadIdx.x == 0) bar[2] = done;
}

// K personalization vectors per launch (replica mode, SURVEY.md §8e: one
// vector per experiment or fault hypothesis): the in-edge CSR is read once
// for all K, x is node-major [N][K] so an edge gathers K contiguous doubles.
// Per vector the arithmetic, the block partition and the reduction order are
// those of ppr_iter_kernel, so each column equals its single-vector solve
// bit for bit.  Vectors whose bit is set in `frozen` (converged in tolerance
// mode) are carried unchanged.
template <int K>
__global__ __launch_bounds__(kPprThreads) void ppr_batch_iter_kernel(
    uint32_t N, const uint32_t* __restrict__ in_ptr, const uint32_t* __restrict__ in_col,
    const float* __restrict__ in_w, const uint8_t* __restrict__ dangling,
    const double* __restrict__ p, double alpha, const double* __restrict__ x_in,
    double* __restrict__ x_out, const unsigned long long* __restrict__ d_in,
    unsigned long long* d_out, unsigned long long* d_zero, unsigned long long* e_out,
    unsigned long long* e_zero, uint32_t frozen) {
  __shared__ double red[kPprThreads / 64];
  __shared__ double s_dsum[K];
  const uint32_t r = blockIdx.x * kRowsPerBlock + threadIdx.x;
  double acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0.0;
  if (r < N) {
    const uint32_t b = in_ptr[r], e = in_ptr[r + 1];
    for (uint32_t k0 = b; k0 < e; k0 += kEdgeBatch) {
      uint32_t c[kEdgeBatch];
      float wv[kEdgeBatch];
#pragma unroll
      for (int j = 0; j < kEdgeBatch; ++j) {
        const bool ok = k0 + j < e;
        c[j] = ok ? in_col[k0 + j] : r;  // padding: the row's own x (weight 0)
        wv[j] = ok ? in_w[k0 + j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < kEdgeBatch; ++j) {
        if (k0 + j < e) {
          const double* xr = x_in + (uint64_t)c[j] * K;
#pragma unroll
          for (int k = 0; k < K; ++k) acc[k] = ppr_edge(acc[k], xr[k], wv[j]);
        }
      }
    }
  }
  // dangling mass of every vector of x_in (fixed-point slots, exact)
  for (int k = threadIdx.x >> 6; k < K; k += kPprThreads / 64) {
    unsigned long long v = d_in[k * kAccSlots + (threadIdx.x & 63)];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) s_dsum[k] = (double)v * (1.0 / kDScale);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double dacc = 0.0, eacc = 0.0;
    if (r < N) {
      const double pr = p[(uint64_t)r * K + k];
      const double xo = x_in[(uint64_t)r * K + k];
      const double y = (frozen >> k) & 1u ? xo
                                           : ppr_row(alpha, acc[k], s_dsum[k], pr);
      x_out[(uint64_t)r * K + k] = y;
      if (dangling[r]) dacc = y;
      eacc = fabs(y - xo);
    }
    const double ds = block_sum(dacc, red);
    const double es = block_sum(eacc, red);
    if (threadIdx.x == 0) {
      const int slot = k * kAccSlots + (blockIdx.x & (kAccSlots - 1));
      atomicAdd(&d_out[slot], __double2ull_rn(ds * kDScale));
      atomicAdd(&e_out[slot], __double2ull_rn(es * kEScale));
    }
  }
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < K * kAccSlots; i += kPprThreads) {
      d_zero[i] = 0ull;
      e_zero[i] = 0ull;
    }
}

// All iterations of a K-vector batch in one launch: ppr_persistent_kernel's
// grid barrier, LDS-staged in-edges and vector ring, with the per-vector
// arithmetic, edge order, 256-row block partition, reduction tree and
// fixed-point slots of ppr_batch_iter_kernel, so every column equals its
// per-launch batch (and single-vector) solve bit for bit.  Tolerance mode:
// every block reads iteration it-1's per-vector L1 changes at the top of
// iteration it, freezes the converged vectors (carried unchanged, as the
// host loop of the per-launch batch does) and stops once all are frozen.
// The final vectors land in x0 ([N][K], node-major); bar[2] = iterations.
// One 16-B store written through to the coherent level (`sc1`, what an
// agent-scope relaxed store compiles to, at 16 B: HIP has no 16-B atomic
// store).  Drained by grid_barrier's wait before the arrival.
using v4u32 = uint32_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store16_wt(void* p, v4u32 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
}

// SUB: a workgroup holds SUB consecutive 256-row blocks (SUB * 256 threads);
// each block keeps its rows, edge order, reduction tree and fixed-point slot,
// only the number of workgroups meeting at the grid barrier shrinks — K = 16
// (216 VGPRs) at SUB = 2 puts N = 10^5's 391 blocks in 196 resident workgroups.
template <int K, bool RING, int SUB = 1>
__global__ __launch_bounds__(kPprThreads * SUB) void ppr_batch_persistent_kernel(
    uint32_t N, const uint32_t* __restrict__ in_ptr, const uint32_t* __restrict__ in_col,
    const float* __restrict__ in_w, const uint8_t* __restrict__ dangling,
    const double* __restrict__ p, double alpha, double* x0, double* x1, unsigned long long* acc,
    uint32_t iters, double ntol, unsigned int* bar, uint32_t spin_limit, double* ring,
    uint64_t slot) {
  // 24 KB of (col, w) (~1 800 in-edges per 256-row block at N = 10^5; the
  // rest from global memory) + the store staging: three workgroups per CU
  // (the residency check admits per-CU occupancy minus one)
  constexpr uint32_t kLdsE = 3072u * SUB;
  constexpr int S = kAccSlots * K;   // one accumulator block: K x kAccSlots
  constexpr int kNW = kPprThreads / 64;  // waves per 256-row block
  constexpr int kWaves = kNW * SUB;
  __shared__ uint32_t lcol[kLdsE];
  __shared__ float lw[kLdsE];
  __shared__ double red[SUB * 2 * K * kNW];
  __shared__ double s_dsum[K];
  __shared__ v4u32 stg[kWaves * 64 * (K / 2 + 1)];  // per wave: 64 rows of K doubles (+ a pad piece)
  __shared__ uint32_t s_conv;
  __shared__ int s_flag;
  const uint32_t sub = threadIdx.x / kPprThreads, lt = threadIdx.x % kPprThreads;
  const uint32_t gb = blockIdx.x * SUB + sub;  // the 256-row block of this thread
  const uint32_t r = blockIdx.x * SUB * kRowsPerBlock + threadIdx.x;
  const uint32_t r0 = blockIdx.x * SUB * kRowsPerBlock;
  const uint32_t r0e = r0 < N ? r0 : N;
  const uint32_t r1 = r0 + SUB * kRowsPerBlock < N ? r0 + SUB * kRowsPerBlock : N;
  const uint32_t e0 = in_ptr[r0e], e1 = in_ptr[r1];
  const uint32_t nc = e1 - e0 < kLdsE ? e1 - e0 : kLdsE;
  for (uint32_t i = threadIdx.x; i < nc; i += kPprThreads * SUB) {
    lcol[i] = in_col[e0 + i];
    lw[i] = in_w[e0 + i];
  }
  uint32_t rb = 0, re = 0;
  double pr[K], xr[K];
  bool dg = false;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    pr[k] = 0.0;
    xr[k] = 0.0;
  }
  if (r < N) {
    rb = in_ptr[r];
    re = in_ptr[r + 1];
    dg = dangling[r] != 0;
    // x0 = 1/N everywhere (the host fills it so): the row's previous value
    // without a plain load of a buffer later iterations rewrite
    const double x0v = 1.0 / (double)N;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      pr[k] = p[(uint64_t)r * K + k];
      xr[k] = x0v;
    }
  }
  if (threadIdx.x == 0) s_conv = 0u;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t all = K >= 32 ? 0xFFFFFFFFu : ((1u << K) - 1u);
  uint32_t frozen = 0, done = iters;
  for (uint32_t it = 0; it < iters; ++it) {
    const bool odd = it & 1u;
    const double* x_in = RING ? (it == 0 ? x0 : ring + (uint64_t)(it - 1u) * slot) : odd ? x1 : x0;
    double* x_out = RING ? ring + (uint64_t)it * slot : odd ? x0 : x1;
    const int rr = it % 3, w = (it + 1) % 3, z = (it + 2) % 3;
    // the previous iteration's per-vector slots: dangling mass, and (tolerance
    // mode) L1 change -> the vectors converged by then
    const bool check = ntol > 0.0 && it > 0;
    for (int k = wid; k < K; k += kWaves) {
      unsigned long long dv = __hip_atomic_load(&acc[rr * S + k * kAccSlots + lane],
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned long long ev = check ? __hip_atomic_load(&acc[(3 + rr) * S + k * kAccSlots + lane],
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                    : 0ull;
      for (int off = 32; off > 0; off >>= 1) {
        dv += __shfl_xor(dv, off);
        ev += __shfl_xor(ev, off);
      }
      if (lane == 0) {
        s_dsum[k] = (double)dv * (1.0 / kDScale);
        if (check && (double)ev * (1.0 / kEScale) < ntol) atomicOr(&s_conv, 1u << k);
      }
    }
    double sum[K];
#pragma unroll
    for (int k = 0; k < K; ++k) sum[k] = 0.0;
    if (r < N) {
      for (uint32_t k0 = rb; k0 < re; k0 += kEdgeBatch) {
        uint32_t c[kEdgeBatch];
        float wv[kEdgeBatch];
#pragma unroll
        for (int j = 0; j < kEdgeBatch; ++j) {
          const uint32_t e = k0 + j, li = e - e0;
          const bool ok = e < re;
          c[j] = !ok ? r : li < nc ? lcol[li] : in_col[e];
          wv[j] = !ok ? 0.f : li < nc ? lw[li] : in_w[e];
        }
#pragma unroll
        for (int j = 0; j < kEdgeBatch; ++j) {
          if (k0 + j < re) {
            const double* xs = x_in + (uint64_t)c[j] * K;
            double xv[K];
            if constexpr (RING) {
#pragma unroll
              for (int k = 0; k < K; k += 2) {
                const double2 v2 = *reinterpret_cast<const double2*>(xs + k);
                xv[k] = v2.x;
                xv[k + 1] = v2.y;
              }
            } else {
#pragma unroll
              for (int k = 0; k < K; ++k)
                xv[k] = __hip_atomic_load(&xs[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int k = 0; k < K; ++k) sum[k] = ppr_edge(sum[k], xv[k], wv[j]);
          }
        }
      }
    }
    __syncthreads();
    frozen |= s_conv;
    if (check && (frozen & all) == all) {
      done = it;
      break;
    }
    double dacc[K], eacc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      dacc[k] = 0.0;
      eacc[k] = 0.0;
      if (r < N) {
        const double y = (frozen >> k) & 1u ? xr[k] : ppr_row(alpha, sum[k], s_dsum[k], pr[k]);
        if (dg) dacc[k] = y;
        eacc[k] = fabs(y - xr[k]);
        xr[k] = y;
      }
    }
    // The wave's 64 rows x K doubles, written through (16-B sc1 stores): lane
    // l stages its row in LDS, then every store instruction covers 1 KiB of
    // consecutive rows — 8-B stores per lane and value wrote each line in
    // eight partial pieces (4x the bytes at the fabric, PMC r04).
    {
      constexpr int Q = K / 2;  // 16-B pieces per row
      v4u32* st = stg + wid * (64 * (Q + 1));
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const uint64_t a0 = __double_as_longlong(xr[2 * q]), a1 = __double_as_longlong(xr[2 * q + 1]);
        st[lane * (Q + 1) + q] = v4u32{(uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a1,
                                      (uint32_t)(a1 >> 32)};
      }
      __builtin_amdgcn_wave_barrier();
      const uint32_t row0 = r - (uint32_t)lane;  // the wave's first row
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        const uint32_t i = (uint32_t)(j * 64 + lane), row = i / Q, q = i % Q;
        if (row0 + row < N)
          store16_wt(x_out + (uint64_t)(row0 + row) * K + 2 * q, st[row * (Q + 1) + q]);
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      for (int off = 32; off > 0; off >>= 1) {
        dacc[k] += __shfl_xor(dacc[k], off);
        eacc[k] += __shfl_xor(eacc[k], off);
      }
      if (lane == 0) {
        red[sub * 2 * K * kNW + (2 * k) * kNW + (wid % kNW)] = dacc[k];
        red[sub * 2 * K * kNW + (2 * k + 1) * kNW + (wid % kNW)] = eacc[k];
      }
    }
    __syncthreads();
    // block_sum's order: thread 0 of the per-launch kernel adds the 4 wave
    // partials from 0.0 in wave order; here thread k does it for vector k
    if (lt < (uint32_t)K) {
      const int k = (int)lt;
      double ds = 0.0, es = 0.0;
      for (int q = 0; q < kNW; ++q) {
        ds += red[sub * 2 * K * kNW + (2 * k) * kNW + q];
        es += red[sub * 2 * K * kNW + (2 * k + 1) * kNW + q];
      }
      const int sl = k * kAccSlots + (int)(gb & (kAccSlots - 1));
      atomicAdd(&acc[w * S + sl], __double2ull_rn(ds * kDScale));
      atomicAdd(&acc[(3 + w) * S + sl], __double2ull_rn(es * kEScale));
    }
    if (blockIdx.x == 0)
      for (int i = threadIdx.x; i < S; i += kPprThreads * SUB) {
        __hip_atomic_store(&acc[z * S + i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&acc[(3 + z) * S + i], 0ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    if (threadIdx.x == 0) s_conv = 0u;  // (read by every thread before the barrier above)
    if (!grid_barrier(bar, it, &s_flag, spin_limit)) {
      done = it;
      break;
    }
  }
  if (r < N)
#pragma unroll
    for (int k = 0; k < K; ++k)
      __hip_atomic_store(&x0[(uint64_t)r * K + k], xr[k], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  if (blockIdx.x == 0 && threadIdx.x == 0) bar[2] = done;
}

// K = 16 in halves: a workgroup holds two 256-row blocks and, for each, two
// halves of 256 lanes — lane (block, half, row) computes vectors 8 h .. 8 h + 7
// of its row, so a lane carries the K = 8 kernel's state (252 VGPRs at one
// row of 16 vectors per lane left two waves per SIMD).  The vector ring holds
// each slot as two node-major [N'][8] halves, so a half's gather is the K = 8
// kernel's 64-B row read; iteration 0 reads no vector at all (x0 = 1/N
// everywhere: the same double the per-launch path loads).  Per vector the
// edge order, the 256-row block partition, the wave reduction tree (a wave
// holds 64 consecutive rows of one half) and the fixed-point slots are those
// of ppr_batch_iter_kernel<16>, so every column is bit-equal to it; the final
// vectors land in x0 as [N][16].  RING only (the caller falls back to the
// SUB form without a ring).
constexpr int kSplitH = 8;  // vectors per half
#ifndef ANOMOD_PPR_SPLIT_BATCH
#define ANOMOD_PPR_SPLIT_BATCH 4
#endif
constexpr int kSplitBatch = ANOMOD_PPR_SPLIT_BATCH;  // in-edges gathered together per lane
__global__ __launch_bounds__(4 * kPprThreads) void ppr_batch_split_kernel(
    uint32_t N, const uint32_t* __restrict__ in_ptr, const uint32_t* __restrict__ in_col,
    const float* __restrict__ in_w, const uint8_t* __restrict__ dangling,
    const double* __restrict__ p, double alpha, double* x0, double* x1, unsigned long long* acc,
    uint32_t iters, double ntol, unsigned int* bar, uint32_t spin_limit, double* ring,
    uint64_t slot) {
  (void)x1;
  constexpr int K = 16, H = kSplitH, SUB = 2;
  constexpr uint32_t kLdsE = 3072u * SUB;
  constexpr int S = kAccSlots * K;
  constexpr int kNW = kPprThreads / 64;  // waves per 256-row block and half
  constexpr int kWaves = 4 * kNW;
  constexpr int Q = H / 2;               // 16-B pieces per half row
  __shared__ uint32_t lcol[kLdsE];
  __shared__ float lw[kLdsE];
  __shared__ double red[SUB * 2 * 2 * H * kNW];
  __shared__ double s_dsum[K];
  __shared__ v4u32 stg[kWaves * 64 * (Q + 1)];
  __shared__ uint32_t s_conv;
  __shared__ int s_flag;
  const uint32_t qq = threadIdx.x / kPprThreads, lt = threadIdx.x % kPprThreads;
  const uint32_t sub = qq >> 1, h = qq & 1u;
  const uint32_t gb = blockIdx.x * SUB + sub;  // the 256-row block of this lane
  const uint32_t r = gb * kRowsPerBlock + lt;
  const uint32_t r0 = blockIdx.x * SUB * kRowsPerBlock;
  const uint32_t r0e = r0 < N ? r0 : N;
  const uint32_t r1 = r0 + SUB * kRowsPerBlock < N ? r0 + SUB * kRowsPerBlock : N;
  const uint32_t e0 = in_ptr[r0e], e1 = in_ptr[r1];
  const uint32_t nc = e1 - e0 < kLdsE ? e1 - e0 : kLdsE;
  for (uint32_t i = threadIdx.x; i < nc; i += 4 * kPprThreads) {
    lcol[i] = in_col[e0 + i];
    lw[i] = in_w[e0 + i];
  }
  uint32_t rb = 0, re = 0;
  double xr[H];  // (the personalization is re-read per iteration: registers)
  bool dg = false;
  const double x0v = 1.0 / (double)N;
  const double* pr = p + (uint64_t)(r < N ? r : 0u) * K + h * H;
#pragma unroll
  for (int k = 0; k < H; ++k) xr[k] = 0.0;
  if (r < N) {
    rb = in_ptr[r];
    re = in_ptr[r + 1];
    dg = dangling[r] != 0;
#pragma unroll
    for (int k = 0; k < H; ++k) xr[k] = x0v;
  }
  if (threadIdx.x == 0) s_conv = 0u;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t hs = slot / 2;  // doubles per half of a ring slot
  uint32_t frozen = 0, done = iters;
  double* const red_me = red + (sub * 2 + h) * 2 * H * kNW;
  for (uint32_t it = 0; it < iters; ++it) {
    const double* x_in = it == 0 ? nullptr : ring + (uint64_t)(it - 1u) * slot + h * hs;
    double* x_out = ring + (uint64_t)it * slot + h * hs;
    const int rr = it % 3, w = (it + 1) % 3, z = (it + 2) % 3;
    const bool check = ntol > 0.0 && it > 0;
    {  // wave wid reads vector wid's slots of the previous iteration
      const int k = wid;
      unsigned long long dv = __hip_atomic_load(&acc[rr * S + k * kAccSlots + lane],
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned long long ev = check ? __hip_atomic_load(&acc[(3 + rr) * S + k * kAccSlots + lane],
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                    : 0ull;
      for (int off = 32; off > 0; off >>= 1) {
        dv += __shfl_xor(dv, off);
        ev += __shfl_xor(ev, off);
      }
      if (lane == 0) {
        s_dsum[k] = (double)dv * (1.0 / kDScale);
        if (check && (double)ev * (1.0 / kEScale) < ntol) atomicOr(&s_conv, 1u << k);
      }
    }
    double sum[H];
#pragma unroll
    for (int k = 0; k < H; ++k) sum[k] = 0.0;
    if (r < N) {
      for (uint32_t k0 = rb; k0 < re; k0 += kSplitBatch) {
        uint32_t c[kSplitBatch];
        float wv[kSplitBatch];
#pragma unroll
        for (int j = 0; j < kSplitBatch; ++j) {
          const uint32_t e = k0 + j, li = e - e0;
          const bool ok = e < re;
          c[j] = !ok ? r : li < nc ? lcol[li] : in_col[e];
          wv[j] = !ok ? 0.f : li < nc ? lw[li] : in_w[e];
        }
#pragma unroll
        for (int j = 0; j < kSplitBatch; ++j) {
          if (k0 + j < re) {
            double xv[H];
            if (x_in) {
              const double* xs = x_in + (uint64_t)c[j] * H;
#pragma unroll
              for (int k = 0; k < H; k += 2) {
                const double2 v2 = *reinterpret_cast<const double2*>(xs + k);
                xv[k] = v2.x;
                xv[k + 1] = v2.y;
              }
            } else {
#pragma unroll
              for (int k = 0; k < H; ++k) xv[k] = x0v;
            }
#pragma unroll
            for (int k = 0; k < H; ++k) sum[k] = ppr_edge(sum[k], xv[k], wv[j]);
          }
        }
      }
    }
    __syncthreads();
    frozen |= s_conv;
    if (check && (frozen & 0xFFFFu) == 0xFFFFu) {
      done = it;
      break;
    }
    // per vector: the new value, then at once its wave's reduction tree of
    // the dangling mass and the L1 change (no per-vector arrays kept live)
#pragma unroll
    for (int k = 0; k < H; ++k) {
      double dacc = 0.0, eacc = 0.0;
      if (r < N) {
        const uint32_t kk = h * H + (uint32_t)k;
        const double y = (frozen >> kk) & 1u ? xr[k] : ppr_row(alpha, sum[k], s_dsum[kk], pr[k]);
        if (dg) dacc = y;
        eacc = fabs(y - xr[k]);
        xr[k] = y;
      }
      for (int off = 32; off > 0; off >>= 1) {
        dacc += __shfl_xor(dacc, off);
        eacc += __shfl_xor(eacc, off);
      }
      if (lane == 0) {
        red_me[(2 * k) * kNW + (wid % kNW)] = dacc;
        red_me[(2 * k + 1) * kNW + (wid % kNW)] = eacc;
      }
    }
    {  // the wave's 64 half rows, written through as 1-KiB store instructions
      v4u32* st = stg + wid * (64 * (Q + 1));
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const uint64_t a0 = __double_as_longlong(xr[2 * q]), a1 = __double_as_longlong(xr[2 * q + 1]);
        st[lane * (Q + 1) + q] = v4u32{(uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a1,
                                      (uint32_t)(a1 >> 32)};
      }
      __builtin_amdgcn_wave_barrier();
      const uint32_t row0 = r - (uint32_t)lane;
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        const uint32_t i = (uint32_t)(j * 64 + lane), row = i / Q, q = i % Q;
        if (row0 + row < N)
          store16_wt(x_out + (uint64_t)(row0 + row) * H + 2 * q, st[row * (Q + 1) + q]);
      }
    }
    __syncthreads();
    if (lt < (uint32_t)H) {  // block_sum's order: the 4 wave partials from 0.0, in wave order
      const int k = (int)lt;
      double ds = 0.0, es = 0.0;
      for (int q = 0; q < kNW; ++q) {
        ds += red_me[(2 * k) * kNW + q];
        es += red_me[(2 * k + 1) * kNW + q];
      }
      const int sl = (int)(h * H + (uint32_t)k) * kAccSlots + (int)(gb & (kAccSlots - 1));
      atomicAdd(&acc[w * S + sl], __double2ull_rn(ds * kDScale));
      atomicAdd(&acc[(3 + w) * S + sl], __double2ull_rn(es * kEScale));
    }
    if (blockIdx.x == 0)
      for (int i = threadIdx.x; i < S; i += 4 * kPprThreads) {
        __hip_atomic_store(&acc[z * S + i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&acc[(3 + z) * S + i], 0ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    if (threadIdx.x == 0) s_conv = 0u;  // (read by every thread before the barrier above)
    if (!grid_barrier(bar, it, &s_flag, spin_limit)) {
      done = it;
      break;
    }
  }
  if (r < N)
#pragma unroll
    for (int k = 0; k < H; ++k)
      __hip_atomic_store(&x0[(uint64_t)r * K + h * H + k], xr[k], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  if (blockIdx.x == 0 && threadIdx.x == 0) bar[2] = done;
}

#ifndef ANOMOD_PPR_SUB
#define ANOMOD_PPR_SUB 1
#endif
constexpr int kPprSub = ANOMOD_PPR_SUB;  // 256-row blocks per persistent workgroup
using PersistentFn = void (*)(uint32_t, const uint32_t*, const uint32_t*, const float*,
                              const uint8_t*, const double*, double, double, double*, double*,
                              unsigned long long*, uint32_t, double, unsigned int*, uint32_t,
                              double*, uint64_t);
PersistentFn persistent_fn(int sub, bool ring) {
  if (ring)
    return sub >= 4 ? ppr_persistent_kernel<4, true> : sub == 2 ? ppr_persistent_kernel<2, true>
                                                                : ppr_persistent_kernel<1, true>;
  return sub >= 4 ? ppr_persistent_kernel<4, false> : sub == 2 ? ppr_persistent_kernel<2, false>
                                                               : ppr_persistent_kernel<1, false>;
}

// A batch's personalizations: raw [K][N] -> normalised node-major [N][kb]
// (padded vectors repeat vector 0), p / sum with the host's sum.
struct BatchNorm {
  double psum[16];
};
__global__ __launch_bounds__(kPprThreads) void ppr_batch_norm_kernel(const double* __restrict__ raw,
                                                                     uint32_t N, uint32_t K,
                                                                     uint32_t kb, BatchNorm bn,
                                                                     double* __restrict__ bp) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x)
    for (uint32_t k = 0; k < kb; ++k) {
      const uint32_t src = k < K ? k : 0u;
      bp[(uint64_t)i * kb + k] = raw[(uint64_t)src * N + i] / bn.psum[src];
    }
}
// node-major [N][kb] -> [K][N]
__global__ __launch_bounds__(kPprThreads) void ppr_batch_out_kernel(const double* __restrict__ x,
                                                                    uint32_t N, uint32_t K,
                                                                    uint32_t kb,
                                                                    double* __restrict__ out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x)
    for (uint32_t k = 0; k < K; ++k) out[(uint64_t)k * N + i] = x[(uint64_t)i * kb + k];
}

using BatchFn = void (*)(uint32_t, const uint32_t*, const uint32_t*, const float*, const uint8_t*,
                        const double*, double, double*, double*, unsigned long long*, uint32_t,
                        double, unsigned int*, uint32_t, double*, uint64_t);
// 256-row blocks per workgroup of the batched persistent solve: K = 16 takes
// 2 (216 VGPRs: one block per workgroup left N = 10^5's 391 blocks
// non-resident, the batch ran per launch); ANOMOD_PPR_BSUB overrides (1 / 2).
uint32_t batch_sub(uint32_t kb) {
  const char* e = getenv("ANOMOD_PPR_BSUB");
  if (e && *e) return atoi(e) >= 2 ? 2u : 1u;
  return kb >= 16 ? 2u : 1u;
}

BatchFn batch_persistent_fn(uint32_t kb, bool ring, uint32_t sub = 1) {
  if (sub >= 2) {
    if (ring)
      return kb == 2 ? ppr_batch_persistent_kernel<2, true, 2> : kb == 4 ? ppr_batch_persistent_kernel<4, true, 2>
           : kb == 8 ? ppr_batch_persistent_kernel<8, true, 2> : ppr_batch_persistent_kernel<16, true, 2>;
    return kb == 2 ? ppr_batch_persistent_kernel<2, false, 2> : kb == 4 ? ppr_batch_persistent_kernel<4, false, 2>
         : kb == 8 ? ppr_batch_persistent_kernel<8, false, 2> : ppr_batch_persistent_kernel<16, false, 2>;
  }
  if (ring)
    return kb == 2 ? ppr_batch_persistent_kernel<2, true> : kb == 4 ? ppr_batch_persistent_kernel<4, true>
         : kb == 8 ? ppr_batch_persistent_kernel<8, true> : ppr_batch_persistent_kernel<16, true>;
  return kb == 2 ? ppr_batch_persistent_kernel<2, false> : kb == 4 ? ppr_batch_persistent_kernel<4, false>
       : kb == 8 ? ppr_batch_persistent_kernel<8, false> : ppr_batch_persistent_kernel<16, false>;
}

// The batch result x ([N][kb] on the device) -> X ([K][N] on the host)
// through `tmp` (a free device vector buffer) and the pinned staging.
hipError_t batch_out(anomod_ctx* ctx, anomod_graph* g, const double* x, double* tmp, uint32_t N,
                     uint32_t K, uint32_t kb, double* X) {
  hipLaunchKernelGGL(ppr_batch_out_kernel, dim3(std::min<uint32_t>((N + kPprThreads - 1) / kPprThreads, 2048)),
                     dim3(kPprThreads), 0, ctx->stream, x, N, K, kb, tmp);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess)
    e = hipMemcpyAsync(g->h_bpin, tmp, (size_t)N * K * 8, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e == hipSuccess) memcpy(X, g->h_bpin, (size_t)N * K * 8);
  return e;
}

void free_graph(anomod_graph* g) {
  if (!g) return;
  (void)hipSetDevice(g->device);
  if (g->exec) (void)hipGraphExecDestroy(g->exec);
  if (g->h_pin) (void)hipHostFree(g->h_pin);
  if (g->h_bpin) (void)hipHostFree(g->h_bpin);
  void* ps[] = {g->in_ptr, g->in_col, g->in_w, g->dangling, g->p,    g->x[0], g->x[1],
                g->acc,    g->bp,     g->bx[0], g->bx[1],    g->bacc, g->bar, g->ring};
  for (void* q : ps)
    if (q) (void)hipFree(q);
  delete g;
}

// The per-iteration vector ring of the persistent solves, grown to `bytes`
// (false: no ring — the caller takes the two-buffer form).
bool ensure_ring(anomod_ctx* ctx, anomod_graph* g, uint64_t bytes) {
  (void)ctx;
  if (g->ring_bytes >= bytes) return true;
  if (g->ring) (void)hipFree(g->ring);
  g->ring = nullptr;
  g->ring_bytes = 0;
  if (hipMalloc(&g->ring, bytes) == hipSuccess) g->ring_bytes = bytes;
  (void)hipGetLastError();
  return g->ring != nullptr;
}

// Launch iteration `it` (x[it&1] -> x[(it+1)&1]) over row blocks
// [block0, block0 + nblocks) (default: all rows).
void launch_iter(anomod_ctx* ctx, anomod_graph* g, double alpha, uint32_t it, uint32_t block0 = 0,
                 uint32_t nblocks = 0) {
  const int a = it & 1, b = a ^ 1;
  const int r = it % 3, w = (it + 1) % 3, z = (it + 2) % 3;
  unsigned long long* A = g->acc;
  const int S = kAccSlots;
  hipLaunchKernelGGL(ppr_iter_kernel, dim3(nblocks ? nblocks : g->grid), dim3(kPprThreads), 0,
                     ctx->stream, g->N, g->in_ptr, g->in_col, g->in_w, g->dangling, g->p, alpha,
                     g->x[a], g->x[b], A + r * S, A + w * S, A + z * S, A + (3 + w) * S,
                     A + (3 + z) * S, block0);
}

// Row shards of the sharded solve: whole 256-row blocks, ceil(grid / G) per
// shard (the last may be short or empty), so every block's rows and its
// fixed-point partials are the unsharded solve's.
struct RowShard {
  uint32_t block0, nblocks, rows_per_shard;
};
RowShard row_shard(const anomod_graph* g, uint32_t G, uint32_t k) {
  const uint32_t per = (g->grid + G - 1) / G;
  const uint32_t b0 = std::min(g->grid, k * per);
  return {b0, std::min(g->grid, b0 + per) - b0, per * kRowsPerBlock};
}

// Size the x buffers for a G-way all-gather (G * rows_per_shard doubles).
int ensure_shard_x(anomod_ctx* ctx, anomod_graph* g, uint32_t G) {
  const uint64_t need = (uint64_t)row_shard(g, G, 0).rows_per_shard * G;
  if (need <= g->x_cap) return ANOMOD_OK;
  for (int i = 0; i < 2; ++i) {
    double* nx = nullptr;
    ANOMOD_HIP(ctx, hipMalloc(&nx, need * 8ull));
    ANOMOD_HIP(ctx, hipFree(g->x[i]));
    g->x[i] = nx;
  }
  g->x_cap = need;
  if (g->exec) {  // the cached graph captured the old buffers
    ANOMOD_HIP(ctx, hipGraphExecDestroy(g->exec));
    g->exec = nullptr;
  }
  return ANOMOD_OK;
}

// Sum of a personalization vector in the one order every solve entry uses
// (8 interleaved partial sums joined by a fixed tree: eight independent add
// chains instead of one N long), copied to `dst` in the same pass when COPY.
// Returns the index of the first entry that is negative or not finite, or N.
template <bool COPY>
uint32_t personalization_sum(const double* __restrict__ p, uint32_t N, double* __restrict__ dst,
                             double& sum) {
  double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  unsigned bad = 0;
  uint32_t i = 0;
  for (; i + 8 <= N; i += 8)
    for (int j = 0; j < 8; ++j) {
      const double v = p[i + j];
      if constexpr (COPY) dst[i + j] = v;
      bad |= !(v >= 0.0 && v <= DBL_MAX);
      a[j] += v;
    }
  for (; i < N; ++i) {
    const double v = p[i];
    if constexpr (COPY) dst[i] = v;
    bad |= !(v >= 0.0 && v <= DBL_MAX);
    a[i & 7] += v;
  }
  sum = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  if (!bad) return N;
  for (uint32_t k = 0; k < N; ++k)
    if (!(p[k] >= 0.0 && p[k] <= DBL_MAX)) return k;
  return N;
}

}  // namespace
}  // namespace anomod

using namespace anomod;

extern "C" {

int anomod_graph_create(anomod_ctx* ctx, const uint32_t* row_ptr, const uint32_t* col,
                        const float* w, uint32_t N, anomod_graph** out) {
  ANOMOD_REQUIRE(nullptr, ctx && out, "anomod_graph_create: NULL argument");
  *out = nullptr;
  ANOMOD_REQUIRE(ctx, N >= 1 && row_ptr && col && w, "graph needs N >= 1 and CSR arrays");
  ANOMOD_REQUIRE(ctx, row_ptr[0] == 0, "row_ptr[0] must be 0");
  for (uint32_t u = 0; u < N; ++u)
    ANOMOD_REQUIRE(ctx, row_ptr[u] <= row_ptr[u + 1], "row_ptr decreases at row %u", u);
  const uint64_t nnz = row_ptr[N];
  std::vector<double> outw(N, 0.0);
  std::vector<uint32_t> indeg(N + 1, 0);
  for (uint32_t u = 0; u < N; ++u) {
    for (uint32_t k = row_ptr[u]; k < row_ptr[u + 1]; ++k) {
      ANOMOD_REQUIRE(ctx, col[k] < N, "col[%u]=%u out of range", k, col[k]);
      ANOMOD_REQUIRE(ctx, std::isfinite(w[k]) && w[k] >= 0.f, "weight %u is negative or not finite",
                     k);
      outw[u] += (double)w[k];
      indeg[col[k] + 1]++;
    }
  }
  for (uint32_t v = 0; v < N; ++v) indeg[v + 1] += indeg[v];
  std::vector<uint32_t> in_col(nnz ? nnz : 1), fill(indeg.begin(), indeg.end() - 1);
  std::vector<float> in_w(nnz ? nnz : 1);
  std::vector<uint8_t> dang(N);
  for (uint32_t u = 0; u < N; ++u) {
    dang[u] = outw[u] == 0.0;
    for (uint32_t k = row_ptr[u]; k < row_ptr[u + 1]; ++k) {
      const uint32_t pos = fill[col[k]]++;
      in_col[pos] = u;
      in_w[pos] = (float)((double)w[k] / outw[u]);
    }
  }
  if (int rc = bind(ctx)) return rc;
  auto* g = new anomod_graph();
  g->device = ctx->device;
  g->N = N;
  g->nnz = nnz;
  g->grid = (N + kRowsPerBlock - 1) / kRowsPerBlock;
  for (uint32_t u = 0; u < N; ++u) g->n_dangling += dang[u];
  bool ok = hipMalloc(&g->in_ptr, (N + 1) * 4ull) == hipSuccess;
  ok = ok && hipMalloc(&g->in_col, in_col.size() * 4) == hipSuccess;
  ok = ok && hipMalloc(&g->in_w, in_w.size() * 4) == hipSuccess;
  ok = ok && hipMalloc(&g->dangling, N) == hipSuccess;
  ok = ok && hipMalloc(&g->p, N * 8ull) == hipSuccess;
  for (int i = 0; i < 2; ++i) ok = ok && hipMalloc(&g->x[i], N * 8ull) == hipSuccess;
  g->x_cap = N;
  ok = ok && hipMalloc(&g->acc, 6 * kAccSlots * 8) == hipSuccess;
  ok = ok && hipMalloc(&g->bar, kBarWords * sizeof(unsigned int)) == hipSuccess;
  g->host_acc.assign(6 * kAccSlots, 0ull);
  if (!ok) {
    free_graph(g);
    set_error(ctx, "hipMalloc failed for a graph of %u nodes / %llu edges", N,
              (unsigned long long)nnz);
    return ANOMOD_ENOMEM;
  }
  hipError_t e = hipMemcpyAsync(g->in_ptr, indeg.data(), (N + 1) * 4ull, hipMemcpyHostToDevice,
                                ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(g->in_col, in_col.data(), in_col.size() * 4, hipMemcpyHostToDevice,
                       ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(g->in_w, in_w.data(), in_w.size() * 4, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(g->dangling, dang.data(), N, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    free_graph(g);
    set_error(ctx, "graph upload failed: %s", hipGetErrorString(e));
    return ANOMOD_EHIP;
  }
  *out = g;
  return ANOMOD_OK;
}

}  // extern "C"

namespace {
// The synthetic service/pod graph of SURVEY.md §8d config 5 (host side, so
// the CPU baseline and the parity tests see the very graph the GPU solves):
// power-law (Pareto, a = 2.2) out-degrees scaled to the requested mean, 2 %
// dangling nodes, uniform callees, call-count weights in [1, 1000].
void synthetic_csr(uint32_t N, uint32_t mean_degree, uint64_t seed, std::vector<uint32_t>& row_ptr,
                   std::vector<uint32_t>& col, std::vector<float>& w) {
  row_ptr.assign(N + 1, 0);
  col.clear();
  w.clear();
  uint64_t st = seed;
  auto next = [&]() { st += 0x9E3779B97F4A7C15ull; return splitmix64(st); };
  const double a = 2.2, xmin = mean_degree * (a - 2.0) / (a - 1.0);
  for (uint32_t u = 0; u < N; ++u) {
    uint64_t d = 0;
    if (next() % 50 != 0) {
      const double uu = ((next() >> 11) + 0.5) * (1.0 / 9007199254740992.0);
      d = (uint64_t)(xmin * std::pow(uu, -1.0 / (a - 1.0)));
      d = std::min<uint64_t>(std::max<uint64_t>(d, 1), std::min<uint64_t>(N - 1, 1000));
    }
    for (uint64_t j = 0; j < d; ++j) {
      col.push_back((uint32_t)(next() % N));
      w.push_back((float)(1 + next() % 1000));
    }
    row_ptr[u + 1] = (uint32_t)col.size();
  }
}
}  // namespace

extern "C" {

int anomod_graph_synthetic(anomod_ctx* ctx, uint32_t N, uint32_t mean_degree, uint64_t seed,
                           anomod_graph** out) {
  ANOMOD_REQUIRE(nullptr, ctx && out, "anomod_graph_synthetic: NULL argument");
  ANOMOD_REQUIRE(ctx, N >= 2 && mean_degree >= 1, "need N >= 2 and mean_degree >= 1");
  std::vector<uint32_t> row_ptr, col;
  std::vector<float> w;
  synthetic_csr(N, mean_degree, seed, row_ptr, col, w);
  return anomod_graph_create(ctx, row_ptr.data(), col.data(), w.data(), N, out);
}

int anomod_graph_synthetic_csr(uint32_t N, uint32_t mean_degree, uint64_t seed,
                               uint32_t* row_ptr, uint32_t* col, float* w, uint64_t cap,
                               uint64_t* nnz) {
  ANOMOD_REQUIRE(nullptr, nnz, "anomod_graph_synthetic_csr: NULL nnz");
  ANOMOD_REQUIRE(nullptr, N >= 2 && mean_degree >= 1, "need N >= 2 and mean_degree >= 1");
  std::vector<uint32_t> rp, c;
  std::vector<float> ww;
  synthetic_csr(N, mean_degree, seed, rp, c, ww);
  *nnz = c.size();
  if (!row_ptr && !col && !w) return ANOMOD_OK;  // size query
  ANOMOD_REQUIRE(nullptr, row_ptr && col && w, "anomod_graph_synthetic_csr: NULL output array");
  ANOMOD_REQUIRE(nullptr, cap >= c.size(), "anomod_graph_synthetic_csr: cap %llu < nnz %llu",
                 (unsigned long long)cap, (unsigned long long)c.size());
  std::copy(rp.begin(), rp.end(), row_ptr);
  std::copy(c.begin(), c.end(), col);
  std::copy(ww.begin(), ww.end(), w);
  return ANOMOD_OK;
}

int anomod_graph_info(const anomod_graph* g, uint32_t* N, uint64_t* nnz) {
  ANOMOD_REQUIRE(nullptr, g, "anomod_graph_info: graph is NULL");
  if (N) *N = g->N;
  if (nnz) *nnz = g->nnz;
  return ANOMOD_OK;
}

int anomod_graph_pagerank(anomod_ctx* ctx, anomod_graph* g, const double* p, double alpha,
                          uint32_t iters, double tol, double* x_out, uint32_t* iters_done) {
  ANOMOD_REQUIRE(nullptr, ctx && g && p && x_out, "anomod_graph_pagerank: NULL argument");
  ANOMOD_REQUIRE(ctx, alpha > 0.0 && alpha < 1.0, "alpha=%g outside (0, 1)", alpha);
  ANOMOD_REQUIRE(ctx, iters >= 1, "iters must be >= 1");
  ANOMOD_REQUIRE(ctx, g->device == ctx->device, "graph lives on another device");
  const uint32_t N = g->N;
  if (int rc = bind(ctx)) return rc;
  // p goes up raw through pinned staging and is normalised on the device
  // (the host-side copy, division and pageable DMA were ~30 % of a
  // 100-iteration solve at N = 10^5); the copy to staging is the checking
  // and summing pass.
  if (!g->h_pin)
    ANOMOD_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&g->h_pin), N * 8ull + 16,
                                  hipHostMallocDefault));  // + the barrier words
  double psum = 0.0;
  const uint32_t bad = personalization_sum<true>(p, N, g->h_pin, psum);
  ANOMOD_REQUIRE(ctx, bad == N, "personalization[%u] invalid", bad);
  ANOMOD_REQUIRE(ctx, psum > 0.0, "personalization sums to zero");
  ANOMOD_HIP(ctx, hipMemcpyAsync(g->p, g->h_pin, N * 8ull, hipMemcpyHostToDevice, ctx->stream));
  // x0 = 1/N; its dangling mass n_dangling/N seeds iteration 0 (slot 0); the
  // slots iteration 0 adds into must start at zero (the init kernel writes
  // them, and clears the barrier words).
  const unsigned long long acc0 =
      (unsigned long long)std::llround((double)g->n_dangling / N * kDScale);
  hipLaunchKernelGGL(ppr_init_norm_kernel, dim3(std::min<uint32_t>(g->grid, 1024)),
                     dim3(kPprThreads), 0, ctx->stream, N, 1.0 / N, g->x[0], g->p, psum, g->acc,
                     (uint32_t)g->host_acc.size(), acc0, g->bar, (uint32_t)kBarWords);
  ANOMOD_HIP(ctx, hipGetLastError());
  uint32_t done = 0;
  // One persistent launch for the whole solve when every workgroup fits on
  // the chip at once (N = 10^5: 391 blocks): the stopping test runs on the
  // device; 8.7 us per iteration (fixed) / 9.4 (tolerance) against 9.8 for
  // the replayed hipGraph of per-iteration launches and 30 us with a host
  // read-back per launch (r02, scripts/time_pagerank.py).  Larger graphs take
  // the graph (fixed iterations) or per-launch read-backs (tolerance).
  // ANOMOD_PPR_MODE=1 forces the per-launch paths, 2 the persistent one
  // (tests: same bits).  ANOMOD_PPR_SUB = 256-row blocks per persistent
  // workgroup: 1, 2 or 4 (anything else: the default).
  const char* sub_env = getenv("ANOMOD_PPR_SUB");
  int sub = sub_env ? atoi(sub_env) : kPprSub;
  if (sub != 1 && sub != 2 && sub != 4) sub = kPprSub;
  if (g->coop_blocks < 0 || g->coop_sub != sub) {
    // Workgroups resident at once.  The persistent solve is a PLAIN launch: the
    // cooperative launch API only adds a launch-time check of this same
    // bound (MI355X_MICROARCH.md, coop-launch row), and a process that made
    // one segfaulted at exit under rocprofv3 --kernel-trace (r01,
    // scripts/coop_exit_probe.py) — so the bound is checked here, one block
    // per CU below the occupancy answer (the hardware may admit one fewer
    // than the API reports for 256-thread blocks).  Residency can still fail
    // when another process holds CUs: the grid barrier's bounded spin then
    // ends the launch and the solve reruns per launch (below), not a hang.
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_fn(sub, true),
                                                     kPprThreads * sub, 0) != hipSuccess)
      per_cu = 0;
    g->coop_blocks = (per_cu > 1 ? per_cu - 1 : per_cu) * ctx->num_cus;
    g->coop_sub = sub;
  }
  const char* mode_env = getenv("ANOMOD_PPR_MODE");
  const int mode = mode_env ? atoi(mode_env) : 0;
  // test knob: a tiny limit (0: no wait at all) forces the timeout and the rerun
  const char* spin_env = getenv("ANOMOD_PPR_SPIN");
  const long spin_v = spin_env && *spin_env ? atol(spin_env) : -1;
  const uint32_t spin = spin_v >= 0 && spin_v < (long)kSpinLimit ? (uint32_t)spin_v : kSpinLimit;
  const uint32_t pgrid = (g->grid + sub - 1) / sub;
  bool persistent = (int)pgrid <= g->coop_blocks && mode != 1;
  unsigned int* hb = reinterpret_cast<unsigned int*>(g->h_pin + N);  // pinned, past the vector
  // a fresh vector slot per iteration for the persistent solve (grow-only;
  // ANOMOD_PPR_RING=0, or more than kRingBytes of slots — e.g. a tolerance
  // solve allowed 1000 iterations —: the two-buffer form, agent-scope gathers)
  const uint64_t slot = (uint64_t)g->grid * kRowsPerBlock;
  const char* ring_env = getenv("ANOMOD_PPR_RING");
  bool ring = persistent && !(ring_env && ring_env[0] == '0') &&
              (uint64_t)iters * slot * 8 <= kRingBytes;
  if (ring) ring = ensure_ring(ctx, g, (uint64_t)iters * slot * 8);
  if (int rc = stage_begin(ctx, kStagePagerank)) return rc;
  g->last_path = 0;
  bool fell_back = false;
  if (persistent) {
    const double ntol = tol > 0.0 ? (double)N * tol : 0.0;
    double x0v = 1.0 / N;
    hipLaunchKernelGGL(persistent_fn(sub, ring), dim3(pgrid), dim3(kPprThreads * sub), 0,
                       ctx->stream, g->N, g->in_ptr, g->in_col, g->in_w, g->dangling, g->p, alpha,
                       x0v, g->x[0], g->x[1], g->acc, iters, ntol, g->bar, spin,
                       ring ? g->ring : nullptr, slot);
    ANOMOD_HIP(ctx, hipGetLastError());
    if (int rc = stage_end(ctx, kStagePagerank)) return rc;  // the copies are not timed
    // the persistent solve leaves its result in x[0]: one copy, one wait
    ANOMOD_HIP(ctx, hipMemcpyAsync(hb, g->bar, 4 * sizeof(unsigned int), hipMemcpyDeviceToHost,
                                   ctx->stream));
    ANOMOD_HIP(ctx, hipMemcpyAsync(g->h_pin, g->x[0], N * 8ull, hipMemcpyDeviceToHost,
                                   ctx->stream));
    ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (hb[1] == 0u) {
      done = hb[2];
      g->last_path = ANOMOD_PPR_PATH_PERSISTENT;
    } else {
      // A workgroup never became resident (another process held CUs) and the
      // grid barrier gave up: start over from x0 on the per-launch path.  p
      // is already normalised on the device (p / 1.0 is p); x, the slots and
      // the barrier words are re-initialised.  Same bits as the persistent
      // solve would have produced (tested).
      ++g->fallbacks;
      fell_back = true;
      hipLaunchKernelGGL(ppr_init_norm_kernel, dim3(std::min<uint32_t>(g->grid, 1024)),
                         dim3(kPprThreads), 0, ctx->stream, N, 1.0 / N, g->x[0], g->p, 1.0,
                         g->acc, (uint32_t)g->host_acc.size(), acc0, g->bar,
                         (uint32_t)kBarWords);
      ANOMOD_HIP(ctx, hipGetLastError());
      persistent = false;
    }
  }
  if (!persistent) {
    if (tol > 0.0) {
      // Convergence mode: host reads the L1 change after every iteration.
      for (uint32_t it = 0; it < iters; ++it) {
        launch_iter(ctx, g, alpha, it);
        ANOMOD_HIP(ctx, hipGetLastError());
        const int w = (it + 1) % 3;
        unsigned long long* eh = g->host_acc.data() + (3 + w) * kAccSlots;
        ANOMOD_HIP(ctx, hipMemcpyAsync(eh, g->acc + (3 + w) * kAccSlots, kAccSlots * 8,
                                       hipMemcpyDeviceToHost, ctx->stream));
        ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
        done = it + 1;
        unsigned long long et = 0;
        for (int i = 0; i < kAccSlots; ++i) et += eh[i];
        if ((double)et * (1.0 / kEScale) < (double)N * tol) break;
      }
      g->last_path = ANOMOD_PPR_PATH_READBACK;
    } else {
      // Fixed-iteration mode: replay a captured graph of `iters` launches.
      if (!g->exec || g->exec_iters != iters || g->exec_alpha != alpha) {
        if (g->exec) ANOMOD_HIP(ctx, hipGraphExecDestroy(g->exec));
        g->exec = nullptr;
        hipGraph_t graph = nullptr;
        ANOMOD_HIP(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
        for (uint32_t it = 0; it < iters; ++it) launch_iter(ctx, g, alpha, it);
        ANOMOD_HIP(ctx, hipStreamEndCapture(ctx->stream, &graph));
        hipError_t e = hipGraphInstantiate(&g->exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        ANOMOD_HIP(ctx, e);
        g->exec_iters = iters;
        g->exec_alpha = alpha;
      }
      ANOMOD_HIP(ctx, hipGraphLaunch(g->exec, ctx->stream));
      done = iters;
      g->last_path = ANOMOD_PPR_PATH_GRAPH;
    }
    if (fell_back) g->last_path |= ANOMOD_PPR_PATH_FALLBACK;
    // (after a fallback the stage spans the failed attempt and the rerun)
    if (int rc = stage_end(ctx, kStagePagerank)) return rc;
    ANOMOD_HIP(ctx, hipMemcpyAsync(g->h_pin, g->x[done & 1], N * 8ull, hipMemcpyDeviceToHost,
                                   ctx->stream));
    ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  memcpy(x_out, g->h_pin, N * 8ull);
  if (iters_done) *iters_done = done;
  return ANOMOD_OK;
}

int anomod_graph_last_solve(const anomod_graph* g, uint32_t* path, uint32_t* fallbacks) {
  ANOMOD_REQUIRE(nullptr, g, "anomod_graph_last_solve: graph is NULL");
  if (path) *path = g->last_path;
  if (fallbacks) *fallbacks = g->fallbacks;
  return ANOMOD_OK;
}

int anomod_graph_pagerank_batch(anomod_ctx* ctx, anomod_graph* g, const double* P, uint32_t K,
                                double alpha, uint32_t iters, double tol, double* X,
                                uint32_t* iters_done) {
  ANOMOD_REQUIRE(nullptr, ctx && g && P && X, "anomod_graph_pagerank_batch: NULL argument");
  ANOMOD_REQUIRE(ctx, K >= 1 && K <= 16, "K=%u outside [1, 16]", K);
  ANOMOD_REQUIRE(ctx, alpha > 0.0 && alpha < 1.0, "alpha=%g outside (0, 1)", alpha);
  ANOMOD_REQUIRE(ctx, iters >= 1, "iters must be >= 1");
  ANOMOD_REQUIRE(ctx, g->device == ctx->device, "graph lives on another device");
  const uint32_t N = g->N;
  const uint32_t kb = K <= 2 ? 2 : K <= 4 ? 4 : K <= 8 ? 8 : 16;  // padded with vector 0
  // node-major, normalised personalizations
  if (int rc = bind(ctx)) return rc;
  // pinned staging of P in and X out, [K][N] as the caller's (grow-only)
  if (g->h_bpin_n < (uint64_t)N * kb) {
    if (g->h_bpin) ANOMOD_HIP(ctx, hipHostFree(g->h_bpin));
    g->h_bpin = nullptr;
    g->h_bpin_n = 0;
    ANOMOD_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&g->h_bpin), (uint64_t)N * kb * 8,
                                  hipHostMallocDefault));
    g->h_bpin_n = (uint64_t)N * kb;
  }
  // the checking-and-summing pass copies each vector into the staging (the
  // single solve's order); the device divides (the same IEEE division: the
  // same bits) and transposes to node-major
  BatchNorm bn{};
  for (uint32_t k = 0; k < K; ++k) {
    double s = 0.0;
    const uint32_t bad = personalization_sum<true>(P + (size_t)k * N, N, g->h_bpin + (size_t)k * N, s);
    ANOMOD_REQUIRE(ctx, bad == N, "personalization[%u][%u] invalid", k, bad);
    ANOMOD_REQUIRE(ctx, s > 0.0, "personalization %u sums to zero", k);
    bn.psum[k] = s;
  }
  if (g->kb < kb) {
    for (void* q : {(void*)g->bp, (void*)g->bx[0], (void*)g->bx[1], (void*)g->bacc})
      if (q) (void)hipFree(q);
    g->bp = g->bx[0] = g->bx[1] = nullptr;
    g->bacc = nullptr;
    g->kb = 0;
    bool ok = hipMalloc(&g->bp, (size_t)N * kb * 8) == hipSuccess;
    for (int i = 0; i < 2; ++i) ok = ok && hipMalloc(&g->bx[i], (size_t)N * kb * 8) == hipSuccess;
    ok = ok && hipMalloc(&g->bacc, 6ull * kb * kAccSlots * 8) == hipSuccess;
    if (!ok) {
      set_error(ctx, "hipMalloc failed for a %u-vector PageRank batch", kb);
      return ANOMOD_ENOMEM;
    }
    g->kb = kb;
    g->host_bacc.assign(6ull * kb * kAccSlots, 0ull);
  }
  const int S = kAccSlots * (int)kb;  // one accumulator block = kb x kAccSlots
  // raw vectors through bx[1] (free until the first iteration writes it)
  ANOMOD_HIP(ctx, hipMemcpyAsync(g->bx[1], g->h_bpin, (size_t)N * K * 8, hipMemcpyHostToDevice,
                                 ctx->stream));
  hipLaunchKernelGGL(ppr_batch_norm_kernel, dim3(std::min<uint32_t>((N + kPprThreads - 1) / kPprThreads, 2048)),
                     dim3(kPprThreads), 0, ctx->stream, g->bx[1], N, K, kb, bn, g->bp);
  ANOMOD_HIP(ctx, hipGetLastError());
  const uint32_t nx = N * kb;  // x0 = 1/N everywhere, on the device
  auto init_x0 = [&]() {
    hipLaunchKernelGGL(ppr_init_kernel, dim3(std::min<uint32_t>((nx + kPprThreads - 1) / kPprThreads, 2048)),
                       dim3(kPprThreads), 0, ctx->stream, nx, 1.0 / N, g->bx[0]);
    return hipGetLastError();
  };
  ANOMOD_HIP(ctx, init_x0());
  std::fill(g->host_bacc.begin(), g->host_bacc.end(), 0ull);
  for (uint32_t k = 0; k < kb; ++k)
    g->host_bacc[k * kAccSlots] =
        (unsigned long long)std::llround((double)g->n_dangling / N * kDScale);
  ANOMOD_HIP(ctx, hipMemcpyAsync(g->bacc, g->host_bacc.data(), g->host_bacc.size() * 8,
                                 hipMemcpyHostToDevice, ctx->stream));
  auto launch = [&](uint32_t it, uint32_t frozen) {
    const int a = it & 1, b = a ^ 1;
    const int rr = it % 3, w = (it + 1) % 3, z = (it + 2) % 3;
    unsigned long long* A = g->bacc;
#define ANOMOD_PPR_BATCH(KK)                                                                   \
  hipLaunchKernelGGL(ppr_batch_iter_kernel<KK>, dim3(g->grid), dim3(kPprThreads), 0, ctx->stream, \
                     N, g->in_ptr, g->in_col, g->in_w, g->dangling, g->bp, alpha, g->bx[a],      \
                     g->bx[b], A + rr * S, A + w * S, A + z * S, A + (3 + w) * S,               \
                     A + (3 + z) * S, frozen)
    switch (kb) {
      case 2: ANOMOD_PPR_BATCH(2); break;
      case 4: ANOMOD_PPR_BATCH(4); break;
      case 8: ANOMOD_PPR_BATCH(8); break;
      default: ANOMOD_PPR_BATCH(16); break;
    }
#undef ANOMOD_PPR_BATCH
  };
  uint32_t done = 0, frozen = 0;
  const uint32_t all = kb >= 32 ? 0xFFFFFFFFu : ((1u << kb) - 1u);
  // One persistent launch for the whole batch when its workgroups are all
  // resident (ANOMOD_PPR_MODE=1: the per-launch loop below); a barrier
  // timeout reruns the batch per launch from x0.
  const char* mode_env = getenv("ANOMOD_PPR_MODE");
  const int mode = mode_env ? atoi(mode_env) : 0;
  const char* spin_env = getenv("ANOMOD_PPR_SPIN");
  const long spin_v = spin_env && *spin_env ? atol(spin_env) : -1;
  const uint32_t spin = spin_v >= 0 && spin_v < (long)kSpinLimit ? (uint32_t)spin_v : kSpinLimit;
  const uint64_t slot = (uint64_t)g->grid * kRowsPerBlock * kb;  // doubles per ring slot
  const char* ring_env = getenv("ANOMOD_PPR_RING");
  bool ring = !(ring_env && ring_env[0] == '0') && (uint64_t)iters * slot * 8 <= kRingBytes;
  const uint32_t bsub = batch_sub(kb);
  // K = 16 with a ring: the split kernel (two 256-row blocks x two halves of
  // 8 vectors per 1024-thread workgroup); ANOMOD_PPR_SPLIT=0 keeps the SUB form
  const char* split_env = getenv("ANOMOD_PPR_SPLIT");
  const bool split = kb == 16 && ring && !(split_env && split_env[0] == '0');
  const uint32_t bthreads = split ? 4u * kPprThreads : kPprThreads * bsub;
  const uint32_t bgrid = split ? (g->grid + 1) / 2 : (g->grid + bsub - 1) / bsub;  // workgroups
  const BatchFn bfn = split ? ppr_batch_split_kernel : batch_persistent_fn(kb, ring, bsub);
  if (g->bcoop_kb != kb || g->bcoop_ring != ring || g->bcoop_sub != bsub + (split ? 16u : 0u)) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bfn, bthreads, 0) != hipSuccess)
      per_cu = 0;
    (void)hipGetLastError();
    g->bcoop_blocks = (per_cu > 1 ? per_cu - 1 : per_cu) * ctx->num_cus;
    g->bcoop_kb = kb;
    g->bcoop_ring = ring;
    g->bcoop_sub = bsub + (split ? 16u : 0u);
  }
  bool persistent = mode != 1 && (int)bgrid <= g->bcoop_blocks;
  if (persistent && ring) {
    ring = ensure_ring(ctx, g, (uint64_t)iters * slot * 8);
    if (!ring && split) persistent = false;  // (the split kernel needs the ring)
    if (!ring && !split) {  // no ring: the two-buffer instantiation (its own residency)
      int per_cu = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, batch_persistent_fn(kb, false, bsub),
                                                       kPprThreads * bsub, 0) != hipSuccess)
        per_cu = 0;
      (void)hipGetLastError();
      persistent = (int)bgrid <= (per_cu > 1 ? per_cu - 1 : per_cu) * ctx->num_cus;
    }
  }
  if (persistent) ANOMOD_HIP(ctx, hipMemsetAsync(g->bar, 0, kBarWords * sizeof(unsigned int),
                                                 ctx->stream));
  if (int rc = stage_begin(ctx, kStagePagerank)) return rc;
  g->last_path = 0;
  bool fell_back = false;
  if (persistent) {
    const double ntol = tol > 0.0 ? (double)N * tol : 0.0;
    hipLaunchKernelGGL(split ? ppr_batch_split_kernel : batch_persistent_fn(kb, ring, bsub),
                       dim3(bgrid), dim3(bthreads), 0,
                       ctx->stream, N, g->in_ptr, g->in_col, g->in_w, g->dangling, g->bp, alpha,
                       g->bx[0], g->bx[1], g->bacc, iters, ntol, g->bar, spin,
                       ring ? g->ring : nullptr, slot);
    ANOMOD_HIP(ctx, hipGetLastError());
    if (int rc = stage_end(ctx, kStagePagerank)) return rc;
    unsigned int hb[4];
    ANOMOD_HIP(ctx, hipMemcpyAsync(hb, g->bar, sizeof(hb), hipMemcpyDeviceToHost, ctx->stream));
    ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (hb[1] == 0u) {
      done = hb[2];
      g->last_path = ANOMOD_PPR_PATH_PERSISTENT;
      ANOMOD_HIP(ctx, batch_out(ctx, g, g->bx[0], g->bx[1], N, K, kb, X));
      if (iters_done) *iters_done = done;
      return ANOMOD_OK;
    }
    // a workgroup never became resident: start over per launch from x0
    ++g->fallbacks;
    fell_back = true;
    ANOMOD_HIP(ctx, init_x0());
    ANOMOD_HIP(ctx, hipMemcpyAsync(g->bacc, g->host_bacc.data(), g->host_bacc.size() * 8,
                                   hipMemcpyHostToDevice, ctx->stream));
    if (int rc = stage_begin(ctx, kStagePagerank)) return rc;
  }
  for (uint32_t it = 0; it < iters; ++it) {
    launch(it, frozen);
    ANOMOD_HIP(ctx, hipGetLastError());
    done = it + 1;
    if (tol > 0.0) {  // per-vector L1 test; converged vectors are carried unchanged
      const int w = (it + 1) % 3;
      unsigned long long* eh = g->host_bacc.data() + (3 + w) * S;
      ANOMOD_HIP(ctx, hipMemcpyAsync(eh, g->bacc + (3 + w) * S, S * 8ull, hipMemcpyDeviceToHost,
                                     ctx->stream));
      ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
      for (uint32_t k = 0; k < kb; ++k) {
        unsigned long long et = 0;
        for (int i = 0; i < kAccSlots; ++i) et += eh[k * kAccSlots + i];
        if (!((frozen >> k) & 1u) && (double)et * (1.0 / kEScale) < (double)N * tol)
          frozen |= 1u << k;
      }
      if ((frozen & all) == all) break;
    }
  }
  g->last_path = tol > 0.0 ? ANOMOD_PPR_PATH_READBACK : ANOMOD_PPR_PATH_GRAPH;
  if (fell_back) g->last_path |= ANOMOD_PPR_PATH_FALLBACK;
  if (int rc = stage_end(ctx, kStagePagerank)) return rc;
  ANOMOD_HIP(ctx, batch_out(ctx, g, g->bx[done & 1], g->bx[(done & 1) ^ 1], N, K, kb, X));
  if (iters_done) *iters_done = done;
  return ANOMOD_OK;
}

int anomod_graph_pagerank_sharded(anomod_ctx* ctx, anomod_graph* g, const double* p,
                                  double alpha, uint32_t iters, double tol,
                                  uint32_t virtual_shards, double* x_out, uint32_t* iters_done) {
  ANOMOD_REQUIRE(nullptr, ctx && g && p && x_out, "anomod_graph_pagerank_sharded: NULL argument");
  ANOMOD_REQUIRE(ctx, alpha > 0.0 && alpha < 1.0, "alpha=%g outside (0, 1)", alpha);
  ANOMOD_REQUIRE(ctx, iters >= 1, "iters must be >= 1");
  ANOMOD_REQUIRE(ctx, g->device == ctx->device, "graph lives on another device");
  const bool ranks = comm_attached(ctx) || ctx->comm_aborted;
  ANOMOD_REQUIRE(ctx, !ranks || virtual_shards <= 1,
                 "virtual_shards=%u needs a context without a communicator", virtual_shards);
  const uint32_t G = ranks ? (uint32_t)ctx->nranks : (virtual_shards ? virtual_shards : 1u);
  ANOMOD_REQUIRE(ctx, G <= 4096, "%u shards", G);
  const uint32_t N = g->N;
  // Checks that can fail on one rank only go through the status agreement
  // (the other ranks would otherwise wait in the first exchange forever).
  int local = ANOMOD_OK;
  double psum = 0.0;
  std::vector<double> pn(N);
  const uint32_t bad = personalization_sum<true>(p, N, pn.data(), psum);
  ANOMOD_CHECK_LOCAL(ctx, local, bad == N, "personalization[%u] invalid", bad);
  ANOMOD_CHECK_LOCAL(ctx, local, psum > 0.0, "personalization sums to zero");
  for (double& v : pn) v /= psum;
  if (local == ANOMOD_OK) local = bind(ctx);
  if (local == ANOMOD_OK) local = ensure_shard_x(ctx, g, G);
  if (ranks) {
    if (int rc = comm_agree(ctx, local)) return rc;
  } else if (local != ANOMOD_OK) {
    return local;
  }
  ANOMOD_HIP(ctx, hipMemcpyAsync(g->p, pn.data(), N * 8ull, hipMemcpyHostToDevice, ctx->stream));
  for (unsigned long long& v : g->host_acc) v = 0ull;
  g->host_acc[0] = (unsigned long long)std::llround((double)g->n_dangling / N * kDScale);
  ANOMOD_HIP(ctx, hipMemcpyAsync(g->acc, g->host_acc.data(), g->host_acc.size() * 8,
                                 hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(ppr_init_kernel, dim3(std::min<uint32_t>(g->grid, 1024)), dim3(kPprThreads),
                     0, ctx->stream, N, 1.0 / N, g->x[0]);
  ANOMOD_HIP(ctx, hipGetLastError());
  unsigned long long* A = g->acc;
  const int S = kAccSlots;
  uint32_t done = iters;
  if (int rc = stage_begin(ctx, kStagePagerank)) return rc;
  for (uint32_t it = 0; it < iters; ++it) {
    const int b = (it & 1) ^ 1, w = (it + 1) % 3, z = (it + 2) % 3;
    if (ranks) {
      // This rank's rows, then one grouped exchange: the fixed-point partials
      // (u64 sums: order-free, so every rank holds the unsharded scalars)
      // and an in-place all-gather of the new vector's row shards.
      const RowShard sh = row_shard(g, G, (uint32_t)ctx->rank);
      if (sh.nblocks) {
        launch_iter(ctx, g, alpha, it, sh.block0, sh.nblocks);
      } else {  // nothing to launch: still clear the slots iteration it+1 adds into
        ANOMOD_HIP(ctx, hipMemsetAsync(A + z * S, 0, S * 8ull, ctx->stream));
        ANOMOD_HIP(ctx, hipMemsetAsync(A + (3 + z) * S, 0, S * 8ull, ctx->stream));
      }
      ANOMOD_HIP(ctx, hipGetLastError());
      double* xb = g->x[b];
      if (int rc = coll_begin(ctx)) return rc;
      if (int rc = coll_allreduce(ctx, A + w * S, S, kCollU64, kCollSum)) return rc;
      if (int rc = coll_allreduce(ctx, A + (3 + w) * S, S, kCollU64, kCollSum)) return rc;
      if (int rc = coll_allgather(ctx, xb, sh.rows_per_shard, kCollF64)) return rc;
      if (int rc = coll_end(ctx)) return rc;
    } else {
      // Virtual shards on one device (the same row split, sequential
      // launches into shared accumulators): rehearses the sharding exactly.
      for (uint32_t k = 0; k < G; ++k) {
        const RowShard sh = row_shard(g, G, k);
        if (sh.nblocks) launch_iter(ctx, g, alpha, it, sh.block0, sh.nblocks);
      }
      ANOMOD_HIP(ctx, hipGetLastError());
    }
    if (tol > 0.0) {
      unsigned long long* eh = g->host_acc.data() + (3 + w) * S;
      ANOMOD_HIP(ctx, hipMemcpyAsync(eh, A + (3 + w) * S, S * 8, hipMemcpyDeviceToHost,
                                     ctx->stream));
      if (int rc = stream_wait(ctx)) return rc;
      unsigned long long et = 0;
      for (int i = 0; i < S; ++i) et += eh[i];
      if ((double)et * (1.0 / kEScale) < (double)N * tol) {
        done = it + 1;
        break;
      }
    }
  }
  if (int rc = stage_end(ctx, kStagePagerank)) return rc;
  ANOMOD_HIP(ctx, hipMemcpyAsync(x_out, g->x[done & 1], N * 8ull, hipMemcpyDeviceToHost,
                                 ctx->stream));
  if (int rc = stream_wait(ctx)) return rc;
  if (iters_done) *iters_done = done;
  return ANOMOD_OK;
}

int anomod_graph_free(anomod_graph* g) {
  free_graph(g);
  return ANOMOD_OK;
}

int anomod_pagerank(anomod_ctx* ctx, const uint32_t* row_ptr, const uint32_t* col, const float* w,
                    uint32_t N, const double* p, double alpha, uint32_t iters, double tol,
                    double* x_out, uint32_t* iters_done) {
  anomod_graph* g = nullptr;
  if (int rc = anomod_graph_create(ctx, row_ptr, col, w, N, &g)) return rc;
  const int rc = anomod_graph_pagerank(ctx, g, p, alpha, iters, tol, x_out, iters_done);
  free_graph(g);
  return rc;
}

}  // extern "C"
