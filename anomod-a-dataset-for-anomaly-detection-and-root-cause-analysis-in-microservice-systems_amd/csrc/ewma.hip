// Windowed EWMA / z-score anomaly scoring over the metric matrix
// (build-defined — the reference only exports the raw
// series: metric_collector.py:427-443 long CSV rows, fetch_prometheus_
// metrics.py:53-67 per-query CSV).
//
// X lives in one of two layouts, chosen per call by the kernel that reads it:
//  * tiled  Xt[ceil(T/16)][4][S][4] — a tile holds 16 steps of every series
//    as four planes of float4 (steps 4q .. 4q+3 of series s at plane q), so
//    one load instruction of a wave reads 1 KiB contiguously (series-major
//    tiles [S][16], each lane's 64 B contiguous, read the same bytes at a
//    64-B lane stride: 1.5 % slower at the config-4 chunk, 5-10 % at
//    T = 7680).  The sequential kernel (one series per lane down T) reads
//    it; with S/64 waves on the chip the row-major form (one 256-B row
//    segment per instruction) tops out near 2 TB/s, the tiled one is ~1.4x
//    faster.  Steps past T in the last tile hold NaN.
//  * rows   X[T][S] — the time-parallel kernel (small S) gives each wave U
//    consecutive rows, which a 16-step tiling would misalign for W % 16 != 0.
// Upload takes row-major host data and tiles it on the device in bounded
// chunks; a series is re-laid-out (one extra pass) only when a forced kernel
// choice (ANOMOD_EWMA_MODE) disagrees with its current layout.
// The recurrence runs in registers; the state (m, v in f64, sample count)
// lives in HBM between calls so an arbitrarily long T is streamed in chunks
// (400 GB at 10^6 x 10^5 does not fit 288 GB of HBM).  HBM-bound: 4 B/sample
// read + 4/W B/sample written.
#include <cmath>
#include <cstdlib>

#include "common.h"
#include "synth.h"

struct anomod_series {
  int device = 0;
  uint64_t T = 0, S = 0;
  float* X = nullptr;      // [T][S] rows or [ceil(T/16)][S][16] tiles (sized for the tiles)
  bool tiled = false;
  float* Z = nullptr;      // [T/W][S] (allocated lazily for the largest W seen)
  size_t z_cap = 0;
  double* m = nullptr;     // [S]
  double* v = nullptr;     // [S]
  uint32_t* n = nullptr;   // [S] valid samples seen
};

namespace anomod {
namespace {

#ifndef ANOMOD_EWMA_U
#define ANOMOD_EWMA_U 32
#endif
constexpr int kU = ANOMOD_EWMA_U;  // time steps per load block (x2 buffers in flight)

struct EwmaState {
  double m, v;
  uint32_t n;
};

// 1/sqrt(v + eps) with the hardware reciprocal square root (v_rsq_f32, 1 ulp):
// v + eps is never denormal for eps >= 2^-126, so rsqrtf's denormal rescaling
// is dead weight on the recurrence's critical path.
__device__ __forceinline__ float zscale(double v, float eps) {
  return __builtin_amdgcn_rsqf((float)v + eps);
}

// One step of the recurrence (spec.ewma_step): a NaN sample is missing (state
// carried, z = 0); the first valid sample starts the state (m = x, v = 0,
// z = 0); otherwise d = x - m, z = d / sqrt(v + eps), m += alpha*d,
// v = beta*(v + alpha*d^2).  Branch-free (every update computed, then
// selected): per-lane branches cost more than the arithmetic on a wave whose
// only work is this dependent chain.
__device__ __forceinline__ float ewma_step_bf(EwmaState& st, float x, double alpha, double beta,
                                              float eps) {
  const bool valid = x == x;
  const bool init = valid && st.n == 0u;
  const bool upd = valid && st.n != 0u;
  const double xd = (double)x;
  const double d = xd - st.m;
  const float zr = (float)d * zscale(st.v, eps);  // computed unconditionally, then selected
  const float z = upd ? zr : 0.f;
  const double m1 = fma(alpha, d, st.m);
  const double v1 = beta * fma(alpha * d, d, st.v);
  st.m = init ? xd : (upd ? m1 : st.m);
  st.v = init ? 0.0 : (upd ? v1 : st.v);
  st.n += valid ? 1u : 0u;
  return z;
}

// The same step for a sample known valid on a started state (n != 0): the
// `upd` arm of ewma_step_bf with the same expressions, so the same roundings.
// The caller adds the block's sample count to n.
__device__ __forceinline__ float ewma_step_dense(EwmaState& st, float x, double alpha,
                                                 double beta, float eps) {
  const double d = (double)x - st.m;
  const float z = (float)d * zscale(st.v, eps);
  const double m1 = fma(alpha, d, st.m);
  const double v1 = beta * fma(alpha * d, d, st.v);
  st.m = m1;
  st.v = v1;
  return z;
}

__global__ __launch_bounds__(64) void ewma_z_kernel(const float* __restrict__ X, uint64_t T,
                                                     uint64_t S, double alpha, uint32_t W,
                                                     float eps, float* __restrict__ Z,
                                                     double* __restrict__ gm,
                                                     double* __restrict__ gv,
                                                     uint32_t* __restrict__ gn) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const double beta = 1.0 - alpha;
  EwmaState st{gm[s], gv[s], gn[s]};
  float a[kU], b[kU];
  const float* col = X + s;
  auto load = [&](float* buf, uint64_t t0) {
#pragma unroll
    for (int u = 0; u < kU; ++u) buf[u] = (t0 + u < T) ? col[(t0 + u) * S] : NAN;
  };
  float wmax = 0.f;
  uint32_t wpos = 0;
  uint64_t w = 0;
  auto consume = [&](const float* buf, uint64_t t0) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (t0 + u < T) {
        wmax = fmaxf(wmax, fabsf(ewma_step_bf(st, buf[u], alpha, beta, eps)));
        if (++wpos == W) {
          Z[w * S + s] = wmax;
          ++w;
          wpos = 0;
          wmax = 0.f;
        }
      }
    }
  };
  load(a, 0);
  uint64_t t0 = 0;
  while (t0 < T) {
    if (t0 + kU < T) load(b, t0 + kU);
    consume(a, t0);
    t0 += kU;
    if (t0 >= T) break;
    if (t0 + kU < T) load(a, t0 + kU);
    consume(b, t0);
    t0 += kU;
  }
  gm[s] = st.m;
  gv[s] = st.v;
  gn[s] = st.n;
}

// Sequential recurrence over the tiled layout.  kTiles tiles (16 steps each)
// per load block, two blocks in flight; blocks wholly inside T run without
// per-step bounds checks.
#ifndef ANOMOD_EWMA_TILE
#define ANOMOD_EWMA_TILE 16
#endif
constexpr int kTile = ANOMOD_EWMA_TILE;  // steps per tile (one lane's contiguous run)
static_assert(kTile % 16 == 0 && 64 % kTile == 0, "tile steps");
#ifndef ANOMOD_EWMA_QMAJOR
#define ANOMOD_EWMA_QMAJOR 1
#endif
// Float index of steps 4q .. 4q+3 of series s in tile `tile` (a tile holds
// kTile steps of every series: S * kTile floats).  q-major (default): the
// float4 groups of one q for all series contiguous, so a wave's load
// instruction reads 1 KiB contiguously; series-major (ANOMOD_EWMA_QMAJOR=0,
// the r01/r02 layout): each series' kTile steps contiguous.
__host__ __device__ __forceinline__ uint64_t tile_off(uint64_t tile, uint64_t S, uint64_t s,
                                                      uint64_t q) {
  if constexpr (ANOMOD_EWMA_QMAJOR) return tile * S * kTile + (q * S + s) * 4;
  else return (tile * S + s) * kTile + 4 * q;
}
#ifndef ANOMOD_ZT_TILES
#define ANOMOD_ZT_TILES 4
#endif
constexpr int kZtTiles = ANOMOD_ZT_TILES;  // tiles per load block (two blocks in flight)
constexpr int kPadTiles = 2 * kZtTiles;  // slack tiles past ceil(T/16) read by the prefetch

// kChk: steps between window-end checks in dense blocks — 4 when W % 4 == 0
// (every window then ends on a float4 boundary: the window position starts at
// 0 and a block advances it by a multiple of 4), else 1.  The per-step max
// sequence is the same either way; only the scalar compare-and-branch of the
// window end runs once per 4 steps.
#ifndef ANOMOD_EWMA_CHK
#define ANOMOD_EWMA_CHK 4
#endif
#ifndef ANOMOD_EWMA_NT
#define ANOMOD_EWMA_NT 0
#endif
#ifndef ANOMOD_EWMA_ABL
#define ANOMOD_EWMA_ABL 0
#endif
constexpr int kEwmaChk = ANOMOD_EWMA_CHK;  // 1: check every step (experiment builds)
template <int kTiles, int kChk>
__global__ __launch_bounds__(64) void ewma_zt_kernel(const float* __restrict__ Xt, uint64_t T,
                                                      uint64_t S, double alpha, uint32_t W,
                                                      float eps, float* __restrict__ Z,
                                                      double* __restrict__ gm,
                                                      double* __restrict__ gv,
                                                      uint32_t* __restrict__ gn) {
  constexpr int kV = kTile / 4;  // float4 per tile
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const double beta = 1.0 - alpha;
  EwmaState st{gm[s], gv[s], gn[s]};
  float4 a[kTiles * kV], b[kTiles * kV];
  const uint64_t nt = (T + kTile - 1) / kTile;
  // unconditional loads (X carries kPadTiles tiles of slack past the last
  // one): a load under a branch would make the wait counts path-dependent
  // and the compiler would drain every load in flight before each use
  auto load = [&](float4* buf, uint64_t tile0) {
#pragma unroll
    for (int k = 0; k < kTiles; ++k) {
#pragma unroll
      for (int q = 0; q < kV; ++q) {
        const float4* p = reinterpret_cast<const float4*>(Xt + tile_off(tile0 + k, S, s, q));
#if ANOMOD_EWMA_NT  // experiment builds: nontemporal sample loads
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
        buf[k * kV + q] = make_float4(v.x, v.y, v.z, v.w);
#else
        buf[k * kV + q] = *p;
#endif
      }
    }
  };
  float wmax = 0.f;
  uint32_t wpos = 0;
  float* zp = Z + s;
  auto step = [&](float x) {
    wmax = fmaxf(wmax, fabsf(ewma_step_bf(st, x, alpha, beta, eps)));
    if (++wpos == W) {
      *zp = wmax;
      zp += S;
      wpos = 0;
      wmax = 0.f;
    }
  };
  auto step_dense_nc = [&](float x) {  // window end checked by the caller
#if ANOMOD_EWMA_ABL & 1  // timing only: the loads and window stores without the recurrence
    wmax = fmaxf(wmax, x);
#else
    wmax = fmaxf(wmax, fabsf(ewma_step_dense(st, x, alpha, beta, eps)));
#endif
  };
  auto check4 = [&]() {
    wpos += 4;
    if (wpos == W) {
      *zp = wmax;
      zp += S;
      wpos = 0;
      wmax = 0.f;
    }
  };
  auto step_dense = [&](float x) {
    wmax = fmaxf(wmax, fabsf(ewma_step_dense(st, x, alpha, beta, eps)));
    if (++wpos == W) {
      *zp = wmax;
      zp += S;
      wpos = 0;
      wmax = 0.f;
    }
  };
  bool started = __all(st.n != 0u);  // every lane of the wave has seen a valid sample
  auto consume = [&](const float4* buf, uint64_t tile0) __attribute__((always_inline)) {
    if ((tile0 + kTiles) * kTile <= T) {  // whole block inside T (wave-uniform)
      // Dense block: no NaN in any lane's samples (a NaN makes the sum NaN;
      // inf - inf only sends a dense block down the general path) and every
      // lane started.  Then every step is the `upd` arm: ~14 VALU instead of
      // ~31 (no selects, n counted once per block).
      bool dense = false;
      if (started) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < kTiles * kV; ++i) acc += (buf[i].x + buf[i].y) + (buf[i].z + buf[i].w);
        dense = __all(acc == acc);
      }
      if (dense && kChk == 4) {
#pragma unroll
        for (int i = 0; i < kTiles * kV; ++i) {
          step_dense_nc(buf[i].x);
          step_dense_nc(buf[i].y);
          step_dense_nc(buf[i].z);
          step_dense_nc(buf[i].w);
          check4();
        }
        st.n += kTiles * kTile;
      } else if (dense) {
#pragma unroll
        for (int i = 0; i < kTiles * kV; ++i) {
          step_dense(buf[i].x);
          step_dense(buf[i].y);
          step_dense(buf[i].z);
          step_dense(buf[i].w);
        }
        st.n += kTiles * kTile;
      } else {
#pragma unroll
        for (int i = 0; i < kTiles * kV; ++i) {
          step(buf[i].x);
          step(buf[i].y);
          step(buf[i].z);
          step(buf[i].w);
        }
        started = started || __all(st.n != 0u);
      }
    } else {
      const uint64_t t0 = tile0 * kTile;
#pragma unroll
      for (int i = 0; i < kTiles * kV; ++i) {
        const float xs[4] = {buf[i].x, buf[i].y, buf[i].z, buf[i].w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (t0 + i * 4 + e < T) step(xs[e]);
      }
    }
  };
  load(a, 0);
  uint64_t t0 = 0;
  while (t0 < nt) {
    load(b, t0 + kTiles);
    consume(a, t0);
    t0 += kTiles;
    if (t0 >= nt) break;
    load(a, t0 + kTiles);
    consume(b, t0);
    t0 += kTiles;
  }
  gm[s] = st.m;
  gv[s] = st.v;
  gn[s] = st.n;
}

// rows X[T][S] <-> tiles Xt[ceil(T/16)][S][16] for steps [r0, r0 + R) (R a
// multiple of 16 unless it reaches T); one thread per (tile, series): 16
// coalesced row reads, one 64-B tile write (or the reverse).  `rows` holds
// the R rows starting at r0.  Tile steps past T are written as NaN.
__global__ void series_relayout_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                       uint64_t T, uint64_t S, uint64_t r0, uint64_t R,
                                       int to_tiles) {
  const uint64_t ntile = (R + kTile - 1) / kTile;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ntile * S;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = i / S, s = i % S;
    const uint64_t tile = r0 / kTile + k;
    if (to_tiles) {
      float v[kTile];
#pragma unroll
      for (int e = 0; e < kTile; ++e) {
        const uint64_t r = k * kTile + e;
        v[e] = (r < R && r0 + r < T) ? src[r * S + s] : NAN;
      }
#pragma unroll
      for (int q = 0; q < kTile / 4; ++q)
        *reinterpret_cast<float4*>(dst + tile_off(tile, S, s, q)) =
            make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    } else {
      float v[kTile];
#pragma unroll
      for (int q = 0; q < kTile / 4; ++q) {
        const float4 f = *reinterpret_cast<const float4*>(src + tile_off(tile, S, s, q));
        v[4 * q] = f.x;
        v[4 * q + 1] = f.y;
        v[4 * q + 2] = f.z;
        v[4 * q + 3] = f.w;
      }
#pragma unroll
      for (int e = 0; e < kTile; ++e) {
        const uint64_t r = k * kTile + e;
        if (r < R && r0 + r < T) dst[r * S + s] = v[e];
      }
    }
  }
}

// Time-parallel form.  A 64-series strip is one workgroup of kNW waves; a
// super-chunk of kNW*U steps gives every wave U consecutive steps (U a
// multiple of W, so every window lies inside one wave's steps).
//  phase A  each wave summarises its U samples as a transfer of the state:
//           with r = its first valid sample x_f, the samples after x_f map an
//           incoming (m = r + delta, v) to
//             m' = M + A*delta,  v' = A*v + Q0 + Q1*delta + Q2*delta^2
//           (M: the mean run from r; A = beta^c; Q*: the variance recurrence
//           expanded in delta).  Exact algebra, f64, terms of the size of the
//           signal around r, so no cancellation at large means.
//  combine  every wave folds the transfers of the waves before it onto the
//           carried state, sub-chunk by sub-chunk in time order (x_f first:
//           the fresh start m = x_f, v = 0 when no sample was seen yet), so
//           its incoming state is the same fold whatever the super-chunk
//           grouping — results do not depend on how T is cut into calls when
//           the cuts fall on multiples of U;
//  phase C  each wave re-runs its U samples from registers with that exact
//           incoming state (the sequential recurrence, unchanged) and writes
//           its window maxima.
// HBM: every sample is read once (4 B) and every window score written once.
constexpr int kTpWaves = 12;
constexpr int kTpThreads = kTpWaves * 64;

struct Transfer {
  double xf, M, A, Q0, Q1, Q2;
  uint32_t c;  // valid samples after x_f; bit 31 set when x_f exists
};

__device__ __forceinline__ void apply_transfer(const Transfer& t, double alpha, double beta,
                                               double& m, double& v, uint32_t& n) {
  if (!(t.c & 0x80000000u)) return;  // no valid sample in this sub-chunk
  const uint32_t c = t.c & 0x7FFFFFFFu;
  double delta, v1;
  if (n == 0u) {  // fresh start at x_f: m = x_f, v = 0
    delta = 0.0;
    v1 = 0.0;
  } else {
    const double d = t.xf - m;
    const double m1 = fma(alpha, d, m);
    v1 = beta * fma(alpha * d, d, v);
    delta = m1 - t.xf;
  }
  m = fma(t.A, delta, t.M);
  v = fma(t.A, v1, fma(fma(t.Q2, delta, t.Q1), delta, t.Q0));
  n += 1u + c;
}

template <int kCap>
__global__ __launch_bounds__(kTpThreads) void ewma_tp_kernel(
    const float* __restrict__ X, uint64_t T, uint64_t S, double alpha, uint32_t W, uint32_t U,
    float eps, float* __restrict__ Z, double* __restrict__ gm, double* __restrict__ gv,
    uint32_t* __restrict__ gn) {
  __shared__ double ls[6][kTpWaves][64];
  __shared__ uint32_t lc[kTpWaves][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const uint64_t s = (uint64_t)blockIdx.x * 64 + lane;
  const bool sv = s < S;
  const double beta = 1.0 - alpha;
  double m = sv ? gm[s] : 0.0, v = sv ? gv[s] : 0.0;
  uint32_t n = sv ? gn[s] : 0u;
  const uint64_t SC = (uint64_t)kTpWaves * U;
  const uint32_t row_bytes = (uint32_t)(S * 4u);
  for (uint64_t t0 = 0; t0 < T; t0 += SC) {
    const uint64_t tw = __builtin_amdgcn_readfirstlane((uint32_t)(t0 >> 32)) * 0x100000000ull +
                        __builtin_amdgcn_readfirstlane((uint32_t)t0) + (uint64_t)w * U;
    const uint32_t cnt = tw < T ? (uint32_t)((T - tw) < U ? (T - tw) : U) : 0u;  // wave-uniform
    // rows [tw, tw + cnt) through one descriptor: a scalar row offset per load,
    // one lane offset for all (rows past cnt read as 0 and are never used)
    const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(X + tw * S), (short)0,
                                                      (int)(cnt * row_bytes), 0x00020000);
    float x[kCap];
#pragma unroll
    for (int u = 0; u < kCap; ++u)
      x[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                           rx, (int)(s * 4u), (int)(u * row_bytes), 0));
#pragma unroll
    for (int u = 0; u < kCap; ++u)
      if ((uint32_t)u >= cnt || !sv) x[u] = NAN;
    // phase A (branch-free: every update is computed and selected)
    Transfer tr{0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0u};
    bool seen = false;
#pragma unroll
    for (int u = 0; u < kCap; ++u) {
      const float xv = x[u];
      const bool valid = xv == xv;
      const bool upd = valid && seen;
      const bool first = valid && !seen;
      const double xd = (double)xv;
      const double d = xd - tr.M;
      const double ad = alpha * d;
      const double q0 = beta * fma(ad, d, tr.Q0);
      const double q1 = beta * fma(-2.0 * ad, tr.A, tr.Q1);
      const double q2 = beta * fma(alpha * tr.A, tr.A, tr.Q2);
      tr.Q0 = upd ? q0 : tr.Q0;
      tr.Q1 = upd ? q1 : tr.Q1;
      tr.Q2 = upd ? q2 : tr.Q2;
      tr.M = first ? xd : (upd ? tr.M + ad : tr.M);
      tr.xf = first ? xd : tr.xf;
      tr.A = upd ? tr.A * beta : tr.A;
      tr.c += upd ? 1u : 0u;
      seen = seen || valid;
    }
    if (seen) tr.c |= 0x80000000u;
    ls[0][w][lane] = tr.xf;
    ls[1][w][lane] = tr.M;
    ls[2][w][lane] = tr.A;
    ls[3][w][lane] = tr.Q0;
    ls[4][w][lane] = tr.Q1;
    ls[5][w][lane] = tr.Q2;
    lc[w][lane] = tr.c;
    __syncthreads();
    // combine: fold the sub-chunks in time order; remember the state entering
    // this wave's sub-chunk; the fold of all of them is the carried state
    double mw = m, vw = v;
    uint32_t nw = n;
    for (int j = 0; j < kTpWaves; ++j) {
      if (j == w) {
        mw = m;
        vw = v;
        nw = n;
      }
      const Transfer tj{ls[0][j][lane], ls[1][j][lane], ls[2][j][lane], ls[3][j][lane],
                        ls[4][j][lane], ls[5][j][lane], lc[j][lane]};
      apply_transfer(tj, alpha, beta, m, v, n);
    }
    // (opaque to the optimiser: keeps it from carrying phase A's 64 f64
    // conversions of x into phase C — 128 extra registers)
#pragma unroll
    for (int u = 0; u < kCap; ++u) asm volatile("" : "+v"(x[u]));
    // phase C: the sequential recurrence from the exact incoming state
    EwmaState st{mw, vw, nw};
    float wmax = 0.f;
    uint32_t wpos = 0;
    float* zp = Z + (tw / W) * S + s;  // this wave's first window row
#pragma unroll
    for (int u = 0; u < kCap; ++u) {
      if ((uint32_t)u < cnt) {
        wmax = fmaxf(wmax, fabsf(ewma_step_bf(st, x[u], alpha, beta, eps)));
        if (++wpos == W) {
          if (sv) *zp = wmax;
          zp += S;
          wpos = 0;
          wmax = 0.f;
        }
      }
    }
    __syncthreads();
  }
  if (w == 0 && sv) {
    gm[s] = m;
    gv[s] = v;
    gn[s] = n;
  }
}

// Synthetic metric matrix: x = mu_s + sigma_s*N(0,1)
// with a +6 sigma level shift on ~0.1 % of series over a random window.
__global__ void series_fill_kernel(float* X, uint64_t T, uint64_t S, uint64_t seed, uint64_t t0,
                                   int tiled) {
  const uint64_t total = tiled ? (T + kTile - 1) / kTile * kTile * S : T * S;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t tl, s;  // step within this matrix, series
    if (tiled) {
      const uint64_t st = (uint64_t)kTile * S;
      const uint64_t r = i % st;
      if constexpr (ANOMOD_EWMA_QMAJOR) {
        tl = i / st * kTile + r / (4 * S) * 4 + r % 4;
        s = r % (4 * S) / 4;
      } else {
        tl = i / st * kTile + r % kTile;
        s = r / kTile;
      }
      if (tl >= T) {
        X[i] = NAN;
        continue;
      }
    } else {
      tl = i / S;
      s = i % S;
    }
    const uint64_t t = tl + t0;
    const uint64_t hs = splitmix64(seed ^ (s * 0x9E3779B97F4A7C15ull));
    const float mu = 10.f + (float)(hs & 1023u);
    const float sigma = 0.5f + (float)((hs >> 10) & 255u) / 32.f;
    uint32_t c[4] = {(uint32_t)t, (uint32_t)(t >> 32), (uint32_t)s, (uint32_t)(s >> 32)};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ 0x7u);
    const float u1 = ((float)(c[0] >> 8) + 0.5f) * (1.0f / 16777216.0f);
    const float u2 = (float)(c[1] >> 8) * (1.0f / 16777216.0f);
    float x = mu + sigma * sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
    if (((hs >> 20) % 1000u) == 0u) {
      const uint64_t start = (hs >> 32) % 1000003ull, len = 2000ull + ((hs >> 52) & 4095u);
      if ((t % 1000003ull) >= start && (t % 1000003ull) < start + len) x += 6.f * sigma;
    }
    X[i] = x;
  }
}

void free_series(anomod_series* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  void* p[] = {s->X, s->Z, s->m, s->v, s->n};
  for (void* q : p)
    if (q) (void)hipFree(q);
  delete s;
}

uint64_t padded_steps(uint64_t T) { return (T + kTile - 1) / kTile * kTile; }
// bytes of X: the tiles plus the prefetch slack
size_t x_bytes(uint64_t T, uint64_t S) { return (padded_steps(T) + kPadTiles * kTile) * S * 4; }

// Which kernel a call runs.  ANOMOD_EWMA_MODE (read per call): 0 auto,
// 1 sequential (tiles), 2 time-parallel (rows), 3 sequential over rows (the
// untiled kernel, kept as the measured comparison).  Auto: one series per
// lane down T while the strips alone fill the chip (>= 4 waves per CU: the
// sequential recurrence does half the arithmetic), the time-parallel form
// when they do not (small S, e.g. one GPU's shard of series).
enum class EwmaKernel { kSeqTiles, kSeqRows, kTimeParallel };

int ewma_mode() {
  const char* e = getenv("ANOMOD_EWMA_MODE");
  return e ? atoi(e) : 0;
}

EwmaKernel pick_kernel(const anomod_ctx* ctx, uint64_t S, uint32_t W, int mode) {
  const uint64_t strips = (S + 63) / 64;
  if (mode == 3) return EwmaKernel::kSeqRows;
  if (W <= 128 && (mode == 2 || (mode == 0 && strips < 4ull * (uint64_t)ctx->num_cus)))
    return EwmaKernel::kTimeParallel;
  return EwmaKernel::kSeqTiles;
}

// Re-lay X out in place of itself (through a temporary of the same size).
int relayout(anomod_ctx* ctx, anomod_series* ser, bool to_tiles) {
  if (ser->tiled == to_tiles) return ANOMOD_OK;
  const size_t bytes = x_bytes(ser->T, ser->S);
  float* tmp = nullptr;
  if (hipMalloc(&tmp, bytes) != hipSuccess) {
    set_error(ctx, "hipMalloc(%zu) to re-lay out the series matrix failed", bytes);
    return ANOMOD_ENOMEM;
  }
  hipLaunchKernelGGL(series_relayout_kernel, dim3(ctx->num_cus * 8), dim3(256), 0, ctx->stream,
                     ser->X, tmp, ser->T, ser->S, 0ull, ser->T, to_tiles ? 1 : 0);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    (void)hipFree(tmp);
    set_error(ctx, "series re-layout failed: %s", hipGetErrorString(e));
    return ANOMOD_EHIP;
  }
  (void)hipFree(ser->X);
  ser->X = tmp;
  ser->tiled = to_tiles;
  return ANOMOD_OK;
}

// Steps per launch of the sequential tiled kernel (ANOMOD_EWMA_SEG, 0 = one
// launch for the whole T).
uint64_t ewma_seg_steps() {
  const char* e = getenv("ANOMOD_EWMA_SEG");
  return e ? strtoull(e, nullptr, 10) : 16384ull;
}

}  // namespace
}  // namespace anomod

using namespace anomod;

extern "C" {

int anomod_series_create(anomod_ctx* ctx, uint64_t T, uint64_t S, anomod_series** out) {
  ANOMOD_REQUIRE(nullptr, ctx && out, "anomod_series_create: NULL argument");
  *out = nullptr;
  ANOMOD_REQUIRE(ctx, S >= 1 && T >= 1, "series matrix must be non-empty (T=%llu S=%llu)",
                 (unsigned long long)T, (unsigned long long)S);
  if (int rc = bind(ctx)) return rc;
  auto* s = new anomod_series();
  s->device = ctx->device;
  s->T = T;
  s->S = S;
  s->tiled = pick_kernel(ctx, S, 1, ewma_mode()) != EwmaKernel::kTimeParallel &&
             ewma_mode() != 3;
  bool ok = hipMalloc(&s->X, x_bytes(T, S)) == hipSuccess;
  ok = ok && hipMalloc(&s->m, S * 8) == hipSuccess;
  ok = ok && hipMalloc(&s->v, S * 8) == hipSuccess;
  ok = ok && hipMalloc(&s->n, S * 4) == hipSuccess;
  if (!ok) {
    free_series(s);
    set_error(ctx, "hipMalloc failed for a %llu x %llu series matrix", (unsigned long long)T,
              (unsigned long long)S);
    return ANOMOD_ENOMEM;
  }
  ANOMOD_HIP(ctx, hipMemsetAsync(s->m, 0, S * 8, ctx->stream));
  ANOMOD_HIP(ctx, hipMemsetAsync(s->v, 0, S * 8, ctx->stream));
  ANOMOD_HIP(ctx, hipMemsetAsync(s->n, 0, S * 4, ctx->stream));
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  *out = s;
  return ANOMOD_OK;
}

int anomod_series_upload(anomod_ctx* ctx, anomod_series* ser, const float* X) {
  ANOMOD_REQUIRE(nullptr, ctx && ser && X, "anomod_series_upload: NULL argument");
  if (int rc = bind(ctx)) return rc;
  if (!ser->tiled) {
    ANOMOD_HIP(ctx, hipMemcpyAsync(ser->X, X, ser->T * ser->S * 4, hipMemcpyHostToDevice,
                                   ctx->stream));
    ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return ANOMOD_OK;
  }
  // tiles: stage up to ~256 MiB of rows (a multiple of 16) at a time and tile
  // them on the device
  const uint64_t T = ser->T, S = ser->S;
  uint64_t R = ((256ull << 20) / (S * 4)) / kTile * kTile;
  if (R < (uint64_t)kTile) R = kTile;
  if (R > padded_steps(T)) R = padded_steps(T);
  float* stage = nullptr;
  if (hipMalloc(&stage, R * S * 4) != hipSuccess) {
    set_error(ctx, "hipMalloc(%llu) for the upload staging buffer failed",
              (unsigned long long)(R * S * 4));
    return ANOMOD_ENOMEM;
  }
  hipError_t e = hipSuccess;
  for (uint64_t r0 = 0; r0 < T && e == hipSuccess; r0 += R) {
    const uint64_t rows = T - r0 < R ? T - r0 : R;
    e = hipMemcpyAsync(stage, X + r0 * S, rows * S * 4, hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) break;
    hipLaunchKernelGGL(series_relayout_kernel, dim3(ctx->num_cus * 8), dim3(256), 0, ctx->stream,
                       stage, ser->X, T, S, r0, rows, 1);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  (void)hipFree(stage);
  if (e != hipSuccess) {
    set_error(ctx, "series upload failed: %s", hipGetErrorString(e));
    return ANOMOD_EHIP;
  }
  return ANOMOD_OK;
}

int anomod_series_download(anomod_ctx* ctx, const anomod_series* ser, float* X) {
  ANOMOD_REQUIRE(nullptr, ctx && ser && X, "anomod_series_download: NULL argument");
  if (int rc = bind(ctx)) return rc;
  const uint64_t T = ser->T, S = ser->S;
  if (!ser->tiled) {
    ANOMOD_HIP(ctx, hipMemcpyAsync(X, ser->X, T * S * 4, hipMemcpyDeviceToHost, ctx->stream));
    ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return ANOMOD_OK;
  }
  // tiles -> rows on the device, up to ~256 MiB of rows (whole tiles) at a time
  uint64_t R = ((256ull << 20) / (S * 4)) / kTile * kTile;
  if (R < (uint64_t)kTile) R = kTile;
  if (R > padded_steps(T)) R = padded_steps(T);
  float* stage = nullptr;
  if (hipMalloc(&stage, R * S * 4) != hipSuccess) {
    set_error(ctx, "hipMalloc(%llu) for the download staging buffer failed",
              (unsigned long long)(R * S * 4));
    return ANOMOD_ENOMEM;
  }
  hipError_t e = hipSuccess;
  for (uint64_t r0 = 0; r0 < T && e == hipSuccess; r0 += R) {
    const uint64_t rows = T - r0 < R ? T - r0 : R;
    hipLaunchKernelGGL(series_relayout_kernel, dim3(ctx->num_cus * 8), dim3(256), 0, ctx->stream,
                       ser->X, stage, T, S, r0, rows, 0);
    e = hipGetLastError();
    if (e == hipSuccess)
      e = hipMemcpyAsync(X + r0 * S, stage, rows * S * 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  }
  (void)hipFree(stage);
  if (e != hipSuccess) {
    set_error(ctx, "series download failed: %s", hipGetErrorString(e));
    return ANOMOD_EHIP;
  }
  return ANOMOD_OK;
}

int anomod_series_fill_synthetic(anomod_ctx* ctx, anomod_series* ser, uint64_t seed,
                                 uint64_t t0) {
  ANOMOD_REQUIRE(nullptr, ctx && ser, "anomod_series_fill_synthetic: NULL argument");
  if (int rc = bind(ctx)) return rc;
  hipLaunchKernelGGL(series_fill_kernel, dim3(ctx->num_cus * 8), dim3(256), 0, ctx->stream,
                     ser->X, ser->T, ser->S, seed, t0, ser->tiled ? 1 : 0);
  ANOMOD_HIP(ctx, hipGetLastError());
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ANOMOD_OK;
}

int anomod_series_reset_state(anomod_ctx* ctx, anomod_series* ser) {
  ANOMOD_REQUIRE(nullptr, ctx && ser, "anomod_series_reset_state: NULL argument");
  if (int rc = bind(ctx)) return rc;
  ANOMOD_HIP(ctx, hipMemsetAsync(ser->m, 0, ser->S * 8, ctx->stream));
  ANOMOD_HIP(ctx, hipMemsetAsync(ser->v, 0, ser->S * 8, ctx->stream));
  ANOMOD_HIP(ctx, hipMemsetAsync(ser->n, 0, ser->S * 4, ctx->stream));
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ANOMOD_OK;
}

int anomod_series_ewma_z(anomod_ctx* ctx, anomod_series* ser, float alpha, uint32_t W, float eps,
                         float* Z_host) {
  ANOMOD_REQUIRE(nullptr, ctx && ser, "anomod_series_ewma_z: NULL argument");
  ANOMOD_REQUIRE(ctx, W >= 1 && ser->T % W == 0, "T=%llu must be a multiple of W=%u",
                 (unsigned long long)ser->T, W);
  ANOMOD_REQUIRE(ctx, alpha > 0.f && alpha <= 1.f, "alpha=%g outside (0, 1]", (double)alpha);
  ANOMOD_REQUIRE(ctx, eps >= 0.f, "eps must be >= 0");
  if (int rc = bind(ctx)) return rc;
  const uint64_t nw = ser->T / W;
  const size_t zbytes = nw * ser->S * 4;
  if (ser->z_cap < zbytes) {
    if (ser->Z) ANOMOD_HIP(ctx, hipFree(ser->Z));
    ser->Z = nullptr;
    ser->z_cap = 0;
    if (hipMalloc(&ser->Z, zbytes) != hipSuccess) {
      set_error(ctx, "hipMalloc(%zu) for window scores failed", zbytes);
      return ANOMOD_ENOMEM;
    }
    ser->z_cap = zbytes;
  }
  const EwmaKernel kern = pick_kernel(ctx, ser->S, W, ewma_mode());
  if (int rc = relayout(ctx, ser, kern == EwmaKernel::kSeqTiles)) return rc;
  if (int rc = stage_begin(ctx, kStageEwma)) return rc;
  const unsigned strips = (unsigned)((ser->S + 63) / 64);
  if (kern == EwmaKernel::kTimeParallel) {
    // time-parallel: U = the most whole windows that fit the register block
    const uint32_t cap = W <= 64 ? 64u : 128u;
    const uint32_t U = W * (cap / W);
    if (cap == 64)
      hipLaunchKernelGGL(ewma_tp_kernel<64>, dim3(strips), dim3(kTpThreads), 0, ctx->stream,
                         ser->X, ser->T, ser->S, (double)alpha, W, U, eps, ser->Z, ser->m, ser->v,
                         ser->n);
    else
      hipLaunchKernelGGL(ewma_tp_kernel<128>, dim3(strips), dim3(kTpThreads), 0, ctx->stream,
                         ser->X, ser->T, ser->S, (double)alpha, W, U, eps, ser->Z, ser->m, ser->v,
                         ser->n);
  } else if (kern == EwmaKernel::kSeqTiles) {
    // Long T in time segments (state carried through HBM between launches,
    // segment = a multiple of lcm(W, 64) steps so windows and dense blocks
    // line up): one lane walks its series sequentially and the waves drift
    // apart over a long launch; measured at S = 10^5: 4.9-5.0 TB/s for
    // T = 32 760 against 3.7-4.6 TB/s for T = 131 040 in one launch.
    uint64_t l = 64;
    while (l % W) l += 64;  // lcm(W, 64)
    const uint64_t seg_env = ewma_seg_steps();
    const uint64_t seg = seg_env ? std::max<uint64_t>(l, seg_env / l * l) : ser->T;
    for (uint64_t t0 = 0; t0 < ser->T; t0 += seg) {
      const uint64_t Ts = std::min<uint64_t>(seg, ser->T - t0);
      hipLaunchKernelGGL((W % 4 == 0 && kEwmaChk == 4 ? ewma_zt_kernel<kZtTiles, 4>
                                                       : ewma_zt_kernel<kZtTiles, 1>),
                         dim3(strips), dim3(64), 0, ctx->stream,
                         ser->X + t0 / kTile * ser->S * kTile, Ts, ser->S, (double)alpha, W, eps,
                         ser->Z + t0 / W * ser->S, ser->m, ser->v, ser->n);
    }
  } else {
    hipLaunchKernelGGL(ewma_z_kernel, dim3(strips), dim3(64), 0, ctx->stream, ser->X, ser->T,
                       ser->S, (double)alpha, W, eps, ser->Z, ser->m, ser->v, ser->n);
  }
  ANOMOD_HIP(ctx, hipGetLastError());
  if (int rc = stage_end(ctx, kStageEwma)) return rc;
  if (Z_host)
    ANOMOD_HIP(ctx, hipMemcpyAsync(Z_host, ser->Z, zbytes, hipMemcpyDeviceToHost, ctx->stream));
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ANOMOD_OK;
}

int anomod_series_free(anomod_series* ser) {
  free_series(ser);
  return ANOMOD_OK;
}

int anomod_ewma_z(anomod_ctx* ctx, const float* X, uint64_t T, uint64_t S, float alpha,
                  uint32_t W, float eps, float* Z) {
  ANOMOD_REQUIRE(nullptr, ctx && X && Z, "anomod_ewma_z: NULL argument");
  ANOMOD_REQUIRE(ctx, W >= 1 && T % W == 0, "T=%llu must be a multiple of W=%u",
                 (unsigned long long)T, W);
  if (T == 0 || S == 0) return ANOMOD_OK;
  if (int rc = bind(ctx)) return rc;
  // X may exceed HBM (config 4: 10^5 series x 10^6 steps = 400 GB on a
  // 288 GB GPU): stream it through one device series in chunks of Tc steps
  // with the (m, v, n) state carried — Tc a multiple of 16 (tiles) and of the
  // time-parallel sub-chunk U (a multiple of W), so the chunked scores equal
  // the one-pass scores bit for bit.
  const uint32_t cap = W <= 64 ? 64u : 128u;
  const uint64_t U = W <= 128 ? (uint64_t)W * (cap / W) : (uint64_t)W;
  uint64_t q = U;
  while (q % kTile) q += U;  // lcm(U, 16)
  size_t free_b = 0, total_b = 0;
  ANOMOD_HIP(ctx, hipMemGetInfo(&free_b, &total_b));
  // X, a possible re-layout copy of X and the window scores must fit, plus
  // 2 GiB for the upload staging and everything else
  const double per_step = (double)S * 4.0 * 2.0 + (double)S * 4.0 / W;
  const double avail = (double)free_b - (double)(2ull << 30);
  uint64_t Tc = avail > per_step * q ? (uint64_t)(avail / per_step) / q * q : q;
  if (const char* e = getenv("ANOMOD_EWMA_CHUNK_STEPS")) {  // tests: force chunking
    const unsigned long long f = strtoull(e, nullptr, 10);
    if (f > 0) Tc = ((f + q - 1) / q) * q;
  }
  if (Tc >= T) Tc = T;
  anomod_series* ser = nullptr;
  if (int rc = anomod_series_create(ctx, Tc, S, &ser)) return rc;
  int rc = ANOMOD_OK;
  for (uint64_t t0 = 0; t0 < T && rc == ANOMOD_OK; t0 += Tc) {
    ser->T = T - t0 < Tc ? T - t0 : Tc;  // the last chunk reuses the allocation
    rc = anomod_series_upload(ctx, ser, X + t0 * S);
    if (rc == ANOMOD_OK) rc = anomod_series_ewma_z(ctx, ser, alpha, W, eps, Z + (t0 / W) * S);
  }
  free_series(ser);
  return rc;
}

}  // extern "C"
