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
// fixed-iteration loop is captured once into a hipGraph and replayed.
#include <algorithm>
#include <cmath>
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
  // cached fixed-iteration graph
  hipGraphExec_t exec = nullptr;
  uint32_t exec_iters = 0;
  double exec_alpha = 0.0;
};

namespace anomod {
namespace {

constexpr int kPprThreads = 256;
constexpr int kRowsPerBlock = kPprThreads;  // one row per lane
constexpr int kEdgeBatch = 8;              // in-edge loads issued together per lane
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

__global__ __launch_bounds__(kPprThreads) void ppr_init_kernel(uint32_t N, double x0,
                                                               double* __restrict__ x) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x)
    x[i] = x0;
}

// One power iteration x_in -> x_out.  Eight lanes per row pull the in-edges.
// The block's share of the new vector's dangling mass and of |x_out - x_in|
// is rounded to 64-bit fixed point and added with one integer atomic each:
// integer adds commute, so the next launch reads a bit-reproducible scalar
// without a reduction kernel or an inter-block hand-off.
__global__ __launch_bounds__(kPprThreads) void ppr_iter_kernel(
    uint32_t N, const uint32_t* __restrict__ in_ptr, const uint32_t* __restrict__ in_col,
    const float* __restrict__ in_w, const uint8_t* __restrict__ dangling,
    const double* __restrict__ p, double alpha, const double* __restrict__ x_in,
    double* __restrict__ x_out, const unsigned long long* __restrict__ d_in,
    unsigned long long* d_out, unsigned long long* d_zero, unsigned long long* e_out,
    unsigned long long* e_zero) {
  __shared__ double red[kPprThreads / 64];
  __shared__ double s_dsum;
  const uint32_t r = blockIdx.x * kRowsPerBlock + threadIdx.x;
  double acc = 0.0;
  if (r < N) {
    const uint32_t b = in_ptr[r], e = in_ptr[r + 1];
    // In-degrees are short (uniform callees): one lane per row, kEdgeBatch
    // (col, w) pairs loaded together, then the x gathers together.
    for (uint32_t k0 = b; k0 < e; k0 += kEdgeBatch) {
      uint32_t c[kEdgeBatch];
      float wv[kEdgeBatch];
#pragma unroll
      for (int j = 0; j < kEdgeBatch; ++j) {
        const bool ok = k0 + j < e;
        c[j] = ok ? in_col[k0 + j] : 0u;
        wv[j] = ok ? in_w[k0 + j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < kEdgeBatch; ++j)
        if (k0 + j < e) acc += x_in[c[j]] * (double)wv[j];
    }
  }
  // Dangling mass of x_in: wave 0 folds the fixed-point slots (exact).
  if (threadIdx.x < 64) {
    unsigned long long v = d_in[threadIdx.x];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (threadIdx.x == 0) s_dsum = (double)v * (1.0 / kDScale);
  }
  __syncthreads();
  const double dsum = s_dsum;
  double dacc = 0.0, eacc = 0.0;
  if (r < N) {
    const double pr = p[r];
    const double y = alpha * (acc + dsum * pr) + (1.0 - alpha) * pr;
    x_out[r] = y;
    if (dangling[r]) dacc = y;
    eacc = fabs(y - x_in[r]);
  }
  const double ds = block_sum(dacc, red);
  const double es = block_sum(eacc, red);
  if (threadIdx.x == 0) {
    const int slot = blockIdx.x & (kAccSlots - 1);
    atomicAdd(&d_out[slot], __double2ull_rn(ds * kDScale));
    atomicAdd(&e_out[slot], __double2ull_rn(es * kEScale));
  }
  if (blockIdx.x == 0 && threadIdx.x < kAccSlots) {
    d_zero[threadIdx.x] = 0ull;
    e_zero[threadIdx.x] = 0ull;
  }
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
        c[j] = ok ? in_col[k0 + j] : 0u;
        wv[j] = ok ? in_w[k0 + j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < kEdgeBatch; ++j) {
        if (k0 + j < e) {
          const double* xr = x_in + (uint64_t)c[j] * K;
#pragma unroll
          for (int k = 0; k < K; ++k) acc[k] += xr[k] * (double)wv[j];
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
                                           : alpha * (acc[k] + s_dsum[k] * pr) + (1.0 - alpha) * pr;
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

void free_graph(anomod_graph* g) {
  if (!g) return;
  (void)hipSetDevice(g->device);
  if (g->exec) (void)hipGraphExecDestroy(g->exec);
  void* ps[] = {g->in_ptr, g->in_col, g->in_w, g->dangling, g->p,  g->x[0],
                g->x[1],   g->acc,    g->bp,   g->bx[0],    g->bx[1], g->bacc};
  for (void* q : ps)
    if (q) (void)hipFree(q);
  delete g;
}

// Launch iteration `it` (x[it&1] -> x[(it+1)&1]).
void launch_iter(anomod_ctx* ctx, anomod_graph* g, double alpha, uint32_t it) {
  const int a = it & 1, b = a ^ 1;
  const int r = it % 3, w = (it + 1) % 3, z = (it + 2) % 3;
  unsigned long long* A = g->acc;
  const int S = kAccSlots;
  hipLaunchKernelGGL(ppr_iter_kernel, dim3(g->grid), dim3(kPprThreads), 0, ctx->stream, g->N,
                     g->in_ptr, g->in_col, g->in_w, g->dangling, g->p, alpha, g->x[a], g->x[b],
                     A + r * S, A + w * S, A + z * S, A + (3 + w) * S, A + (3 + z) * S);
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
  ok = ok && hipMalloc(&g->acc, 6 * kAccSlots * 8) == hipSuccess;
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

int anomod_graph_synthetic(anomod_ctx* ctx, uint32_t N, uint32_t mean_degree, uint64_t seed,
                           anomod_graph** out) {
  ANOMOD_REQUIRE(nullptr, ctx && out, "anomod_graph_synthetic: NULL argument");
  ANOMOD_REQUIRE(ctx, N >= 2 && mean_degree >= 1, "need N >= 2 and mean_degree >= 1");
  // Power-law (Pareto, a = 2.2) out-degrees scaled to the requested mean,
  // 2 % dangling nodes, uniform callees, call-count weights in [1, 1000].
  std::vector<uint32_t> row_ptr(N + 1, 0), col;
  std::vector<float> w;
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
  return anomod_graph_create(ctx, row_ptr.data(), col.data(), w.data(), N, out);
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
  double psum = 0.0;
  for (uint32_t i = 0; i < N; ++i) {
    ANOMOD_REQUIRE(ctx, std::isfinite(p[i]) && p[i] >= 0.0, "personalization[%u] invalid", i);
    psum += p[i];
  }
  ANOMOD_REQUIRE(ctx, psum > 0.0, "personalization sums to zero");
  std::vector<double> pn(p, p + N);
  for (double& v : pn) v /= psum;
  if (int rc = bind(ctx)) return rc;
  ANOMOD_HIP(ctx, hipMemcpyAsync(g->p, pn.data(), N * 8ull, hipMemcpyHostToDevice, ctx->stream));
  // x0 = 1/N; its dangling mass n_dangling/N seeds iteration 0 (slot 0); the
  // slots iteration 0 adds into must start at zero.
  for (unsigned long long& v : g->host_acc) v = 0ull;
  g->host_acc[0] = (unsigned long long)std::llround((double)g->n_dangling / N * kDScale);
  ANOMOD_HIP(ctx, hipMemcpyAsync(g->acc, g->host_acc.data(), g->host_acc.size() * 8,
                                 hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(ppr_init_kernel, dim3(std::min<uint32_t>(g->grid, 1024)), dim3(kPprThreads),
                     0, ctx->stream, N, 1.0 / N, g->x[0]);
  ANOMOD_HIP(ctx, hipGetLastError());
  uint32_t done = 0;
  if (int rc = stage_begin(ctx, kStagePagerank)) return rc;
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
  }
  if (int rc = stage_end(ctx, kStagePagerank)) return rc;
  ANOMOD_HIP(ctx, hipMemcpyAsync(x_out, g->x[done & 1], N * 8ull, hipMemcpyDeviceToHost,
                                 ctx->stream));
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (iters_done) *iters_done = done;
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
  std::vector<double> pn((size_t)N * kb);
  for (uint32_t k = 0; k < kb; ++k) {
    const double* pk = P + (size_t)(k < K ? k : 0) * N;
    double s = 0.0;
    for (uint32_t i = 0; i < N; ++i) {
      ANOMOD_REQUIRE(ctx, std::isfinite(pk[i]) && pk[i] >= 0.0,
                     "personalization[%u][%u] invalid", k, i);
      s += pk[i];
    }
    ANOMOD_REQUIRE(ctx, s > 0.0, "personalization %u sums to zero", k);
    for (uint32_t i = 0; i < N; ++i) pn[(size_t)i * kb + k] = pk[i] / s;
  }
  if (int rc = bind(ctx)) return rc;
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
  ANOMOD_HIP(ctx, hipMemcpyAsync(g->bp, pn.data(), pn.size() * 8, hipMemcpyHostToDevice,
                                 ctx->stream));
  std::vector<double> x0((size_t)N * kb, 1.0 / N);
  ANOMOD_HIP(ctx, hipMemcpyAsync(g->bx[0], x0.data(), x0.size() * 8, hipMemcpyHostToDevice,
                                 ctx->stream));
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
  if (int rc = stage_begin(ctx, kStagePagerank)) return rc;
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
  if (int rc = stage_end(ctx, kStagePagerank)) return rc;
  std::vector<double> xs((size_t)N * kb);
  ANOMOD_HIP(ctx, hipMemcpyAsync(xs.data(), g->bx[done & 1], xs.size() * 8, hipMemcpyDeviceToHost,
                                 ctx->stream));
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  for (uint32_t k = 0; k < K; ++k)
    for (uint32_t i = 0; i < N; ++i) X[(size_t)k * N + i] = xs[(size_t)i * kb + k];
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
