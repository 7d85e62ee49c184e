// API-response summary (second half): the latency
// statistics and distributions of
//   SN_collection-scripts/Dataset/api_responses/monitor_http_responses.py
//     OpenAPIResponseCollector.generate_summary (:150-207)
//   SN_collection-scripts/Dataset/api_responses/enhanced_openapi_monitor.py
//     EnhancedOpenAPIMonitor.generate_reports (:318-332)
// Both sort the latencies and read nearest-rank order statistics
// (x[n//2], x[int(n*0.95)], x[int(n*0.99)]) plus min / max / sum / count.
//
// Value summary: select (v > 0, generate_summary :167-169; or every non-NaN
// value, generate_reports :324) into order-preserving u64 keys -> the
// hand-written LSD radix sort of radix.hip -> one fixed-order sum over the
// sorted keys -> five gathers.  Order statistics are exact (the sorted values
// themselves); the sum is reproducible run to run and within n * 2^-53
// relative of Python's left-to-right sum.  HBM: the radix sort's passes
// dominate (8 B/key counted + 16 B/key scattered per varying 8-bit digit,
// plus the selection's 8 + 8 + 8 B/value).
// Response summary: the status-code / content-type counts and the error
// count (:163-177) in one pass with LDS-privatised integer counters, plus the
// value summary of the positive latencies.
#include <algorithm>
#include <cmath>

#include "common.h"
#include "radix.h"

namespace anomod {
namespace {

// sorted[0], sorted[c-1] and the three nearest-rank picks (keys -> values)
__global__ void pick_kernel(const uint64_t* __restrict__ sorted, uint64_t c, uint64_t i50,
                            uint64_t i95, uint64_t i99, double* __restrict__ out) {
  if (threadIdx.x == 0) {
    out[0] = key_f64(sorted[0]);
    out[1] = key_f64(sorted[c - 1]);
    out[2] = key_f64(sorted[i50]);
    out[3] = key_f64(sorted[i95]);
    out[4] = key_f64(sorted[i99]);
  }
}

constexpr int kCatThreads = 1024;
constexpr uint32_t kCatLds = 4096;

template <bool LDS_A, bool LDS_B>
__global__ __launch_bounds__(kCatThreads) void category_count_kernel(
    const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
    const uint8_t* __restrict__ flag, uint64_t n, uint32_t na, uint32_t nb,
    unsigned long long* __restrict__ ca, unsigned long long* __restrict__ cb,
    unsigned long long* __restrict__ cflag) {
  __shared__ uint32_t la[LDS_A ? kCatLds : 1];
  __shared__ uint32_t lb[LDS_B ? kCatLds : 1];
  const int tid = threadIdx.x;
  if constexpr (LDS_A)
    for (uint32_t i = tid; i < na; i += kCatThreads) la[i] = 0u;
  if constexpr (LDS_B)
    for (uint32_t i = tid; i < nb; i += kCatThreads) lb[i] = 0u;
  __syncthreads();
  uint32_t flags = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kCatThreads + tid; i < n;
       i += (uint64_t)gridDim.x * kCatThreads) {
    if constexpr (LDS_A) atomicAdd(&la[a[i]], 1u);
    else atomicAdd(&ca[a[i]], 1ull);
    if constexpr (LDS_B) atomicAdd(&lb[b[i]], 1u);
    else atomicAdd(&cb[b[i]], 1ull);
    flags += flag[i] != 0;
  }
  for (int off = 32; off > 0; off >>= 1) flags += __shfl_xor(flags, off);
  if ((tid & 63) == 0 && flags) atomicAdd(cflag, (unsigned long long)flags);
  __syncthreads();
  if constexpr (LDS_A)
    for (uint32_t i = tid; i < na; i += kCatThreads)
      if (la[i]) atomicAdd(&ca[i], (unsigned long long)la[i]);
  if constexpr (LDS_B)
    for (uint32_t i = tid; i < nb; i += kCatThreads)
      if (lb[i]) atomicAdd(&cb[i], (unsigned long long)lb[i]);
}

using CatFn = void (*)(const uint32_t*, const uint32_t*, const uint8_t*, uint64_t, uint32_t,
                       uint32_t, unsigned long long*, unsigned long long*, unsigned long long*);

CatFn pick_category_kernel(uint32_t na, uint32_t nb) {
  const bool x = na <= kCatLds, y = nb <= kCatLds;
  if (x && y) return category_count_kernel<true, true>;
  if (x) return category_count_kernel<true, false>;
  if (y) return category_count_kernel<false, true>;
  return category_count_kernel<false, false>;
}

// Python's int(c * q) for q in {0.95, 0.99}: the f64 product truncated
uint64_t py_rank(uint64_t c, double q) { return (uint64_t)((double)c * q); }

// The value summary of n device values already at `vals` (device scratch
// allocated here).  Runs on ctx->stream.
int value_summary_device(anomod_ctx* ctx, const double* vals, uint64_t n, int positive_only,
                         anomod_value_summary_out* out) {
  *out = anomod_value_summary_out{};
  if (n == 0) return ANOMOD_OK;
  const size_t tb = std::max(radix_temp_bytes(n),
                             std::max(select_temp_bytes(n), sum_temp_bytes(n)));
  const size_t keys_b = (n * 8 + 255) & ~size_t(255);
  const size_t bytes = 2 * keys_b + 256 + tb;
  char* base = nullptr;
  if (hipMalloc(&base, bytes) != hipSuccess) {
    set_error(ctx, "hipMalloc(%zu) for the value summary failed", bytes);
    return ANOMOD_ENOMEM;
  }
  auto* sel = reinterpret_cast<uint64_t*>(base);
  auto* sorted = reinterpret_cast<uint64_t*>(base + keys_b);
  auto* res = reinterpret_cast<double*>(base + 2 * keys_b);  // [0..4] picks, [5] sum
  auto* d_count = reinterpret_cast<unsigned long long*>(res + 6);
  void* temp = base + 2 * keys_b + 256;
  unsigned long long c = 0;
  double h[6] = {0, 0, 0, 0, 0, 0};
  hipError_t e = hipSuccess;
  int rc = stage_begin(ctx, kStageSummary);
  if (rc == ANOMOD_OK) {
    e = select_f64_keys(vals, n, positive_only, sel, d_count, temp, tb, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(&c, d_count, 8, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess && c > 0) {
      e = radix_sort_u64(sel, sorted, c, 0, 64, temp, tb, ctx->stream);
      if (e == hipSuccess) e = sum_keys_f64(sorted, c, res + 5, temp, tb, ctx->stream);
      if (e == hipSuccess) {
        hipLaunchKernelGGL(pick_kernel, dim3(1), dim3(64), 0, ctx->stream, sorted, c, c / 2,
                           py_rank(c, 0.95), py_rank(c, 0.99), res);
        e = hipGetLastError();
      }
    }
    if (e == hipSuccess) rc = stage_end(ctx, kStageSummary);
    if (e == hipSuccess && rc == ANOMOD_OK && c > 0)
      e = hipMemcpyAsync(h, res, 6 * 8, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && rc == ANOMOD_OK) e = hipStreamSynchronize(ctx->stream);
  }
  (void)hipFree(base);
  if (rc != ANOMOD_OK) return rc;
  if (e != hipSuccess) {
    set_error(ctx, "value summary failed: %s", hipGetErrorString(e));
    return ANOMOD_EHIP;
  }
  out->count = c;
  if (c > 0) {
    out->min = h[0];
    out->max = h[1];
    out->median = h[2];
    out->p95 = h[3];
    out->p99 = h[4];
    out->sum = h[5];
  }
  return ANOMOD_OK;
}

}  // namespace
}  // namespace anomod

using namespace anomod;

extern "C" {

int anomod_value_summary(anomod_ctx* ctx, const double* values, uint64_t n, int positive_only,
                         anomod_value_summary_out* out) {
  ANOMOD_REQUIRE(nullptr, ctx && out, "anomod_value_summary: NULL argument");
  ANOMOD_REQUIRE(ctx, n == 0 || values, "anomod_value_summary: NULL values");
  ANOMOD_REQUIRE(ctx, n <= kMaxSortKeys, "anomod_value_summary: at most 2^32 - 4097 values");
  if (int rc = bind(ctx)) return rc;
  *out = anomod_value_summary_out{};
  if (n == 0) return ANOMOD_OK;
  double* d = nullptr;
  if (hipMalloc(&d, n * 8) != hipSuccess) {
    set_error(ctx, "hipMalloc(%llu) for the values failed", (unsigned long long)(n * 8));
    return ANOMOD_ENOMEM;
  }
  int rc = ANOMOD_OK;
  if (hipMemcpyAsync(d, values, n * 8, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) {
    set_error(ctx, "value upload failed");
    rc = ANOMOD_EHIP;
  }
  if (rc == ANOMOD_OK) rc = value_summary_device(ctx, d, n, positive_only, out);
  (void)hipFree(d);
  return rc;
}

int anomod_sort_u64(anomod_ctx* ctx, const uint64_t* keys, uint64_t n, int begin_bit,
                    int end_bit, uint64_t* sorted, int* passes) {
  ANOMOD_REQUIRE(nullptr, ctx, "anomod_sort_u64: NULL context");
  ANOMOD_REQUIRE(ctx, n == 0 || (keys && sorted), "anomod_sort_u64: NULL buffer");
  ANOMOD_REQUIRE(ctx, 0 <= begin_bit && begin_bit <= end_bit && end_bit <= 64,
                 "bit range [%d, %d) outside [0, 64]", begin_bit, end_bit);
  ANOMOD_REQUIRE(ctx, n <= kMaxSortKeys, "anomod_sort_u64: at most 2^32 - 4097 keys");
  if (passes) *passes = 0;
  if (n == 0) return ANOMOD_OK;
  if (int rc = bind(ctx)) return rc;
  const size_t kb = (n * 8 + 255) & ~size_t(255), tb = radix_temp_bytes(n);
  char* d = nullptr;
  if (hipMalloc(&d, kb + tb) != hipSuccess) {
    set_error(ctx, "hipMalloc(%zu) for the sort failed", kb + tb);
    return ANOMOD_ENOMEM;
  }
  auto* k = reinterpret_cast<uint64_t*>(d);
  hipError_t e = hipMemcpyAsync(k, keys, n * 8, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = radix_sort_u64(k, k, n, begin_bit, end_bit, d + kb, tb, ctx->stream,
                                          passes);
  if (e == hipSuccess) e = hipMemcpyAsync(sorted, k, n * 8, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  (void)hipFree(d);
  if (e != hipSuccess) {
    set_error(ctx, "anomod_sort_u64 failed: %s", hipGetErrorString(e));
    return ANOMOD_EHIP;
  }
  return ANOMOD_OK;
}

int anomod_response_summary(anomod_ctx* ctx, const uint32_t* status_id, const uint32_t* ctype_id,
                            const uint8_t* has_error, const double* latency_ms, uint64_t n,
                            anomod_response_summary_out* out) {
  ANOMOD_REQUIRE(nullptr, ctx && out, "anomod_response_summary: NULL argument");
  ANOMOD_REQUIRE(ctx, n == 0 || (status_id && ctype_id && has_error && latency_ms),
                 "anomod_response_summary: NULL column");
  ANOMOD_REQUIRE(ctx, out->n_status >= 1 && out->n_ctype >= 1,
                 "n_status and n_ctype must be >= 1");
  ANOMOD_REQUIRE(ctx, out->status_counts && out->ctype_counts,
                 "anomod_response_summary: NULL count buffers");
  for (uint64_t i = 0; i < n; ++i) {
    ANOMOD_REQUIRE(ctx, status_id[i] < out->n_status, "status id %u >= n_status %u",
                   status_id[i], out->n_status);
    ANOMOD_REQUIRE(ctx, ctype_id[i] < out->n_ctype, "content-type id %u >= n_ctype %u",
                   ctype_id[i], out->n_ctype);
  }
  if (int rc = bind(ctx)) return rc;
  out->error_count = 0;
  out->latency = anomod_value_summary_out{};
  const uint32_t na = out->n_status, nb = out->n_ctype;
  if (n == 0) {
    std::fill(out->status_counts, out->status_counts + na, 0ull);
    std::fill(out->ctype_counts, out->ctype_counts + nb, 0ull);
    return ANOMOD_OK;
  }
  // device layout: latency | status | ctype | error flags | counts
  const size_t off_a = n * 8, off_b = off_a + n * 4, off_f = off_b + n * 4;
  const size_t off_ca = (off_f + n + 7) & ~(size_t)7, off_cb = off_ca + na * 8ull;
  const size_t off_cf = off_cb + nb * 8ull, bytes = off_cf + 8;
  char* d = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess) {
    set_error(ctx, "hipMalloc(%zu) for the response summary failed", bytes);
    return ANOMOD_ENOMEM;
  }
  hipError_t e = hipSuccess;
  auto h2d = [&](size_t off, const void* src, size_t nb_) {
    if (e == hipSuccess) e = hipMemcpyAsync(d + off, src, nb_, hipMemcpyHostToDevice, ctx->stream);
  };
  h2d(0, latency_ms, n * 8);
  h2d(off_a, status_id, n * 4);
  h2d(off_b, ctype_id, n * 4);
  h2d(off_f, has_error, n);
  if (e == hipSuccess) e = hipMemsetAsync(d + off_ca, 0, bytes - off_ca, ctx->stream);
  if (e == hipSuccess) {
    const uint64_t want = (n + kCatThreads - 1) / kCatThreads;
    const uint64_t cap = (uint64_t)ctx->num_cus * 2;
    hipLaunchKernelGGL(pick_category_kernel(na, nb), dim3((unsigned)std::min(want, cap)),
                       dim3(kCatThreads), 0, ctx->stream,
                       reinterpret_cast<const uint32_t*>(d + off_a),
                       reinterpret_cast<const uint32_t*>(d + off_b),
                       reinterpret_cast<const uint8_t*>(d + off_f), n, na, nb,
                       reinterpret_cast<unsigned long long*>(d + off_ca),
                       reinterpret_cast<unsigned long long*>(d + off_cb),
                       reinterpret_cast<unsigned long long*>(d + off_cf));
    e = hipGetLastError();
  }
  int rc = ANOMOD_OK;
  if (e == hipSuccess)
    rc = value_summary_device(ctx, reinterpret_cast<const double*>(d), n, 1, &out->latency);
  if (rc == ANOMOD_OK && e == hipSuccess)
    e = hipMemcpyAsync(out->status_counts, d + off_ca, na * 8ull, hipMemcpyDeviceToHost,
                       ctx->stream);
  if (rc == ANOMOD_OK && e == hipSuccess)
    e = hipMemcpyAsync(out->ctype_counts, d + off_cb, nb * 8ull, hipMemcpyDeviceToHost,
                       ctx->stream);
  if (rc == ANOMOD_OK && e == hipSuccess)
    e = hipMemcpyAsync(&out->error_count, d + off_cf, 8, hipMemcpyDeviceToHost, ctx->stream);
  if (rc == ANOMOD_OK && e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  (void)hipFree(d);
  if (rc != ANOMOD_OK) return rc;
  if (e != hipSuccess) {
    set_error(ctx, "response summary failed: %s", hipGetErrorString(e));
    return ANOMOD_EHIP;
  }
  return ANOMOD_OK;
}

}  // extern "C"
