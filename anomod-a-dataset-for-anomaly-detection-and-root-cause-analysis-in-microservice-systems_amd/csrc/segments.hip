// Segment summary: the per-service / per-endpoint
// call counts, error count, latency min/max/sum/count and start-time range of
// TT_collection-scripts/T-Dataset/enhanced_trace_collector.py
// analyze_trace_patterns (:216-296), as one pass over columnar segment
// records (service id, endpoint id, is_error, latency, start_time):
//   service_call_counts[s]   += 1                         (:246-248)
//   endpoint_call_counts[e]  += 1                         (:251-253)
//   error_traces             += is_error == 1             (:256-257)
//   latency min/max/sum/count over latency > 0            (:260-262, 277-283)
//   time_range min/max over start_time != 0               (:265-270)
// HBM-bound: 4 + 4 + 4 + 8 + 8 = 28 B per segment read once.  Counters are
// privatised per workgroup in LDS (ids < 4096) and flushed with integer
// atomics; the scalars are reduced per wave and merged with one atomic each
// per workgroup — integer adds / min / max, so the result is exact.
#include <climits>

#include "common.h"

namespace anomod {
namespace {

constexpr int kSegThreads = 1024;
constexpr uint32_t kLdsIds = 4096;

struct SegScalars {
  unsigned long long errors, lat_count, start_count;
  long long lat_sum, lat_min, lat_max, start_min, start_max;
};

__device__ __forceinline__ long long wave_sum(long long v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ __forceinline__ long long wave_min(long long v) {
  for (int off = 32; off > 0; off >>= 1) v = min(v, (long long)__shfl_xor(v, off));
  return v;
}
__device__ __forceinline__ long long wave_max(long long v) {
  for (int off = 32; off > 0; off >>= 1) v = max(v, (long long)__shfl_xor(v, off));
  return v;
}

template <bool LDS_SVC, bool LDS_EP>
__global__ __launch_bounds__(kSegThreads) void segment_summary_kernel(
    const uint32_t* __restrict__ svc, const uint32_t* __restrict__ ep,
    const int32_t* __restrict__ is_error, const int64_t* __restrict__ latency,
    const int64_t* __restrict__ start, uint64_t n, uint32_t n_svc, uint32_t n_ep,
    unsigned long long* __restrict__ svc_count, unsigned long long* __restrict__ ep_count,
    SegScalars* __restrict__ out) {
  __shared__ uint32_t lsvc[LDS_SVC ? kLdsIds : 1];
  __shared__ uint32_t lep[LDS_EP ? kLdsIds : 1];
  const int tid = threadIdx.x;
  if constexpr (LDS_SVC)
    for (uint32_t i = tid; i < n_svc; i += kSegThreads) lsvc[i] = 0u;
  if constexpr (LDS_EP)
    for (uint32_t i = tid; i < n_ep; i += kSegThreads) lep[i] = 0u;
  __syncthreads();
  long long errors = 0, lat_count = 0, lat_sum = 0, start_count = 0;
  long long lat_min = LLONG_MAX, lat_max = LLONG_MIN, st_min = LLONG_MAX, st_max = LLONG_MIN;
  for (uint64_t i = (uint64_t)blockIdx.x * kSegThreads + tid; i < n;
       i += (uint64_t)gridDim.x * kSegThreads) {
    const uint32_t s = svc[i], e = ep[i];
    const int32_t er = is_error[i];
    const long long lat = latency[i], st = start[i];
    if constexpr (LDS_SVC) atomicAdd(&lsvc[s], 1u);
    else atomicAdd(&svc_count[s], 1ull);
    if constexpr (LDS_EP) atomicAdd(&lep[e], 1u);
    else atomicAdd(&ep_count[e], 1ull);
    errors += er == 1;
    if (lat > 0) {
      ++lat_count;
      lat_sum += lat;
      lat_min = min(lat_min, lat);
      lat_max = max(lat_max, lat);
    }
    if (st != 0) {
      ++start_count;
      st_min = min(st_min, st);
      st_max = max(st_max, st);
    }
  }
  errors = wave_sum(errors);
  lat_count = wave_sum(lat_count);
  lat_sum = wave_sum(lat_sum);
  start_count = wave_sum(start_count);
  lat_min = wave_min(lat_min);
  lat_max = wave_max(lat_max);
  st_min = wave_min(st_min);
  st_max = wave_max(st_max);
  if ((tid & 63) == 0) {
    if (errors) atomicAdd(&out->errors, (unsigned long long)errors);
    if (lat_count) {
      atomicAdd(&out->lat_count, (unsigned long long)lat_count);
      atomicAdd(reinterpret_cast<unsigned long long*>(&out->lat_sum),
                (unsigned long long)lat_sum);  // two's-complement add
      atomicMin(&out->lat_min, lat_min);
      atomicMax(&out->lat_max, lat_max);
    }
    if (start_count) {
      atomicAdd(&out->start_count, (unsigned long long)start_count);
      atomicMin(&out->start_min, st_min);
      atomicMax(&out->start_max, st_max);
    }
  }
  __syncthreads();
  if constexpr (LDS_SVC)
    for (uint32_t i = tid; i < n_svc; i += kSegThreads)
      if (lsvc[i]) atomicAdd(&svc_count[i], (unsigned long long)lsvc[i]);
  if constexpr (LDS_EP)
    for (uint32_t i = tid; i < n_ep; i += kSegThreads)
      if (lep[i]) atomicAdd(&ep_count[i], (unsigned long long)lep[i]);
}

using SegFn = void (*)(const uint32_t*, const uint32_t*, const int32_t*, const int64_t*,
                       const int64_t*, uint64_t, uint32_t, uint32_t, unsigned long long*,
                       unsigned long long*, SegScalars*);

SegFn pick_segment_kernel(uint32_t n_svc, uint32_t n_ep) {
  const bool a = n_svc <= kLdsIds, b = n_ep <= kLdsIds;
  if (a && b) return segment_summary_kernel<true, true>;
  if (a) return segment_summary_kernel<true, false>;
  if (b) return segment_summary_kernel<false, true>;
  return segment_summary_kernel<false, false>;
}

}  // namespace
}  // namespace anomod

using namespace anomod;

extern "C" {

int anomod_segment_summary(anomod_ctx* ctx, const uint32_t* svc, const uint32_t* endpoint,
                           const int32_t* is_error, const int64_t* latency,
                           const int64_t* start_time, uint64_t n, anomod_segment_summary_out* out) {
  ANOMOD_REQUIRE(nullptr, ctx && out, "anomod_segment_summary: NULL argument");
  ANOMOD_REQUIRE(ctx, n == 0 || (svc && endpoint && is_error && latency && start_time),
                 "anomod_segment_summary: NULL column");
  ANOMOD_REQUIRE(ctx, out->n_services >= 1 && out->n_endpoints >= 1,
                 "n_services and n_endpoints must be >= 1");
  for (uint64_t i = 0; i < n; ++i) {
    ANOMOD_REQUIRE(ctx, svc[i] < out->n_services, "service id %u >= n_services %u", svc[i],
                   out->n_services);
    ANOMOD_REQUIRE(ctx, endpoint[i] < out->n_endpoints, "endpoint id %u >= n_endpoints %u",
                   endpoint[i], out->n_endpoints);
  }
  if (int rc = bind(ctx)) return rc;
  const uint32_t ns = out->n_services, ne = out->n_endpoints;
  // device layout: columns | svc counts | ep counts | scalars
  const size_t off_ep = n * 4, off_er = 2 * n * 4, off_lat = (3 * n * 4 + 7) & ~(size_t)7;
  const size_t off_st = off_lat + n * 8, off_sc = off_st + n * 8, off_ec = off_sc + ns * 8ull;
  const size_t off_out = off_ec + ne * 8ull, bytes = off_out + sizeof(SegScalars);
  char* d = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess) {
    set_error(ctx, "hipMalloc(%zu) for the segment summary failed", bytes);
    return ANOMOD_ENOMEM;
  }
  SegScalars init{0, 0, 0, 0, LLONG_MAX, LLONG_MIN, LLONG_MAX, LLONG_MIN};
  SegScalars res{};
  hipError_t e = hipSuccess;
  auto h2d = [&](size_t off, const void* src, size_t nb) {
    if (e == hipSuccess && nb) e = hipMemcpyAsync(d + off, src, nb, hipMemcpyHostToDevice,
                                                  ctx->stream);
  };
  h2d(0, svc, n * 4);
  h2d(off_ep, endpoint, n * 4);
  h2d(off_er, is_error, n * 4);
  h2d(off_lat, latency, n * 8);
  h2d(off_st, start_time, n * 8);
  h2d(off_out, &init, sizeof(init));
  if (e == hipSuccess) e = hipMemsetAsync(d + off_sc, 0, (ns + ne) * 8ull, ctx->stream);
  int rc = ANOMOD_OK;
  if (e == hipSuccess) rc = stage_begin(ctx, kStageSegments);
  if (e == hipSuccess && rc == ANOMOD_OK && n > 0) {
    const uint64_t want = (n + kSegThreads - 1) / kSegThreads;
    const uint64_t cap = (uint64_t)ctx->num_cus * 2;
    const unsigned grid = (unsigned)(want < cap ? want : cap);
    hipLaunchKernelGGL(pick_segment_kernel(ns, ne), dim3(grid), dim3(kSegThreads), 0, ctx->stream,
                       reinterpret_cast<const uint32_t*>(d),
                       reinterpret_cast<const uint32_t*>(d + off_ep),
                       reinterpret_cast<const int32_t*>(d + off_er),
                       reinterpret_cast<const int64_t*>(d + off_lat),
                       reinterpret_cast<const int64_t*>(d + off_st), n, ns, ne,
                       reinterpret_cast<unsigned long long*>(d + off_sc),
                       reinterpret_cast<unsigned long long*>(d + off_ec),
                       reinterpret_cast<SegScalars*>(d + off_out));
    e = hipGetLastError();
  }
  if (e == hipSuccess && rc == ANOMOD_OK) rc = stage_end(ctx, kStageSegments);
  if (e == hipSuccess && rc == ANOMOD_OK && out->service_counts)
    e = hipMemcpyAsync(out->service_counts, d + off_sc, ns * 8ull, hipMemcpyDeviceToHost,
                       ctx->stream);
  if (e == hipSuccess && rc == ANOMOD_OK && out->endpoint_counts)
    e = hipMemcpyAsync(out->endpoint_counts, d + off_ec, ne * 8ull, hipMemcpyDeviceToHost,
                       ctx->stream);
  if (e == hipSuccess && rc == ANOMOD_OK)
    e = hipMemcpyAsync(&res, d + off_out, sizeof(res), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess && rc == ANOMOD_OK) e = hipStreamSynchronize(ctx->stream);
  (void)hipFree(d);
  if (rc != ANOMOD_OK) return rc;
  if (e != hipSuccess) {
    set_error(ctx, "segment summary failed: %s", hipGetErrorString(e));
    return ANOMOD_EHIP;
  }
  out->total = n;
  out->error_count = res.errors;
  out->latency_count = res.lat_count;
  out->latency_sum = res.lat_sum;
  out->latency_min = res.lat_count ? res.lat_min : 0;
  out->latency_max = res.lat_count ? res.lat_max : 0;
  out->start_count = res.start_count;
  out->start_min = res.start_count ? res.start_min : 0;
  out->start_max = res.start_count ? res.start_max : 0;
  return ANOMOD_OK;
}

}  // extern "C"
