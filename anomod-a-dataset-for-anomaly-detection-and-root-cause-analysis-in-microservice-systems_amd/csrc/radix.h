// Hand-written device sort / compaction / sum primitives (CDNA4), used by the
// cross-check and summary paths: the exact per-edge quantiles (edge_agg.hip,
// SURVEY.md §8a a11) and the API-response value summary (summary.hip, §8f row
// 3).  Both restate the reference's sorted(x)[int(n*q)]
// (SN_collection-scripts/Dataset/api_responses/monitor_http_responses.py:
// 180-190), so they need a stable sort of 64-bit keys; no library sort.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace anomod {

// Device scratch bytes radix_sort_u64 needs for n keys.
size_t radix_temp_bytes(uint64_t n);

// Most keys one radix_sort_u64 call takes (its per-tile counts, scan sums
// and scatter bases are u32): larger n returns hipErrorInvalidValue.
constexpr uint64_t kMaxSortKeys = 0xFFFFFFFFull - 4096;

// Stable LSD radix sort of n u64 keys by bits [begin_bit, end_bit) (keys must
// be < 2^end_bit), 8-bit digits: per pass the digit counts of every
// 4096-key tile, their exclusive scan over tiles, one scatter (wave-ballot
// ranks, the tile staged in LDS in digit order, written as coalesced digit
// runs).  A pass whose digit is the same in every key (from one OR / AND
// reduction of the keys first) is skipped.  `in` may equal `out`.  Blocks on
// `stream` once (the reduction's read-back).  Returns the passes run in
// *passes when not NULL.
hipError_t radix_sort_u64(const uint64_t* in, uint64_t* out, uint64_t n, int begin_bit,
                          int end_bit, void* temp, size_t temp_bytes, hipStream_t stream,
                          int* passes = nullptr);

// Order-preserving u64 key of an f64 (total order: -inf < ... < -0.0 < +0.0
// < ... < +inf; NaN is never a key here) and back.
__host__ __device__ inline uint64_t f64_key(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  return (u >> 63) ? ~u : (u | (1ull << 63));
}
__host__ __device__ inline double key_f64(uint64_t k) {
  return __builtin_bit_cast(double, (k >> 63) ? (k & ~(1ull << 63)) : ~k);
}

// Device scratch bytes of select_f64_keys for n values.
size_t select_temp_bytes(uint64_t n);

// Stable compaction of the values v with v > 0 (positive_only) or v == v
// (every non-NaN value) into order keys f64_key(v); the count lands in
// *d_count (device).
hipError_t select_f64_keys(const double* vals, uint64_t n, int positive_only, uint64_t* keys,
                           unsigned long long* d_count, void* temp, size_t temp_bytes,
                           hipStream_t stream);

// Device scratch bytes of sum_keys_f64 for n keys.
size_t sum_temp_bytes(uint64_t n);

// Sum of key_f64(keys[i]) over n keys in one fixed order (16384-key chunks
// summed by a fixed lane stride and LDS tree, the chunk sums by the same
// rule): the same bits every run, whatever the schedule.  Result to *out
// (device).
hipError_t sum_keys_f64(const uint64_t* keys, uint64_t n, double* out, void* temp,
                        size_t temp_bytes, hipStream_t stream);

}  // namespace anomod
