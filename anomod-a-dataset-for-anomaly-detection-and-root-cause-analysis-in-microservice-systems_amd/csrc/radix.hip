// Hand-written stable LSD radix sort of u64 keys, stable f64 compaction and a
// fixed-order f64 sum (radix.h).  Same tile machinery as the trace grouping
// (group.hip), specialised to bare 8-B keys:
//  * digit counts of every 4096-key tile (per-wave LDS sub-histograms, so a
//    skewed digit — the high bits of latencies — does not serialise one LDS
//    address for the whole block);
//  * their exclusive scan over tiles: column sums of 256-tile blocks, one
//    block scanning those (digit starts added in), the blocks writing every
//    tile's global run start (reduce-then-scan: no look-back chain);
//  * one scatter per pass: a tile (1024 threads x 4 keys) ranked stably with
//    wave ballots (8 ballots give a lane its same-digit peers; rank = popc of
//    the lower peers; per-wave LDS digit counters carry the count down the
//    wave's 4 rows), staged in LDS in digit order and written as coalesced
//    digit runs (~16 keys = 128 B per run at uniform digits).
// Bytes per pass: 8 (count) + 16 (scatter) per key.
#include "radix.h"

#include <algorithm>

#include "chunk.h"

namespace anomod {
namespace {

using chunk::wave_sync;
constexpr int kWv = 64;
constexpr int kDig = 256;
constexpr int kSThreads = 1024;
constexpr int kSWaves = kSThreads / kWv;
constexpr int kSPer = 4;
constexpr int kTile = kSThreads * kSPer;            // 4096 keys
constexpr int kRowsPerWave = kTile / kSWaves / kWv;  // 4
constexpr int kCThreads = 256;                       // count kernel
constexpr int kScanRows = 256;                       // tiles per block of the tile scan
constexpr int kSumThreads = 256;
constexpr int kSumChunk = kSumThreads * 64;          // keys per partial sum

inline size_t al256(size_t x) { return (x + 255) & ~size_t(255); }
inline uint64_t n_tiles(uint64_t n) { return (n + kTile - 1) / kTile; }

// ---- OR / AND of all keys (which digits are constant) ---------------------
__global__ __launch_bounds__(256) void keys_or_and_kernel(const uint64_t* __restrict__ k,
                                                          uint64_t n,
                                                          unsigned long long* __restrict__ oa) {
  uint64_t o = 0, a = ~0ull;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * 256) {
    const uint64_t x = k[i];
    o |= x;
    a &= x;
  }
  for (int off = 32; off > 0; off >>= 1) {
    o |= __shfl_xor(o, off);
    a &= __shfl_xor(a, off);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicOr(&oa[0], (unsigned long long)o);
    atomicAnd(&oa[1], (unsigned long long)a);
  }
}

// ---- per-tile digit counts --------------------------------------------------
__global__ __launch_bounds__(kCThreads) void radix_count_kernel(const uint64_t* __restrict__ k,
                                                                uint64_t n, int shift,
                                                                uint32_t dmask,
                                                                uint32_t* __restrict__ tcnt) {
  constexpr int kW = kCThreads / kWv;
  __shared__ uint32_t lh[kW][kDig];
  const int tid = threadIdx.x, w = tid / kWv;
  for (int i = tid; i < kW * kDig; i += kCThreads) (&lh[0][0])[i] = 0u;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
#pragma unroll 4
  for (int j = 0; j < kTile / kCThreads; ++j) {
    const uint64_t p = t0 + (uint64_t)(j * kCThreads + tid);
    if (p < n) atomicAdd(&lh[w][(uint32_t)(k[p] >> shift) & dmask], 1u);
  }
  __syncthreads();
  uint32_t s = 0;
#pragma unroll
  for (int ww = 0; ww < kW; ++ww) s += lh[ww][tid];
  tcnt[(uint64_t)blockIdx.x * kDig + tid] = s;
}

// ---- exclusive scan of the tile counts over tiles, per digit ---------------
__global__ __launch_bounds__(kDig) void radix_scan_up_kernel(const uint32_t* __restrict__ tcnt,
                                                             uint64_t tiles,
                                                             uint32_t* __restrict__ bsum) {
  const uint64_t a = (uint64_t)blockIdx.x * kScanRows;
  const uint64_t b = a + kScanRows < tiles ? a + kScanRows : tiles;
  uint32_t s = 0;
#pragma unroll 8
  for (uint64_t t = a; t < b; ++t) s += tcnt[t * kDig + threadIdx.x];
  bsum[(uint64_t)blockIdx.x * kDig + threadIdx.x] = s;
}

__global__ __launch_bounds__(kDig) void radix_scan_top_kernel(uint32_t* __restrict__ bsum,
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

__global__ __launch_bounds__(kDig) void radix_scan_down_kernel(uint32_t* __restrict__ tcnt,
                                                               uint64_t tiles,
                                                               const uint32_t* __restrict__ bsum) {
  const uint64_t a = (uint64_t)blockIdx.x * kScanRows;
  const uint64_t b = a + kScanRows < tiles ? a + kScanRows : tiles;
  uint32_t run = bsum[(uint64_t)blockIdx.x * kDig + threadIdx.x];
#pragma unroll 8
  for (uint64_t t = a; t < b; ++t) {
    const uint32_t x = tcnt[t * kDig + threadIdx.x];
    tcnt[t * kDig + threadIdx.x] = run;
    run += x;
  }
}

// ---- one stable pass ----------------------------------------------------------
__global__ __launch_bounds__(kSThreads) void radix_scatter_kernel(
    const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint64_t n, int shift,
    uint32_t dmask, const uint32_t* __restrict__ toff) {
  __shared__ uint64_t stage[kTile];             // 32 KiB
  __shared__ uint16_t wcnt[kSWaves][kDig];      // per-wave digit counts, then wave offsets
  __shared__ uint8_t sdig[kTile];
  __shared__ uint32_t tstart[kDig];
  __shared__ uint32_t gbase[kDig];
  __shared__ uint32_t wsum_t[kDig / kWv];
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  const uint64_t tile = blockIdx.x;
  const uint64_t base = tile * kTile;
  uint64_t key[kSPer];
  bool v[kSPer];
  uint32_t d[kSPer];
#pragma unroll
  for (int k = 0; k < kSPer; ++k) {
    const uint64_t i = base + (uint64_t)(w * (kRowsPerWave * kWv) + k * kWv + lane);
    v[k] = i < n;
    key[k] = v[k] ? in[i] : 0ull;
    d[k] = (uint32_t)(key[k] >> shift) & dmask;
  }
  for (int i = tid; i < kSWaves * kDig / 2; i += kSThreads)
    reinterpret_cast<uint32_t*>(&wcnt[0][0])[i] = 0u;
  if (tid < kDig) gbase[tid] = toff[tile * kDig + tid];
  __syncthreads();

  // wave multisplit, rows in order: peers = lanes of the row with the same
  // digit; rank = lower peers + the wave's running count of that digit
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
  if (tid < kDig) {  // wave offsets per digit, then the tile's digit starts
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
#pragma unroll
  for (int k = 0; k < kSPer; ++k) {
    if (v[k]) {
      const uint32_t lp = tstart[d[k]] + wcnt[w][d[k]] + off[k];
      stage[lp] = key[k];
      sdig[lp] = (uint8_t)d[k];
    }
  }
  __syncthreads();
  const uint64_t nvalid = n - base < (uint64_t)kTile ? n - base : (uint64_t)kTile;
#pragma unroll
  for (int k = 0; k < kSPer; ++k) {
    const uint32_t p = (uint32_t)(tid + k * kSThreads);
    if (p < nvalid) {
      const uint32_t dd = sdig[p];
      out[(uint64_t)gbase[dd] + (p - tstart[dd])] = stage[p];
    }
  }
}

// ---- stable f64 compaction ----------------------------------------------------
__device__ __forceinline__ bool keep_value(double x, int positive_only) {
  return positive_only ? x > 0.0 : x == x;
}

__global__ __launch_bounds__(kCThreads) void select_count_kernel(const double* __restrict__ x,
                                                                 uint64_t n, int positive_only,
                                                                 uint32_t* __restrict__ tcnt) {
  __shared__ uint32_t ws[kCThreads / kWv];
  const int tid = threadIdx.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
  uint32_t c = 0;
  for (int j = 0; j < kTile / kCThreads; ++j) {
    const uint64_t p = t0 + (uint64_t)(j * kCThreads + tid);
    c += (p < n && keep_value(x[p], positive_only)) ? 1u : 0u;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((tid & 63) == 0) ws[tid / kWv] = c;
  __syncthreads();
  if (tid == 0) {
    uint32_t s = 0;
    for (int i = 0; i < kCThreads / kWv; ++i) s += ws[i];
    tcnt[blockIdx.x] = s;
  }
}

// one block: exclusive scan of the tile counts (in place), total to *count
__global__ __launch_bounds__(1024) void select_scan_kernel(uint32_t* __restrict__ tcnt,
                                                           uint64_t tiles,
                                                           unsigned long long* __restrict__ count) {
  __shared__ uint64_t wsum[16];
  __shared__ uint64_t carry;
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (uint64_t b0 = 0; b0 < tiles; b0 += 1024) {
    const uint64_t t = b0 + tid;
    const uint64_t x = t < tiles ? tcnt[t] : 0u;
    uint64_t inc = x;
#pragma unroll
    for (int o = 1; o < kWv; o <<= 1) {
      const uint64_t y = __shfl_up(inc, o);
      if (lane >= o) inc += y;
    }
    if (lane == kWv - 1) wsum[w] = inc;
    __syncthreads();
    uint64_t pre = carry;
    for (int ww = 0; ww < w; ++ww) pre += wsum[ww];
    if (t < tiles) tcnt[t] = (uint32_t)(pre + inc - x);
    __syncthreads();
    if (tid == 1023) carry = pre + inc;
    __syncthreads();
  }
  if (tid == 0) *count = carry;
}

__global__ __launch_bounds__(kCThreads) void select_write_kernel(
    const double* __restrict__ x, uint64_t n, int positive_only,
    const uint32_t* __restrict__ toff, uint64_t* __restrict__ keys) {
  __shared__ uint32_t ws[kTile / kCThreads][kCThreads / kWv];
  const int tid = threadIdx.x, lane = tid & (kWv - 1), w = tid / kWv;
  constexpr int kW = kCThreads / kWv;
  constexpr int kRows = kTile / kCThreads;  // 16 rows of 256 values
  const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
  uint64_t b[kRows];
  uint32_t below[kRows];
#pragma unroll
  for (int j = 0; j < kRows; ++j) {
    const uint64_t p = t0 + (uint64_t)(j * kCThreads + tid);
    const bool keep = p < n && keep_value(x[p], positive_only);
    b[j] = __ballot(keep);
    below[j] = keep ? (uint32_t)__popcll(b[j] & ((1ull << lane) - 1ull)) : 0xFFFFFFFFu;
    if (lane == 0) ws[j][w] = (uint32_t)__popcll(b[j]);
  }
  __syncthreads();
  uint32_t run = toff[blockIdx.x];
#pragma unroll
  for (int j = 0; j < kRows; ++j) {
    uint32_t pre = run;
    for (int ww = 0; ww < w; ++ww) pre += ws[j][ww];
    for (int ww = 0; ww < kW; ++ww) run += ws[j][ww];
    if (below[j] != 0xFFFFFFFFu) {
      const uint64_t p = t0 + (uint64_t)(j * kCThreads + tid);
      keys[(uint64_t)pre + below[j]] = f64_key(x[p]);
    }
  }
}

// ---- fixed-order sum ----------------------------------------------------------
__device__ double block_tree_sum(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = kSumThreads / 2; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  return red[0];
}

// block b sums keys [b * kSumChunk, (b + 1) * kSumChunk): lane i adds i, i +
// 256, ... in order, then a fixed LDS tree
__global__ __launch_bounds__(kSumThreads) void sum_chunks_kernel(const uint64_t* __restrict__ k,
                                                                 uint64_t n,
                                                                 double* __restrict__ part) {
  __shared__ double red[kSumThreads];
  const uint64_t a = (uint64_t)blockIdx.x * kSumChunk;
  double s = 0.0;
  for (int j = 0; j < kSumChunk / kSumThreads; ++j) {
    const uint64_t p = a + (uint64_t)(j * kSumThreads + threadIdx.x);
    if (p < n) s += key_f64(k[p]);
  }
  const double t = block_tree_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ __launch_bounds__(kSumThreads) void sum_parts_kernel(const double* __restrict__ part,
                                                                uint64_t m,
                                                                double* __restrict__ out) {
  __shared__ double red[kSumThreads];
  double s = 0.0;
  for (uint64_t p = threadIdx.x; p < m; p += kSumThreads) s += part[p];
  const double t = block_tree_sum(s, red);
  if (threadIdx.x == 0) *out = t;
}

}  // namespace

size_t radix_temp_bytes(uint64_t n) {
  const uint64_t tiles = n_tiles(n ? n : 1);
  return al256(n * 8) + al256(tiles * kDig * 4) + al256((tiles / kScanRows + 1) * kDig * 4) + 256;
}

hipError_t radix_sort_u64(const uint64_t* in, uint64_t* out, uint64_t n, int begin_bit,
                          int end_bit, void* temp, size_t temp_bytes, hipStream_t stream,
                          int* passes) {
  if (passes) *passes = 0;
  if (temp_bytes < radix_temp_bytes(n) || begin_bit < 0 || end_bit > 64 || begin_bit > end_bit)
    return hipErrorInvalidValue;
  // tile counts, scan sums and scatter bases are u32: n + one tile must fit
  if (n > kMaxSortKeys) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  const uint64_t tiles = n_tiles(n), nb = (tiles + kScanRows - 1) / kScanRows;
  char* t = static_cast<char*>(temp);
  uint64_t* alt = reinterpret_cast<uint64_t*>(t);
  uint32_t* tcnt = reinterpret_cast<uint32_t*>(t + al256(n * 8));
  uint32_t* bsum = reinterpret_cast<uint32_t*>(t + al256(n * 8) + al256(tiles * kDig * 4));
  auto* oa = reinterpret_cast<unsigned long long*>(
      t + al256(n * 8) + al256(tiles * kDig * 4) + al256((tiles / kScanRows + 1) * kDig * 4));
  // which digits vary: OR / AND of every key
  unsigned long long h_oa[2] = {0ull, ~0ull};
  hipError_t e = hipMemcpyAsync(oa, h_oa, 16, hipMemcpyHostToDevice, stream);
  if (e != hipSuccess) return e;
  const unsigned rgrid = (unsigned)std::min<uint64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(keys_or_and_kernel, dim3(rgrid), dim3(256), 0, stream, in, n, oa);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(h_oa, oa, 16, hipMemcpyDeviceToHost, stream)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(stream)) != hipSuccess) return e;
  const uint64_t varies = h_oa[0] ^ h_oa[1];
  int shifts[8], P = 0;
  for (int s = begin_bit; s < end_bit; s += 8) {
    const int w = std::min(8, end_bit - s);
    const uint64_t m = ((1ull << w) - 1ull) << s;
    if (varies & m) shifts[P++] = s;
  }
  if (passes) *passes = P;
  if (P == 0) {
    if (in != out)
      return hipMemcpyAsync(out, in, n * 8, hipMemcpyDeviceToDevice, stream);
    return hipSuccess;
  }
  const uint64_t* src = in;
  for (int p = 0; p < P; ++p) {
    uint64_t* dst = ((P - 1 - p) & 1) == 0 ? out : alt;
    if (dst == src) dst = (dst == out) ? alt : out;  // in == out: never scatter in place
    const int s = shifts[p];
    const uint32_t dmask = (uint32_t)((1ull << std::min(8, end_bit - s)) - 1ull);
    hipLaunchKernelGGL(radix_count_kernel, dim3((unsigned)tiles), dim3(kCThreads), 0, stream, src,
                       n, s, dmask, tcnt);
    hipLaunchKernelGGL(radix_scan_up_kernel, dim3((unsigned)nb), dim3(kDig), 0, stream, tcnt,
                       tiles, bsum);
    hipLaunchKernelGGL(radix_scan_top_kernel, dim3(1), dim3(kDig), 0, stream, bsum, nb);
    hipLaunchKernelGGL(radix_scan_down_kernel, dim3((unsigned)nb), dim3(kDig), 0, stream, tcnt,
                       tiles, bsum);
    hipLaunchKernelGGL(radix_scatter_kernel, dim3((unsigned)tiles), dim3(kSThreads), 0, stream,
                       src, dst, n, s, dmask, tcnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    src = dst;
  }
  if (src != out) return hipMemcpyAsync(out, src, n * 8, hipMemcpyDeviceToDevice, stream);
  return hipSuccess;
}

size_t select_temp_bytes(uint64_t n) { return al256(n_tiles(n ? n : 1) * 4); }

hipError_t select_f64_keys(const double* vals, uint64_t n, int positive_only, uint64_t* keys,
                           unsigned long long* d_count, void* temp, size_t temp_bytes,
                           hipStream_t stream) {
  if (temp_bytes < select_temp_bytes(n)) return hipErrorInvalidValue;
  if (n == 0) return hipMemsetAsync(d_count, 0, 8, stream);
  const uint64_t tiles = n_tiles(n);
  uint32_t* tcnt = static_cast<uint32_t*>(temp);
  hipLaunchKernelGGL(select_count_kernel, dim3((unsigned)tiles), dim3(kCThreads), 0, stream, vals,
                     n, positive_only, tcnt);
  hipLaunchKernelGGL(select_scan_kernel, dim3(1), dim3(1024), 0, stream, tcnt, tiles, d_count);
  hipLaunchKernelGGL(select_write_kernel, dim3((unsigned)tiles), dim3(kCThreads), 0, stream, vals,
                     n, positive_only, tcnt, keys);
  return hipGetLastError();
}

size_t sum_temp_bytes(uint64_t n) { return al256(((n + kSumChunk - 1) / kSumChunk + 1) * 8); }

hipError_t sum_keys_f64(const uint64_t* keys, uint64_t n, double* out, void* temp,
                        size_t temp_bytes, hipStream_t stream) {
  if (temp_bytes < sum_temp_bytes(n)) return hipErrorInvalidValue;
  const uint64_t m = (n + kSumChunk - 1) / kSumChunk;
  double* part = static_cast<double*>(temp);
  if (m)
    hipLaunchKernelGGL(sum_chunks_kernel, dim3((unsigned)m), dim3(kSumThreads), 0, stream, keys, n,
                       part);
  hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(kSumThreads), 0, stream, part, m, out);
  return hipGetLastError();
}

}  // namespace anomod
