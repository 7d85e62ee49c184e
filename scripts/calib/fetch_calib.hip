// FETCH_SIZE calibration for the access patterns of the ungrouped path and the
// batched PageRank (VERDICT r04 "Next" 1a; MI355X_MICROARCH.md "HBM": FETCH_SIZE
// reads exactly 1/2 of a wide coalesced 16-B/lane stream on gfx950, other
// widths are uncalibrated).  Each kernel reads a KNOWN number of bytes:
//
//   stream16      16 B per lane, coalesced, over the whole buffer (the guide's
//                 reference pattern: expect FETCH_SIZE = 1/2 of the bytes)
//   stream8        8 B per lane, coalesced (pair loads: count B, scatter B, join)
//   gather32_far  32-B records (two 16-B loads per lane, as bk_join's q[0], q[1])
//                 at uniform random indices over the whole buffer (>> 256 MiB)
//   gather32_win  the same inside a 72 MiB window (one level-A bucket of the
//                 ungrouped path: the join's gathers)
//   gather16_far  16-B records at uniform random indices (PageRank batch x)
//   gather16_win  the same inside a 8 MiB window (the batch vector is 0.8-6 MB)
//   gather8_far    8-B words at uniform random indices
//
// Each lane issues kPer loads of its pattern; the sums go to one word per lane
// (written bytes: 8 per lane, negligible).  Prints one JSON line per kernel
// with the true bytes read and the hipEvent time; rocprofv3 --pmc FETCH_SIZE on
// the same binary gives the counter, and scripts/calib/summarize.py the ratio.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      std::exit(1);                                                                       \
    }                                                                                     \
  } while (0)

constexpr int kThreads = 256;
constexpr int kPer = 16;  // loads per lane

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <int B>  // 8 or 16 bytes per lane, coalesced
__global__ __launch_bounds__(kThreads) void stream_kernel(const unsigned char* __restrict__ buf,
                                                          uint64_t bytes, uint64_t* __restrict__ out) {
  const uint64_t nv = bytes / B, stride = (uint64_t)gridDim.x * kThreads;
  uint64_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < nv; i += stride) {
    if constexpr (B == 16) {
      const uint4 x = reinterpret_cast<const uint4*>(buf)[i];
      acc += x.x ^ x.y ^ x.z ^ x.w;
    } else {
      acc += reinterpret_cast<const uint64_t*>(buf)[i];
    }
  }
  out[(uint64_t)blockIdx.x * kThreads + threadIdx.x] = acc;
}

template <int B>  // record bytes: 8, 16 or 32 (32 = two 16-B loads)
__global__ __launch_bounds__(kThreads) void gather_kernel(const unsigned char* __restrict__ buf,
                                                          uint64_t win_bytes, uint64_t win_step,
                                                          uint64_t* __restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  const uint64_t nrec = win_bytes / B;
  // win_step = 1: blocks walk the buffer window by window, 2 048 blocks per
  // window (about what is resident at once), as the join's buckets walk the
  // level-A buckets; win_step = 0: one window = the whole buffer
  const unsigned char* w = buf + (win_step ? ((uint64_t)blockIdx.x / 2048) * win_bytes : 0);
  uint64_t idx[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) idx[j] = mix(t * kPer + j + 0x1234567ull) % nrec;
  uint64_t acc = 0;
  if constexpr (B == 32) {
    uint4 a[kPer], b[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const uint4* q = reinterpret_cast<const uint4*>(w + idx[j] * 32);
      a[j] = q[0];
      b[j] = q[1];
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) acc += a[j].x ^ a[j].w ^ b[j].y ^ b[j].z;
  } else if constexpr (B == 16) {
    uint4 a[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) a[j] = reinterpret_cast<const uint4*>(w)[idx[j]];
#pragma unroll
    for (int j = 0; j < kPer; ++j) acc += a[j].x ^ a[j].w;
  } else {
    uint64_t a[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) a[j] = reinterpret_cast<const uint64_t*>(w)[idx[j]];
#pragma unroll
    for (int j = 0; j < kPer; ++j) acc += a[j];
  }
  out[t] = acc;
}

__global__ void fill_kernel(uint64_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = mix(i);
}

int main(int argc, char** argv) {
  const uint64_t gib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 8;
  const uint64_t bytes = gib << 30;
  unsigned char* buf;
  uint64_t* out;
  CHECK(hipMalloc(&buf, bytes));
  const unsigned grid = 256 * 64;  // 16 384 blocks
  CHECK(hipMalloc(&out, (uint64_t)grid * kThreads * 8));
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(buf),
                     bytes / 8);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const uint64_t lanes = (uint64_t)grid * kThreads;
  auto run = [&](const char* name, auto launch, uint64_t true_bytes) {
    launch();  // warm
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      CHECK(hipEventRecord(e0));
      launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    std::printf("{\"kernel\": \"%s\", \"true_bytes\": %llu, \"launches\": 4, \"best_ms\": %.4f, "
                "\"GBps\": %.1f}\n",
                name, (unsigned long long)true_bytes, best, true_bytes / (best * 1e6));
    std::fflush(stdout);
  };
  run("stream16", [&] { hipLaunchKernelGGL(stream_kernel<16>, dim3(grid), dim3(kThreads), 0, 0, buf, bytes, out); }, bytes);
  run("stream8", [&] { hipLaunchKernelGGL(stream_kernel<8>, dim3(grid), dim3(kThreads), 0, 0, buf, bytes, out); }, bytes);
  const uint64_t g = lanes * kPer;  // gathers per launch
  run("gather32_far", [&] { hipLaunchKernelGGL(gather_kernel<32>, dim3(grid), dim3(kThreads), 0, 0, buf, bytes, (uint64_t)0, out); }, g * 32);
  run("gather32_win", [&] { hipLaunchKernelGGL(gather_kernel<32>, dim3(grid), dim3(kThreads), 0, 0, buf, (uint64_t)72 << 20, (uint64_t)1, out); }, g * 32);
  run("gather16_far", [&] { hipLaunchKernelGGL(gather_kernel<16>, dim3(grid), dim3(kThreads), 0, 0, buf, bytes, (uint64_t)0, out); }, g * 16);
  run("gather16_win", [&] { hipLaunchKernelGGL(gather_kernel<16>, dim3(grid), dim3(kThreads), 0, 0, buf, (uint64_t)8 << 20, (uint64_t)1, out); }, g * 16);
  run("gather8_far", [&] { hipLaunchKernelGGL(gather_kernel<8>, dim3(grid), dim3(kThreads), 0, 0, buf, bytes, (uint64_t)0, out); }, g * 8);
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
