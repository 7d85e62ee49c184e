// Minimal probe for the r01 observation "a process that made a cooperative
// launch segfaults at exit under rocprofv3 --kernel-trace": no libanomod, one
// trivial kernel launched cooperatively (argv[1] == "coop") or plainly.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__global__ void touch(int* p) {
  if (threadIdx.x == 0) atomicAdd(p, 1);
}

int main(int argc, char** argv) {
  const bool coop = argc > 1 && std::strcmp(argv[1], "coop") == 0;
  int* d = nullptr;
  if (hipMalloc(&d, sizeof(int)) != hipSuccess) return 2;
  if (hipMemset(d, 0, sizeof(int)) != hipSuccess) return 2;
  void* args[] = {&d};
  hipError_t e = coop ? hipLaunchCooperativeKernel(reinterpret_cast<const void*>(touch), dim3(4),
                                                   dim3(64), args, 0, nullptr)
                      : hipLaunchKernel(reinterpret_cast<const void*>(touch), dim3(4), dim3(64),
                                        args, 0, nullptr);
  if (e != hipSuccess) {
    std::printf("launch failed: %s\n", hipGetErrorString(e));
    return 3;
  }
  int h = 0;
  if (hipMemcpy(&h, d, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return 4;
  (void)hipFree(d);
  std::printf("%s launch ok: %d blocks counted\n", coop ? "cooperative" : "plain", h);
  return h == 4 ? 0 : 5;
}
