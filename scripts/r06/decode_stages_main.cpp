#include <cstdio>
#include <cstdarg>
#include <cstdint>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <chrono>
#include "../../include/anomod.h"
namespace anomod { void set_error(anomod_ctx*, const char* fmt, ...) { va_list a; va_start(a, fmt); vfprintf(stderr, fmt, a); va_end(a); } }
int main(int argc, char** argv) {
  int fd = open(argv[1], O_RDONLY); struct stat st; fstat(fd, &st);
  const char* m = (const char*)mmap(nullptr, st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
  for (int r = 0; r < 3; ++r) {
    auto t0 = std::chrono::steady_clock::now();
    anomod_metrics* out = nullptr;
    // the library's file entry (a fresh mapping per call, as load_experiment
    // uses it); argv[2] == "mem": the in-memory entry on one mapping
    int rc = argc > 2 ? anomod_decode_metric_long_csv(m, st.st_size, &out)
                      : anomod_decode_metric_long_csv_file(argv[1], &out);
    auto t1 = std::chrono::steady_clock::now();
    printf("rc %d %.1f ms\n", rc, std::chrono::duration<double, std::milli>(t1 - t0).count());
    anomod_metrics_free(out);
  }
}
