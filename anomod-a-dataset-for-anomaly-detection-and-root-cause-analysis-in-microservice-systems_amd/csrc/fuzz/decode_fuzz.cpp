// Mutation fuzzer for the host decoders of libanomod (decode.cpp,
// metrics_decode.cpp), built with -fsanitize=address,undefined by
// `make -C csrc sanitize` (host sanitizer builds).  The
// decoders parse untrusted files on up to 16 threads; every mutated input
// must decode or fail with a status, never touch memory it does not own.
//
// usage: decode_fuzz ITERS SEED kind:path ...   (kind: jaeger | skywalking |
//        long | longfile | prom); prints "ok <decoded> <rejected>" on success.
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

#include <unistd.h>

#include "../../../include/anomod.h"

namespace anomod {
void set_error(anomod_ctx*, const char* fmt, ...) {  // the library's lives in ctx.hip
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
}
}  // namespace anomod

namespace {

struct Seed {
  std::string kind;
  std::string data;
};

std::string mutate(const std::string& in, std::mt19937_64& rng) {
  std::string s = in;
  const int n_ops = 1 + (int)(rng() % 8);
  const char* tokens[] = {"\"", "\\", "{", "}", "[", "]", ",", ":", "null", "true", "1e309",
                          "-0", "\"\\u0000\"", "\"\\ud800\"", "\n", "\r\n", "\"\"", "NaN", "9999999999999999999999"};
  for (int k = 0; k < n_ops && !s.empty(); ++k) {
    const size_t at = rng() % (s.size() + 1);
    switch (rng() % 7) {
      case 0: if (at < s.size()) s[at] ^= (char)(1u << (rng() % 8)); break;
      case 1: s.insert(at, tokens[rng() % (sizeof tokens / sizeof *tokens)]); break;
      case 2: if (at < s.size()) s.erase(at, 1 + rng() % 16); break;
      case 3: s.resize(at); break;
      case 4: {
        const size_t b = rng() % (s.size() + 1), len = rng() % 256;
        s.insert(at, s.substr(b, len));
        break;
      }
      case 5: if (at < s.size() && s[at] >= '0' && s[at] <= '9') s[at] = (char)('0' + rng() % 10); break;
      default: if (at < s.size()) s[at] = (char)(rng() & 0xFF); break;
    }
  }
  return s;
}

int run(const Seed& sd, const std::string& data) {
  if (sd.kind == "jaeger" || sd.kind == "skywalking") {
    anomod_decoded* d = nullptr;
    const int rc = sd.kind == "jaeger"
                       ? anomod_decode_jaeger(data.data(), data.size(), nullptr, 0, &d)
                       : anomod_decode_skywalking(data.data(), data.size(), nullptr, 0, &d);
    if (rc != ANOMOD_OK) return 0;
    uint64_t ns = 0, nt = 0;
    uint32_t nsv = 0;
    anomod_decoded_info(d, &ns, &nt, &nsv);
    std::vector<uint64_t> th(ns), sid(ns), pid(ns), ptr(nt + 1);
    std::vector<uint16_t> svc(ns), fl(ns);
    std::vector<uint32_t> dur(ns);
    anomod_span_soa_out o{th.data(), sid.data(), pid.data(), svc.data(), fl.data(), dur.data()};
    anomod_decoded_columns(d, &o, ptr.data());
    for (uint32_t i = 0; i < nsv; ++i) (void)strlen(anomod_decoded_service(d, i));
    anomod_decoded_free(d);
    return 1;
  }
  if (sd.kind == "longfile") {
    // The file API maps the file: no terminator past its last byte.  Sizes
    // are padded (newlines) to a whole number of pages so a read past the
    // end faults instead of landing in the page's zero slack; the result
    // must equal the buffer API's on the same bytes.
    std::string body = data + std::string((4096 - data.size() % 4096) % 4096, '\n');
    char path[] = "/tmp/anomod_fuzz_XXXXXX";
    const int fd = mkstemp(path);
    if (fd < 0) return 0;
    const bool wrote = write(fd, body.data(), body.size()) == (ssize_t)body.size();
    close(fd);
    anomod_metrics *mf = nullptr, *mb = nullptr;
    const int rf = wrote ? anomod_decode_metric_long_csv_file(path, &mf) : ANOMOD_EINVAL;
    unlink(path);
    const int rb = anomod_decode_metric_long_csv(body.data(), body.size(), &mb);
    if (wrote && (rf == ANOMOD_OK) != (rb == ANOMOD_OK)) {
      fprintf(stderr, "file and buffer decodes disagree: %d vs %d\n", rf, rb);
      abort();
    }
    if (rf != ANOMOD_OK) {
      if (mb) anomod_metrics_free(mb);
      return 0;
    }
    uint64_t T1 = 0, S1 = 0, T2 = 0, S2 = 0;
    anomod_metrics_info(mf, &T1, &S1);
    anomod_metrics_info(mb, &T2, &S2);
    if (T1 != T2 || S1 != S2) abort();
    std::vector<float> X1(T1 * S1), X2(T2 * S2);
    std::vector<double> t1(T1), t2(T2);
    anomod_metrics_matrix(mf, X1.data(), t1.data());
    anomod_metrics_matrix(mb, X2.data(), t2.data());
    if ((!X1.empty() && memcmp(X1.data(), X2.data(), X1.size() * 4)) ||
        (T1 && memcmp(t1.data(), t2.data(), T1 * 8)))
      abort();
    for (uint64_t s = 0; s < S1; ++s)
      if (strcmp(anomod_metrics_series_name(mf, s), anomod_metrics_series_name(mb, s))) abort();
    anomod_metrics_free(mf);
    anomod_metrics_free(mb);
    return 1;
  }
  anomod_metrics* m = nullptr;
  int rc;
  if (sd.kind == "long") {
    rc = anomod_decode_metric_long_csv(data.data(), data.size(), &m);
  } else {
    const char* blobs[2] = {data.data(), data.data()};
    const uint64_t lens[2] = {data.size(), data.size() / 2};
    const char* stems[2] = {"a", "b"};
    rc = anomod_decode_prometheus_csvs(blobs, lens, stems, 2, &m);
  }
  if (rc != ANOMOD_OK) return 0;
  uint64_t T = 0, S = 0;
  anomod_metrics_info(m, &T, &S);
  std::vector<float> X(T * S);
  std::vector<double> ts(T);
  anomod_metrics_matrix(m, X.data(), ts.data());
  for (uint64_t s = 0; s < S; ++s) {
    (void)strlen(anomod_metrics_series_name(m, s));
    for (uint32_t j = 0; j < anomod_metrics_series_nlabels(m, s); ++j) {
      const char* v = nullptr;
      (void)strlen(anomod_metrics_series_label(m, s, j, &v));
      (void)strlen(v);
    }
  }
  anomod_metrics_free(m);
  return 1;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s ITERS SEED kind:path ...\n", argv[0]);
    return 2;
  }
  const long iters = atol(argv[1]);
  std::mt19937_64 rng((uint64_t)atoll(argv[2]));
  std::vector<Seed> seeds;
  for (int i = 3; i < argc; ++i) {
    const char* c = strchr(argv[i], ':');
    if (!c) return 2;
    std::ifstream f(c + 1, std::ios::binary);
    if (!f) {
      fprintf(stderr, "cannot read %s\n", c + 1);
      return 2;
    }
    seeds.push_back({std::string(argv[i], (size_t)(c - argv[i])),
                     std::string(std::istreambuf_iterator<char>(f), {})});
  }
  long ok = 0, rej = 0;
  for (const Seed& sd : seeds) {  // the unmutated seeds must decode
    if (!run(sd, sd.data)) {
      fprintf(stderr, "seed of kind %s did not decode\n", sd.kind.c_str());
      return 1;
    }
  }
  for (long it = 0; it < iters; ++it) {
    const Seed& sd = seeds[rng() % seeds.size()];
    if (run(sd, mutate(sd.data, rng))) ++ok; else ++rej;
  }
  printf("ok %ld %ld\n", ok, rej);
  return 0;
}
