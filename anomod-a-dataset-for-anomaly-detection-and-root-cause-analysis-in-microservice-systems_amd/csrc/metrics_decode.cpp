// Native metric-file decoders (host C++): the
// Prometheus CSVs the reference's collectors write -> the time-major series
// matrix X[T][S] the EWMA/z kernels read, without a Python dict per row.
//
//  TT long CSV (metric_collector.py:400-478; rows :427-443, column order
//  :453-467): metric_name,timestamp,datetime,value,<sorted label columns>.
//    series key = (metric_name, the row's non-empty label (name, value) pairs
//    sorted); value '' = missing ('NaN' -> None -> '' at :435); the collector
//    queries three metrics twice (key_metrics :37-109, loop :420-423), so rows
//    are de-duplicated on (series, timestamp), first occurrence kept.
//  SN metric directory (fetch_prometheus_metrics.py:47-67 + main :92-102, one
//    CSV per query as collect_metric.sh names them): timestamp = naive local
//    datetime string, value, metric = the label string (:51), one column per
//    label.  series key = (file stem, the 'metric' column).
//
// Rules shared with anomod/decode.py (decode_metric_long_csv /
// decode_prometheus_csv_dir), whose outputs the tests pin to the reference's
// files: CSV per Python's csv module (excel dialect: "" escapes inside quoted
// fields, \r\n or \n records; a header name repeated keeps the last column),
// values and TT timestamps by strtod (Python float(): correctly rounded),
// datetime strings as datetime.fromisoformat(..).timestamp() (naive = local
// time: seconds + microseconds / 1e6; with an offset: exact microseconds /
// 1e6), timestamps = the sorted distinct values over all rows, series sorted
// as Python sorts the key tuples, X f32 with NaN where a series has no row.
#include <algorithm>
#ifdef ANOMOD_DECODE_TIMING
#include <chrono>
#include <cstdio>
#endif
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <deque>
#include <emmintrin.h>
#include <string>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/anomod.h"

namespace anomod {
void set_error(anomod_ctx* ctx, const char* fmt, ...);
}

struct anomod_metrics {
  struct Series {
    std::string name;                                        // metric_name / file stem
    std::vector<std::pair<std::string, std::string>> labels;  // sorted by (name, value)
  };
  std::vector<Series> series;  // sorted
  std::vector<double> ts;      // sorted distinct timestamps
  std::vector<float> X;        // [T][S]
};

namespace {

#ifdef ANOMOD_DECODE_TIMING  // stage times to stderr (scripts/r06/decode_stages.sh only)
void dt_mark(const char* name) {
  static auto last = std::chrono::steady_clock::now();
  const auto now = std::chrono::steady_clock::now();
  fprintf(stderr, "  %-14s %8.2f ms\n", name,
          std::chrono::duration<double, std::milli>(now - last).count());
  last = now;
}
#define DT_MARK(name) dt_mark(name)
#else
#define DT_MARK(name) ((void)0)
#endif

using Labels = std::vector<std::pair<std::string, std::string>>;

// First byte of [p, end) that is ',', '\n' or '\r' (end if none): eight bytes
// at a time (a zero byte of x ^ c marks a match; the classic haszero test
// can flag a 0x01 byte after a true match, never before one, so the lowest
// flagged byte is exact).
inline const char* field_end(const char* p, const char* end) {
  constexpr uint64_t kOnes = 0x0101010101010101ull, kHigh = 0x8080808080808080ull;
  while (end - p >= 8) {
    uint64_t x;
    memcpy(&x, p, 8);
    const uint64_t a = x ^ (kOnes * (uint8_t)','), n = x ^ (kOnes * (uint8_t)'\n'),
                   r = x ^ (kOnes * (uint8_t)'\r');
    const uint64_t m = ((a - kOnes) & ~a & kHigh) | ((n - kOnes) & ~n & kHigh) |
                       ((r - kOnes) & ~r & kHigh);
    if (m) return p + (__builtin_ctzll(m) >> 3);
    p += 8;
  }
  while (p < end && *p != ',' && *p != '\n' && *p != '\r') ++p;
  return p;
}

// One CSV record: field views (quoted fields with "" escapes are unescaped
// into `scratch`, which stays alive until the next record).
struct CsvReader {
  const char* p;
  const char* end;
  std::deque<std::string> scratch;  // stable addresses: fields view into them
  std::vector<std::string_view> fields;

  CsvReader(const char* b, size_t n) : p(b), end(b + n) {}

  // A record with no quote character, its delimiters found 16 bytes at a
  // time (SSE2 compares + movemask).  false (nothing consumed, no fields)
  // when the record holds a quote or runs into the last 16 bytes of the
  // input: the general loop below takes it.
  bool fast_record() {
    const __m128i kComma = _mm_set1_epi8(','), kNl = _mm_set1_epi8('\n'),
                  kCr = _mm_set1_epi8('\r'), kQuote = _mm_set1_epi8('"');
    const char* f = p;  // current field start
    for (const char* q = p; end - q >= 16; q += 16) {
      const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(q));
      unsigned mc = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(x, kComma));
      const unsigned me = (unsigned)_mm_movemask_epi8(
          _mm_or_si128(_mm_cmpeq_epi8(x, kNl), _mm_cmpeq_epi8(x, kCr)));
      const unsigned mq = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(x, kQuote));
      const unsigned stop = me & (0u - me);            // the record's end, if in this block
      const unsigned below = stop ? stop - 1u : 0xFFFFu;  // the bytes before it
      if (mq & below) break;                             // a quote: the general loop
      for (mc &= below; mc; mc &= mc - 1u) {
        const char* c = q + __builtin_ctz(mc);
        fields.emplace_back(f, (size_t)(c - f));
        f = c + 1;
      }
      if (stop) {
        const char* e = q + __builtin_ctz(stop);
        fields.emplace_back(f, (size_t)(e - f));
        p = e;
        if (p < end && *p == '\r') ++p;
        if (p < end && *p == '\n') ++p;
        return true;
      }
    }
    fields.clear();
    return false;
  }

  bool next() {  // false at end of input
    fields.clear();
    size_t used = 0;
    if (p >= end) return false;
    if (fast_record()) return true;
    while (true) {
      if (p < end && *p == '"') {  // quoted field
        ++p;
        if (used == scratch.size()) scratch.emplace_back();
        std::string& s = scratch[used++];
        s.clear();
        while (p < end) {
          const char* q = static_cast<const char*>(memchr(p, '"', (size_t)(end - p)));
          if (!q) {  // unterminated: the rest of the input
            s.append(p, (size_t)(end - p));
            p = end;
            break;
          }
          s.append(p, (size_t)(q - p));
          p = q + 1;
          if (p < end && *p == '"') {
            s.push_back('"');
            ++p;
            continue;
          }
          break;
        }
        // text after the closing quote up to the delimiter joins the field
        // (the csv module keeps it)
        const char* f = p;
        while (p < end && *p != ',' && *p != '\n' && *p != '\r') ++p;
        s.append(f, (size_t)(p - f));
        fields.emplace_back(s);
      } else {
        const char* f = p;
        p = field_end(p, end);
        fields.emplace_back(f, (size_t)(p - f));
      }
      if (p < end && *p == ',') {
        ++p;
        continue;
      }
      // end of record
      if (p < end && *p == '\r') ++p;
      if (p < end && *p == '\n') ++p;
      return true;
    }
  }
};

// Clinger's fast path: [-]digits[.digits] whose digits, read as one integer
// m, give m <= 2^53 (exactly a double) with <= 22 fraction digits (10^k exact)
// is m / 10^k, the one IEEE division being the correctly rounded value strtod
// returns.  One pass, no per-digit branches beyond the digit test.
bool fast_decimal(std::string_view v, double& out) {
  static const double kPow10[] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                  1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                  1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  const char* p = v.data();
  const char* const e = p + v.size();
  const bool neg = p < e && *p == '-';
  p += neg ? 1 : 0;
  const char* const s = p;
  uint64_t m = 0;  // (wraps past 19 digits: such strings are rejected below)
  while (p < e && (unsigned)(*p - '0') < 10u) m = m * 10u + (unsigned)(*p++ - '0');
  const size_t ni = (size_t)(p - s);
  size_t nf = 0;
  if (p < e && *p == '.') {
    const char* const f = ++p;
    while (p < e && (unsigned)(*p - '0') < 10u) m = m * 10u + (unsigned)(*p++ - '0');
    nf = (size_t)(p - f);
  }
  if (p != e || ni + nf == 0 || ni + nf > 19 || nf > 22 || m > (1ull << 53)) return false;
  const double d = (double)m / kPow10[nf];
  out = neg ? -d : d;
  return true;
}

bool parse_float(std::string_view v, double& out) {  // Python float() of a CSV field
  if (fast_decimal(v, out)) return true;
  char buf[64];
  std::string big;
  const char* b;
  if (v.size() < sizeof buf) {
    if (!v.empty()) memcpy(buf, v.data(), v.size());
    buf[v.size()] = '\0';
    b = buf;
  } else {
    big.assign(v);
    b = big.c_str();
  }
  while (*b == ' ' || *b == '\t') ++b;
  if (!*b) return false;
  char* e = nullptr;
  errno = 0;
  out = strtod(b, &e);
  if (e == b) return false;
  while (*e == ' ' || *e == '\t' || *e == '\n' || *e == '\r') ++e;
  return *e == '\0';
}

int digits(std::string_view s, size_t at, size_t n, int& v) {
  if (at + n > s.size()) return 0;
  v = 0;
  for (size_t i = 0; i < n; ++i) {
    const char c = s[at + i];
    if (c < '0' || c > '9') return 0;
    v = v * 10 + (c - '0');
  }
  return 1;
}

// datetime.fromisoformat(s).timestamp() for the forms pandas writes:
// YYYY-MM-DD[?HH[:MM[:SS[.fff|.ffffff]]]][+HH:MM[:SS[.ffffff]]|-HH:MM...]
bool iso_timestamp(std::string_view s, double& out) {
  int Y, M, D, h = 0, m = 0, sec = 0, us = 0;
  if (!digits(s, 0, 4, Y) || s.size() < 10 || s[4] != '-' || !digits(s, 5, 2, M) || s[7] != '-' ||
      !digits(s, 8, 2, D))
    return false;
  size_t i = 10;
  bool aware = false;
  long long off_us = 0;
  if (i < s.size()) {
    ++i;  // any one separator character
    if (!digits(s, i, 2, h)) return false;
    i += 2;
    if (i < s.size() && s[i] == ':') {
      if (!digits(s, i + 1, 2, m)) return false;
      i += 3;
      if (i < s.size() && s[i] == ':') {
        if (!digits(s, i + 1, 2, sec)) return false;
        i += 3;
        if (i < s.size() && s[i] == '.') {
          size_t j = i + 1;
          while (j < s.size() && s[j] >= '0' && s[j] <= '9') ++j;
          const size_t nd = j - i - 1;
          if (nd != 3 && nd != 6) return false;
          int f = 0;
          digits(s, i + 1, nd, f);
          us = nd == 3 ? f * 1000 : f;
          i = j;
        }
      }
    }
    if (i < s.size()) {  // UTC offset
      if (s[i] != '+' && s[i] != '-') return false;
      const int sign = s[i] == '-' ? -1 : 1;
      int oh, om, os = 0, ous = 0;
      if (!digits(s, i + 1, 2, oh) || i + 3 >= s.size() || s[i + 3] != ':' ||
          !digits(s, i + 4, 2, om))
        return false;
      size_t j = i + 6;
      if (j < s.size() && s[j] == ':') {
        if (!digits(s, j + 1, 2, os)) return false;
        j += 3;
        if (j < s.size() && s[j] == '.') {
          if (!digits(s, j + 1, 6, ous)) return false;
          j += 7;
        }
      }
      if (j != s.size()) return false;
      aware = true;
      off_us = sign * (((long long)oh * 3600 + om * 60 + os) * 1000000LL + ous);
    }
  }
  if (M < 1 || M > 12 || D < 1 || D > 31 || h > 23 || m > 59 || sec > 59) return false;
  struct tm t;
  memset(&t, 0, sizeof t);
  t.tm_year = Y - 1900;
  t.tm_mon = M - 1;
  t.tm_mday = D;
  t.tm_hour = h;
  t.tm_min = m;
  t.tm_sec = sec;
  if (aware) {  // (self - epoch).total_seconds(): exact microseconds / 1e6
    const long long u = (long long)timegm(&t) * 1000000LL + us - off_us;
    out = (double)u / 1e6;
  } else {  // local time: seconds + microseconds / 1e6
    t.tm_isdst = -1;
    const time_t u = mktime(&t);
    out = (double)u + us / 1e6;
  }
  return true;
}

struct Sample {  // kept in row order: the first occurrence of a cell wins
  uint32_t lc;      // the piece's timestamp column (Piece::lts)
  float v;
  uint32_t series;  // the piece's series id
};

// One parser's samples in row order, with what finish() needs to place them
// without another pass over them: the distinct timestamps in first-seen order
// (samples refer to them by index) and the runs of rows of one series.
struct Piece {
  std::vector<Sample> samples;
  std::vector<double> lts;               // distinct timestamps, first-seen order
  std::vector<uint32_t> run_at, run_sid;  // series runs: first sample, series id
  std::vector<uint32_t> map;             // piece series -> builder series (empty: identity)
};

int metric_threads();

struct Builder {
  std::unordered_map<std::string, uint32_t> index;  // serialised key -> provisional series
  std::vector<std::string> keys;                      // by series id (the fast path's keys)
  std::vector<anomod_metrics::Series> series;
  Piece own;                // the rows this builder parsed itself
  std::deque<Piece> parts;  // set by the threaded decode: the pieces, in file order
  std::string key;
  // the timestamp column of the next row: series-major files repeat one
  // series' timestamps in order, so the column after the previous row's is
  // the usual answer (no hash lookup)
  std::unordered_map<double, uint32_t> lidx;
  double last_t = std::nan("");
  uint32_t last_lc = 0, last_s = ~0u;

  void add(double t, float v, uint32_t s) {
    uint32_t lc;
    if (t == last_t) {  // (NaN never matches: timestamps are never NaN)
      lc = last_lc;
    } else if (last_lc + 1 < own.lts.size() && own.lts[last_lc + 1] == t) {
      lc = last_lc + 1;
    } else {
      auto it = lidx.find(t);
      if (it == lidx.end()) {
        it = lidx.emplace(t, (uint32_t)own.lts.size()).first;
        own.lts.push_back(t);
      }
      lc = it->second;
    }
    last_t = t;
    last_lc = lc;
    if (s != last_s) {
      own.run_at.push_back((uint32_t)own.samples.size());
      own.run_sid.push_back(s);
      last_s = s;
    }
    own.samples.push_back({lc, v, s});
  }

  // Series id of a key already serialised as name \0 k1 \0 v1 ...; `make`
  // builds the (name, labels) only when the series is new.
  template <class Make>
  uint32_t series_of_key(const std::string& k, Make&& make) {
    auto it = index.find(k);
    if (it != index.end()) return it->second;
    const uint32_t id = (uint32_t)series.size();
    index.emplace(k, id);
    keys.push_back(k);
    series.push_back(make());
    return id;
  }

  uint32_t series_of(const std::string& name, const Labels& labels) {
    key.assign(name);
    for (const auto& kv : labels) {
      key.push_back('\0');
      key.append(kv.first);
      key.push_back('\0');
      key.append(kv.second);
    }
    auto it = index.find(key);
    if (it != index.end()) return it->second;
    const uint32_t id = (uint32_t)series.size();
    index.emplace(key, id);
    keys.push_back(key);
    series.push_back({name, labels});
    return id;
  }

  anomod_metrics* finish() {
    DT_MARK("decode return");
    auto* out = new anomod_metrics();
    // series in Python tuple order: the serialised keys (name \0 k1 \0 v1 ...,
    // no NUL inside a field) compare bytewise as the (name, labels) tuples do —
    // a name or field that is a prefix of another ends at \0, which sorts first,
    // and a key with fewer labels ends first — so one memcmp per comparison
    std::vector<uint32_t> order(series.size());
    for (uint32_t i = 0; i < order.size(); ++i) order[i] = i;
    bool nul = keys.size() != series.size();
    for (size_t i = 0; !nul && i < series.size(); ++i) {
      nul = series[i].name.find('\0') != std::string::npos;
      for (const auto& kv : series[i].labels)
        nul = nul || kv.first.find('\0') != std::string::npos ||
              kv.second.find('\0') != std::string::npos;
    }
    if (!nul) {
      std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return keys[a] < keys[b]; });
    } else {
      std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        if (series[a].name != series[b].name) return series[a].name < series[b].name;
        return series[a].labels < series[b].labels;
      });
    }
    std::vector<uint32_t> rank(series.size());
    for (uint32_t i = 0; i < order.size(); ++i) rank[order[i]] = i;
    DT_MARK("series sort");
    out->series.reserve(series.size());
    for (uint32_t i : order) out->series.push_back(std::move(series[i]));
    std::vector<const Piece*> ps;
    if (parts.empty()) ps.push_back(&own);
    for (const Piece& p : parts) ps.push_back(&p);
    // distinct timestamps over the pieces (a hash map to a provisional column,
    // then sorted); each piece's columns -> output rows
    std::unordered_map<double, uint32_t> gidx;
    gidx.reserve(1024);
    std::vector<std::vector<uint32_t>> row_of(ps.size());
    size_t n_samples = 0;
    for (size_t k = 0; k < ps.size(); ++k) {
      n_samples += ps[k]->samples.size();
      row_of[k].resize(ps[k]->lts.size());
      for (size_t j = 0; j < ps[k]->lts.size(); ++j) {
        const double t = ps[k]->lts[j];
        auto it = gidx.find(t);
        if (it == gidx.end()) {
          it = gidx.emplace(t, (uint32_t)out->ts.size()).first;
          out->ts.push_back(t);
        }
        row_of[k][j] = it->second;
      }
    }
    std::vector<uint32_t> ord(out->ts.size());
    for (uint32_t k = 0; k < ord.size(); ++k) ord[k] = k;
    std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return out->ts[a] < out->ts[b]; });
    std::vector<uint32_t> crank(ord.size());
    std::vector<double> sorted_ts(ord.size());
    for (uint32_t k = 0; k < ord.size(); ++k) {
      crank[ord[k]] = k;
      sorted_ts[k] = out->ts[ord[k]];
    }
    out->ts.swap(sorted_ts);
    for (auto& r : row_of)
      for (uint32_t& x : r) x = crank[x];
    DT_MARK("timestamps");
    const size_t T = out->ts.size(), S = out->series.size();
    out->X.assign(T * S, std::nanf(""));
    // first occurrence per (series, t): later rows of the same cell skipped.
    // Series-major rows put consecutive samples S cells apart in X[T][S], one
    // cache miss each on one thread; so the series ranks are cut into ranges,
    // one per thread, and every thread walks the pieces' series runs in row
    // order, taking only the runs of its own series (its writes stay in a
    // T x S/threads block).  Cells are disjoint between threads and each cell
    // sees its samples in row order, so the result is the one-thread one.
    std::vector<uint8_t> seen(T * S, 0);
    DT_MARK("X alloc");
    const int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)metric_threads(),
                                                             n_samples / (1u << 16)));
    auto fill = [&](uint32_t lo, uint32_t hi) {
      for (size_t k = 0; k < ps.size(); ++k) {
        const Piece& P = *ps[k];
        const uint32_t* row = row_of[k].data();
        const size_t nr = P.run_at.size();
        for (size_t r = 0; r < nr; ++r) {
          const uint32_t sid = P.run_sid[r];
          const uint32_t rk = rank[P.map.empty() ? sid : P.map[sid]];
          if (rk < lo || rk >= hi) continue;
          const size_t a = P.run_at[r], b = r + 1 < nr ? P.run_at[r + 1] : P.samples.size();
          for (size_t i = a; i < b; ++i) {
            const Sample& sm = P.samples[i];
            const size_t cell = (size_t)row[sm.lc] * S + rk;
            if (seen[cell]) continue;
            seen[cell] = 1;
            out->X[cell] = sm.v;
          }
        }
      }
    };
    if (nt <= 1) {
      fill(0, (uint32_t)S);
    } else {
      std::vector<std::thread> th;
      for (int k = 0; k < nt; ++k)
        th.emplace_back(fill, (uint32_t)(S * (size_t)k / (size_t)nt),
                        (uint32_t)(S * (size_t)(k + 1) / (size_t)nt));
      for (auto& x : th) x.join();
    }
    DT_MARK("fill");
    return out;
  }
};

// Columns of a header: name -> the LAST index with that name (a dict built
// from the row keeps the last value of a repeated name).
std::vector<int> header_last(const std::vector<std::string>& hdr) {
  std::vector<int> keep(hdr.size(), 1);
  for (size_t i = 0; i < hdr.size(); ++i)
    for (size_t j = i + 1; j < hdr.size(); ++j)
      if (hdr[i] == hdr[j]) keep[i] = 0;
  return keep;
}

int find_col(const std::vector<std::string>& hdr, const char* name) {
  int at = -1;
  for (size_t i = 0; i < hdr.size(); ++i)
    if (hdr[i] == name) at = (int)i;
  return at;
}

struct LongHeader {
  std::vector<std::string> hdr;
  std::vector<int> label_cols;  // in label-name order
  int c_name = -1, c_ts = -1, c_val = -1;
};

// The data rows of [p, end) (whole records) into b.
int decode_long_rows(const LongHeader& H, const char* p, const char* end, Builder& b,
                     uint64_t row0) {
  CsvReader rd(p, (size_t)(end - p));
  Labels labels;
  std::string key, prev_key;
  uint32_t prev_s = 0;
  bool have_prev = false;
  // the previous row's series fields (name, then the label columns), when
  // they all view the input itself (a quoted field views the reader's
  // scratch, which the next record reuses)
  std::vector<std::string_view> prev_id(1 + H.label_cols.size());
  bool prev_views = false;
  const auto in_input = [&](std::string_view x) {
    return x.empty() || (x.data() >= p && x.data() + x.size() <= end);
  };
  uint64_t row = row0;
  // room for the rows up front (a collector row is ~80 bytes; one row per 32
  // bytes leaves slack, and shorter rows only fall back to growing): growing
  // by doubling would copy the samples and fault fresh pages for each copy;
  // reserved pages are touched only as rows arrive
  b.own.samples.reserve(b.own.samples.size() + (size_t)(end - p) / 32u);
  while (rd.next()) {
    if (rd.fields.size() == 1 && rd.fields[0].empty()) continue;  // blank line (skipped)
    ++row;
    const auto field = [&](int c) -> std::string_view {
      return c >= 0 && (size_t)c < rd.fields.size() ? rd.fields[c] : std::string_view();
    };
    const std::string_view nm = field(H.c_name);
    // series-major files: the row's series is usually the previous row's,
    // seen here as the same bytes in the same fields (no key built)
    bool same = prev_views && nm == prev_id[0];
    for (size_t j = 0; same && j < H.label_cols.size(); ++j)
      same = field(H.label_cols[j]) == prev_id[j + 1];
    if (!same) {
      key.assign(nm.data(), nm.size());
      for (int c : H.label_cols) {
        const std::string_view v = field(c);
        if (v.empty()) continue;
        key.push_back('\0');
        key.append(H.hdr[c]);
        key.push_back('\0');
        key.append(v.data(), v.size());
      }
    }
    double t;
    if (!parse_float(field(H.c_ts), t) || std::isnan(t)) {
      anomod::set_error(nullptr, "metric CSV row %llu: bad timestamp '%.*s'",
                        (unsigned long long)row, (int)field(H.c_ts).size(), field(H.c_ts).data());
      return ANOMOD_EINVAL;
    }
    const std::string_view vs = field(H.c_val);
    double v = NAN;
    if (!vs.empty() && !parse_float(vs, v)) {
      anomod::set_error(nullptr, "metric CSV row %llu: bad value '%.*s'", (unsigned long long)row,
                        (int)vs.size(), vs.data());
      return ANOMOD_EINVAL;
    }
    // otherwise one compare of the built key before hashing it
    if (!same && (!have_prev || key != prev_key)) {
      prev_s = b.series_of_key(key, [&] {
        labels.clear();
        for (int c : H.label_cols) {
          const std::string_view lv = field(c);
          if (!lv.empty()) labels.emplace_back(H.hdr[c], std::string(lv));
        }
        return anomod_metrics::Series{std::string(nm), labels};
      });
      prev_key.swap(key);
      have_prev = true;
    }
    if (!same) {
      prev_id[0] = nm;
      prev_views = in_input(nm);
      for (size_t j = 0; j < H.label_cols.size(); ++j) {
        prev_id[j + 1] = field(H.label_cols[j]);
        prev_views = prev_views && in_input(prev_id[j + 1]);
      }
    }
    b.add(t, (float)v, prev_s);
  }
  return ANOMOD_OK;
}

int metric_threads() {
  const char* e = getenv("ANOMOD_DECODE_THREADS");
  if (e && atoi(e) > 0) return std::min(atoi(e), 64);
  const unsigned hc = std::thread::hardware_concurrency();
  return (int)std::min<unsigned>(hc ? hc : 1u, 16u);
}

int decode_long(const char* data, uint64_t len, Builder& b) {
  CsvReader rd(data, len);
  if (!rd.next()) return ANOMOD_OK;  // empty file: no rows
  LongHeader H;
  H.hdr.assign(rd.fields.begin(), rd.fields.end());
  const std::vector<int> keep = header_last(H.hdr);
  H.c_name = find_col(H.hdr, "metric_name");
  H.c_ts = find_col(H.hdr, "timestamp");
  H.c_val = find_col(H.hdr, "value");
  for (size_t i = 0; i < H.hdr.size(); ++i)
    if (keep[i] && H.hdr[i] != "metric_name" && H.hdr[i] != "timestamp" &&
        H.hdr[i] != "datetime" && H.hdr[i] != "value")
      H.label_cols.push_back((int)i);
  // label names are distinct: visiting the columns in name order yields each
  // row's non-empty (name, value) pairs already sorted
  std::sort(H.label_cols.begin(), H.label_cols.end(),
            [&](int a, int c) { return H.hdr[a] < H.hdr[c]; });
  if (H.c_name < 0 || H.c_ts < 0) {
    anomod::set_error(nullptr, "metric CSV: no metric_name / timestamp column");
    return ANOMOD_EINVAL;
  }
  const char* body = rd.p;
  const char* end = data + len;
  const int threads = metric_threads();
  // Large files without any quote character (every record ends at a newline)
  // parse in newline-aligned pieces on several threads; the pieces' series
  // and samples are merged in file order, so the result is the one-thread one.
  // (every piece checks itself for quotes in parallel; with one anywhere the
  // parallel result is dropped and the file parses on one thread)
  if (threads > 1 && end - body > (8 << 20)) {
    std::vector<const char*> cut{body};
    for (int t = 1; t < threads; ++t) {
      const char* c = body + (size_t)(end - body) * (size_t)t / (size_t)threads;
      if (c <= cut.back()) continue;
      const char* nl = static_cast<const char*>(memchr(c, '\n', (size_t)(end - c)));
      if (!nl) break;
      if (nl + 1 > cut.back() && nl + 1 < end) cut.push_back(nl + 1);
    }
    cut.push_back(end);
    const size_t np = cut.size() - 1;
    std::vector<Builder> part(np);
    std::vector<int> rc(np, ANOMOD_OK);
    std::vector<uint8_t> quoted(np, 0);
    std::vector<std::thread> th;
    for (size_t k = 0; k < np; ++k)
      th.emplace_back([&, k] {
        quoted[k] = memchr(cut[k], '"', (size_t)(cut[k + 1] - cut[k])) != nullptr;
        try {  // an exception must not leave a worker thread (std::terminate)
          if (!quoted[k]) rc[k] = decode_long_rows(H, cut[k], cut[k + 1], part[k], 0);
        } catch (const std::bad_alloc&) {
          rc[k] = ANOMOD_ENOMEM;
        }
      });
    for (auto& x : th) x.join();
    DT_MARK("parse");
    bool any_quote = false;
    for (size_t k = 0; k < np; ++k) any_quote |= quoted[k] != 0;
    if (any_quote) return decode_long_rows(H, body, end, b, 0);
    for (size_t k = 0; k < np; ++k) {
      if (rc[k] == ANOMOD_ENOMEM)
        anomod::set_error(nullptr, "out of host memory decoding a metric CSV");
      if (rc[k] != ANOMOD_OK) return rc[k];  // (row numbers in the message are per piece)
    }
    // the pieces' series into the builder (file order); their samples move
    // with them, not copied
    for (size_t k = 0; k < np; ++k) {
      Builder& pb = part[k];
      b.parts.push_back(std::move(pb.own));
      std::vector<uint32_t>& map = b.parts.back().map;
      map.resize(pb.series.size());
      for (size_t s = 0; s < pb.series.size(); ++s)
        map[s] = b.series_of_key(pb.keys[s], [&] { return std::move(pb.series[s]); });
    }
    DT_MARK("merge");
    return ANOMOD_OK;
  }
  return decode_long_rows(H, body, end, b, 0);
}

int decode_prom(const char* data, uint64_t len, const std::string& stem, Builder& b) {
  CsvReader rd(data, len);
  if (!rd.next()) return ANOMOD_OK;
  std::vector<std::string> hdr(rd.fields.begin(), rd.fields.end());
  const int c_ts = find_col(hdr, "timestamp"), c_val = find_col(hdr, "value"),
            c_met = find_col(hdr, "metric");
  if (c_ts < 0) {
    anomod::set_error(nullptr, "%s: no timestamp column", stem.c_str());
    return ANOMOD_EINVAL;
  }
  Labels labels(1);
  labels[0].first = "metric";
  uint64_t row = 0;
  while (rd.next()) {
    if (rd.fields.size() == 1 && rd.fields[0].empty()) continue;
    ++row;
    const auto field = [&](int c) -> std::string_view {
      return c >= 0 && (size_t)c < rd.fields.size() ? rd.fields[c] : std::string_view();
    };
    double t;
    if (!iso_timestamp(field(c_ts), t)) {
      anomod::set_error(nullptr, "%s row %llu: bad timestamp '%.*s'", stem.c_str(),
                        (unsigned long long)row, (int)field(c_ts).size(), field(c_ts).data());
      return ANOMOD_EINVAL;
    }
    const std::string_view vs = field(c_val);
    double v = NAN;
    if (!vs.empty() && !parse_float(vs, v)) {
      anomod::set_error(nullptr, "%s row %llu: bad value '%.*s'", stem.c_str(),
                        (unsigned long long)row, (int)vs.size(), vs.data());
      return ANOMOD_EINVAL;
    }
    labels[0].second.assign(field(c_met));
    const uint32_t s = b.series_of(stem, labels);
    b.add(t, (float)v, s);
  }
  return ANOMOD_OK;
}

}  // namespace

extern "C" {

int anomod_decode_metric_long_csv(const char* data, uint64_t len, anomod_metrics** out) {
  if (!out || (!data && len)) {
    anomod::set_error(nullptr, "anomod_decode_metric_long_csv: NULL argument");
    return ANOMOD_EINVAL;
  }
  *out = nullptr;
  try {
    DT_MARK("start");
    {
      Builder b;
      if (int rc = decode_long(data, len, b)) return rc;
      *out = b.finish();
      DT_MARK("finish");
    }
    DT_MARK("builder free");
  } catch (const std::bad_alloc&) {
    anomod::set_error(nullptr, "out of host memory decoding a metric CSV");
    return ANOMOD_ENOMEM;
  }
  return ANOMOD_OK;
}

int anomod_decode_metric_long_csv_file(const char* path, anomod_metrics** out) {
  if (!path || !out) {
    anomod::set_error(nullptr, "anomod_decode_metric_long_csv_file: NULL argument");
    return ANOMOD_EINVAL;
  }
  *out = nullptr;
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    anomod::set_error(nullptr, "metric CSV %s: %s", path, strerror(errno));
    return ANOMOD_EINVAL;
  }
  struct stat st;
  if (fstat(fd, &st) != 0) {
    anomod::set_error(nullptr, "metric CSV %s: %s", path, strerror(errno));
    close(fd);
    return ANOMOD_EINVAL;
  }
  const uint64_t len = (uint64_t)st.st_size;
  if (len == 0) {
    close(fd);
    return anomod_decode_metric_long_csv(nullptr, 0, out);
  }
  // mapped, not read: the parser threads fault their own pieces in parallel
  void* m = mmap(nullptr, (size_t)len, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (m == MAP_FAILED) {
    anomod::set_error(nullptr, "metric CSV %s: mmap: %s", path, strerror(errno));
    return ANOMOD_EINVAL;
  }
  const int rc = anomod_decode_metric_long_csv(static_cast<const char*>(m), len, out);
  munmap(m, (size_t)len);
  return rc;
}

int anomod_decode_prometheus_csvs(const char* const* data, const uint64_t* lens,
                                  const char* const* stems, uint32_t n_files,
                                  anomod_metrics** out) {
  if (!out || (n_files && (!data || !lens || !stems))) {
    anomod::set_error(nullptr, "anomod_decode_prometheus_csvs: NULL argument");
    return ANOMOD_EINVAL;
  }
  *out = nullptr;
  try {
    Builder b;
    for (uint32_t f = 0; f < n_files; ++f)
      if (int rc = decode_prom(data[f], lens[f], stems[f] ? stems[f] : "", b)) return rc;
    *out = b.finish();
  } catch (const std::bad_alloc&) {
    anomod::set_error(nullptr, "out of host memory decoding metric CSVs");
    return ANOMOD_ENOMEM;
  }
  return ANOMOD_OK;
}

int anomod_metrics_info(const anomod_metrics* m, uint64_t* T, uint64_t* S) {
  if (!m) {
    anomod::set_error(nullptr, "anomod_metrics_info: NULL argument");
    return ANOMOD_EINVAL;
  }
  if (T) *T = m->ts.size();
  if (S) *S = m->series.size();
  return ANOMOD_OK;
}

int anomod_metrics_matrix(const anomod_metrics* m, float* X, double* timestamps) {
  if (!m) {
    anomod::set_error(nullptr, "anomod_metrics_matrix: NULL argument");
    return ANOMOD_EINVAL;
  }
  if (X && !m->X.empty()) memcpy(X, m->X.data(), m->X.size() * sizeof(float));
  if (timestamps && !m->ts.empty()) memcpy(timestamps, m->ts.data(), m->ts.size() * sizeof(double));
  return ANOMOD_OK;
}

const char* anomod_metrics_series_name(const anomod_metrics* m, uint64_t s) {
  return m && s < m->series.size() ? m->series[s].name.c_str() : nullptr;
}

uint32_t anomod_metrics_series_nlabels(const anomod_metrics* m, uint64_t s) {
  return m && s < m->series.size() ? (uint32_t)m->series[s].labels.size() : 0u;
}

const char* anomod_metrics_series_label(const anomod_metrics* m, uint64_t s, uint32_t j,
                                        const char** value) {
  if (!m || s >= m->series.size() || j >= m->series[s].labels.size()) return nullptr;
  if (value) *value = m->series[s].labels[j].second.c_str();
  return m->series[s].labels[j].first.c_str();
}

int anomod_metrics_series_packed(const anomod_metrics* m, char* buf, uint64_t cap,
                                 uint32_t* nlabels, uint64_t* bytes) {
  if (!m || !bytes) {
    anomod::set_error(nullptr, "anomod_metrics_series_packed: NULL argument");
    return ANOMOD_EINVAL;
  }
  uint64_t need = 0;
  for (size_t s = 0; s < m->series.size(); ++s) {
    const auto& sr = m->series[s];
    need += sr.name.size() + 1;
    for (const auto& kv : sr.labels) need += kv.first.size() + kv.second.size() + 2;
    if (nlabels) nlabels[s] = (uint32_t)sr.labels.size();
  }
  *bytes = need;
  if (!buf || cap < need) return ANOMOD_OK;
  char* o = buf;
  auto put = [&](const std::string& x) {
    memcpy(o, x.data(), x.size());
    o += x.size();
    *o++ = '\0';
  };
  for (const auto& sr : m->series) {
    put(sr.name);
    for (const auto& kv : sr.labels) {
      put(kv.first);
      put(kv.second);
    }
  }
  return ANOMOD_OK;
}

int anomod_metrics_free(anomod_metrics* m) {
  delete m;
  return ANOMOD_OK;
}

}  // extern "C"
