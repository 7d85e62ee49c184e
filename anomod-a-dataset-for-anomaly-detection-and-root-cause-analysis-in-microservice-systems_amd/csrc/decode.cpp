// Native trace-file decoders: a Jaeger /api/traces dump
// (SN_data/trace_data/*/all_traces.json) or a SkyWalking collector payload
// (TT_data/trace_data/*/*_skywalking_traces_*.json) -> the span SoA the GPU
// kernels read, without a Python object per span.
//
// Column rules (the same as anomod/decode.py, whose outputs are pinned to the
// reference's own CSV / _build_span_records goldens):
//  Jaeger  (jaeger_to_csv.py:21-90)
//    trace_hash = xxh64(traceID)            span_id = id of spanID
//    parent     = id of the first CHILD_OF reference's spanID (:34-38), 0 = none
//    svc        = rank of processes[processID].serviceName among the sorted
//                 service names of the file (:45-46)
//    dur_us     = duration clamped to u32 (:83)
//    flags      = ERROR when the last 'error' tag is true / "true" (any case)
//                 or the last 'http.status_code' tag is an integer >= 500
//    id(s)      = s as hex when it is 1-16 hex digits and not 0, else
//                 xxh64(s) | 2^63; '' -> 0
//  SkyWalking payload (trace_collector.py:564-578, SpanRecord.to_dict :97-123)
//    node ids and parent node ids -> dense per-trace ids (first occurrence
//    + 1; a parent naming no node of the trace -> 2^64 - 1), service_code
//    ranks, duration = max(0, end_ms - start_ms) * 1000 clamped (:87),
//    flags = ERROR when is_error is truthy (:471).
//
// The parser builds a compact DOM (24 B per JSON value) over the caller's
// bytes in one pass; strings are unescaped only when they contain escapes.
// Large documents are decoded element-parallel: a structural scan finds the
// trace array's elements, the rest of the document is validated on its own,
// and byte-balanced runs of elements are parsed and decoded on up to 16
// threads (ANOMOD_DECODE_THREADS), concatenated in file order — the same
// columns as the one-thread path, which is also the fallback for anything
// the scan does not recognise.
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <thread>
#include <vector>
#include <algorithm>

#include "../../include/anomod.h"

namespace anomod {
void set_error(anomod_ctx* ctx, const char* fmt, ...);
}

struct anomod_decoded {
  std::vector<std::string> services;
  std::vector<uint64_t> trace_ptr{0};
  std::vector<uint64_t> trace_hash, span_id, parent;
  std::vector<uint16_t> svc, flags;
  std::vector<uint32_t> dur;
  bool dup_ids = false;  // some trace holds a span id twice (anomod_decoded_unique_ids)
};

namespace {

// ---------------------------------------------------------------- xxh64
constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull,
                   P3 = 1609587929392839161ull, P4 = 9650029242287828579ull,
                   P5 = 2870177450012600261ull;
inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t rd64(const unsigned char* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}
inline uint32_t rd32(const unsigned char* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint64_t round1(uint64_t acc, uint64_t in) {
  acc += in * P2;
  acc = rotl(acc, 31);
  return acc * P1;
}
inline uint64_t merge(uint64_t acc, uint64_t v) {
  acc ^= round1(0, v);
  return acc * P1 + P4;
}

uint64_t xxh64(const void* data, size_t len, uint64_t seed = 0) {
  const auto* p = static_cast<const unsigned char*>(data);
  const unsigned char* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const unsigned char* limit = end - 32;
    do {
      v1 = round1(v1, rd64(p));
      v2 = round1(v2, rd64(p + 8));
      v3 = round1(v3, rd64(p + 16));
      v4 = round1(v4, rd64(p + 24));
      p += 32;
    } while (p <= limit);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = merge(h, v1);
    h = merge(h, v2);
    h = merge(h, v3);
    h = merge(h, v4);
  } else {
    h = seed + P5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    h ^= round1(0, rd64(p));
    h = rotl(h, 27) * P1 + P4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)rd32(p) * P1;
    h = rotl(h, 23) * P2 + P3;
    p += 4;
  }
  while (p < end) {
    h ^= (*p) * P5;
    h = rotl(h, 11) * P1;
    ++p;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

uint64_t hash64(std::string_view s) {
  const uint64_t h = xxh64(s.data(), s.size());
  return h ? h : 1ull;
}

// ---------------------------------------------------------------- JSON DOM
enum : uint8_t { J_NULL, J_FALSE, J_TRUE, J_NUM, J_STR, J_ARR, J_OBJ };
constexpr uint32_t kNone = 0xFFFFFFFFu;

struct Node {
  uint8_t type;
  uint8_t esc;    // string holds escapes
  uint32_t len;   // string / number byte length, or child count
  uint32_t first; // first child (containers); for object members: key, value, key, value...
  uint32_t next;  // next sibling
  uint64_t off;   // byte offset of the string body / number text
};

struct Dom {
  const char* s = nullptr;
  size_t n = 0;
  std::vector<Node> nodes;
  std::string err;

  static bool ws(char c) { return c == ' ' || c == '\n' || c == '\r' || c == '\t'; }

  bool parse(const char* src, size_t len) {
    s = src;
    n = len;
    nodes.clear();
    nodes.reserve(len / 12 + 16);
    struct Frame {
      uint32_t node, last;
    };
    std::vector<Frame> stack;
    size_t i = 0;
    auto skip = [&] {
      while (i < n && ws(s[i])) ++i;
    };
    auto add = [&](uint8_t t, uint64_t off, uint32_t l) -> uint32_t {
      nodes.push_back(Node{t, 0, l, kNone, kNone, off});
      const uint32_t id = (uint32_t)(nodes.size() - 1);
      if (!stack.empty()) {
        Frame& f = stack.back();
        if (f.last == kNone) nodes[f.node].first = id;
        else nodes[f.last].next = id;
        f.last = id;
        nodes[f.node].len++;
      }
      return id;
    };
    auto str = [&]() -> bool {  // at the opening quote
      const size_t start = ++i;
      bool esc = false;
      while (i < n) {
        const char c = s[i];
        if (c == '"') break;
        if (c == '\\') {
          esc = true;
          i += 2;
          continue;
        }
        ++i;
      }
      if (i >= n) return false;
      const uint32_t id = add(J_STR, start, (uint32_t)(i - start));
      nodes[id].esc = esc;
      ++i;
      return true;
    };
    bool expect_key = false;
    bool after_comma = false;  // a ',' must be followed by a value (no trailing commas)
    skip();
    while (true) {
      skip();
      if (i >= n) {
        if (stack.empty() && !nodes.empty()) return true;
        err = "unexpected end of input";
        return false;
      }
      const bool in_obj = !stack.empty() && nodes[stack.back().node].type == J_OBJ;
      char c = s[i];
      const bool closer = c == '}' || c == ']';
      if (closer && after_comma) break;  // trailing comma
      after_comma = false;
      if (closer) {
        if (stack.empty()) break;
        const uint8_t want = c == '}' ? J_OBJ : J_ARR;
        if (nodes[stack.back().node].type != want) break;
        stack.pop_back();
        ++i;
      } else if (in_obj && expect_key) {
        if (c != '"' || !str()) break;
        skip();
        if (i >= n || s[i] != ':') break;
        ++i;
        expect_key = false;
        continue;
      } else if (c == '{' || c == '[') {
        const uint32_t id = add(c == '{' ? J_OBJ : J_ARR, i, 0);
        nodes[id].len = 0;
        stack.push_back(Frame{id, kNone});
        ++i;
        expect_key = c == '{';
        skip();
        if (i < n && (s[i] == '}' || s[i] == ']')) continue;
        if (c == '{') continue;
        continue;
      } else if (c == '"') {
        if (!str()) break;
      } else if (c == 't' && n - i >= 4 && std::memcmp(s + i, "true", 4) == 0) {
        add(J_TRUE, i, 4);
        i += 4;
      } else if (c == 'f' && n - i >= 5 && std::memcmp(s + i, "false", 5) == 0) {
        add(J_FALSE, i, 5);
        i += 5;
      } else if (c == 'n' && n - i >= 4 && std::memcmp(s + i, "null", 4) == 0) {
        add(J_NULL, i, 4);
        i += 4;
      } else if (c == '-' || (c >= '0' && c <= '9')) {
        const size_t start = i++;
        while (i < n && (std::isdigit((unsigned char)s[i]) || s[i] == '.' || s[i] == 'e' ||
                         s[i] == 'E' || s[i] == '+' || s[i] == '-'))
          ++i;
        add(J_NUM, start, (uint32_t)(i - start));
      } else {
        break;
      }
      // after a value: ',' or a closer
      if (stack.empty()) {
        skip();
        if (i == n) return true;
        break;
      }
      skip();
      if (i < n && s[i] == ',') {
        ++i;
        after_comma = true;
        expect_key = nodes[stack.back().node].type == J_OBJ;
      } else if (i < n && (s[i] == '}' || s[i] == ']')) {
        // handled at the top of the loop
      } else {
        break;
      }
    }
    if (err.empty()) err = "invalid JSON at byte " + std::to_string(i);
    return false;
  }

  const Node& at(uint32_t id) const { return nodes[id]; }

  std::string_view raw(uint32_t id) const { return {s + nodes[id].off, nodes[id].len}; }

  // Unescaped string value (JSON \uXXXX incl. surrogate pairs -> UTF-8).
  std::string text(uint32_t id) const {
    const Node& nd = nodes[id];
    std::string_view r = raw(id);
    if (!nd.esc) return std::string(r);
    std::string out;
    out.reserve(r.size());
    for (size_t k = 0; k < r.size(); ++k) {
      char c = r[k];
      if (c != '\\' || k + 1 >= r.size()) {
        out.push_back(c);
        continue;
      }
      c = r[++k];
      switch (c) {
        case 'n': out.push_back('\n'); break;
        case 't': out.push_back('\t'); break;
        case 'r': out.push_back('\r'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'u': {
          auto hex4 = [&](size_t p) -> uint32_t {
            uint32_t v = 0;
            for (size_t q = p; q < p + 4 && q < r.size(); ++q) {
              const char h = r[q];
              v = v * 16 + (uint32_t)(h <= '9' ? h - '0' : (h | 32) - 'a' + 10);
            }
            return v;
          };
          uint32_t cp = hex4(k + 1);
          k += 4;
          if (cp >= 0xD800 && cp < 0xDC00 && k + 6 < r.size() + 1 && r[k + 1] == '\\' &&
              r[k + 2] == 'u') {
            const uint32_t lo = hex4(k + 3);
            if (lo >= 0xDC00 && lo < 0xE000) {
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              k += 6;
            }
          }
          if (cp < 0x80) {
            out.push_back((char)cp);
          } else if (cp < 0x800) {
            out.push_back((char)(0xC0 | (cp >> 6)));
            out.push_back((char)(0x80 | (cp & 63)));
          } else if (cp < 0x10000) {
            out.push_back((char)(0xE0 | (cp >> 12)));
            out.push_back((char)(0x80 | ((cp >> 6) & 63)));
            out.push_back((char)(0x80 | (cp & 63)));
          } else {
            out.push_back((char)(0xF0 | (cp >> 18)));
            out.push_back((char)(0x80 | ((cp >> 12) & 63)));
            out.push_back((char)(0x80 | ((cp >> 6) & 63)));
            out.push_back((char)(0x80 | (cp & 63)));
          }
          break;
        }
        default: out.push_back(c);  // \" \\ \/
      }
    }
    return out;
  }

  // Member `key` of object `obj` (the LAST one, as json.load keeps), or kNone.
  uint32_t get(uint32_t obj, std::string_view key) const {
    if (obj == kNone || nodes[obj].type != J_OBJ) return kNone;
    uint32_t found = kNone;
    for (uint32_t k = nodes[obj].first; k != kNone; k = nodes[nodes[k].next].next) {
      const uint32_t v = nodes[k].next;
      const Node& kn = nodes[k];
      if (!kn.esc ? raw(k) == key : text(k) == key) found = v;
      if (v == kNone) break;
    }
    return found;
  }
};

// ---------------------------------------------------------------- value rules
bool is_hex_id(std::string_view s, uint64_t& v) {
  if (s.empty() || s.size() > 16) return false;
  v = 0;
  for (char c : s) {
    int d;
    if (c >= '0' && c <= '9') d = c - '0';
    else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
    else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
    else return false;
    v = v * 16 + (uint64_t)d;
  }
  return v != 0;
}

// The string form of a scalar JSON value as Python's str() of the json.load
// result prints it for the id fields we hash (strings, integers, booleans).
std::string py_str(const Dom& d, uint32_t id) {
  if (id == kNone) return "";
  switch (d.at(id).type) {
    case J_STR: return d.text(id);
    case J_TRUE: return "True";
    case J_FALSE: return "False";
    case J_NULL: return "None";
    default: return std::string(d.raw(id));
  }
}

uint64_t span_id_of(const Dom& d, uint32_t id) {
  if (id == kNone || d.at(id).type == J_NULL) return 0;
  const std::string s = py_str(d, id);
  if (s.empty()) return 0;
  uint64_t v;
  if (is_hex_id(s, v)) return v;
  return hash64(s) | (1ull << 63);
}

// int(v) of a JSON value as Python would take it, when it is an integer
// (strings: optional sign / surrounding whitespace / underscores between
// digits; floats truncate; bools are 0/1).  false when int() would raise.
bool py_int(const Dom& d, uint32_t id, long double& out) {
  if (id == kNone) return false;
  const Node& nd = d.at(id);
  if (nd.type == J_TRUE || nd.type == J_FALSE) {
    out = nd.type == J_TRUE;
    return true;
  }
  if (nd.type == J_NUM) {
    const std::string r(d.raw(id));
    char* e = nullptr;
    const long double v = std::strtold(r.c_str(), &e);
    if (!std::isfinite((double)v)) return false;
    out = std::trunc(v);
    return true;
  }
  if (nd.type != J_STR) return false;
  std::string t = d.text(id);
  size_t a = 0, b = t.size();
  while (a < b && std::isspace((unsigned char)t[a])) ++a;
  while (b > a && std::isspace((unsigned char)t[b - 1])) --b;
  if (a == b) return false;
  bool neg = false;
  if (t[a] == '+' || t[a] == '-') neg = t[a++] == '-';
  if (a == b) return false;
  long double v = 0;
  bool prev_digit = false;
  for (size_t k = a; k < b; ++k) {
    const char c = t[k];
    if (c == '_' && prev_digit && k + 1 < b && std::isdigit((unsigned char)t[k + 1])) {
      prev_digit = false;
      continue;
    }
    if (!std::isdigit((unsigned char)c)) return false;
    v = v * 10 + (c - '0');
    prev_digit = true;
  }
  out = neg ? -v : v;
  return true;
}

uint32_t clamp_u32(const Dom& d, uint32_t id) {
  long double v;
  if (!py_int(d, id, v)) return 0;
  if (v < 0) return 0;
  if (v > 4294967295.0L) return 0xFFFFFFFFu;
  return (uint32_t)v;
}

bool truthy_error_tag(const Dom& d, uint32_t id) {
  if (id == kNone) return false;
  const Node& nd = d.at(id);
  if (nd.type == J_TRUE) return true;
  if (nd.type != J_STR) return false;
  std::string t = d.text(id);
  for (char& c : t) c = (char)std::tolower((unsigned char)c);
  return t == "true";
}

bool truthy(const Dom& d, uint32_t id) {  // Python bool() of a JSON value
  if (id == kNone) return false;
  const Node& nd = d.at(id);
  switch (nd.type) {
    case J_TRUE: return true;
    case J_FALSE:
    case J_NULL: return false;
    case J_STR: return nd.len > 0;
    case J_NUM: return std::strtold(std::string(d.raw(id)).c_str(), nullptr) != 0;
    default: return nd.len > 0;  // non-empty container
  }
}

// Per-span service names as ids into a small local dictionary (a thread's or
// the whole file's), resolved to sorted-name ranks once at the end — no
// string per span.
struct Names {
  std::unordered_map<std::string, uint32_t> index;
  std::vector<const std::string*> list;  // id -> name (keys of index)
  std::vector<uint32_t> ids;              // per span
  void push(std::string&& nm) {
    auto [it, inserted] = index.try_emplace(std::move(nm), (uint32_t)list.size());
    if (inserted) list.push_back(&it->first);
    ids.push_back(it->second);
  }
};

// Ranks of the names in `parts` (in order, one svc per span) against the
// sorted distinct names (or the caller's fixed list; 0xFFFF = absent).
void resolve_names(const std::vector<Names*>& parts, const std::vector<std::string>* fixed,
                   anomod_decoded* out) {
  std::vector<std::string> svc_names;
  if (fixed) {
    svc_names = *fixed;
  } else {
    for (const Names* p : parts)
      for (const std::string* nm : p->list) svc_names.push_back(*nm);
    std::sort(svc_names.begin(), svc_names.end());
    svc_names.erase(std::unique(svc_names.begin(), svc_names.end()), svc_names.end());
  }
  std::unordered_map<std::string, uint32_t> rank;
  for (uint32_t k = 0; k < svc_names.size(); ++k) rank.emplace(svc_names[k], k);
  size_t ns = 0;
  for (const Names* p : parts) ns += p->ids.size();
  out->svc.resize(ns);
  size_t o = 0;
  for (const Names* p : parts) {
    std::vector<uint16_t> lut(p->list.size());
    for (size_t k = 0; k < p->list.size(); ++k) {
      auto it = rank.find(*p->list[k]);
      lut[k] = it == rank.end() ? 0xFFFF : (uint16_t)it->second;
    }
    for (uint32_t id : p->ids) out->svc[o++] = lut[id];
  }
  out->services = std::move(svc_names);
}

// One element of the dump's "data" array -> its spans (jaeger_to_csv.py:21-90).
void jaeger_trace(const Dom& d, uint32_t tr, anomod_decoded* out, Names& names,
                  std::unordered_map<std::string, std::string>& proc) {
  const uint64_t th = hash64(py_str(d, d.get(tr, "traceID")));
  proc.clear();
  const uint32_t procs = d.get(tr, "processes");
  if (procs != kNone && d.at(procs).type == J_OBJ) {
    for (uint32_t k = d.at(procs).first; k != kNone; k = d.at(d.at(k).next).next) {
      const uint32_t info = d.at(k).next;
      const uint32_t sn = d.get(info, "serviceName");
      proc[d.text(k)] = sn == kNone ? std::string() : py_str(d, sn);
      if (info == kNone) break;
    }
  }
  const uint32_t spans = d.get(tr, "spans");
  if (spans != kNone && d.at(spans).type == J_ARR) {
    for (uint32_t sp = d.at(spans).first; sp != kNone; sp = d.at(sp).next) {
      uint64_t parent = 0;
      const uint32_t refs = d.get(sp, "references");
      if (refs != kNone && d.at(refs).type == J_ARR) {
        for (uint32_t r = d.at(refs).first; r != kNone; r = d.at(r).next) {
          const uint32_t rt = d.get(r, "refType");
          if (rt != kNone && d.at(rt).type == J_STR && d.text(rt) == "CHILD_OF") {
            parent = span_id_of(d, d.get(r, "spanID"));
            break;
          }
        }
      }
      uint32_t err_tag = kNone, status = kNone;
      const uint32_t tags = d.get(sp, "tags");
      if (tags != kNone && d.at(tags).type == J_ARR) {
        for (uint32_t t = d.at(tags).first; t != kNone; t = d.at(t).next) {
          const uint32_t key = d.get(t, "key");
          const std::string ks = key == kNone ? std::string() : py_str(d, key);
          if (ks == "error") err_tag = d.get(t, "value");
          else if (ks == "http.status_code") status = d.get(t, "value");
        }
      }
      long double code = 0;
      const bool error = truthy_error_tag(d, err_tag) || (py_int(d, status, code) && code >= 500);
      const uint32_t pid = d.get(sp, "processID");
      auto it = proc.find(pid == kNone ? std::string() : py_str(d, pid));
      names.push(it == proc.end() ? std::string() : it->second);
      out->trace_hash.push_back(th);
      out->span_id.push_back(span_id_of(d, d.get(sp, "spanID")));
      out->parent.push_back(parent);
      out->flags.push_back(error ? ANOMOD_FLAG_ERROR : 0);
      out->dur.push_back(clamp_u32(d, d.get(sp, "duration")));
    }
  }
  // span ids unique inside the trace? (lets the GPU parent scans run from
  // both ends; a sort of the trace's ids, O(L log L))
  if (!out->dup_ids) {
    thread_local std::vector<uint64_t> ids;
    ids.assign(out->span_id.begin() + (std::ptrdiff_t)out->trace_ptr.back(), out->span_id.end());
    std::sort(ids.begin(), ids.end());
    out->dup_ids = std::adjacent_find(ids.begin(), ids.end()) != ids.end();
  }
  out->trace_ptr.push_back(out->span_id.size());
}

// One element of the payload's "traces" array (trace_collector.py:564-578).
void skywalking_trace(const Dom& d, uint32_t tr, anomod_decoded* out, Names& names,
                      std::unordered_map<std::string, uint64_t>& first) {
  const uint32_t spans = d.get(tr, "spans");
  if (spans == kNone || d.at(spans).type != J_ARR || d.at(spans).len == 0) return;
  std::string tid;
  const uint32_t summ = d.get(tr, "summary");
  const uint32_t st = d.get(summ, "trace_id");
  if (st != kNone && truthy(d, st)) tid = py_str(d, st);
  else {
    const uint32_t s0 = d.get(d.at(spans).first, "trace_id");
    if (s0 != kNone && truthy(d, s0)) tid = py_str(d, s0);
  }
  const uint64_t th = hash64(tid);
  first.clear();
  uint64_t k = 0;
  for (uint32_t sp = d.at(spans).first; sp != kNone; sp = d.at(sp).next, ++k)
    if (!first.emplace(py_str(d, d.get(sp, "node_id")), k + 1).second)
      out->dup_ids = true;  // a node id twice: both spans get its first occurrence's id
  for (uint32_t sp = d.at(spans).first; sp != kNone; sp = d.at(sp).next) {
    out->trace_hash.push_back(th);
    out->span_id.push_back(first[py_str(d, d.get(sp, "node_id"))]);
    const uint32_t pn = d.get(sp, "parent_node_id");
    uint64_t p = 0;
    if (pn != kNone && d.at(pn).type != J_NULL) {
      auto it = first.find(py_str(d, pn));
      p = it == first.end() ? ~0ull : it->second;
    }
    out->parent.push_back(p);
    const uint32_t sc = d.get(sp, "service_code");
    names.push(sc != kNone && truthy(d, sc) ? py_str(d, sc) : std::string());
    long double a = 0, b = 0;
    const uint32_t sa = d.get(sp, "start_timestamp_ms"), sb = d.get(sp, "end_timestamp_ms");
    const bool ok = (!truthy(d, sa) || py_int(d, sa, a)) && (!truthy(d, sb) || py_int(d, sb, b));
    if (!truthy(d, sa)) a = 0;
    if (!truthy(d, sb)) b = 0;
    long double us = ok ? (b - a) * 1000.0L : 0;
    if (us < 0) us = 0;
    out->dur.push_back(us > 4294967295.0L ? 0xFFFFFFFFu : (uint32_t)us);
    out->flags.push_back(truthy(d, d.get(sp, "is_error")) ? ANOMOD_FLAG_ERROR : 0);
  }
  out->trace_ptr.push_back(out->span_id.size());
}

constexpr const char* kTopKey[2] = {"data", "traces"};  // Jaeger dump, SkyWalking payload

bool decode_sequential(const Dom& d, int kind, anomod_decoded* out, Names& names,
                       std::string& err) {
  const uint32_t root = 0;
  if (d.at(root).type != J_OBJ) {
    err = kind == 0 ? "Jaeger dump: top level is not an object"
                    : "SkyWalking payload: top level is not an object";
    return false;
  }
  const uint32_t arr = d.get(root, kTopKey[kind]);
  if (arr == kNone || d.at(arr).type != J_ARR) return true;  // no traces
  std::unordered_map<std::string, std::string> proc;
  std::unordered_map<std::string, uint64_t> first;
  for (uint32_t tr = d.at(arr).first; tr != kNone; tr = d.at(tr).next) {
    if (kind == 0) jaeger_trace(d, tr, out, names, proc);
    else skywalking_trace(d, tr, out, names, first);
  }
  return true;
}

// ------------------------------------------------------- parallel decode
// Structural scan: the byte ranges of the elements of the array that is the
// value of the LAST top-level member `key` (the one json.load keeps).  Only
// strings (with escapes) and nesting are tracked; anything unexpected makes
// it return false and the caller takes the sequential path, whose parser
// reports the error.
struct ByteRange {
  size_t b, e;
};

bool top_array_elements(const char* s, size_t n, std::string_view key, size_t& open, size_t& close,
                        std::vector<ByteRange>& elems) {
  auto ws = [](char c) { return c == ' ' || c == '\n' || c == '\r' || c == '\t'; };
  size_t i = 0;
  while (i < n && ws(s[i])) ++i;
  if (i >= n || s[i] != '{') return false;
  int depth = 0;
  bool expect_key = false, found = false, in_target = false, want_value = false;
  bool key_is_target = false;
  size_t elem_start = 0;
  bool elem_open = false;
  auto end_string = [&](size_t q) -> size_t {  // q just past the opening quote -> closing quote
    while (true) {
      const void* hit = std::memchr(s + q, '"', n - q);
      if (!hit) return n;
      const size_t c = (size_t)((const char*)hit - s);
      size_t bs = 0;
      while (c > bs && s[c - 1 - bs] == '\\') ++bs;
      if ((bs & 1u) == 0) return c;
      q = c + 1;
    }
  };
  for (; i < n; ++i) {
    const char c = s[i];
    if (ws(c)) {
      // indentation runs: skip 8 spaces at a time
      while (i + 9 <= n) {
        uint64_t w;
        std::memcpy(&w, s + i + 1, 8);
        if (w != 0x2020202020202020ull) break;
        i += 8;
      }
      continue;
    }
    if (in_target && depth == 2 && !elem_open && c != ']' && c != ',') {
      elem_start = i;
      elem_open = true;
    }
    if (c == '"') {
      const size_t q = end_string(i + 1);
      if (q >= n) return false;
      if (depth == 1 && expect_key) {
        const std::string_view k(s + i + 1, q - i - 1);
        if (k.find('\\') != std::string_view::npos) return false;  // escaped key: rare, bail
        key_is_target = k == key;
        expect_key = false;
        want_value = true;
      }
      i = q;
      continue;
    }
    if (c == ':') continue;
    if (c == '{' || c == '[') {
      ++depth;
      if (depth == 1) {
        expect_key = true;
      } else if (depth == 2 && want_value) {
        want_value = false;
        if (key_is_target && c == '[') {
          in_target = true;
          found = true;
          open = i;
          elems.clear();
          elem_open = false;
        }
      }
      continue;
    }
    if (c == '}' || c == ']') {
      if (in_target && depth == 2) {
        if (elem_open) {
          size_t e = i;
          while (e > elem_start && ws(s[e - 1])) --e;
          elems.push_back({elem_start, e});
          elem_open = false;
        } else if (!elems.empty()) {
          return false;  // trailing comma
        }
        close = i;
        in_target = false;
      } else if (in_target && depth == 3) {
        // closing an element's container: the element continues to the separator
      }
      --depth;
      if (depth < 0) return false;
      if (depth == 0) {
        // root closed: only whitespace may follow
        for (++i; i < n; ++i)
          if (!ws(s[i])) return false;
        return found;
      }
      continue;
    }
    if (c == ',') {
      if (depth == 1) {
        expect_key = true;
        want_value = false;
      } else if (in_target && depth == 2) {
        if (!elem_open) return false;  // empty element
        size_t e = i;
        while (e > elem_start && ws(s[e - 1])) --e;
        elems.push_back({elem_start, e});
        elem_open = false;
      }
      continue;
    }
    // scalar byte (number / literal)
    if (depth == 1) want_value = false;
  }
  return false;
}

int decode_threads() {
  const char* e = getenv("ANOMOD_DECODE_THREADS");
  if (e && atoi(e) > 0) return atoi(e);
  const unsigned hc = std::thread::hardware_concurrency();
  return (int)std::min<unsigned>(hc ? hc : 1u, 16u);
}

// Element-parallel decode: the skeleton (the document with the array
// emptied) is parsed to validate everything outside the elements; the
// elements are split into contiguous byte-balanced runs, one per thread, each
// parsed and decoded independently and concatenated in order.  Returns false
// when the document is not in that shape or an element fails to parse (the
// caller then runs the sequential path).
bool decode_parallel(const char* json, size_t len, int kind, anomod_decoded* out,
                     std::vector<Names>& names, int threads) {
  size_t open = 0, close = 0;
  std::vector<ByteRange> elems;
  if (!top_array_elements(json, len, kTopKey[kind], open, close, elems)) return false;
  if (elems.size() < 2 * (size_t)threads) return false;  // not worth it
  {
    std::string skel(json, open + 1);
    skel.append(json + close, len - close);
    Dom sd;
    if (!sd.parse(skel.data(), skel.size()) || sd.at(0).type != J_OBJ) return false;
    const uint32_t arr = sd.get(0, kTopKey[kind]);
    if (arr == kNone || sd.at(arr).type != J_ARR) return false;
  }
  const size_t total = elems.back().e - elems.front().b;
  std::vector<size_t> cut{0};
  for (int t = 1; t < threads; ++t) {
    const size_t target = elems.front().b + total * (size_t)t / (size_t)threads;
    size_t k = cut.back();
    while (k < elems.size() && elems[k].b < target) ++k;
    cut.push_back(k);
  }
  cut.push_back(elems.size());
  std::vector<anomod_decoded> part(threads);
  names.assign(threads, Names());
  std::vector<char> ok(threads, 1), oom(threads, 0);
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) {
    pool.emplace_back([&, t] {
      try {  // an exception must not leave a worker thread (std::terminate)
        Dom d;
        std::unordered_map<std::string, std::string> proc;
        std::unordered_map<std::string, uint64_t> first;
        for (size_t k = cut[t]; k < cut[t + 1]; ++k) {
          if (!d.parse(json + elems[k].b, elems[k].e - elems[k].b)) {
            ok[t] = 0;
            return;
          }
          if (kind == 0) jaeger_trace(d, 0, &part[t], names[t], proc);
          else skywalking_trace(d, 0, &part[t], names[t], first);
        }
      } catch (const std::bad_alloc&) {
        oom[t] = 1;
      }
    });
  }
  for (auto& th : pool) th.join();
  for (int t = 0; t < threads; ++t)
    if (oom[t]) throw std::bad_alloc();  // reported by decode_common as ANOMOD_ENOMEM
  for (int t = 0; t < threads; ++t)
    if (!ok[t]) return false;
  size_t ns = 0, nt = 0;
  for (const auto& p : part) {
    ns += p.span_id.size();
    nt += p.trace_ptr.size() - 1;
  }
  out->trace_hash.reserve(ns);
  out->span_id.reserve(ns);
  out->parent.reserve(ns);
  out->flags.reserve(ns);
  out->dur.reserve(ns);
  out->trace_ptr.reserve(nt + 1);
  for (int t = 0; t < threads; ++t) {
    const uint64_t base = out->span_id.size();
    auto app = [](auto& dst, const auto& src) { dst.insert(dst.end(), src.begin(), src.end()); };
    app(out->trace_hash, part[t].trace_hash);
    app(out->span_id, part[t].span_id);
    app(out->parent, part[t].parent);
    app(out->flags, part[t].flags);
    app(out->dur, part[t].dur);
    out->dup_ids = out->dup_ids || part[t].dup_ids;
    for (size_t k = 1; k < part[t].trace_ptr.size(); ++k)
      out->trace_ptr.push_back(base + part[t].trace_ptr[k]);
  }
  return true;
}

thread_local std::string g_decode_err;

int decode_common_impl(const char* json, uint64_t len, const char* const* services,
                       uint32_t n_services, int kind, anomod_decoded** out);

int decode_common(const char* json, uint64_t len, const char* const* services, uint32_t n_services,
                  int kind, anomod_decoded** out) {
  try {
    return decode_common_impl(json, len, services, n_services, kind, out);
  } catch (const std::bad_alloc&) {
    if (out) *out = nullptr;
    anomod::set_error(nullptr, "anomod_decode: out of host memory");
    return ANOMOD_ENOMEM;
  }
}

int decode_common_impl(const char* json, uint64_t len, const char* const* services,
                       uint32_t n_services, int kind, anomod_decoded** out) {
  if (!out || (!json && len)) {
    anomod::set_error(nullptr, "anomod_decode: NULL argument");
    return ANOMOD_EINVAL;
  }
  *out = nullptr;
  std::unique_ptr<anomod_decoded> owned(new anomod_decoded());  // freed if anything throws
  anomod_decoded* res = owned.get();
  std::vector<Names> names;
  const int threads = decode_threads();
  if (threads <= 1 || len < (64u << 10) ||
      !decode_parallel(json, (size_t)len, kind, res, names, threads)) {
    *res = anomod_decoded();
    names.assign(1, Names());
    Dom d;
    if (!d.parse(json, (size_t)len)) {
      anomod::set_error(nullptr, "anomod_decode: %s", d.err.c_str());
      return ANOMOD_EINVAL;
    }
    std::string err;
    if (!decode_sequential(d, kind, res, names[0], err)) {
      anomod::set_error(nullptr, "anomod_decode: %s", err.c_str());
      return ANOMOD_EINVAL;
    }
  }
  std::vector<std::string> fixed;
  if (services) {
    for (uint32_t k = 0; k < n_services; ++k) fixed.emplace_back(services[k] ? services[k] : "");
  }
  std::vector<Names*> parts;
  for (Names& nm : names) parts.push_back(&nm);
  resolve_names(parts, services ? &fixed : nullptr, res);
  for (uint16_t v : res->svc) {
    if (v == 0xFFFF) {
      anomod::set_error(nullptr, "anomod_decode: a span's service is not in the service list");
      return ANOMOD_EINVAL;
    }
  }
  if (res->services.size() > 0xFFFF) {
    anomod::set_error(nullptr, "anomod_decode: more than 65535 services");
    return ANOMOD_EINVAL;
  }
  *out = owned.release();
  return ANOMOD_OK;
}

}  // namespace

extern "C" {

int anomod_decode_jaeger(const char* json, uint64_t len, const char* const* services,
                         uint32_t n_services, anomod_decoded** out) {
  return decode_common(json, len, services, n_services, 0, out);
}

int anomod_decode_skywalking(const char* json, uint64_t len, const char* const* services,
                             uint32_t n_services, anomod_decoded** out) {
  return decode_common(json, len, services, n_services, 1, out);
}

int anomod_decoded_info(const anomod_decoded* d, uint64_t* n_spans, uint64_t* n_traces,
                        uint32_t* n_services) {
  if (!d) {
    anomod::set_error(nullptr, "anomod_decoded_info: NULL argument");
    return ANOMOD_EINVAL;
  }
  if (n_spans) *n_spans = d->span_id.size();
  if (n_traces) *n_traces = d->trace_ptr.size() - 1;
  if (n_services) *n_services = (uint32_t)d->services.size();
  return ANOMOD_OK;
}

int anomod_decoded_unique_ids(const anomod_decoded* d, int* unique) {
  if (!d || !unique) {
    anomod::set_error(nullptr, "anomod_decoded_unique_ids: NULL argument");
    return ANOMOD_EINVAL;
  }
  *unique = d->dup_ids ? 0 : 1;
  return ANOMOD_OK;
}

const char* anomod_decoded_service(const anomod_decoded* d, uint32_t i) {
  if (!d || i >= d->services.size()) return nullptr;
  return d->services[i].c_str();
}

int anomod_decoded_columns(const anomod_decoded* d, const anomod_span_soa_out* dst,
                           uint64_t* trace_ptr) {
  if (!d || !dst) {
    anomod::set_error(nullptr, "anomod_decoded_columns: NULL argument");
    return ANOMOD_EINVAL;
  }
  const size_t n = d->span_id.size();
  auto cp = [&](void* to, const void* from, size_t bytes) {
    if (to && bytes) std::memcpy(to, from, bytes);
  };
  cp(dst->trace_hash, d->trace_hash.data(), n * 8);
  cp(dst->span_id, d->span_id.data(), n * 8);
  cp(dst->parent_span_id, d->parent.data(), n * 8);
  cp(dst->svc, d->svc.data(), n * 2);
  cp(dst->flags, d->flags.data(), n * 2);
  cp(dst->dur_us, d->dur.data(), n * 4);
  cp(trace_ptr, d->trace_ptr.data(), d->trace_ptr.size() * 8);
  return ANOMOD_OK;
}

int anomod_decoded_free(anomod_decoded* d) {
  delete d;
  return ANOMOD_OK;
}

uint64_t anomod_hash64(const char* s, uint64_t len) {
  return hash64(std::string_view(s ? s : "", s ? (size_t)len : 0));
}

}  // extern "C"
