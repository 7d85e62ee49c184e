// Synthetic span workloads + device span sets (upload / generate / download).
//
// Topologies:
//  * SN — DeathStarBench SocialNetwork: the 12 services Jaeger lists in
//    SN_data/trace_data/*/available_services.json; request mix 60 % read
//    home timeline / 30 % read user timeline / 10 % compose post
//    (DeathStarBench/socialNetwork/wrk2/scripts/social-network/
//    mixed-workload.lua:113-115); call trees follow the Thrift client pools
//    seen in SN_data/coverage_data/*/<svc>/*Handler.h.gcov (compose-post ->
//    {unique-id, text, media, user, post-storage, user-timeline,
//    home-timeline}; text -> {url-shorten, user-mention}; home-timeline ->
//    {post-storage, social-graph}; user-timeline -> post-storage).
//  * TT — TrainTicket: the ts-*-service deployments of
//    train-ticket/deployment/kubernetes-manifests (+ ts-ui-dashboard) with
//    SkyWalking-style span trees (Entry span per service visit, one Exit span
//    per downstream call, one MySQL Exit span for database-backed services).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "synth.h"

namespace anomod {

struct HostTopo {
  std::vector<std::string> services;  // sorted
  std::vector<uint32_t> tmpl_cdf;
  std::vector<uint32_t> tmpl_off;
  std::vector<int32_t> span_parent;
  std::vector<uint16_t> span_svc;
  std::vector<uint16_t> span_op;
  std::vector<uint32_t> dur_q;
  uint32_t dur_quant = 1;  // us
};

namespace {

// Acklam's rational approximation of the standard normal quantile.
double norm_ppf(double p) {
  static const double a[] = {-3.969683028665376e+01, 2.209460984245205e+02,
                             -2.759285104469687e+02, 1.383577518672690e+02,
                             -3.066479806614716e+01, 2.506628277459239e+00};
  static const double b[] = {-5.447609879822406e+01, 1.615858368580409e+02,
                             -1.556989798598866e+02, 6.680131188771972e+01,
                             -1.328068155288572e+01};
  static const double c[] = {-7.784894002430293e-03, -3.223964580411365e-01,
                             -2.400758277161838e+00, -2.549732539343734e+00,
                             4.374664141464968e+00,  2.938163982698783e+00};
  static const double d[] = {7.784695709041462e-03, 3.224671290700398e-01,
                             2.445134137142996e+00, 3.754408661907416e+00};
  const double pl = 0.02425, ph = 1 - pl;
  if (p < pl) {
    double q = std::sqrt(-2 * std::log(p));
    return (((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
           ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1);
  }
  if (p > ph) {
    double q = std::sqrt(-2 * std::log(1 - p));
    return -(((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
           ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1);
  }
  double q = p - 0.5, r = q * q;
  return (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * q /
         (((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1);
}

struct SpanDef {
  int parent;
  std::string svc;
  double median_us;
  double sigma;
};

struct Builder {
  HostTopo topo;
  std::map<std::string, uint16_t> svc_index;
  std::vector<double> weights;

  explicit Builder(std::vector<std::string> services) {
    std::sort(services.begin(), services.end());
    topo.services = services;
    for (size_t i = 0; i < services.size(); ++i) svc_index[services[i]] = (uint16_t)i;
    topo.tmpl_off.push_back(0);
  }

  void add_template(const std::vector<SpanDef>& spans, double weight) {
    for (const SpanDef& s : spans) {
      topo.span_parent.push_back(s.parent);
      topo.span_svc.push_back(svc_index.at(s.svc));
      const uint16_t op = (uint16_t)(topo.dur_q.size() / kDurQuantiles);
      topo.span_op.push_back(op);
      for (int i = 0; i < kDurQuantiles; ++i) {
        const double z = norm_ppf((i + 0.5) / kDurQuantiles);
        const double v = std::llround(s.median_us * std::exp(s.sigma * z));
        topo.dur_q.push_back((uint32_t)std::min(std::max(v, 1.0), 4.0e9));
      }
    }
    topo.tmpl_off.push_back((uint32_t)topo.span_parent.size());
    weights.push_back(weight);
  }

  HostTopo finish() {
    double tot = 0;
    for (double w : weights) tot += w;
    double acc = 0;
    for (size_t i = 0; i < weights.size(); ++i) {
      acc += weights[i];
      const double thr = (i + 1 == weights.size()) ? 4294967295.0 : acc / tot * 4294967296.0;
      topo.tmpl_cdf.push_back((uint32_t)std::min(thr, 4294967295.0));
    }
    return topo;
  }
};

HostTopo build_sn() {
  const std::string NG = "nginx-web-server", HT = "home-timeline-service",
                    UT = "user-timeline-service", PS = "post-storage-service",
                    CP = "compose-post-service", UI = "unique-id-service", TX = "text-service",
                    US = "url-shorten-service", UM = "user-mention-service",
                    ME = "media-service", USR = "user-service", SG = "social-graph-service";
  Builder b({CP, HT, ME, NG, PS, SG, TX, UI, US, UM, USR, UT});
  b.add_template({{-1, NG, 2500, 0.45},
                  {0, NG, 2200, 0.45},
                  {1, HT, 1900, 0.45},
                  {2, HT, 250, 0.5},
                  {2, PS, 1200, 0.5},
                  {4, PS, 300, 0.5},
                  {4, PS, 700, 0.6}},
                 0.60);
  b.add_template({{-1, NG, 2800, 0.45},
                  {0, NG, 2500, 0.45},
                  {1, UT, 2200, 0.45},
                  {2, UT, 240, 0.5},
                  {2, UT, 600, 0.6},
                  {2, PS, 1100, 0.5},
                  {5, PS, 280, 0.5},
                  {5, PS, 650, 0.6}},
                 0.30);
  b.add_template({{-1, NG, 9000, 0.4},  {0, NG, 8500, 0.4},   {1, CP, 8000, 0.4},
                  {2, UI, 120, 0.4},    {2, TX, 2500, 0.45},  {4, US, 900, 0.5},
                  {5, US, 500, 0.6},    {4, UM, 800, 0.5},    {7, UM, 200, 0.5},
                  {2, ME, 150, 0.4},    {2, USR, 400, 0.5},   {2, PS, 1300, 0.5},
                  {11, PS, 900, 0.6},   {2, UT, 1800, 0.5},   {13, UT, 800, 0.6},
                  {13, UT, 300, 0.5},   {2, HT, 2600, 0.5},   {16, SG, 900, 0.5},
                  {17, SG, 250, 0.5},   {16, HT, 600, 0.5}},
                 0.10);
  return b.finish();
}

// --- TrainTicket: span trees from a nested call expression -----------------
struct CallNode {
  std::string svc;
  std::vector<CallNode> calls;
};

CallNode parse_call(const char*& p) {
  CallNode n;
  while (*p && *p != '(' && *p != ',' && *p != ')') n.svc.push_back(*p++);
  n.svc = (n.svc == "ui-dashboard") ? "ts-ui-dashboard" : "ts-" + n.svc + "-service";
  if (*p == '(') {
    ++p;
    while (true) {
      n.calls.push_back(parse_call(p));
      if (*p == ',') { ++p; continue; }
      if (*p == ')') { ++p; break; }
      break;
    }
  }
  return n;
}

const char* kTTdb[] = {"order",      "order-other",    "user",         "auth",
                       "contacts",   "route",          "train",        "station",
                       "config",     "price",          "assurance",    "consign",
                       "consign-price", "food-delivery", "payment",    "inside-payment",
                       "security",   "travel",         "travel2",      "station-food",
                       "train-food", "notification",   "delivery",     "wait-order",
                       "voucher"};

bool tt_has_db(const std::string& svc) {
  for (const char* d : kTTdb)
    if (svc == std::string("ts-") + d + "-service") return true;
  return false;
}

// Java services behind the SkyWalking agent: an entry span costs ~1.2 ms of
// its own, a MySQL exit ~1.5 ms, an HTTP hop ~0.45 ms on top of the callee's
// entry span (r03: 3x the r01/r02 medians, so that the whole-millisecond
// durations SkyWalking records keep most spans above 0 ms).
double entry_median(const CallNode& n) {
  double m = 1200.0 + (tt_has_db(n.svc) ? 1500.0 : 0.0);
  for (const CallNode& c : n.calls) m += 0.7 * (entry_median(c) + 450.0);
  return m;
}

void expand(const CallNode& n, int parent, std::vector<SpanDef>& out) {
  const int entry = (int)out.size();
  out.push_back({parent, n.svc, entry_median(n), 0.45});
  for (const CallNode& c : n.calls) {
    const int exit = (int)out.size();
    out.push_back({entry, n.svc, entry_median(c) + 450.0, 0.5});
    expand(c, exit, out);
  }
  if (tt_has_db(n.svc)) out.push_back({entry, n.svc, 1500.0, 0.6});
}

HostTopo build_tt() {
  static const char* kServices[] = {
      "admin-basic-info", "admin-order", "admin-route", "admin-travel", "admin-user",
      "assurance", "auth", "avatar", "basic", "cancel", "config", "consign-price",
      "consign", "contacts", "delivery", "execute", "food-delivery", "food", "gateway",
      "inside-payment", "news", "notification", "order-other", "order", "payment",
      "preserve-other", "preserve", "price", "rebook", "route-plan", "route", "seat",
      "security", "station-food", "station", "ticket-office", "train-food", "train",
      "travel-plan", "travel", "travel2", "user", "verification-code", "voucher",
      "wait-order"};
  std::vector<std::string> names;
  for (const char* s : kServices) names.push_back(std::string("ts-") + s + "-service");
  names.push_back("ts-ui-dashboard");
  Builder b(names);
  static const struct { const char* expr; double w; } kReq[] = {
      {"gateway(travel(route,train,basic(station,train,route,price),seat(config,order)))", 0.22},
      {"gateway(travel2(route,train,basic(station,train,route,price),seat(config,order-other)))",
       0.08},
      {"gateway(preserve(security(order,order-other),contacts,travel(basic(station,train,route,"
       "price),seat(config,order)),station,seat(config,order),order,assurance,food(station-food,"
       "train-food),consign(consign-price),user,notification))",
       0.08},
      {"gateway(preserve-other(security(order,order-other),contacts,travel2(basic(station,train,"
       "route,price),seat(config,order-other)),station,order-other,user,notification))",
       0.02},
      {"gateway(auth(verification-code,user))", 0.10},
      {"gateway(order)", 0.10},
      {"gateway(order-other)", 0.05},
      {"gateway(food(station-food,train-food,travel(route)))", 0.05},
      {"gateway(inside-payment(order,payment))", 0.05},
      {"gateway(cancel(order,inside-payment(payment),user,notification))", 0.04},
      {"gateway(rebook(order,travel(basic(station,train,route,price),seat(config,order)),"
       "inside-payment(payment)))",
       0.03},
      {"gateway(execute(order))", 0.03},
      {"gateway(route-plan(travel(basic(station,train,route,price)),travel2(basic(station,"
       "train,route,price)),station,route))",
       0.02},
      {"gateway(travel-plan(route-plan(travel,travel2),seat(config,order),train,station))",
       0.01},
      {"gateway(consign(consign-price))", 0.02},
      {"gateway(admin-order(order,order-other))", 0.015},
      {"gateway(admin-basic-info(station,train,config,price,contacts))", 0.01},
      {"gateway(admin-route(route))", 0.005},
      {"gateway(admin-travel(travel,travel2,train,route,station))", 0.005},
      {"gateway(admin-user(user))", 0.005},
      {"gateway(wait-order(order,contacts))", 0.01},
      {"gateway(news)", 0.005},
      {"gateway(voucher(order))", 0.005},
      {"gateway(avatar)", 0.002},
      {"gateway(food-delivery(station-food,delivery))", 0.005},
      {"gateway(ticket-office)", 0.003},
      {"gateway(price)", 0.005},
      {"gateway(contacts)", 0.02},
      {"gateway(user)", 0.01},
      {"gateway(station)", 0.01},
      {"gateway(verification-code)", 0.005},
  };
  for (const auto& r : kReq) {
    const char* p = r.expr;
    CallNode root = parse_call(p);
    std::vector<SpanDef> spans;
    expand(root, -1, spans);
    b.add_template(spans, r.w);
  }
  b.topo.dur_quant = 1000;  // whole milliseconds (SkyWalking)
  return b.finish();
}

// --- LONG: SocialNetwork services in traces of 16 .. 4000 spans -----------
// Not a reference topology: the length / depth stress case beside SN and TT
// (batch jobs, fan-out crawls, retried chains).  Random trees from a fixed
// seed: each span's parent is the previous span with p = 0.6 (long chains),
// else a uniformly drawn earlier span.  Span shares by trace length: 16 / 48
// / 128 spans 20 % each, 256 / 600 / 1500 / 4000 spans 10 % each, so 30 % of
// the spans sit in traces longer than a 256-span wave chunk.
HostTopo build_long() {
  static const char* kSvc[] = {"compose-post-service", "home-timeline-service", "media-service",
                               "nginx-web-server",     "post-storage-service",  "social-graph-service",
                               "text-service",         "unique-id-service",     "url-shorten-service",
                               "user-mention-service", "user-service",          "user-timeline-service"};
  static const double kMedian[] = {8000, 1900, 150, 2500, 1200, 900, 2500, 120, 900, 800, 400, 1800};
  std::vector<std::string> names(std::begin(kSvc), std::end(kSvc));
  Builder b(names);
  static const struct { int len; double share; } kLen[] = {
      {16, 0.2}, {48, 0.2}, {128, 0.2}, {256, 0.1}, {600, 0.1}, {1500, 0.1}, {4000, 0.1}};
  uint64_t st = 0x4C4F4E47ull;  // "LONG"
  auto next = [&]() { st += 0x9E3779B97F4A7C15ull; return splitmix64(st); };
  for (const auto& t : kLen) {
    std::vector<SpanDef> spans;
    for (int j = 0; j < t.len; ++j) {
      const int par = j == 0 ? -1 : (next() % 10 < 6 ? j - 1 : (int)(next() % (uint64_t)j));
      const int sv = j == 0 ? 3 : (int)(next() % 12);
      spans.push_back({par, kSvc[sv], kMedian[sv], 0.5});
    }
    b.add_template(spans, t.share / t.len);
  }
  return b.finish();
}

std::once_flag g_topo_once;
std::unique_ptr<HostTopo> g_topo[3];

}  // namespace

const HostTopo* host_topo(uint32_t topology) {
  std::call_once(g_topo_once, [] {
    g_topo[0].reset(new HostTopo(build_sn()));
    g_topo[1].reset(new HostTopo(build_tt()));
    g_topo[2].reset(new HostTopo(build_long()));
  });
  if (topology > 2) return nullptr;
  return g_topo[topology].get();
}

TopoView topo_view(const HostTopo* h) {
  TopoView v;
  v.n_services = (uint32_t)h->services.size();
  v.n_templates = (uint32_t)h->tmpl_cdf.size();
  v.n_ops = (uint32_t)(h->dur_q.size() / kDurQuantiles);
  v.tmpl_cdf = h->tmpl_cdf.data();
  v.tmpl_off = h->tmpl_off.data();
  v.span_parent = h->span_parent.data();
  v.span_svc = h->span_svc.data();
  v.span_op = h->span_op.data();
  v.dur_q = h->dur_q.data();
  v.dur_quant = h->dur_quant;
  return v;
}

SynthParams synth_params(const anomod_synth_spec* spec) {
  auto thr = [](uint32_t ppm) -> uint32_t {
    const uint64_t t = (uint64_t)ppm * 4294967296ull / 1000000ull;
    return t > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)t;
  };
  SynthParams p;
  p.k0 = (uint32_t)spec->seed;
  p.k1 = (uint32_t)(spec->seed >> 32);
  p.fault_svc = spec->fault_service;
  p.fault_mult = spec->fault_latency_mult ? spec->fault_latency_mult : 1u;
  p.thr_err = thr(spec->p_error_ppm);
  p.thr_fault_err = thr(spec->p_fault_error_ppm);
  p.thr_orphan = thr(spec->p_orphan_ppm);
  return p;
}

namespace {

__global__ void synth_sizes_kernel(TopoView tp, SynthParams sp, uint64_t shard, uint64_t n_traces,
                                   uint64_t* sizes) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_traces;
       t += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h;
    const uint32_t k = synth_trace(tp, sp, shard, t, &h);
    sizes[t] = tp.tmpl_off[k + 1] - tp.tmpl_off[k];
  }
}

__global__ void synth_fill_kernel(TopoView tp, SynthParams sp, uint64_t shard, uint64_t n_traces,
                                  const uint64_t* __restrict__ trace_ptr, uint64_t* trace_hash,
                                  uint64_t* span_id, uint64_t* parent, uint32_t* svc_flags,
                                  uint32_t* dur) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_traces;
       t += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h;
    const uint32_t k = synth_trace(tp, sp, shard, t, &h);
    const uint32_t n = tp.tmpl_off[k + 1] - tp.tmpl_off[k];
    const uint64_t base = trace_ptr[t];
    for (uint32_t j = 0; j < n; ++j) {
      const SynthSpan s = synth_span(tp, sp, shard, t, h, k, j);
      trace_hash[base + j] = h;
      span_id[base + j] = s.span_id;
      parent[base + j] = s.parent_span_id;
      svc_flags[base + j] = (uint32_t)s.svc | ((uint32_t)s.flags << 16);
      dur[base + j] = s.dur_us;
    }
  }
}

}  // namespace

void free_spans(anomod_spans* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  void* ptrs[] = {s->trace_hash, s->span_id, s->parent_span_id, s->svc_flags, s->dur_us,
                  s->trace_ptr};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  delete s;
}

// Allocate every array of a span set (trace_hash optional).
int alloc_spans(anomod_ctx* ctx, uint64_t n_spans, uint64_t n_traces, bool with_hash,
                anomod_spans** out) {
  auto* s = new anomod_spans();
  s->device = ctx->device;
  s->n_spans = n_spans;
  s->n_traces = n_traces;
  const uint64_t ns = n_spans ? n_spans : 1;
  // (a failed allocation is retried once after the ctx's scratch is released)
  auto dm = [ctx](void* p, size_t b) {
    return dev_malloc(ctx, static_cast<void**>(p), b) == hipSuccess;
  };
  bool ok = dm(&s->trace_ptr, (n_traces + 1) * 8);
  if (ok && with_hash) ok = dm(&s->trace_hash, ns * 8);
  ok = ok && dm(&s->span_id, ns * 8);
  ok = ok && dm(&s->parent_span_id, ns * 8);
  ok = ok && dm(&s->svc_flags, ns * 4);
  ok = ok && dm(&s->dur_us, ns * 4);
  if (!ok) {
    free_spans(s);
    set_error(ctx, "hipMalloc failed for a span set of %llu spans / %llu traces",
              (unsigned long long)n_spans, (unsigned long long)n_traces);
    return ANOMOD_ENOMEM;
  }
  *out = s;
  return ANOMOD_OK;
}

}  // namespace anomod

using namespace anomod;

extern "C" {

int anomod_synth_n_services(uint32_t topology, uint32_t* out) {
  const HostTopo* h = host_topo(topology);
  ANOMOD_REQUIRE(nullptr, h && out, "unknown topology %u", topology);
  *out = (uint32_t)h->services.size();
  return ANOMOD_OK;
}

const char* anomod_synth_service_name(uint32_t topology, uint32_t i) {
  const HostTopo* h = host_topo(topology);
  if (!h || i >= h->services.size()) return nullptr;
  return h->services[i].c_str();
}

int anomod_synth_count_host(const anomod_synth_spec* spec, uint64_t shard, uint64_t n_traces,
                            uint64_t* n_spans) {
  ANOMOD_REQUIRE(nullptr, spec && n_spans, "anomod_synth_count_host: NULL argument");
  const HostTopo* h = host_topo(spec->topology);
  ANOMOD_REQUIRE(nullptr, h, "unknown topology %u", spec->topology);
  const TopoView tp = topo_view(h);
  const SynthParams sp = synth_params(spec);
  uint64_t n = 0;
  for (uint64_t t = 0; t < n_traces; ++t) {
    uint64_t th;
    const uint32_t k = synth_trace(tp, sp, shard, t, &th);
    n += tp.tmpl_off[k + 1] - tp.tmpl_off[k];
  }
  *n_spans = n;
  return ANOMOD_OK;
}

int anomod_synth_generate_host(const anomod_synth_spec* spec, uint64_t shard, uint64_t n_traces,
                               const anomod_span_soa_out* dst, uint64_t* trace_ptr) {
  ANOMOD_REQUIRE(nullptr, spec && dst && trace_ptr, "anomod_synth_generate_host: NULL argument");
  ANOMOD_REQUIRE(nullptr, dst->span_id && dst->parent_span_id && dst->svc && dst->flags &&
                              dst->dur_us,
                 "anomod_synth_generate_host: span arrays must be non-NULL");
  const HostTopo* h = host_topo(spec->topology);
  ANOMOD_REQUIRE(nullptr, h, "unknown topology %u", spec->topology);
  const TopoView tp = topo_view(h);
  const SynthParams sp = synth_params(spec);
  uint64_t pos = 0;
  trace_ptr[0] = 0;
  for (uint64_t t = 0; t < n_traces; ++t) {
    uint64_t th;
    const uint32_t k = synth_trace(tp, sp, shard, t, &th);
    const uint32_t n = tp.tmpl_off[k + 1] - tp.tmpl_off[k];
    for (uint32_t j = 0; j < n; ++j) {
      const SynthSpan s = synth_span(tp, sp, shard, t, th, k, j);
      if (dst->trace_hash) dst->trace_hash[pos] = th;
      dst->span_id[pos] = s.span_id;
      dst->parent_span_id[pos] = s.parent_span_id;
      dst->svc[pos] = s.svc;
      dst->flags[pos] = s.flags;
      dst->dur_us[pos] = s.dur_us;
      ++pos;
    }
    trace_ptr[t + 1] = pos;
  }
  return ANOMOD_OK;
}

int anomod_spans_generate(anomod_ctx* ctx, const anomod_synth_spec* spec, uint64_t shard,
                          uint64_t n_traces, anomod_spans** out) {
  ANOMOD_REQUIRE(nullptr, ctx && spec && out, "anomod_spans_generate: NULL argument");
  *out = nullptr;
  const HostTopo* h = host_topo(spec->topology);
  ANOMOD_REQUIRE(ctx, h, "unknown topology %u", spec->topology);
  ANOMOD_REQUIRE(ctx, n_traces < (1ull << 36), "n_traces %llu too large",
                 (unsigned long long)n_traces);
  if (int rc = bind(ctx)) return rc;
  // Topology tables -> device (one buffer).
  const size_t b_cdf = h->tmpl_cdf.size() * 4, b_off = h->tmpl_off.size() * 4,
               b_par = h->span_parent.size() * 4, b_svc = h->span_svc.size() * 2,
               b_op = h->span_op.size() * 2, b_dur = h->dur_q.size() * 4;
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t total = al(b_cdf) + al(b_off) + al(b_par) + al(b_svc) + al(b_op) + al(b_dur);
  char* dtopo = nullptr;
  ANOMOD_HIP(ctx, hipMalloc(&dtopo, total));
  TopoView tp = topo_view(h);
  size_t off = 0;
  auto put = [&](const void* src, size_t bytes) {
    char* dst = dtopo + off;
    (void)hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream);
    off += al(bytes);
    return (const void*)dst;
  };
  tp.tmpl_cdf = (const uint32_t*)put(h->tmpl_cdf.data(), b_cdf);
  tp.tmpl_off = (const uint32_t*)put(h->tmpl_off.data(), b_off);
  tp.span_parent = (const int32_t*)put(h->span_parent.data(), b_par);
  tp.span_svc = (const uint16_t*)put(h->span_svc.data(), b_svc);
  tp.span_op = (const uint16_t*)put(h->span_op.data(), b_op);
  tp.dur_q = (const uint32_t*)put(h->dur_q.data(), b_dur);
  const SynthParams sp = synth_params(spec);

  int rc = ANOMOD_OK;
  uint64_t* sizes = nullptr;
  void* tmp = nullptr;
  anomod_spans* s = nullptr;
  uint64_t n_spans = 0;
  const int threads = 256;
  const int blocks = (int)std::min<uint64_t>((n_traces + threads - 1) / threads,
                                             (uint64_t)ctx->num_cus * 16);
  do {
    if (n_traces == 0) {
      rc = alloc_spans(ctx, 0, 0, true, &s);
      if (rc) break;
      (void)hipMemsetAsync(s->trace_ptr, 0, 8, ctx->stream);
      break;
    }
    if (dev_malloc(ctx, reinterpret_cast<void**>(&sizes), n_traces * 8) != hipSuccess) {
      set_error(ctx, "hipMalloc sizes failed");
      rc = ANOMOD_ENOMEM;
      break;
    }
    hipLaunchKernelGGL(synth_sizes_kernel, dim3(blocks), dim3(threads), 0, ctx->stream, tp, sp,
                       shard, n_traces, sizes);
    // trace_ptr = [0, inclusive_scan(sizes)]
    uint64_t* tptr = nullptr;
    if (dev_malloc(ctx, reinterpret_cast<void**>(&tptr), (n_traces + 1) * 8) != hipSuccess) {
      set_error(ctx, "hipMalloc trace_ptr failed");
      rc = ANOMOD_ENOMEM;
      break;
    }
    size_t tmp_bytes = 0;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, sizes, tptr + 1, n_traces,
                                           ctx->stream);
    if (dev_malloc(ctx, &tmp, tmp_bytes) != hipSuccess) {
      (void)hipFree(tptr);
      set_error(ctx, "hipMalloc scan workspace failed");
      rc = ANOMOD_ENOMEM;
      break;
    }
    (void)hipMemsetAsync(tptr, 0, 8, ctx->stream);
    if (hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, sizes, tptr + 1, n_traces,
                                         ctx->stream) != hipSuccess) {
      (void)hipFree(tptr);
      set_error(ctx, "hipcub InclusiveSum failed");
      rc = ANOMOD_EHIP;
      break;
    }
    if (hipMemcpyAsync(&n_spans, tptr + n_traces, 8, hipMemcpyDeviceToHost, ctx->stream) !=
            hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess) {
      (void)hipFree(tptr);
      set_error(ctx, "reading the span count failed: %s", hipGetErrorString(hipGetLastError()));
      rc = ANOMOD_EHIP;
      break;
    }
    rc = alloc_spans(ctx, n_spans, n_traces, true, &s);
    if (rc) {
      (void)hipFree(tptr);
      break;
    }
    (void)hipFree(s->trace_ptr);
    s->trace_ptr = tptr;
    hipLaunchKernelGGL(synth_fill_kernel, dim3(blocks), dim3(threads), 0, ctx->stream, tp, sp,
                       shard, n_traces, s->trace_ptr, s->trace_hash, s->span_id,
                       s->parent_span_id, s->svc_flags, s->dur_us);
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) {
      set_error(ctx, "synthetic span generation failed: %s", hipGetErrorString(e));
      rc = ANOMOD_EHIP;
    }
  } while (false);
  (void)hipStreamSynchronize(ctx->stream);
  if (sizes) (void)hipFree(sizes);
  if (tmp) (void)hipFree(tmp);
  (void)hipFree(dtopo);
  if (rc != ANOMOD_OK) {
    free_spans(s);
    return rc;
  }
  s->max_svc = (uint32_t)h->services.size() - 1u;
  s->unique_ids = true;  // synth_span_id is injective in the span index
  s->order = 1;          // the generator emits a callee's spans after its caller's
  s->max_trace_len = 0;
  for (size_t k = 0; k + 1 < h->tmpl_off.size(); ++k)
    s->max_trace_len = std::max<uint64_t>(s->max_trace_len, h->tmpl_off[k + 1] - h->tmpl_off[k]);
  *out = s;
  return ANOMOD_OK;
}

int anomod_spans_set_unique_ids(anomod_spans* spans, int unique) {
  ANOMOD_REQUIRE(nullptr, spans, "anomod_spans_set_unique_ids: NULL span set");
  spans->unique_ids = unique != 0;
  return ANOMOD_OK;
}

int anomod_spans_hist_compact(const anomod_spans* spans, int* compact) {
  ANOMOD_REQUIRE(nullptr, spans && compact, "anomod_spans_hist_compact: NULL argument");
  *compact = spans->hist_form == 1 ? 1 : 0;
  return ANOMOD_OK;
}

int anomod_spans_hints(const anomod_spans* spans, int* scan_order, int* hist_form) {
  ANOMOD_REQUIRE(nullptr, spans && scan_order && hist_form, "anomod_spans_hints: NULL argument");
  *scan_order = spans->order;
  *hist_form = spans->hist_form;
  return ANOMOD_OK;
}

int anomod_spans_set_hints(anomod_spans* spans, int scan_order, int hist_form) {
  ANOMOD_REQUIRE(nullptr, spans, "anomod_spans_set_hints: NULL span set");
  ANOMOD_REQUIRE(nullptr, scan_order >= -1 && scan_order <= 1 && hist_form >= -1 && hist_form <= 1,
                 "anomod_spans_set_hints: scan_order=%d / hist_form=%d outside [-1, 1]", scan_order,
                 hist_form);
  spans->order = (int8_t)scan_order;
  spans->hist_form = (int8_t)hist_form;
  return ANOMOD_OK;
}

int anomod_spans_scan_order(const anomod_spans* spans, int* order) {
  ANOMOD_REQUIRE(nullptr, spans && order, "anomod_spans_scan_order: NULL argument");
  *order = spans->order;
  return ANOMOD_OK;
}

int anomod_spans_unique_ids(const anomod_spans* spans, int* unique) {
  ANOMOD_REQUIRE(nullptr, spans && unique, "anomod_spans_unique_ids: NULL argument");
  *unique = spans->unique_ids ? 1 : 0;
  return ANOMOD_OK;
}

namespace {

// Validates an upload's arguments (kernels index by these values) and returns
// the longest trace in *max_len.
int check_upload(anomod_ctx* ctx, const anomod_span_soa* soa, uint64_t n_spans,
                 const uint64_t* trace_ptr, uint64_t n_traces, uint64_t* max_len) {
  ANOMOD_REQUIRE(ctx, n_traces == 0 || trace_ptr, "trace_ptr is NULL");
  ANOMOD_REQUIRE(ctx, n_spans == 0 || (soa->span_id && soa->parent_span_id && soa->svc &&
                                       soa->flags && soa->dur_us),
                 "span arrays must be non-NULL");
  ANOMOD_REQUIRE(ctx, n_traces < (1ull << 36), "n_traces too large");
  uint64_t ml = 0;
  for (uint64_t t = 0; t < n_traces; ++t) {
    ANOMOD_REQUIRE(ctx, trace_ptr[t] <= trace_ptr[t + 1],
                   "trace_ptr is not non-decreasing at trace %llu", (unsigned long long)t);
    ml = std::max<uint64_t>(ml, trace_ptr[t + 1] - trace_ptr[t]);
  }
  if (n_traces) {
    ANOMOD_REQUIRE(ctx, trace_ptr[n_traces] <= n_spans,
                   "trace_ptr[n_traces]=%llu exceeds n_spans=%llu",
                   (unsigned long long)trace_ptr[n_traces], (unsigned long long)n_spans);
  }
  *max_len = ml;
  return ANOMOD_OK;
}

// The columns of soa (trace_hash only when with_hash and given) and trace_ptr
// into s through the staging pipeline; s->max_svc from the packing pass.
int fill_set(anomod_ctx* ctx, anomod_spans* s, const anomod_span_soa* soa, uint64_t n_spans,
             const uint64_t* trace_ptr, uint64_t n_traces, bool with_hash) {
  UpItem it[7];
  int k = 0;
  if (n_traces) it[k++] = {s->trace_ptr, trace_ptr, nullptr, (n_traces + 1) * 8, 0};
  else ANOMOD_HIP(ctx, hipMemsetAsync(s->trace_ptr, 0, 8, ctx->stream));
  if (with_hash && soa->trace_hash && s->trace_hash)
    it[k++] = {s->trace_hash, soa->trace_hash, nullptr, n_spans * 8, 0};
  it[k++] = {s->span_id, soa->span_id, nullptr, n_spans * 8, 0};
  it[k++] = {s->parent_span_id, soa->parent_span_id, nullptr, n_spans * 8, 0};
  it[k++] = {s->svc_flags, soa->svc, soa->flags, n_spans, 1};
  it[k++] = {s->dur_us, soa->dur_us, nullptr, n_spans * 4, 0};
  uint32_t mx = 0;
  if (int rc = upload_items(ctx, it, k, &mx)) return rc;
  s->max_svc = mx;
  return ANOMOD_OK;
}

}  // namespace

int anomod_spans_upload(anomod_ctx* ctx, const anomod_span_soa* soa, uint64_t n_spans,
                        const uint64_t* trace_ptr, uint64_t n_traces, anomod_spans** out) {
  ANOMOD_REQUIRE(nullptr, ctx && soa && out, "anomod_spans_upload: NULL argument");
  *out = nullptr;
  uint64_t max_len = 0;
  if (int rc = check_upload(ctx, soa, n_spans, trace_ptr, n_traces, &max_len)) return rc;
  if (int rc = bind(ctx)) return rc;
  anomod_spans* s = nullptr;
  if (int rc = alloc_spans(ctx, n_spans, n_traces, soa->trace_hash != nullptr, &s)) return rc;
  // (no trace_ptr: an ungrouped set, its trace lengths unknown until grouped)
  s->max_trace_len = n_traces || !n_spans ? max_len : ~0ull;
  if (int rc = fill_set(ctx, s, soa, n_spans, trace_ptr, n_traces, true)) {
    free_spans(s);
    return rc;
  }
  *out = s;
  return ANOMOD_OK;
}

int anomod_edge_aggregate_host(anomod_ctx* ctx, const anomod_span_soa* soa, uint64_t n_spans,
                               const uint64_t* trace_ptr, uint64_t n_traces, uint32_t n_services,
                               int unique_ids, int* scan_order, int* hist_form,
                               anomod_edge_table* out) {
  ANOMOD_REQUIRE(nullptr, ctx && soa && out && scan_order && hist_form,
                 "anomod_edge_aggregate_host: NULL argument");
  uint64_t max_len = 0;
  // every check goes through `local`: the hints come from this rank's own
  // host set, so a bad one on one rank must reach comm_agree too
  int local = ANOMOD_OK;
  ANOMOD_CHECK_LOCAL(ctx, local,
                     *scan_order >= -1 && *scan_order <= 1 && *hist_form >= -1 && *hist_form <= 1,
                     "scan_order=%d / hist_form=%d outside [-1, 1]", *scan_order, *hist_form);
  if (local == ANOMOD_OK) local = check_upload(ctx, soa, n_spans, trace_ptr, n_traces, &max_len);
  if (local == ANOMOD_OK) local = bind(ctx);
  // the ctx's grow-only set: no trace_hash (a grouped aggregation reads none)
  if (local == ANOMOD_OK &&
      (!ctx->host_set || ctx->host_set_spans < n_spans || ctx->host_set_traces < n_traces)) {
    if (ctx->host_set) {
      (void)hipStreamSynchronize(ctx->stream);
      free_spans(ctx->host_set);
      ctx->host_set = nullptr;
    }
    const uint64_t cs = std::max<uint64_t>(n_spans, ctx->host_set_spans);
    const uint64_t ct = std::max<uint64_t>(n_traces, ctx->host_set_traces);
    const double t0 = host_now_ms();
    local = alloc_spans(ctx, cs, ct, false, &ctx->host_set);
    host_record(ctx, kHostSetAlloc, host_now_ms() - t0);
    ctx->host_set_spans = local == ANOMOD_OK ? cs : 0;
    ctx->host_set_traces = local == ANOMOD_OK ? ct : 0;
  }
  anomod_spans* s = ctx->host_set;
  if (local == ANOMOD_OK) {
    s->n_spans = n_spans;
    s->n_traces = n_traces;
    s->grouped = true;
    s->unique_ids = unique_ids != 0;
    s->order = (int8_t)*scan_order;
    s->hist_form = (int8_t)*hist_form;
    s->max_trace_len = max_len;
    local = fill_set(ctx, s, soa, n_spans, trace_ptr, n_traces, false);
  }
  if (local != ANOMOD_OK) return comm_agree(ctx, local);  // peers learn of it before their reduce
  const int rc = anomod_edge_aggregate_spans(ctx, s, n_services, out);
  *scan_order = s->order;
  *hist_form = s->hist_form;
  return rc;
}

int anomod_spans_info(const anomod_spans* spans, uint64_t* n_spans, uint64_t* n_traces) {
  ANOMOD_REQUIRE(nullptr, spans, "anomod_spans_info: spans is NULL");
  if (n_spans) *n_spans = spans->n_spans;
  if (n_traces) *n_traces = spans->n_traces;
  return ANOMOD_OK;
}

int anomod_spans_download(anomod_ctx* ctx, const anomod_spans* s, const anomod_span_soa_out* dst,
                          uint64_t* trace_ptr) {
  ANOMOD_REQUIRE(nullptr, ctx && s && dst, "anomod_spans_download: NULL argument");
  ANOMOD_REQUIRE(ctx, s->device == ctx->device, "span set lives on another device");
  if (int rc = bind(ctx)) return rc;
  const uint64_t n = s->n_spans;
  hipError_t e = hipSuccess;
  auto cp = [&](void* d, const void* src, size_t bytes) {
    if (e == hipSuccess && d && src && bytes)
      e = hipMemcpyAsync(d, src, bytes, hipMemcpyDeviceToHost, ctx->stream);
  };
  cp(trace_ptr, s->trace_ptr, (s->n_traces + 1) * 8);
  if (dst->trace_hash && !s->trace_hash && n) memset(dst->trace_hash, 0, n * 8);
  cp(dst->trace_hash, s->trace_hash, n * 8);
  cp(dst->span_id, s->span_id, n * 8);
  cp(dst->parent_span_id, s->parent_span_id, n * 8);
  std::vector<uint32_t> packed((dst->svc || dst->flags) ? n : 0);
  if (!packed.empty()) cp(packed.data(), s->svc_flags, n * 4);
  cp(dst->dur_us, s->dur_us, n * 4);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  ANOMOD_HIP(ctx, e);
  for (uint64_t i = 0; i < packed.size(); ++i) {
    if (dst->svc) dst->svc[i] = (uint16_t)(packed[i] & 0xFFFFu);
    if (dst->flags) dst->flags[i] = (uint16_t)(packed[i] >> 16);
  }
  return ANOMOD_OK;
}

int anomod_spans_free(anomod_spans* spans) {
  free_spans(spans);
  return ANOMOD_OK;
}

}  // extern "C"
