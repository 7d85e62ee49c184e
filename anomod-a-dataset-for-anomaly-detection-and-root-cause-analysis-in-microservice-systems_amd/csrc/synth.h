// Synthetic DeathStarBench-SocialNetwork / TrainTicket span workload
// (SURVEY.md §8d configs 2-3).  The same __host__ __device__ code generates a
// trace on the CPU and on the GPU, so a span set built in HBM is
// bit-identical to the one built on the host: integer-only arithmetic
// (Philox4x32-10 counters + SplitMix64 ids + integer inverse-CDF duration
// tables), no transcendental functions on the generation path.
#pragma once

#include <cstdint>

#include "common.h"

namespace anomod {

constexpr int kDurQuantiles = 1024;  // inverse-CDF table entries per operation

// Flattened trace templates (span trees) and duration tables.
struct TopoView {
  uint32_t n_services = 0;
  uint32_t n_templates = 0;
  uint32_t n_ops = 0;
  const uint32_t* tmpl_cdf = nullptr;    // [n_templates] selection thresholds
  const uint32_t* tmpl_off = nullptr;    // [n_templates + 1] span offsets
  const int32_t* span_parent = nullptr;  // [total] parent index in template, -1 = root
  const uint16_t* span_svc = nullptr;    // [total]
  const uint16_t* span_op = nullptr;     // [total]
  const uint32_t* dur_q = nullptr;       // [n_ops * kDurQuantiles] microseconds
  uint32_t dur_quant = 1;                // durations are whole multiples of this (us)
};

struct SynthParams {
  uint32_t k0 = 0, k1 = 0;  // Philox key (seed)
  uint32_t fault_svc = 0xFFFFFFFFu;
  uint32_t fault_mult = 1;
  uint32_t thr_err = 0;        // error iff draw < thr
  uint32_t thr_fault_err = 0;
  uint32_t thr_orphan = 0;
};

__host__ __device__ inline uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * b) >> 32);
}

// Philox4x32-10 (Salmon et al., SC'11).
__host__ __device__ inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = mulhi32(0xD2511F53u, c[0]);
    const uint32_t lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = mulhi32(0xCD9E8D57u, c[2]);
    const uint32_t lo1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0;
    const uint32_t n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Span id j of a trace: injective in j (odd multiplier, xor, bijective mix).
__host__ __device__ inline uint64_t synth_span_id(uint64_t trace_hash, uint32_t j) {
  uint64_t s = splitmix64(trace_hash ^ (0xA0761D6478BD642Full * (uint64_t)(j + 1)));
  return s ? s : 1ull;
}

// Trace-level draw: 96-bit trace id -> trace_hash, and the template index.
__host__ __device__ inline uint32_t synth_trace(const TopoView& tp, const SynthParams& sp,
                                                uint64_t shard, uint64_t t,
                                                uint64_t* trace_hash) {
  uint32_t c[4] = {(uint32_t)t, (uint32_t)(t >> 32), (uint32_t)shard, 0u};
  philox4x32_10(c, sp.k0, sp.k1);
  *trace_hash = splitmix64((((uint64_t)c[0] << 32) | c[1]) ^ splitmix64(c[2]));
  uint32_t i = 0;
  while (i + 1 < tp.n_templates && c[3] >= tp.tmpl_cdf[i]) ++i;
  return i;
}

struct SynthSpan {
  uint64_t span_id, parent_span_id;
  uint16_t svc, flags;
  uint32_t dur_us;
};

__host__ __device__ inline SynthSpan synth_span(const TopoView& tp, const SynthParams& sp,
                                                uint64_t shard, uint64_t t,
                                                uint64_t trace_hash, uint32_t tmpl,
                                                uint32_t j) {
  uint32_t c[4] = {(uint32_t)t, (uint32_t)(t >> 32), (uint32_t)shard, j + 1u};
  philox4x32_10(c, sp.k0, sp.k1);
  const uint32_t g = tp.tmpl_off[tmpl] + j;
  const int32_t par = tp.span_parent[g];
  SynthSpan s;
  s.svc = tp.span_svc[g];
  s.span_id = synth_span_id(trace_hash, j);
  if (par < 0) {
    s.parent_span_id = 0;
  } else if (c[2] < sp.thr_orphan) {
    // dropped parent: a reference to a span that is not in the trace
    s.parent_span_id = splitmix64(s.span_id ^ 0x5BD1E9955BD1E995ull) | 1ull;
  } else {
    s.parent_span_id = synth_span_id(trace_hash, (uint32_t)par);
  }
  const uint32_t base = tp.dur_q[(uint32_t)tp.span_op[g] * kDurQuantiles + (c[0] >> 22)];
  uint64_t d = (uint64_t)base + (c[3] % (base / 16u + 1u));
  const bool faulty = (uint32_t)s.svc == sp.fault_svc;
  if (faulty) d *= sp.fault_mult;
  if (d > 0xFFFFFFFFull) d = 0xFFFFFFFFull;
  // TrainTicket: SkyWalking records whole milliseconds (duration = end_ms -
  // start_ms, trace_collector.py:87), so the topology's durations are floored
  // to a multiple of 1000 us, as the decoder reads them back (ms x 1000)
  s.dur_us = (uint32_t)(d - d % tp.dur_quant);
  const uint32_t thr = faulty ? sp.thr_fault_err : sp.thr_err;
  s.flags = (c[1] < thr) ? (uint16_t)ANOMOD_FLAG_ERROR : (uint16_t)0;
  return s;
}

// Host-side topology owner (vectors behind a TopoView).
struct HostTopo;
const HostTopo* host_topo(uint32_t topology);  // nullptr if unknown
TopoView topo_view(const HostTopo* h);
uint64_t topo_bytes(const HostTopo* h);
SynthParams synth_params(const anomod_synth_spec* spec);

}  // namespace anomod
