/*
 * anomod.h — C ABI of the MI355X-native AnoMod RCA-feature engine (libanomod.so).
 *
 * The reference (EvoTestOps/AnoMod, /root/reference) has no FFI: its hot path is
 * a CLI + file boundary driven by bash.  Each entry point below
 * names the reference code it replaces (path:line relative to the reference
 * root).  Everything is `extern "C"`, plain pointers and sizes; no torch types.
 *
 * Conventions
 *  - Every function returns an int status: ANOMOD_OK (0) or a negative code; a
 *    human-readable message is available from anomod_last_error(ctx) (or
 *    anomod_last_error(NULL) for errors raised before a ctx exists).
 *  - Host buffers are caller-owned; no pointer is retained after a call
 *    returns and inputs are never mutated (unlike trace_collector.py:415, which
 *    mutates the span dicts it is handed).
 *  - Empty input (n == 0) is not an error: outputs are zero/empty tables and
 *    status is ANOMOD_OK (mirrors jaeger_to_csv.py:92-97, which writes a
 *    header-only CSV and exits 0).
 *  - One ctx per host thread; a ctx owns one HIP device, one stream and,
 *    optionally, one RCCL communicator.
 */
#ifndef ANOMOD_H
#define ANOMOD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ANOMOD_ABI_VERSION 2

/* ---- status codes ------------------------------------------------------- */
#define ANOMOD_OK 0
#define ANOMOD_EINVAL (-1)  /* bad argument / shape                           */
#define ANOMOD_EHIP (-2)    /* HIP runtime error (no device, launch failure)  */
#define ANOMOD_ERCCL (-3)   /* RCCL error                                     */
#define ANOMOD_ENOMEM (-4)  /* device or host allocation failed               */
#define ANOMOD_ESTATE (-5)  /* call not valid in this state                   */

/* ---- span flags (anomod_span_soa.flags) --------------------------------- */
/* Error bit.  SN/Jaeger: tags["error"] == true or http.status_code >= 500
 * (tags kept at jaeger_to_csv.py:55-67,88).  TT/SkyWalking: isError
 * (trace_collector.py:471).                                                 */
#define ANOMOD_FLAG_ERROR 0x1u

/* ---- latency histogram (build-defined) ---------------
 * Integer log-linear ("HDR") binning of a u32 microsecond latency v:
 *   v <  64 : bin = v                                 (exact)
 *   v >= 64 : e = floor(log2 v) - 5 ; bin = 32*e + (v >> e)
 * 32 sub-buckets per octave (<= 3.1 % relative bin width), 896 bins cover the
 * whole u32 range.                                                          */
#define ANOMOD_HIST_SUB_BITS 5
#define ANOMOD_HIST_BINS 896

/* ---- edge table layout ---------------------------------------------------
 * For S services the table has E = (S + 2) * S rows; row = p * S + c where c
 * is the child span's service and p is the parent span's service, or
 *   p == S     : ROOT   — the span carries no parent reference
 *                (jaeger_to_csv.py:34-38 leaves parent_span_id = '';
 *                 trace_collector.py:427-437 yields parent_node None)
 *   p == S + 1 : ORPHAN — a parent reference that names no span of the same
 *                trace (trace_collector.py:443 counts these among the roots). */
#define ANOMOD_ROOT_ROWS 2

typedef struct anomod_ctx anomod_ctx;       /* device + stream + comm      */
typedef struct anomod_spans anomod_spans;   /* device-resident span set    */
typedef struct anomod_series anomod_series; /* device-resident metric matrix */
typedef struct anomod_graph anomod_graph;   /* device-resident CSR graph   */

/* Span set in struct-of-arrays form, grouped by trace: the spans of trace t
 * are [trace_ptr[t], trace_ptr[t+1]).  span_id 0 is reserved; a
 * parent_span_id of 0 means "no parent reference".  Collectors already emit
 * spans grouped by trace (jaeger_to_csv.py:21-32 iterates trace -> spans;
 * trace_collector.py:539-546 emits per-trace span lists).                   */
typedef struct {
  const uint64_t* trace_hash;      /* [n] shard key (may be NULL)          */
  const uint64_t* span_id;         /* [n]                                  */
  const uint64_t* parent_span_id;  /* [n]                                  */
  const uint16_t* svc;             /* [n] service index (< n_services)     */
  const uint16_t* flags;           /* [n] ANOMOD_FLAG_*                    */
  const uint32_t* dur_us;          /* [n] latency in microseconds          */
} anomod_span_soa;

/* Writable twin of anomod_span_soa (download / host generation targets). */
typedef struct {
  uint64_t* trace_hash;
  uint64_t* span_id;
  uint64_t* parent_span_id;
  uint16_t* svc;
  uint16_t* flags;
  uint32_t* dur_us;
} anomod_span_soa_out;

/* Per-edge aggregate.  Every pointer may be NULL (that output is skipped).
 * Arrays have E = (n_services + 2) * n_services rows; hist has E * n_bins. */
typedef struct {
  uint32_t n_services;  /* in : S                                         */
  uint32_t n_bins;      /* in : must equal ANOMOD_HIST_BINS               */
  uint64_t* count;      /* [E] spans on the edge                          */
  uint64_t* errors;     /* [E] spans with ANOMOD_FLAG_ERROR               */
  uint64_t* sum_us;     /* [E] sum of latencies                           */
  uint32_t* min_us;     /* [E] UINT32_MAX when count == 0                 */
  uint32_t* max_us;     /* [E] 0 when count == 0                          */
  uint64_t* hist;       /* [E * n_bins] latency histogram                 */
  double* p50_us;       /* [E] histogram quantile, rank (n*50)//100       */
  double* p99_us;       /* [E] histogram quantile, rank (n*99)//100       */
} anomod_edge_table;

/* ---- library / context ---------------------------------------------------*/
int anomod_abi_version(void);
const char* anomod_last_error(const anomod_ctx* ctx);
int anomod_device_count(int* out);
int anomod_ctx_create(int device, anomod_ctx** out);
int anomod_ctx_destroy(anomod_ctx* ctx);
int anomod_ctx_synchronize(anomod_ctx* ctx);
/* Milliseconds of the last launch of a stage, measured with hipEvents on the
 * ctx stream.  stage: 0 = edge aggregation kernel, 1 = edge finalize kernel,
 * 2 = edge all-reduce, 3 = ewma kernel, 4 = pagerank iterations,
 * 5 = trace-structure kernel, 6 = segment-summary kernel,
 * 7 = value summary (select + sort + sum + picks),
 * 8 = trace grouping of an ungrouped span set (radix passes + copy + trace_ptr). */
int anomod_ctx_stage_ms(const anomod_ctx* ctx, int stage, double* ms);
/* Host wall milliseconds of the last occurrence of a one-off setup step or of
 * a call phase the stage events above cannot see, and how many times it
 * happened on this ctx (count may be NULL; a caller compares counts around a
 * call to learn whether that call paid it).  Slots: */
#define ANOMOD_HOST_GROUP_ALLOC 0  /* grouping workspace: device hipMalloc     */
#define ANOMOD_HOST_GROUP_PINNED 1 /* grouping workspace: pinned read-back     */
#define ANOMOD_HOST_GROUP_WALL 2   /* an ungrouped aggregation's grouping:
                                      first launch to counters read back       */
#define ANOMOD_HOST_UPLOAD_SETUP 3 /* upload pipeline: threads, streams, pinned
                                      buffers                                  */
#define ANOMOD_HOST_SET_ALLOC 4    /* the device set anomod_edge_aggregate_host
                                      keeps: (re)allocation                    */
#define ANOMOD_HOST_SLOTS 5
int anomod_ctx_host_ms(const anomod_ctx* ctx, int slot, double* ms, uint64_t* count);

/* ---- histogram helpers (host) ------------------------------------------- */
uint32_t anomod_hist_bin(uint32_t v);
int anomod_hist_bin_bounds(uint32_t bin, uint32_t* lo, uint32_t* hi);

/* ---- span sets -----------------------------------------------------------*/
/* Span ids unique within every trace: the producer's declaration (the
 * synthetic generator sets it by construction; the native decoders report it
 * per decoded document, anomod_decoded_unique_ids).  With it, parent
 * lookups may stop at the nearest match from either end of the trace (any
 * match is the first match).  Declaring it for a set that holds a duplicated
 * id inside a trace gives unspecified parents for those spans.  Default 0
 * (unknown: the first-match scan).  Grouping and shuffling keep it.         */
int anomod_spans_set_unique_ids(anomod_spans* spans, int unique);
int anomod_spans_unique_ids(const anomod_spans* spans, int* unique);
/* Order hint of a unique-id set (a performance hint the library keeps):
 * 1 = collector order, most child spans right after their parent (the
 * bidirectional scan from the trace start and from the span pays off);
 * 0 = not (e.g. spans shuffled inside their traces: the forward scan);
 * -1 = not known yet — the first aggregation probes the set's first 2^20
 * spans on the device.  Generated sets are 1; results never depend on it.   */
int anomod_spans_scan_order(const anomod_spans* spans, int* order);
/* 1 once an aggregation of this set overflowed the workgroups' 8 Ki-slot
 * (pair-form) LDS histogram: its later aggregations use the 16 Ki packed-slot
 * (compact) form (same results; a performance hint the library keeps).     */
int anomod_spans_hist_compact(const anomod_spans* spans, int* compact);
/* Both hints of a set, for callers that keep a span set on the host and
 * upload it per call (the Python SpanSet does): *scan_order as
 * anomod_spans_scan_order; *hist_form 0 = pair, 1 = compact, -1 = not known
 * yet (the aggregation starts in the pair form and a workgroup whose table
 * saturates hands its remaining traces to a compact-form launch — no
 * first-call cliff either way).  set_hints puts learned values on a freshly
 * uploaded set (each in [-1, 1]); results never depend on them.           */
int anomod_spans_hints(const anomod_spans* spans, int* scan_order, int* hist_form);
int anomod_spans_set_hints(anomod_spans* spans, int scan_order, int hist_form);
/* Copy a host span set to HBM.  Replaces the in-memory hand-off between
 * json.load and the per-span loop of jaeger_to_csv.py:12-32 /
 * trace_collector.py:519-531.                                              */
int anomod_spans_upload(anomod_ctx* ctx, const anomod_span_soa* soa, uint64_t n_spans,
                        const uint64_t* trace_ptr, uint64_t n_traces, anomod_spans** out);
int anomod_spans_info(const anomod_spans* spans, uint64_t* n_spans, uint64_t* n_traces);
int anomod_spans_download(anomod_ctx* ctx, const anomod_spans* spans,
                          const anomod_span_soa_out* dst, uint64_t* trace_ptr);
int anomod_spans_free(anomod_spans* spans);

/* ---- ungrouped span sets (BASELINE.json north_star (2)) ------------------
 * Spans that arrive interleaved across traces — the Elasticsearch path of
 * enhanced_trace_collector.py:80-90,109-110 pulls sw_segment-* hits sorted by
 * start_time over all traces — carry their trace only in trace_hash (equal
 * hash = same trace).  anomod_spans_group groups them on the device with a
 * segmented radix sort: traces ordered by mix64(trace_hash) ascending (the
 * SplitMix64 finaliser), the spans of a trace in arrival order (stable), so
 * every grouped-set kernel then sees each trace's spans in the order they
 * arrived (first-match parent rule, trace_collector.py:424-443).            */
int anomod_spans_upload_ungrouped(anomod_ctx* ctx, const anomod_span_soa* soa, uint64_t n_spans,
                                  anomod_spans** out);
int anomod_spans_grouped(const anomod_spans* spans, int* grouped);
int anomod_spans_group(anomod_ctx* ctx, const anomod_spans* ungrouped, anomod_spans** grouped);
/* How the ctx's last grouping ran (csrc/group.hip, csrc/bucket.hip):
 * *path = 1 bucket path (two stable MSD scatters over the top *bits bits of
 * mix64(trace_hash), then one workgroup per bucket), 2 the same scatters then
 * the per-bucket hash join of anomod_edge_aggregate_ungrouped (edge records,
 * no grouped columns), 3 the same scatters then the sorting bucket kernels'
 * edge records (the fused aggregation with ANOMOD_FUSED_JOIN=0), 0 LSD path (8-bit radix passes + bucket fix-up); *levels = scatter levels / radix passes run;
 * *bits = bucket bits (bucket path) or 8 * passes.  All 0 before any grouping. */
int anomod_ctx_group_info(const anomod_ctx* ctx, int* path, int* levels, int* bits);
/* Size the ctx's grouping workspace (grow-only, kept until the ctx is
 * destroyed) for sets of up to n_spans spans ahead of their first
 * aggregation: ~58 B per span for the ungrouped aggregation's join path,
 * + 32 B with both_records (grouping into columns, the LSD path).  A
 * workspace of tens of GB can take seconds to obtain from the driver when
 * the memory it gets was in use earlier in the process; reserving it when the
 * set is made keeps that out of the aggregation call.  Context.upload_ungrouped
 * and Context.shuffle (interleaving) in the Python package reserve for the
 * set they return.                                                         */
int anomod_ctx_reserve_grouping(anomod_ctx* ctx, uint64_t n_spans, int both_records);
/* Rearranged copies of a grouped set (synthetic arrival orders for tests
 * and benchmarks): window_traces = 0 shuffles the spans inside every trace
 * (the result stays grouped); window_traces = W interleaves the spans of
 * every W consecutive traces in a random order (the result is ungrouped).  */
int anomod_spans_shuffle(anomod_ctx* ctx, const anomod_spans* grouped, uint64_t seed,
                         uint64_t window_traces, anomod_spans** out);

/* ---- synthetic workload ----------------------*/
#define ANOMOD_TOPO_SN 0 /* DeathStarBench SocialNetwork, 12 services        */
#define ANOMOD_TOPO_TT 1 /* TrainTicket, 46 services                         */
#define ANOMOD_TOPO_LONG 2 /* SN services, traces of 16..4000 spans (stress) */

typedef struct {
  uint32_t topology;          /* ANOMOD_TOPO_*                               */
  uint32_t fault_service;     /* service index with an injected fault, or
                                 UINT32_MAX for a normal run                 */
  uint64_t seed;              /* Philox4x32-10 key                           */
  uint32_t fault_latency_mult;/* latency multiplier on the faulty service    */
  uint32_t p_error_ppm;       /* base error probability (parts per million)  */
  uint32_t p_fault_error_ppm; /* error probability on the faulty service     */
  uint32_t p_orphan_ppm;      /* probability a non-root span loses its parent*/
} anomod_synth_spec;

int anomod_synth_n_services(uint32_t topology, uint32_t* out);
/* Service name of index i (sorted-name order, cf. trace_collector.py:536). */
const char* anomod_synth_service_name(uint32_t topology, uint32_t i);
/* Host generation (same code path as the device generator): first count the
 * spans of traces [0, n_traces) of shard `shard`, then fill caller buffers.
 * dst arrays have n_spans entries, trace_ptr has n_traces + 1.             */
int anomod_synth_count_host(const anomod_synth_spec* spec, uint64_t shard, uint64_t n_traces,
                            uint64_t* n_spans);
int anomod_synth_generate_host(const anomod_synth_spec* spec, uint64_t shard, uint64_t n_traces,
                               const anomod_span_soa_out* dst, uint64_t* trace_ptr);
/* Device generation straight into HBM (no PCIe), bit-identical to host.    */
int anomod_spans_generate(anomod_ctx* ctx, const anomod_synth_spec* spec, uint64_t shard,
                          uint64_t n_traces, anomod_spans** out);

/* ---- native trace-file decoders --------------------
 * Parse a whole file image (caller's bytes, UTF-8 JSON) into span columns
 * without a Python object per span:
 *   anomod_decode_jaeger      Jaeger /api/traces dump (all_traces.json), the
 *                             columns jaeger_to_csv.py:21-90 derives
 *   anomod_decode_skywalking  trace_collector.py collector payload
 *                             ({metadata, traces:[{summary, spans}]}, :564-578)
 * services (may be NULL): the service-name list to index against; NULL =
 * the sorted distinct names of the file.  Ids: Jaeger spanIDs of 1-16 hex
 * digits are their value, other ids xxh64 | 2^63; SkyWalking node ids become
 * dense per-trace ids (first occurrence + 1; a parent naming no node of the
 * trace = UINT64_MAX).  trace_hash = xxh64 of the trace id.                 */
typedef struct anomod_decoded anomod_decoded;
int anomod_decode_jaeger(const char* json, uint64_t len, const char* const* services,
                         uint32_t n_services, anomod_decoded** out);
int anomod_decode_skywalking(const char* json, uint64_t len, const char* const* services,
                             uint32_t n_services, anomod_decoded** out);
int anomod_decoded_info(const anomod_decoded* d, uint64_t* n_spans, uint64_t* n_traces,
                        uint32_t* n_services);
/* *unique = 1 when no trace of the document holds a span id twice (checked
 * exactly while decoding: Jaeger spanIDs after their id mapping, SkyWalking
 * node ids), else 0 — what anomod_spans_set_unique_ids takes.              */
int anomod_decoded_unique_ids(const anomod_decoded* d, int* unique);
const char* anomod_decoded_service(const anomod_decoded* d, uint32_t i);
int anomod_decoded_columns(const anomod_decoded* d, const anomod_span_soa_out* dst,
                           uint64_t* trace_ptr /* [n_traces + 1] */);
int anomod_decoded_free(anomod_decoded* d);
/* The 64-bit id hash of the decoders (xxh64, seed 0; 0 maps to 1).       */
uint64_t anomod_hash64(const char* s, uint64_t len);

/* ---- native metric-file decoders --------------
 * Prometheus CSVs -> the time-major series matrix X[T][S] (f32, NaN = no
 * sample) the EWMA/z kernels read:
 *   anomod_decode_metric_long_csv   TT long CSV of metric_collector.py:400-478
 *                                   (series = (metric_name, sorted non-empty
 *                                   labels); rows de-duplicated on (series,
 *                                   timestamp), first kept, :420-423)
 *   anomod_decode_prometheus_csvs   SN metric directory, one CSV per query as
 *                                   fetch_prometheus_metrics.py:47-67,99 writes
 *                                   it (series = (file stem, 'metric' label
 *                                   string); naive datetimes read as local time)
 * Timestamps are the sorted distinct values of all rows; series are sorted
 * by (name, labels).  The same rules as anomod/decode.py's Python decoders. */
typedef struct anomod_metrics anomod_metrics;
int anomod_decode_metric_long_csv(const char* data, uint64_t len, anomod_metrics** out);
/* the same from a file path (mapped, not read; pieces faulted in by the
 * parser threads) */
int anomod_decode_metric_long_csv_file(const char* path, anomod_metrics** out);
int anomod_decode_prometheus_csvs(const char* const* data, const uint64_t* lens,
                                  const char* const* stems, uint32_t n_files,
                                  anomod_metrics** out);
int anomod_metrics_info(const anomod_metrics* m, uint64_t* T, uint64_t* S);
int anomod_metrics_matrix(const anomod_metrics* m, float* X /* [T][S] */,
                          double* timestamps /* [T] */);
const char* anomod_metrics_series_name(const anomod_metrics* m, uint64_t s);
uint32_t anomod_metrics_series_nlabels(const anomod_metrics* m, uint64_t s);
const char* anomod_metrics_series_label(const anomod_metrics* m, uint64_t s, uint32_t j,
                                        const char** value);
/* every series at once: name \0 (label name \0 label value \0) x nlabels[s],
 * series after series; *bytes = the size needed.  buf == NULL or cap < *bytes
 * writes nothing but *bytes (and nlabels, when given: [S]). */
int anomod_metrics_series_packed(const anomod_metrics* m, char* buf, uint64_t cap,
                                 uint32_t* nlabels, uint64_t* bytes);
int anomod_metrics_free(anomod_metrics* m);

/* ---- edge aggregation (the hot path) -------------------------------------
 * Call-graph edge table with per-edge latency histogram, count, errors,
 * sum/min/max and p50/p99.  Replaces and extends the per-span loops of
 * jaeger_to_csv.py:21-90 (parent = first CHILD_OF ref, service from
 * processID) and trace_collector.py:401-481 (_build_span_records parent
 * resolution) + the per-service aggregation of
 * enhanced_trace_collector.py:216-296.  Integer results are bit-exact and
 * independent of launch geometry, shard count and span order within a trace
 * set.  When a communicator is attached the table is summed over all ranks
 * (RCCL all-reduce) before quantiles are taken.                            */
int anomod_edge_aggregate_spans(anomod_ctx* ctx, const anomod_spans* spans, uint32_t n_services,
                                anomod_edge_table* out);
/* Edge table of a host span set grouped by trace (trace_ptr), in one call:
 * the columns go to a device set the ctx keeps and regrows only when a
 * larger set comes (no trace_hash: the aggregation reads none) through the
 * pinned staging pipeline (worker threads pack svc|flags into pinned
 * buffers, several DMA streams), then anomod_edge_aggregate_spans.  The
 * set's hints (anomod_spans_hints) go in through *scan_order / *hist_form
 * and come back with what the call learned; unique_ids as
 * anomod_spans_set_unique_ids.  The product path's one conversion per
 * experiment (collect_trace.sh:70: each dump is converted once, then every
 * feature comes from it).                                                  */
int anomod_edge_aggregate_host(anomod_ctx* ctx, const anomod_span_soa* soa, uint64_t n_spans,
                               const uint64_t* trace_ptr, uint64_t n_traces, uint32_t n_services,
                               int unique_ids, int* scan_order, int* hist_form,
                               anomod_edge_table* out);
/* Edge table of an ungrouped set; a grouped set is aggregated as is.  By
 * default the set is bucketed by trace (the grouping's two scatter levels) and
 * each bucket finds its spans' parents by an LDS hash join on (trace, span id),
 * writing one edge record per span that the table is taken from (no grouped
 * columns).  A set whose buckets hold several traces of thousands of spans,
 * or ANOMOD_UNGROUPED_FUSED=0, takes group (anomod_spans_group, into a
 * workspace the ctx keeps) then aggregate.  Same table either way. */
int anomod_edge_aggregate_ungrouped(anomod_ctx* ctx, const anomod_spans* spans,
                                    uint32_t n_services, anomod_edge_table* out);
/* Exact per-edge order statistics (SURVEY.md §8a a11 cross-check mode): the
 * same per-span edges as the aggregation, one radix sort of (edge, latency)
 * keys, then per edge x[int(c * q)] of its sorted latencies with q the double
 * q_pct[k] / 100.0 and the product truncated — the reference's
 * sorted(x)[int(n*q)] for any q_pct (monitor_http_responses.py:180-190).
 * out: [E][nq] doubles (NaN for an empty edge); count: [E] (may be NULL).
 * Needs a grouped set of at most 2^32 - 4097 spans (one sort); q_pct[k] in
 * [0, 99], nq <= 16.                                                        */
int anomod_edge_quantiles_exact(anomod_ctx* ctx, const anomod_spans* spans, uint32_t n_services,
                                const uint32_t* q_pct, uint32_t nq, double* out, uint64_t* count);
/* One-shot host convenience: upload + aggregate + download.               */
int anomod_edge_aggregate(anomod_ctx* ctx, const anomod_span_soa* soa, uint64_t n_spans,
                          const uint64_t* trace_ptr, uint64_t n_traces, anomod_edge_table* out);

/* ---- trace structure -------------------------------
 * Per span and per trace, what _build_span_records / collect_traces compute
 * one dict at a time (trace_collector.py:401-481, 536-547).  Spans are nodes
 * keyed by their id; with duplicated ids the reference keeps the LAST span's
 * parent (:437) while every span joins its own parent's child list (:438-439).
 *   parent_pos  position in the trace of the node's parent (first span whose
 *               id equals the parent reference of the LAST span carrying the
 *               node's id), ANOMOD_NO_PARENT when the reference is 0 or names
 *               no span of the trace (:427-437, :443)
 *   depth       the BFS of :441-449: the node's deepest visit from the roots,
 *               i.e. the longest path along "node of a span's own parent
 *               reference -> the span's node" (with unique ids: the distance
 *               along the parents); 0 when no root reaches the node (:477) or
 *               a cycle the BFS reaches feeds it (the reference never ends)
 *   n_children  spans whose own parent reference names the node (:438-439)
 *   span_flags  ANOMOD_SPAN_ROOT | ANOMOD_SPAN_FIRST (first span with its id)
 *   n_roots     distinct root nodes of the trace (len(root_span_node_ids))
 *   svc_mask    services_involved (:536): bit s of word s/64, ceil(S/64) words
 * Every pointer may be NULL (that output is skipped).                      */
#define ANOMOD_NO_PARENT 0xFFFFFFFFu
#define ANOMOD_SPAN_ROOT 0x1u
#define ANOMOD_SPAN_FIRST 0x2u
typedef struct {
  uint32_t n_services;  /* in : S (sizes svc_mask)                          */
  uint32_t* parent_pos; /* [n_spans]                                        */
  uint32_t* depth;      /* [n_spans]                                        */
  uint32_t* n_children; /* [n_spans]                                        */
  uint8_t* span_flags;  /* [n_spans]                                        */
  uint32_t* n_roots;    /* [n_traces]                                       */
  uint64_t* svc_mask;   /* [n_traces * ceil(S / 64)]                        */
} anomod_trace_struct_out;
int anomod_trace_structure_spans(anomod_ctx* ctx, const anomod_spans* spans,
                                 anomod_trace_struct_out* out);
int anomod_trace_structure(anomod_ctx* ctx, const anomod_span_soa* soa, uint64_t n_spans,
                           const uint64_t* trace_ptr, uint64_t n_traces,
                           anomod_trace_struct_out* out);

/* ---- segment summary -------------------------------
 * analyze_trace_patterns (enhanced_trace_collector.py:216-296) over columnar
 * segment records: svc / endpoint are indices into the caller's name lists
 * (service_name decoded as extract_trace_info does, :130-150), is_error the
 * raw value, latency and start_time in ms.
 *   service_counts[s], endpoint_counts[e]  call counts (:246-253)
 *   error_count        records with is_error == 1 (:256-257)
 *   latency_*          count / sum / min / max over latency > 0 (:260-283;
 *                      avg = sum / count)
 *   start_*            count / min / max over start_time != 0 (:265-270)
 * min/max are 0 when their count is 0.                                      */
typedef struct {
  uint32_t n_services;       /* in : service ids are < n_services          */
  uint32_t n_endpoints;      /* in : endpoint ids are < n_endpoints        */
  uint64_t* service_counts;  /* [n_services] (may be NULL)                 */
  uint64_t* endpoint_counts; /* [n_endpoints] (may be NULL)                */
  uint64_t total;            /* out                                        */
  uint64_t error_count;      /* out                                        */
  uint64_t latency_count;    /* out                                        */
  int64_t latency_sum, latency_min, latency_max; /* out                    */
  uint64_t start_count;      /* out                                        */
  int64_t start_min, start_max; /* out                                     */
} anomod_segment_summary_out;
int anomod_segment_summary(anomod_ctx* ctx, const uint32_t* svc, const uint32_t* endpoint,
                           const int32_t* is_error, const int64_t* latency,
                           const int64_t* start_time, uint64_t n, anomod_segment_summary_out* out);

/* ---- API-response summary ----------------------------
 * Latency statistics of monitor_http_responses.py generate_summary
 * (:150-207) and enhanced_openapi_monitor.py generate_reports (:318-332):
 * the selected values (positive_only: v > 0, as generate_summary :167-169;
 * else every non-NaN value, as generate_reports :324) sorted, then
 *   min = x[0], max = x[c-1], median = x[c//2],
 *   p95 = x[int(c*0.95)], p99 = x[int(c*0.99)]   (f64 product, truncated)
 * exactly, and sum over the sorted values (fixed tree order: reproducible,
 * within c*2^-53 relative of Python's left-to-right sum).  All 0 when c = 0.
 * n <= 2^32 - 4097 (the sort's limit).                                     */
typedef struct {
  uint64_t count;             /* out: values selected                      */
  double min, max, sum;       /* out                                       */
  double median, p95, p99;    /* out                                       */
} anomod_value_summary_out;
int anomod_value_summary(anomod_ctx* ctx, const double* values, uint64_t n, int positive_only,
                         anomod_value_summary_out* out);
/* The device sort under the exact-order-statistic paths (the exact per-edge
 * quantiles and the value summary above): a stable LSD radix sort of n u64
 * keys by bits [begin_bit, end_bit) (every key < 2^end_bit), hand-written
 * for CDNA4 (csrc/radix.hip).  Host buffers in and out (may alias);
 * *passes (may be NULL) = 8-bit digit passes run (digits equal in every key
 * are skipped).  n <= 2^32 - 4097 (u32 tile offsets).                      */
int anomod_sort_u64(anomod_ctx* ctx, const uint64_t* keys, uint64_t n, int begin_bit,
                    int end_bit, uint64_t* sorted, int* passes);
/* generate_summary's distributions in the same pass: status_id / ctype_id
 * index the caller's first-appearance lists of status codes and content
 * types (content_type.split(';')[0], 'unknown' when absent: :163-173),
 * has_error = the response carries an 'error' key (:176-177); latency is
 * the value summary of latency_ms > 0.                                       */
typedef struct {
  uint32_t n_status;          /* in : status ids are < n_status            */
  uint32_t n_ctype;           /* in : content-type ids are < n_ctype       */
  uint64_t* status_counts;    /* [n_status] out                            */
  uint64_t* ctype_counts;     /* [n_ctype] out                             */
  uint64_t error_count;       /* out                                       */
  anomod_value_summary_out latency; /* out                                 */
} anomod_response_summary_out;
int anomod_response_summary(anomod_ctx* ctx, const uint32_t* status_id, const uint32_t* ctype_id,
                            const uint8_t* has_error, const double* latency_ms, uint64_t n,
                            anomod_response_summary_out* out);

/* ---- windowed EWMA / z-score -------------------------
 * X is time-major [T][S] f32 (NaN = missing sample).  Per series:
 *   d_t = x_t - m_{t-1};  z_t = d_t / sqrt(v_{t-1} + eps)
 *   m_t = m_{t-1} + alpha*d_t;  v_t = (1-alpha)*(v_{t-1} + alpha*d_t^2)
 * with m = x, v = 0, z = 0 at the first valid sample; NaN samples leave the
 * state untouched and score 0.  Z[w][s] = max |z_t| over t in window w of W
 * steps (T must be a multiple of W).  m/v equal pandas
 * Series.ewm(alpha, adjust=False).mean() / .var(bias=True).  The metric
 * matrix replaces the long CSV rows of metric_collector.py:427-443 and
 * fetch_prometheus_metrics.py:53-67.                                       */
int anomod_ewma_z(anomod_ctx* ctx, const float* X, uint64_t T, uint64_t S, float alpha,
                  uint32_t W, float eps, float* Z);
/* Device-resident streaming variant: X stays in HBM, the (m, v, n) state is
 * carried across calls so T can be processed in chunks.  upload takes
 * row-major host X[T][S]; the device copy is laid out for the kernel that
 * reads it (16-step tiles for the sequential kernel, rows for the
 * time-parallel one; ANOMOD_EWMA_MODE=1/2/3 forces sequential-tiles /
 * time-parallel / sequential-rows) — opaque to the caller.                */
int anomod_series_create(anomod_ctx* ctx, uint64_t T, uint64_t S, anomod_series** out);
int anomod_series_upload(anomod_ctx* ctx, anomod_series* ser, const float* X);
int anomod_series_fill_synthetic(anomod_ctx* ctx, anomod_series* ser, uint64_t seed,
                                 uint64_t t0);
int anomod_series_reset_state(anomod_ctx* ctx, anomod_series* ser);
/* The resident matrix back as host rows X[T][S] (whatever the device layout). */
int anomod_series_download(anomod_ctx* ctx, const anomod_series* ser, float* X);
int anomod_series_ewma_z(anomod_ctx* ctx, anomod_series* ser, float alpha, uint32_t W,
                         float eps, float* Z_host /* may be NULL */);
int anomod_series_free(anomod_series* ser);

/* ---- personalized PageRank RCA -----------------------
 * networkx 3.4.2 pagerank convention: out-edge CSR (row = caller) with
 * weights; rows are normalised by out-weight; dangling mass is sent along
 * the personalization p; x0 = 1/N;
 *   x <- alpha*(x A + sum_{dangling} x * p) + (1 - alpha)*p
 * stop when ||x - x_last||_1 < N*tol (tol > 0) or after `iters` iterations.
 * iters_done = iterations executed; status ANOMOD_OK even when tol was not
 * reached (caller checks iters_done == iters).                            */
int anomod_pagerank(anomod_ctx* ctx, const uint32_t* row_ptr, const uint32_t* col,
                    const float* w, uint32_t N, const double* p, double alpha, uint32_t iters,
                    double tol, double* x_out, uint32_t* iters_done);
int anomod_graph_create(anomod_ctx* ctx, const uint32_t* row_ptr, const uint32_t* col,
                        const float* w, uint32_t N, anomod_graph** out);
int anomod_graph_synthetic(anomod_ctx* ctx, uint32_t N, uint32_t mean_degree, uint64_t seed,
                           anomod_graph** out);
/* The same synthetic graph as host CSR (config 5: Pareto out-degrees of the
 * given mean, 2 % dangling, call-count weights): *nnz always; with every
 * array NULL a size query, else row_ptr [N + 1], col / w [cap >= nnz].     */
int anomod_graph_synthetic_csr(uint32_t N, uint32_t mean_degree, uint64_t seed,
                               uint32_t* row_ptr, uint32_t* col, float* w, uint64_t cap,
                               uint64_t* nnz);
int anomod_graph_info(const anomod_graph* g, uint32_t* N, uint64_t* nnz);
int anomod_graph_pagerank(anomod_ctx* ctx, anomod_graph* g, const double* p, double alpha,
                          uint32_t iters, double tol, double* x_out, uint32_t* iters_done);
/* Which path the last anomod_graph_pagerank / _batch solve of g took: 1 =
 * replayed hipGraph of per-iteration launches (fixed iterations; a batch:
 * per-iteration launches), 2 = per-iteration
 * launches with a host read-back of the L1 change (tolerance), 3 = one
 * persistent launch (grid barrier); | 4 = the persistent launch timed out at
 * its grid barrier (a workgroup never became resident, e.g. another process
 * held CUs) and the solve was rerun from x0 on path 1 or 2 — same result
 * bits.  fallbacks = such reruns over the graph's lifetime.              */
#define ANOMOD_PPR_PATH_GRAPH 1
#define ANOMOD_PPR_PATH_READBACK 2
#define ANOMOD_PPR_PATH_PERSISTENT 3
#define ANOMOD_PPR_PATH_FALLBACK 4
int anomod_graph_last_solve(const anomod_graph* g, uint32_t* path, uint32_t* fallbacks);
/* K (<= 16) personalizations solved together (replica mode, SURVEY.md §8e:
 * one vector per experiment / fault hypothesis): the CSR is read once per
 * iteration for all K.  P and X are [K][N]; every column equals its
 * anomod_graph_pagerank solve bit for bit (same arithmetic and reduction
 * order).  tol > 0: each vector stops at its own convergence iteration
 * (later iterations carry it unchanged); iters_done = iterations run.  One
 * persistent launch (grid barrier) when the batch's workgroups are all
 * resident (N = 10^5: K <= 16), else one launch per iteration.             */
int anomod_graph_pagerank_batch(anomod_ctx* ctx, anomod_graph* g, const double* P, uint32_t K,
                                double alpha, uint32_t iters, double tol, double* X,
                                uint32_t* iters_done);
/* Row-sharded solve (SURVEY.md §8e "sharded" series): with a communicator
 * attached (anomod_ctx_attach_comm) each rank computes its share of whole
 * 256-row blocks of the pull SpMV and every iteration ends in one grouped
 * RCCL exchange — u64 sums of the fixed-point dangling / L1 partials and an
 * in-place all-gather of the new vector.  Without a communicator,
 * virtual_shards = G > 1 runs the same G-way row split on this one device
 * (the single-GPU rehearsal of the sharded path).  Every rank returns the
 * whole vector, equal bit for bit to anomod_graph_pagerank's per-launch
 * solve for any G (same blocks, same integer-summed scalars).           */
int anomod_graph_pagerank_sharded(anomod_ctx* ctx, anomod_graph* g, const double* p,
                                  double alpha, uint32_t iters, double tol,
                                  uint32_t virtual_shards, double* x_out, uint32_t* iters_done);
int anomod_graph_free(anomod_graph* g);

/* ---- multi-GPU (one process per GPU, RCCL over xGMI) ---------------------*/
#define ANOMOD_UNIQUE_ID_BYTES 128
int anomod_comm_unique_id(uint8_t* out /* ANOMOD_UNIQUE_ID_BYTES */);
int anomod_ctx_attach_comm(anomod_ctx* ctx, const uint8_t* unique_id, int nranks, int rank);
int anomod_ctx_comm_info(const anomod_ctx* ctx, int* nranks, int* rank);

/* Host collective transport instead of RCCL (ranks that share one device —
 * RCCL refuses two ranks on a GPU —, or any host-side library such as gloo):
 * libanomod stages every collective through pinned host memory and calls
 *   allreduce(user, buf, count, dtype, op): in place over all ranks
 *   allgather(user, buf, bytes_per_rank): buf holds nranks blocks, this
 *     rank's (at rank * bytes_per_rank) filled; afterwards all are
 * returning 0 on success.  The same calls, in the same order, as the RCCL
 * path (status agreement, edge-table merge, sharded PageRank exchange). */
#define ANOMOD_DTYPE_I32 0
#define ANOMOD_DTYPE_U32 1
#define ANOMOD_DTYPE_U64 2
#define ANOMOD_DTYPE_F64 3
#define ANOMOD_OP_SUM 0
#define ANOMOD_OP_MIN 1
#define ANOMOD_OP_MAX 2
typedef int (*anomod_host_allreduce_fn)(void* user, void* buf, uint64_t count, int dtype, int op);
typedef int (*anomod_host_allgather_fn)(void* user, void* buf, uint64_t bytes_per_rank);
int anomod_ctx_attach_host_comm(anomod_ctx* ctx, int nranks, int rank,
                                anomod_host_allreduce_fn allreduce,
                                anomod_host_allgather_fn allgather, void* user);

#ifdef __cplusplus
}
#endif
#endif /* ANOMOD_H */
