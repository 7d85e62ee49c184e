"""anomod — MI355X-native RCA-feature engine for the AnoMod dataset.

Call surface:

    exp = anomod.load_experiment(path_or_SynthSpec, metrics=...)
    feats = anomod.features(exp)          # GPU: edge table, p50/p99, window z
    ranking = anomod.rank(feats)          # GPU: personalized PageRank

All compute runs in libanomod.so (hand-written HIP for gfx950) through a
ctypes C ABI (include/anomod.h); there is no CPU fallback.
"""
from ._lib import (FLAG_ERROR, HIST_BINS, HIST_SUB_BITS, AnomodError, EXPORTED_SYMBOLS,
                   LIB_PATH, lib)
from .decode import (MetricMatrix, decode_jaeger, decode_native, load_trace_file, decode_metric_long_csv,
                     decode_metric_long_csv_native, decode_prometheus_csv_dir,
                     decode_prometheus_csv_dir_native, decode_skywalking_payload, decode_skywalking_raw,
                     jaeger_span_rows, merge_jaeger_dumps, skywalking_parents)
from .device import (Context, DeviceGraph, DeviceSeries, DeviceSpans, SynthSpec, device_count,
                     device_count_safe, synth_generate_host, synth_graph_csr, synth_services)
from .engine import (Experiment, Features, default_context, fault_target, features, hit_at,
                     load_experiment, rank)
from . import api
from .segments import SegmentSet, service_name_of, trace_infos
from .writers import jaeger_to_csv, write_jaeger_csv, write_metric_long_csv
from .spans import EdgeTable, SpanSet, TraceStructure, edge_rows

__all__ = [
    "AnomodError", "Context", "DeviceGraph", "DeviceSeries", "DeviceSpans", "EdgeTable",
    "EXPORTED_SYMBOLS", "Experiment", "FLAG_ERROR", "Features", "HIST_BINS", "HIST_SUB_BITS",
    "LIB_PATH", "MetricMatrix", "SpanSet", "SynthSpec", "decode_jaeger",
    "decode_metric_long_csv", "decode_metric_long_csv_native", "decode_prometheus_csv_dir",
    "decode_prometheus_csv_dir_native", "decode_skywalking_payload",
    "decode_skywalking_raw", "default_context", "device_count", "device_count_safe", "edge_rows", "fault_target",
    "features", "hit_at", "jaeger_span_rows", "lib", "load_experiment", "merge_jaeger_dumps",
    "rank", "skywalking_parents", "synth_generate_host", "synth_graph_csr", "synth_services", "TraceStructure",
    "SegmentSet", "service_name_of", "trace_infos", "analyze_trace_patterns",
    "jaeger_to_csv", "write_jaeger_csv", "write_metric_long_csv", "decode_native",
    "load_trace_file", "api",
]


def analyze_trace_patterns(traces_or_segments, ctx: "Context | None" = None) -> dict:
    """Drop-in for EnhancedTraceCollector.analyze_trace_patterns
    (enhanced_trace_collector.py:216-296): accepts its input (a list of
    extract_trace_info dicts), a raw Elasticsearch segment response, or a
    SegmentSet; the reductions run on the GPU."""
    if isinstance(traces_or_segments, SegmentSet):
        seg = traces_or_segments
    elif isinstance(traces_or_segments, dict):
        seg = SegmentSet.from_es(traces_or_segments)
    else:
        seg = SegmentSet.from_traces(list(traces_or_segments or []))
    return (ctx or default_context()).segment_summary(seg)
