"""ctypes binding of libanomod.so (the C ABI declared in include/anomod.h).

The library is the only compute path: if it cannot be loaded, every entry
point raises :class:`AnomodError` — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("ANOMOD_LIB", _HERE / "libanomod.so"))

ABI_VERSION = 2
HIST_SUB_BITS = 5
HIST_BINS = 896
ROOT_ROWS = 2
FLAG_ERROR = 0x1
UNIQUE_ID_BYTES = 128
TOPO_SN = 0
TOPO_TT = 1
TOPO_LONG = 2

OK, EINVAL, EHIP, ERCCL, ENOMEM, ESTATE = 0, -1, -2, -3, -4, -5
_STATUS = {EINVAL: "EINVAL", EHIP: "EHIP", ERCCL: "ERCCL", ENOMEM: "ENOMEM", ESTATE: "ESTATE"}

(STAGE_EDGE_AGG, STAGE_EDGE_FINAL, STAGE_EDGE_REDUCE, STAGE_EWMA, STAGE_PAGERANK,
 STAGE_TRACE_STRUCT, STAGE_SEGMENTS, STAGE_SUMMARY, STAGE_GROUP) = range(9)
(HOST_GROUP_ALLOC, HOST_GROUP_PINNED, HOST_GROUP_WALL, HOST_UPLOAD_SETUP,
 HOST_SET_ALLOC) = range(5)
HOST_SLOTS = 5
HOST_SLOT_NAMES = ("group_alloc", "group_pinned", "group_wall", "upload_setup", "set_alloc")
NO_PARENT = 0xFFFFFFFF
SPAN_ROOT, SPAN_FIRST = 0x1, 0x2


class AnomodError(RuntimeError):
    """A libanomod call failed (status code + anomod_last_error message)."""

    def __init__(self, status: int, message: str):
        super().__init__(f"{_STATUS.get(status, status)}: {message}")
        self.status = status


class SpanSoA(C.Structure):
    _fields_ = [
        ("trace_hash", C.POINTER(C.c_uint64)),
        ("span_id", C.POINTER(C.c_uint64)),
        ("parent_span_id", C.POINTER(C.c_uint64)),
        ("svc", C.POINTER(C.c_uint16)),
        ("flags", C.POINTER(C.c_uint16)),
        ("dur_us", C.POINTER(C.c_uint32)),
    ]


class EdgeTableC(C.Structure):
    _fields_ = [
        ("n_services", C.c_uint32),
        ("n_bins", C.c_uint32),
        ("count", C.POINTER(C.c_uint64)),
        ("errors", C.POINTER(C.c_uint64)),
        ("sum_us", C.POINTER(C.c_uint64)),
        ("min_us", C.POINTER(C.c_uint32)),
        ("max_us", C.POINTER(C.c_uint32)),
        ("hist", C.POINTER(C.c_uint64)),
        ("p50_us", C.POINTER(C.c_double)),
        ("p99_us", C.POINTER(C.c_double)),
    ]


class TraceStructC(C.Structure):
    _fields_ = [
        ("n_services", C.c_uint32),
        ("parent_pos", C.POINTER(C.c_uint32)),
        ("depth", C.POINTER(C.c_uint32)),
        ("n_children", C.POINTER(C.c_uint32)),
        ("span_flags", C.POINTER(C.c_uint8)),
        ("n_roots", C.POINTER(C.c_uint32)),
        ("svc_mask", C.POINTER(C.c_uint64)),
    ]


class ValueSummaryC(C.Structure):
    _fields_ = [
        ("count", C.c_uint64),
        ("min", C.c_double),
        ("max", C.c_double),
        ("sum", C.c_double),
        ("median", C.c_double),
        ("p95", C.c_double),
        ("p99", C.c_double),
    ]


class ResponseSummaryC(C.Structure):
    _fields_ = [
        ("n_status", C.c_uint32),
        ("n_ctype", C.c_uint32),
        ("status_counts", C.POINTER(C.c_uint64)),
        ("ctype_counts", C.POINTER(C.c_uint64)),
        ("error_count", C.c_uint64),
        ("latency", ValueSummaryC),
    ]


class SegmentSummaryC(C.Structure):
    _fields_ = [
        ("n_services", C.c_uint32),
        ("n_endpoints", C.c_uint32),
        ("service_counts", C.POINTER(C.c_uint64)),
        ("endpoint_counts", C.POINTER(C.c_uint64)),
        ("total", C.c_uint64),
        ("error_count", C.c_uint64),
        ("latency_count", C.c_uint64),
        ("latency_sum", C.c_int64),
        ("latency_min", C.c_int64),
        ("latency_max", C.c_int64),
        ("start_count", C.c_uint64),
        ("start_min", C.c_int64),
        ("start_max", C.c_int64),
    ]


class SynthSpec(C.Structure):
    _fields_ = [
        ("topology", C.c_uint32),
        ("fault_service", C.c_uint32),
        ("seed", C.c_uint64),
        ("fault_latency_mult", C.c_uint32),
        ("p_error_ppm", C.c_uint32),
        ("p_fault_error_ppm", C.c_uint32),
        ("p_orphan_ppm", C.c_uint32),
    ]


_vp = C.c_void_p
_u32, _u64, _i32 = C.c_uint32, C.c_uint64, C.c_int
_f32, _f64 = C.c_float, C.c_double
_P = C.POINTER

# name -> (restype, argtypes)
_SIGS = {
    "anomod_abi_version": (_i32, []),
    "anomod_last_error": (C.c_char_p, [_vp]),
    "anomod_device_count": (_i32, [_P(_i32)]),
    "anomod_ctx_create": (_i32, [_i32, _P(_vp)]),
    "anomod_ctx_destroy": (_i32, [_vp]),
    "anomod_ctx_synchronize": (_i32, [_vp]),
    "anomod_ctx_stage_ms": (_i32, [_vp, _i32, _P(_f64)]),
    "anomod_ctx_host_ms": (_i32, [_vp, _i32, _P(_f64), _P(_u64)]),
    "anomod_hist_bin": (_u32, [_u32]),
    "anomod_hist_bin_bounds": (_i32, [_u32, _P(_u32), _P(_u32)]),
    "anomod_spans_upload": (_i32, [_vp, _P(SpanSoA), _u64, _P(_u64), _u64, _P(_vp)]),
    "anomod_spans_info": (_i32, [_vp, _P(_u64), _P(_u64)]),
    "anomod_spans_download": (_i32, [_vp, _vp, _P(SpanSoA), _P(_u64)]),
    "anomod_spans_free": (_i32, [_vp]),
    "anomod_spans_set_unique_ids": (_i32, [_vp, C.c_int]),
    "anomod_spans_unique_ids": (_i32, [_vp, _P(C.c_int)]),
    "anomod_spans_scan_order": (_i32, [_vp, _P(C.c_int)]),
    "anomod_spans_hist_compact": (_i32, [_vp, _P(C.c_int)]),
    "anomod_spans_hints": (_i32, [_vp, _P(C.c_int), _P(C.c_int)]),
    "anomod_spans_set_hints": (_i32, [_vp, C.c_int, C.c_int]),
    "anomod_spans_upload_ungrouped": (_i32, [_vp, _P(SpanSoA), _u64, _P(_vp)]),
    "anomod_spans_grouped": (_i32, [_vp, _P(_i32)]),
    "anomod_spans_group": (_i32, [_vp, _vp, _P(_vp)]),
    "anomod_ctx_group_info": (_i32, [_vp, _P(_i32), _P(_i32), _P(_i32)]),
    "anomod_ctx_reserve_grouping": (_i32, [_vp, _u64, C.c_int]),
    "anomod_spans_shuffle": (_i32, [_vp, _vp, _u64, _u64, _P(_vp)]),
    "anomod_edge_aggregate_ungrouped": (_i32, [_vp, _vp, _u32, _P(EdgeTableC)]),
    "anomod_edge_quantiles_exact": (_i32, [_vp, _vp, _u32, _P(_u32), _u32, _P(_f64), _P(_u64)]),
    "anomod_synth_n_services": (_i32, [_u32, _P(_u32)]),
    "anomod_synth_service_name": (C.c_char_p, [_u32, _u32]),
    "anomod_synth_count_host": (_i32, [_P(SynthSpec), _u64, _u64, _P(_u64)]),
    "anomod_synth_generate_host": (_i32, [_P(SynthSpec), _u64, _u64, _P(SpanSoA), _P(_u64)]),
    "anomod_spans_generate": (_i32, [_vp, _P(SynthSpec), _u64, _u64, _P(_vp)]),
    "anomod_edge_aggregate_spans": (_i32, [_vp, _vp, _u32, _P(EdgeTableC)]),
    "anomod_edge_aggregate_host": (_i32, [_vp, _P(SpanSoA), _u64, _P(_u64), _u64, _u32, _i32,
                                          _P(_i32), _P(_i32), _P(EdgeTableC)]),
    "anomod_edge_aggregate": (_i32, [_vp, _P(SpanSoA), _u64, _P(_u64), _u64, _P(EdgeTableC)]),
    "anomod_trace_structure_spans": (_i32, [_vp, _vp, _P(TraceStructC)]),
    "anomod_trace_structure": (_i32, [_vp, _P(SpanSoA), _u64, _P(_u64), _u64, _P(TraceStructC)]),
    "anomod_value_summary": (_i32, [_vp, _P(C.c_double), _u64, C.c_int, _P(ValueSummaryC)]),
    "anomod_sort_u64": (_i32, [_vp, _P(_u64), _u64, C.c_int, C.c_int, _P(_u64), _P(C.c_int)]),
    "anomod_response_summary": (_i32, [_vp, _P(_u32), _P(_u32), _P(C.c_uint8), _P(C.c_double),
                                       _u64, _P(ResponseSummaryC)]),
    "anomod_segment_summary": (_i32, [_vp, _P(_u32), _P(_u32), _P(C.c_int32), _P(C.c_int64),
                                      _P(C.c_int64), _u64, _P(SegmentSummaryC)]),
    "anomod_decode_jaeger": (_i32, [C.c_char_p, _u64, _P(C.c_char_p), _u32, _P(_vp)]),
    "anomod_decode_skywalking": (_i32, [C.c_char_p, _u64, _P(C.c_char_p), _u32, _P(_vp)]),
    "anomod_decoded_info": (_i32, [_vp, _P(_u64), _P(_u64), _P(_u32)]),
    "anomod_decoded_service": (C.c_char_p, [_vp, _u32]),
    "anomod_decoded_unique_ids": (_i32, [_vp, _P(C.c_int)]),
    "anomod_decoded_columns": (_i32, [_vp, _P(SpanSoA), _P(_u64)]),
    "anomod_decoded_free": (_i32, [_vp]),
    "anomod_hash64": (_u64, [C.c_char_p, _u64]),
    "anomod_decode_metric_long_csv": (_i32, [C.c_char_p, _u64, _P(_vp)]),
    "anomod_decode_metric_long_csv_file": (_i32, [C.c_char_p, _P(_vp)]),
    "anomod_decode_prometheus_csvs": (_i32, [_P(C.c_char_p), _P(_u64), _P(C.c_char_p), _u32,
                                             _P(_vp)]),
    "anomod_metrics_info": (_i32, [_vp, _P(_u64), _P(_u64)]),
    "anomod_metrics_matrix": (_i32, [_vp, _P(_f32), _P(_f64)]),
    "anomod_metrics_series_name": (C.c_char_p, [_vp, _u64]),
    "anomod_metrics_series_nlabels": (_u32, [_vp, _u64]),
    "anomod_metrics_series_label": (C.c_char_p, [_vp, _u64, _u32, _P(C.c_char_p)]),
    "anomod_metrics_series_packed": (_i32, [_vp, C.c_char_p, _u64, _P(_u32), _P(_u64)]),
    "anomod_metrics_free": (_i32, [_vp]),
    "anomod_ewma_z": (_i32, [_vp, _P(_f32), _u64, _u64, _f32, _u32, _f32, _P(_f32)]),
    "anomod_series_create": (_i32, [_vp, _u64, _u64, _P(_vp)]),
    "anomod_series_upload": (_i32, [_vp, _vp, _P(_f32)]),
    "anomod_series_fill_synthetic": (_i32, [_vp, _vp, _u64, _u64]),
    "anomod_series_reset_state": (_i32, [_vp, _vp]),
    "anomod_series_download": (_i32, [_vp, _vp, _P(_f32)]),
    "anomod_series_ewma_z": (_i32, [_vp, _vp, _f32, _u32, _f32, _P(_f32)]),
    "anomod_series_free": (_i32, [_vp]),
    "anomod_pagerank": (_i32, [_vp, _P(_u32), _P(_u32), _P(_f32), _u32, _P(_f64), _f64, _u32,
                               _f64, _P(_f64), _P(_u32)]),
    "anomod_graph_create": (_i32, [_vp, _P(_u32), _P(_u32), _P(_f32), _u32, _P(_vp)]),
    "anomod_graph_synthetic": (_i32, [_vp, _u32, _u32, _u64, _P(_vp)]),
    "anomod_graph_synthetic_csr": (_i32, [_u32, _u32, _u64, _P(_u32), _P(_u32), _P(_f32), _u64,
                                          _P(_u64)]),
    "anomod_graph_info": (_i32, [_vp, _P(_u32), _P(_u64)]),
    "anomod_graph_last_solve": (_i32, [_vp, _P(_u32), _P(_u32)]),
    "anomod_graph_pagerank": (_i32, [_vp, _vp, _P(_f64), _f64, _u32, _f64, _P(_f64), _P(_u32)]),
    "anomod_graph_pagerank_sharded": (_i32, [_vp, _vp, _P(_f64), _f64, _u32, _f64, _u32,
                                             _P(_f64), _P(_u32)]),
    "anomod_graph_pagerank_batch": (_i32, [_vp, _vp, _P(_f64), _u32, _f64, _u32, _f64, _P(_f64),
                                           _P(_u32)]),
    "anomod_graph_free": (_i32, [_vp]),
    "anomod_comm_unique_id": (_i32, [_P(C.c_uint8)]),
    "anomod_ctx_attach_comm": (_i32, [_vp, _P(C.c_uint8), _i32, _i32]),
    "anomod_ctx_comm_info": (_i32, [_vp, _P(_i32), _P(_i32)]),
    "anomod_ctx_attach_host_comm": (_i32, [_vp, _i32, _i32, _vp, _vp, _vp]),
}

# Host collective transport (include/anomod.h anomod_ctx_attach_host_comm).
DTYPE_I32, DTYPE_U32, DTYPE_U64, DTYPE_F64 = 0, 1, 2, 3
OP_SUM, OP_MIN, OP_MAX = 0, 1, 2
HostAllreduceFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_int)
HostAllgatherFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64)

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


def lib() -> C.CDLL:
    """Load libanomod.so once; raise loudly if it is missing or stale."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise AnomodError(
            ESTATE,
            f"{LIB_PATH} not found: build the HIP library first "
            "(python -c 'import __graft_entry__ as g; g.build()')",
        )
    handle = C.CDLL(str(LIB_PATH))
    for name, (res, args) in _SIGS.items():
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    v = handle.anomod_abi_version()
    if v != ABI_VERSION:
        raise AnomodError(ESTATE, f"libanomod ABI {v} != expected {ABI_VERSION}")
    _lib = handle
    return _lib


def check(status: int, ctx=None) -> None:
    if status != OK:
        msg = lib().anomod_last_error(ctx)
        raise AnomodError(status, msg.decode() if msg else "unknown error")


def ptr(a: np.ndarray | None, ctype):
    """ctypes pointer into a C-contiguous numpy array (None -> NULL)."""
    if a is None:
        return C.cast(None, C.POINTER(ctype))
    assert a.flags["C_CONTIGUOUS"], "arrays passed to libanomod must be C-contiguous"
    return a.ctypes.data_as(C.POINTER(ctype))
