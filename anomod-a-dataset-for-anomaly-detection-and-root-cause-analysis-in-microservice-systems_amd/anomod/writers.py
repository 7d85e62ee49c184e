"""File-boundary writers: the CSVs the reference's
collectors write, byte for byte, so the engine can stand in for them where
bash expects files.

* Jaeger dump -> 13-column span CSV: SN_collection-scripts/Dataset/trace_data/
  jaeger_to_csv.py:19-101 (rows :21-90, empty input :92-97, pandas to_csv
  :99-100).  Written with the csv module; the column typing pandas applies
  (a column of ints prints ints, a numeric column holding a float prints
  every value as a float, anything mixed prints str(value)) is restated.
* Prometheus range results -> TT long metric CSV:
  TT_collection-scripts/T-Dataset/metric_collector.py:400-478 (rows :427-443,
  'NaN' -> empty :435, columns fixed + sorted labels :453-467).
"""
from __future__ import annotations

import csv
import io
import json
import math
from datetime import datetime
from pathlib import Path

JAEGER_COLUMNS = ["trace_id", "span_id", "parent_span_id", "service", "operation", "start_time",
                  "duration_us", "http_status_code", "http_method", "http_url", "component",
                  "tags", "logs"]
_TAG_COLUMNS = {"http.status_code": 7, "http.method": 8, "http.url": 9, "component": 10}


def _local_us(seconds: float) -> str:
    return datetime.fromtimestamp(seconds).strftime("%Y-%m-%d %H:%M:%S.%f")


def jaeger_csv_rows(doc: dict) -> list[list]:
    """One 13-value row per span of a Jaeger /api/traces dump, in file order
    (the values jaeger_to_csv.py:76-90 puts in its DataFrame)."""
    rows = []
    for trace in doc.get("data", []):
        tid = trace.get("traceID", "")
        services = {pid: info.get("serviceName", "")
                    for pid, info in trace.get("processes", {}).items()}
        for span in trace.get("spans", []):
            parent = next((ref.get("spanID", "") for ref in span.get("references", [])
                           if ref.get("refType") == "CHILD_OF"), "")
            start_us = span.get("startTime", 0)
            tags, special = {}, ["", "", "", ""]
            for tag in span.get("tags", []):
                key, value = tag.get("key", ""), tag.get("value", "")
                tags[key] = value
                if key in _TAG_COLUMNS:
                    special[_TAG_COLUMNS[key] - 7] = value
            logs = []
            for log in span.get("logs", []):
                fields = {f.get("key", ""): f.get("value", "") for f in log.get("fields", [])}
                logs.append(f"{_local_us(log.get('timestamp', 0) / 1000000)}: "
                            f"{json.dumps(fields)}")
            rows.append([tid, span.get("spanID", ""), parent,
                         services.get(span.get("processID", ""), ""),
                         span.get("operationName", ""),
                         _local_us(start_us / 1000 / 1000),  # µs -> ms -> s, as :41-43
                         span.get("duration", 0), *special, json.dumps(tags), "; ".join(logs)])
    return rows


def _column_formatter(values: list):
    """How pandas.DataFrame.to_csv prints one inferred column."""
    def is_int(v):
        return isinstance(v, int) and not isinstance(v, bool)

    def is_num(v):
        return is_int(v) or isinstance(v, float)

    if values and all(is_num(v) for v in values) and any(isinstance(v, float) for v in values):
        return lambda v: "" if math.isnan(float(v)) else repr(float(v))  # float64 column
    return lambda v: "" if v is None else str(v)


def write_jaeger_csv(doc: dict, out) -> int:
    """Write the span CSV of a Jaeger dump to a path or text file; returns the
    number of span rows (0 -> header-only file, :92-97)."""
    rows = jaeger_csv_rows(doc)
    fmts = [_column_formatter([r[c] for r in rows]) for c in range(len(JAEGER_COLUMNS))]
    own = isinstance(out, (str, Path))
    fh = open(out, "w", newline="", encoding="utf-8") if own else out
    try:
        w = csv.writer(fh, lineterminator="\n")
        w.writerow(JAEGER_COLUMNS)
        for r in rows:
            w.writerow([f(v) for f, v in zip(fmts, r)])
    finally:
        if own:
            fh.close()
    return len(rows)


def jaeger_to_csv(in_json, out_csv) -> int:
    """CLI twin of ``python jaeger_to_csv.py <in> <out>`` (collect_trace.sh:70):
    returns the process exit status (1 on invalid JSON, :15-17)."""
    try:
        with open(in_json, encoding="utf-8") as fh:
            doc = json.load(fh)
    except json.JSONDecodeError:
        print("Error: invalid JSON payload.")
        return 1
    n = write_jaeger_csv(doc, out_csv)
    print(f"Exported {n} spans to {out_csv}" if n else "Warning: no trace data detected.")
    return 0


METRIC_FIXED = ["metric_name", "timestamp", "datetime", "value"]


def metric_long_rows(results) -> list[dict]:
    """Rows of the TT long metric CSV from (query, Prometheus matrix result)
    pairs in query order (metric_collector.py:427-443)."""
    items = results.items() if isinstance(results, dict) else results
    rows = []
    for query, result in items:
        for series in result or []:
            if "values" not in series:
                continue
            labels = {k: v for k, v in series.get("metric", {}).items() if k != "__name__"}
            for ts, value in series["values"]:
                row = {"metric_name": query, "timestamp": ts,
                       "datetime": datetime.fromtimestamp(ts).isoformat(),
                       "value": float(value) if value != "NaN" else None}
                row.update(labels)
                rows.append(row)
    return rows


def write_metric_long_csv(results, out) -> int:
    """The long CSV (fixed columns, then the sorted union of label names;
    missing labels and NaN values empty: metric_collector.py:453-467)."""
    rows = metric_long_rows(results)
    labels = sorted({k for r in rows for k in r} - set(METRIC_FIXED))
    cols = METRIC_FIXED + labels
    own = isinstance(out, (str, Path))
    fh = open(out, "w", newline="", encoding="utf-8") if own else out
    try:
        w = csv.writer(fh)  # DictWriter defaults: excel dialect, \r\n rows
        w.writerow(cols)
        for r in rows:
            w.writerow(["" if r.get(c) is None else r.get(c, "") for c in cols])
    finally:
        if own:
            fh.close()
    return len(rows)


def to_text(writer, *args) -> str:
    buf = io.StringIO(newline="")
    writer(*args, buf)
    return buf.getvalue()


# --------------------------------------------------------------------------
# TT files of one experiment from a span set / metric matrix (the layouts
# load_experiment reads: trace_collector.py:564-581 payload, json.dump
# indent=2; metric_collector.py:453-467 long CSV).  Used to stage the
# dataset's file formats at their LFS sizes for end-to-end timing.
# --------------------------------------------------------------------------
def _utc_iso_ms(ms: int) -> str:  # utc_iso (trace_collector.py:126-131)
    return datetime.utcfromtimestamp(ms / 1000).isoformat(timespec="milliseconds") + "Z"


def skywalking_payload(spans, experiment_name: str, t0_ms: int = 1762178400000) -> dict:
    """A collector payload ({metadata, traces}) holding `spans`: one segment
    per trace, node ids "{segment}:{k}", SpanRecord.to_dict fields
    (trace_collector.py:86-123), durations in whole ms."""
    import numpy as np  # noqa: F401  (spans columns are numpy arrays)

    traces = []
    services_seen = set()
    ptr = spans.trace_ptr.tolist()
    sid = spans.span_id.tolist()
    pid = spans.parent_span_id.tolist()
    svc = spans.svc.tolist()
    fl = spans.flags.tolist()
    dur = spans.dur_us.tolist()
    names = spans.services
    for t in range(spans.n_traces):
        a, b = ptr[t], ptr[t + 1]
        if a == b:
            continue
        tid = f"{t:08x}.{spans.trace_hash[a]:016x}"
        seg = f"seg{t:08x}"
        pos = {}
        for i in range(a, b):
            pos.setdefault(sid[i], i - a)
        start = t0_ms + t
        recs, roots, svcs = [], [], set()
        for i in range(a, b):
            k = i - a
            p = pos.get(pid[i]) if pid[i] else None
            node, pnode = f"{seg}:{k}", (f"{seg}:{p}" if p is not None else None)
            if pnode is None:
                roots.append(node)
            s_ms = start + k
            e_ms = s_ms + dur[i] // 1000
            sc = names[svc[i]]
            svcs.add(sc)
            tags = [{"key": "http.method", "value": "GET"},
                    {"key": "url", "value": f"http://{sc}:8080/api/v1/op{k}"}]
            recs.append({
                "node_id": node, "trace_id": tid, "segment_id": seg, "span_id": k,
                "parent_span_id": p if p is not None else -1, "parent_node_id": pnode,
                "depth": 0, "children_node_ids": [], "service_code": sc,
                "service_instance": f"{sc}-7d9c4b6f5-x2x9k", "start_time_utc": _utc_iso_ms(s_ms),
                "end_time_utc": _utc_iso_ms(e_ms), "start_timestamp_ms": s_ms,
                "end_timestamp_ms": e_ms, "duration_ms": e_ms - s_ms,
                "endpoint_name": f"/api/v1/op{k}", "type": "Entry" if p is None else "Exit",
                "peer": None if p is None else f"{sc}:8080", "component": "SpringMVC",
                "layer": "Http", "is_error": bool(fl[i] & 1), "tags": tags,
                "tags_map": {d["key"]: d["value"] for d in tags}, "logs": [], "refs": []})
        services_seen |= svcs
        traces.append({"summary": {"trace_id": tid, "segment_id": seg, "duration": 0,
                                   "start": str(start), "endpoint_names": ["/api"],
                                   "is_error": False},
                       "span_count": len(recs), "services_involved": sorted(svcs),
                       "root_span_node_ids": roots, "spans": recs})
    return {"metadata": {"generated_at": "2025-11-03T14:02:00Z", "lookback_hours": 1,
                         "requested_trace_limit": len(traces), "min_trace_duration_ms": 0,
                         "collected_traces": len(traces), "available_total": len(traces),
                         "services_discovered": sorted(services_seen),
                         "experiment_name": experiment_name,
                         "skywalking_base_url": "http://skywalking-oap:12800",
                         "skywalking_graphql": "http://skywalking-oap:12800/graphql"},
            "traces": traces}


def write_metric_long_csv_matrix(X, timestamps, series, out) -> int:
    """A metric matrix as the TT long CSV (metric_collector.py:453-467:
    metric_name, timestamp, datetime, value, then the sorted label columns;
    NaN -> empty), one row per (series, timestamp), series-major as the
    collector emits them.  Vectorised over a series' samples."""
    import numpy as np

    label_names = sorted({k for _, labels in series for k, _ in labels})
    ts = np.asarray(timestamps)
    ts_txt = np.array([repr(float(t)) if not float(t).is_integer() else str(int(t)) for t in ts],
                      dtype=object)
    dt_txt = np.array([datetime.utcfromtimestamp(float(t)).strftime("%Y-%m-%d %H:%M:%S")
                       for t in ts], dtype=object)
    head = ",".join(["metric_name", "timestamp", "datetime", "value"] + label_names) + "\n"
    rows = 0
    with open(out, "w", encoding="utf-8", newline="") as fh:
        fh.write(head)
        for j, (name, labels) in enumerate(series):
            d = dict(labels)
            tail = "," + ",".join(_csv_field(d.get(k, "")) for k in label_names) + "\n"
            col = X[:, j].astype(np.float64)
            vals = np.char.mod("%.9g", col).astype(object)
            vals[np.isnan(col)] = ""
            pre = _csv_field(name) + ","
            fh.write("".join((pre + ts_txt + "," + dt_txt + "," + vals + tail).tolist()))
            rows += col.shape[0]
    return rows


def _csv_field(v: str) -> str:
    v = str(v)
    if any(c in v for c in ',"\r\n'):
        return '"' + v.replace('"', '""') + '"'
    return v
