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
