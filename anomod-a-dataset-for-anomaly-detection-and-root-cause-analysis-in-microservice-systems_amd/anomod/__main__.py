"""CLI:  python -m anomod features <trace file|dir> [--metrics PATH] [--out FILE]
       python -m anomod jaeger-to-csv <all_traces.json> <all_traces.csv>

Computes the RCA features of one experiment on the GPU and writes them as JSON:
the call-graph edge table (count, errors, mean/min/max, p50/p99 per edge), the
per-service anomaly scores and the PageRank root-cause ranking.  It slots in
where the reference's bash orchestration calls its converters
(collect_trace.sh:70 ``python jaeger_to_csv.py ...``;
collect_all_modalities.sh:238 ``python3 trace_collector.py ...``).
"""
from __future__ import annotations

import argparse
import json
import sys

from . import features, load_experiment, rank


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m anomod")
    sub = ap.add_subparsers(dest="cmd", required=True)
    f = sub.add_parser("features", help="edge table + anomaly scores + ranking of one experiment")
    f.add_argument("traces", help="Jaeger all_traces.json / SkyWalking payload (file or dir)")
    f.add_argument("--metrics", help="SN metric dir (one CSV per query) or TT long metric CSV")
    f.add_argument("--window", type=int, default=60)
    f.add_argument("--alpha", type=float, default=0.85, help="PageRank damping")
    f.add_argument("--out", help="output JSON (default: stdout)")
    j = sub.add_parser("jaeger-to-csv",
                       help="span CSV identical to jaeger_to_csv.py's (collect_trace.sh:70)")
    j.add_argument("input")
    j.add_argument("output")
    args = ap.parse_args(argv)
    if args.cmd == "jaeger-to-csv":
        from .writers import jaeger_to_csv
        return jaeger_to_csv(args.input, args.output)

    exp = load_experiment(args.traces, metrics=args.metrics)
    feats = features(exp, W=args.window)
    ranking = rank(feats, alpha=args.alpha)
    doc = {
        "experiment": exp.name,
        "label": exp.label,
        "services": feats.edges.services,
        "spans": exp.spans.n_spans,
        "traces": exp.spans.n_traces,
        "edges": feats.edges.records(),
        "service_scores": dict(zip(feats.edges.services, map(float, feats.service_scores))),
        "ranking": ranking,
    }
    text = json.dumps(doc, indent=2)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(text)
    else:
        print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
