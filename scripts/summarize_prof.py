#!/usr/bin/env python3
"""Turn a gpurun_out/prof run (scripts/gpu_round.sh) into the committed
profile summaries under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_bench.json         the bench line of the same round
  profiles/edge_agg_pmc.json        HBM bytes per edge-aggregation launch
                                    (FETCH_SIZE x 2 per the gfx950 correction
                                    in MI355X_MICROARCH.md "HBM", + WRITE_SIZE;
                                    both KiB), read back by bench.py

usage: python scripts/summarize_prof.py TAG [gpurun_out/prof] [gpurun_out/bench.log]
"""
from __future__ import annotations

import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def counter(path: Path, name: str, kernel: str) -> list[float]:
    vals = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]))
    return vals


def main() -> int:
    tag = sys.argv[1]
    prof = Path(sys.argv[2]) if len(sys.argv) > 2 else ROOT / "gpurun_out" / "prof"
    blog = Path(sys.argv[3]) if len(sys.argv) > 3 else ROOT / "gpurun_out" / "bench.log"
    out = ROOT / "profiles"
    out.mkdir(exist_ok=True)
    shutil.copy(prof / "trace" / "run_kernel_stats.csv", out / f"{tag}_kernel_stats.csv")
    bench = None
    for line in blog.read_text().splitlines():
        if line.startswith("{"):
            bench = json.loads(line)
    if bench:
        (out / f"{tag}_bench.json").write_text(json.dumps(bench, indent=1) + "\n")
    fetch = counter(prof / "pmc_fetch" / "run_counter_collection.csv", "FETCH_SIZE", "edge_agg_kernel")
    write = counter(prof / "pmc_write" / "run_counter_collection.csv", "WRITE_SIZE", "edge_agg_kernel")
    if fetch and bench:
        f_b = sum(fetch) / len(fetch) * 1024 * 2
        w_b = sum(write) / len(write) * 1024 if write else 0.0
        alg = bench["roofline"]["bytes_per_launch"]
        d = {"kernel": "edge_agg_kernel", "round": tag,
             "n_spans": bench["config"]["spans_per_gpu"],
             "fetch_size_kib": sum(fetch) / len(fetch), "write_size_kib": sum(write) / len(write)
             if write else None,
             "read_bytes_per_launch": f_b, "write_bytes_per_launch": w_b,
             "hbm_bytes_per_launch": f_b + w_b, "algorithmic_bytes_per_launch": alg,
             "traffic_over_algorithmic": (f_b + w_b) / alg,
             "correction": "FETCH_SIZE (KiB) x 1024 x 2 (gfx950: FETCH_SIZE counts half of a "
                           "wide coalesced read); WRITE_SIZE x 1024"}
        (out / "edge_agg_pmc.json").write_text(json.dumps(d, indent=1) + "\n")
        print(json.dumps(d, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
