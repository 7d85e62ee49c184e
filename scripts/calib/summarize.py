#!/usr/bin/env python3
"""FETCH_SIZE calibration summary (scripts/calib/fetch_calib.hip run plain,
under rocprofv3 --pmc FETCH_SIZE and under --pmc TCC_HIT_sum TCC_MISS_sum) ->
profiles/<tag>_fetch_calibration.json: per access pattern, the true bytes one
launch reads, FETCH_SIZE (bytes), their ratio and the factor that turns a
kernel's FETCH_SIZE of that pattern into bytes requested from the memory side.

usage: python scripts/calib/summarize.py gpurun_out/r5a r05
"""
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
src = Path(sys.argv[1])
tag = sys.argv[2] if len(sys.argv) > 2 else "r05"
ORDER = ["stream16", "stream8", "gather32_far", "gather32_win", "gather16_far", "gather16_win",
         "gather8_far"]
DESC = {
    "stream16": "16 B per lane, coalesced, 8 GiB (the guide's reference pattern)",
    "stream8": "8 B per lane, coalesced, 8 GiB (pair loads)",
    "gather32_far": "32-B records (two 16-B loads per lane) at uniform random indices over 8 GiB",
    "gather32_win": "32-B records at random indices inside 72 MiB windows (one level-A bucket: "
                    "the join's gathers)",
    "gather16_far": "16-B records at random indices over 8 GiB",
    "gather16_win": "16-B records at random indices inside 8 MiB windows (batched PageRank x)",
    "gather8_far": "8-B words at random indices over 8 GiB",
}
timing = [json.loads(l) for l in (src / "calib_time.log").read_text().splitlines()
          if l.startswith("{")]


def per_kernel(path, counter):
    """counter values of the calibration kernels in dispatch order (fill excluded)."""
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter
            and "fill_kernel" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [float(r["Counter_Value"]) for r in rows]


fetch = per_kernel(src / "calib_fetch.csv", "FETCH_SIZE")
hit = per_kernel(src / "calib_hitmiss.csv", "TCC_HIT_sum")
miss = per_kernel(src / "calib_hitmiss.csv", "TCC_MISS_sum")
out = {"what": "FETCH_SIZE against known byte counts (scripts/calib/fetch_calib.hip, 4 "
               "launches per pattern: one warm + 3 timed; values per launch)",
       "source": str(src), "patterns": {}}
for i, t in enumerate(timing):
    name = t["kernel"]
    f = fetch[4 * i:4 * i + 4]
    h, m = hit[4 * i:4 * i + 4], miss[4 * i:4 * i + 4]
    fb = sum(f) / len(f) * 1024.0
    mm = sum(m) / len(m)
    out["patterns"][name] = {
        "desc": DESC.get(name, ""), "true_bytes": t["true_bytes"],
        "fetch_size_bytes": round(fb), "fetch_over_true": round(fb / t["true_bytes"], 4),
        "true_over_fetch": round(t["true_bytes"] / fb, 4),
        "tcc_miss": round(mm), "tcc_hit": round(sum(h) / len(h)),
        "fetch_bytes_per_miss": round(fb / mm, 2),
        "best_ms": t["best_ms"], "true_GBps": t["GBps"],
        "requested_GBps": round(2 * fb / (t["best_ms"] * 1e6), 1),
    }
out["conclusion"] = (
    "FETCH_SIZE = 64 B per L2 miss (fetch_bytes_per_miss) for every pattern, streams and "
    "gathers alike.  For the streams the true bytes are exactly 2 x FETCH_SIZE, i.e. 128 B per "
    "miss.  A gather's request size cannot be read off FETCH_SIZE (a 64-B and a 128-B request "
    "tally the same); 128-B lines are consistent with the rates (gather8_far: 67 M misses in "
    "1.44 ms = 6.0 TB/s of 128-B lines, the stream's rate).  Calibrated factors, FETCH_SIZE -> "
    "useful bytes: stream 2.0 (8 or 16 B per lane), gather32 0.50, gather16 0.25, gather8 0.125; "
    "memory-side line traffic = 2 x FETCH_SIZE for all.  Infinity-Cache hits are counted: the "
    "72-MiB-window gathers miss L2 as often as the 8-GiB ones (gather32_win) at twice the rate.")
dst = ROOT / "profiles" / f"{tag}_fetch_calibration.json"
dst.write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out, indent=1))
