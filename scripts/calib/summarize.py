#!/usr/bin/env python3
"""FETCH_SIZE calibration summary (scripts/calib/fetch_calib.hip run plain,
under rocprofv3 --pmc FETCH_SIZE and under --pmc TCC_HIT_sum TCC_MISS_sum) ->
profiles/<tag>_fetch_calibration.json: per access pattern, the true bytes one
launch reads, FETCH_SIZE (bytes), their ratio and the factor that turns a
kernel's FETCH_SIZE of that pattern into bytes requested from the memory side.

usage: python scripts/calib/summarize.py gpurun_out/r5a r05 [gpurun_out/r5d]
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
# request sizes and DRAM-bound requests (a second run: gpurun_out/r5d)
src2 = Path(sys.argv[3]) if len(sys.argv) > 3 else None
req = {}
if src2 and (src2 / "calib_reqsize.csv").exists():
    for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum",
              "TCC_EA0_RDREQ_128B_sum"):
        req[c] = per_kernel(src2 / "calib_reqsize.csv", c)
    req["TCC_EA0_RDREQ_DRAM_sum"] = per_kernel(src2 / "calib_dram.csv", "TCC_EA0_RDREQ_DRAM_sum")
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
    if req:
        q = {c: round(sum(v[4 * i:4 * i + 4]) / 4) for c, v in req.items()}
        out["patterns"][name]["requests"] = q
        out["patterns"][name]["useful_bytes_per_128B_request"] = round(
            t["true_bytes"] / max(q["TCC_EA0_RDREQ_128B_sum"], 1), 2)
out["conclusion"] = (
    "Every L2 miss is one 128-B read request (TCC_EA0_RDREQ_128B = TCC_EA0_RDREQ, no 32- or "
    "64-B requests) for streams and gathers alike, and FETCH_SIZE tallies each at 64 B: "
    "memory-side read bytes = 2 x FETCH_SIZE exactly, for every pattern.  TCC_EA0_RDREQ_DRAM "
    "equals TCC_EA0_RDREQ, so Infinity-Cache hits are not told apart from HBM reads: the "
    "72-MiB-window gathers request as many lines as the 8-GiB ones (gather32_win) and run at "
    "twice the rate, so 2 x FETCH_SIZE is line traffic at the memory side, an upper bound on "
    "HBM bytes.  Useful bytes per request: 128 for a coalesced stream (8 or 16 B per lane), 32 "
    "/ 16 / 8 for a gather of that width; FETCH_SIZE per useful byte 0.5 / 2 / 4 / 8.")
dst = ROOT / "profiles" / f"{tag}_fetch_calibration.json"
dst.write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out, indent=1))
