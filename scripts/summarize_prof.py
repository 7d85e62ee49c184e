#!/usr/bin/env python3
"""Turn a gpurun_out/prof run (scripts/gpu_round.sh) into the committed
profile summaries under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_bench.json         the bench line of the same round
  profiles/<tag>_pmc.json           HBM bytes per launch of the edge, trace-structure
                                    and EWMA kernels
  profiles/edge_agg_pmc.json        HBM bytes per edge-aggregation launch
                                    (FETCH_SIZE x 2 per the gfx950 correction
                                    in MI355X_MICROARCH.md "HBM", + WRITE_SIZE;
                                    both KiB), read back by bench.py

usage: python scripts/summarize_prof.py TAG [gpurun_out/prof] [gpurun_out/bench.log]
       (scripts/profile_r03.sh layout: TAG gpurun_out/r03prof gpurun_out/r03prof/bench_profiled.log
        — the bench line printed BY the profiled process, so the headline kernel's
        rocprof dispatch times and ms_per_step come from one run)
"""
from __future__ import annotations

import csv
import json
import math
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


# PMC runs: `bench.py --steps 2 --warmup 0 --legs ...` — the SN-width edge
# kernel's first 2 dispatches are the headline's, later ones other legs'
FIRST_N = {"edge_agg_kernel": 2}


def counter(path: Path, name: str, kernel: str) -> list[float]:
    vals = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == name:
                vals.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    vals.sort()
    n = FIRST_N.get(kernel)
    return [v for _, v in (vals[:n] if n else vals)]


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
    # HBM bytes per launch of each profiled kernel (PMC passes of
    # scripts/profile.sh), against the algorithmic bytes of the same launch
    # from the bench line of the same box
    alg = {}
    per_unit = {}  # launches per algorithmic unit (EWMA: a chunk runs as time segments)
    if bench:
        alg["edge_agg_kernel"] = bench["roofline"]["bytes_per_launch"]
        if "trace_structure" in bench:
            alg["trace_struct_kernel"] = bench["trace_structure"]["bytes_per_launch"]
        if "ewma" in bench:
            e = bench["ewma"]
            samples = e["steps_per_chunk"] * e["S"]
            alg["ewma_zt_kernel"] = 4 * samples + 4 * samples // e["W"] + 40 * e["S"]
            # ewma.hip: segments of floor(16384 / lcm(W, 64)) * lcm(W, 64) steps
            l = e["W"] * 64 // math.gcd(e["W"], 64)
            seg = max(l, 16384 // l * l)
            per_unit["ewma_zt_kernel"] = -(-e["steps_per_chunk"] // seg)
        if "ungrouped" in bench:
            u = bench["ungrouped"]
            info = u.get("group_path", {"path": "lsd", "levels": u.get("radix_passes", 4)})
            if info["path"] == "bucket":
                # a scatter level reads and writes one 32-B record per span (the
                # first also writes the next level's 2-B digit: averaged); the
                # bucket kernel reads the records and writes the SoA columns
                lv = info["levels"]
                alg["bk_scatter_kernel"] = (64 + 2 * (lv - 1) / lv) * u["spans"]
                alg["bk_bucket_kernel"] = 64 * u["spans"]
            else:
                # a radix pass reads and writes one 32-B record per span; every
                # pass but the last also writes the next pass's 1-B digit
                P = info["levels"]
                alg["group_scatter_kernel"] = (64 + (P - 1) / P) * u["spans"]
    kernels = {}
    for k, a in alg.items():
        fetch = counter(prof / "pmc_fetch" / "run_counter_collection.csv", "FETCH_SIZE", k)
        write = counter(prof / "pmc_write" / "run_counter_collection.csv", "WRITE_SIZE", k)
        if not fetch:
            continue
        u = per_unit.get(k, 1)  # launches summed per algorithmic unit
        f_b = sum(fetch) / len(fetch) * u * 1024 * 2
        w_b = sum(write) / len(write) * u * 1024 if write else 0.0
        kernels[k] = {"launches": len(fetch), "launches_per_unit": u,
                      "fetch_size_kib": sum(fetch) / len(fetch),
                      "write_size_kib": sum(write) / len(write) if write else None,
                      "read_bytes_per_launch": f_b, "write_bytes_per_launch": w_b,
                      "hbm_bytes_per_launch": f_b + w_b, "algorithmic_bytes_per_launch": a,
                      "traffic_over_algorithmic": (f_b + w_b) / a}
    # SQ counters of the same kernels (two passes), per launch
    for k in list(kernels):
        sq = {}
        for sub in ("pmc_sq", "pmc_sq2"):
            path = prof / sub / "run_counter_collection.csv"
            if not path.exists():
                continue
            with open(path) as f:
                acc: dict = {}
                for r in csv.DictReader(f):
                    if k in r["Kernel_Name"]:
                        acc.setdefault(r["Counter_Name"], []).append(
                            (int(r["Dispatch_Id"]), float(r["Counter_Value"])))
            for name, v in acc.items():
                v = [x for _, x in sorted(v)][:FIRST_N.get(k, len(v))]
                sq[name] = sum(v) / len(v)
        if sq:
            if sq.get("SQ_WAVE_CYCLES"):
                sq["wait_any_frac"] = sq.get("SQ_WAIT_ANY", 0.0) / sq["SQ_WAVE_CYCLES"]
            if sq.get("SQ_ACTIVE_INST_LDS"):
                sq["lds_bank_conflict_frac"] = (sq.get("SQ_LDS_BANK_CONFLICT", 0.0)
                                                / sq["SQ_ACTIVE_INST_LDS"])
            kernels[k]["sq"] = sq
    corr = ("FETCH_SIZE (KiB) x 1024 x 2 (gfx950: FETCH_SIZE counts half of a wide coalesced "
            "read, MI355X_MICROARCH.md HBM); WRITE_SIZE x 1024")
    # The headline kernel's own dispatches in the kernel trace (the first
    # warmup + steps launches of the SN-width edge kernel; later launches of
    # the same kernel belong to other legs), against the bench's hipEvent time
    trace = prof / "trace" / "run_kernel_trace.csv"
    if bench and trace.exists():
        rows = []
        with open(trace) as f:
            for r in csv.DictReader(f):
                if "edge_agg_kernel<1, 1" in r["Kernel_Name"]:  # <1, 1> or <1, 1, UNI>
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        rows.sort()
        k = bench["warmup"] + bench["steps"]
        head = [(e - b) * 1e-6 for b, e in rows[:k]]
        timed = head[bench["warmup"]:]
        if timed:
            hk = {"round": tag, "kernel": "edge_agg_kernel<1, 1> (SN width: lds_hist, lds_stats)",
                  "dispatches": len(timed), "rocprof_avg_ms": sum(timed) / len(timed),
                  "rocprof_min_ms": min(timed), "rocprof_max_ms": max(timed),
                  "bench_hipevent_kernel_ms": bench["roofline"]["kernel_ms"],
                  "bench_ms_per_step": bench["ms_per_step"],
                  "bytes_per_launch": bench["roofline"]["bytes_per_launch"],
                  "line_frac": bench["roofline"]["frac"],
                  "note": "bench line and dispatch times from the same profiled process"
                          if "bench_profiled" in blog.name else
                          "the profiled run repeats the bench command on the same box right "
                          "after the unprofiled bench run"}
            hk["frac_from_rocprof_avg"] = hk["bytes_per_launch"] / (hk["rocprof_avg_ms"] * 1e-3) / 8e12
            hk["frac_rel_diff"] = hk["frac_from_rocprof_avg"] / hk["line_frac"] - 1.0
            hk["avg_le_ms_per_step"] = hk["rocprof_avg_ms"] <= hk["bench_ms_per_step"]
            (out / f"{tag}_headline_kernel.json").write_text(json.dumps(hk, indent=1) + "\n")
            print(json.dumps(hk, indent=1))
    if kernels:
        (out / f"{tag}_pmc.json").write_text(json.dumps(
            {"round": tag, "correction": corr, "kernels": kernels}, indent=1) + "\n")
        print(json.dumps(kernels, indent=1))
    if "edge_agg_kernel" in kernels:
        d = dict(kernel="edge_agg_kernel", round=tag, n_spans=bench["config"]["spans_per_gpu"],
                 correction=corr, **kernels["edge_agg_kernel"])
        (out / "edge_agg_pmc.json").write_text(json.dumps(d, indent=1) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
