#!/usr/bin/env python3
"""Turn a scripts/profile_r06.sh run into the committed profile summaries:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats of the bench process
  profiles/<tag>_bench.json         the bench line that same process printed
  profiles/<tag>_headline_kernel.json  the headline kernel's dispatch times from the
                                    trace against the line's hipEvent time and frac
  profiles/<tag>_pmc.json           per kernel: HBM bytes per launch (FETCH_SIZE x 2 per
                                    the gfx950 correction of MI355X_MICROARCH.md "HBM", +
                                    WRITE_SIZE; both KiB) against its algorithmic bytes,
                                    plus the SQ / LDS counters per launch
  profiles/edge_agg_pmc.json        the headline kernel's HBM bytes (read by bench.py)

Every kernel's traffic ratio names its calibration (VERDICT r04 "Next" 1a):
the FETCH_SIZE it should report for its algorithmic reads, priced per access
pattern with the factors measured by scripts/calib/fetch_calib.hip
(profiles/r05_fetch_calibration.json: FETCH_SIZE = 0.5 x the bytes of a
coalesced stream, 8 or 16 B per lane; 1.89 x the bytes of 32-B gathers inside
a 72-MiB window; ...), against the FETCH_SIZE it does report.

usage: python scripts/summarize_r06.py TAG PROFILE_DIR COMMIT
"""
from __future__ import annotations

import csv
import json
import math
import re
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CORR = ("hbm_bytes = FETCH_SIZE (KiB) x 1024 x 2 + WRITE_SIZE x 1024 (memory-side line traffic: "
        "FETCH_SIZE tallies 64 B per 128-B line request, profiles/r05_fetch_calibration.json); "
        "calibrated_ratio = FETCH_SIZE / (sum over the kernel's read patterns of bytes x the "
        "pattern's measured FETCH_SIZE per byte)")
CALIB = json.loads((ROOT / "profiles" / "r05_fetch_calibration.json").read_text())["patterns"]


def expected_fetch(parts) -> float:
    """FETCH_SIZE bytes a kernel should report for its reads: parts = [(bytes,
    pattern)] priced with the calibration kernel's FETCH_SIZE per true byte."""
    return sum(b * CALIB[p]["fetch_over_true"] for b, p in parts)


def bench_line(path: Path) -> dict | None:
    line = None
    for ln in path.read_text().splitlines():
        if ln.startswith("{"):
            line = json.loads(ln)
    return line


def pmc(paths: list[Path]) -> dict:
    """(kernel name, counter) -> values in dispatch order."""
    acc: dict = {}
    for p in paths:
        if not p.exists():
            continue
        with open(p) as f:
            for r in csv.DictReader(f):
                acc.setdefault((r["Kernel_Name"], r["Counter_Name"]), []).append(
                    (int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return {k: [v for _, v in sorted(vals)] for k, vals in acc.items()}


def select(data: dict, match: str, counter: str, sl: slice) -> list[float]:
    """Values of `counter` for kernels whose name contains `match` (or, with a
    "re:" prefix, matches that regular expression), in dispatch order."""
    vals = []
    for (k, c), v in data.items():
        hit = re.search(match[3:], k) if match.startswith("re:") else match in k
        if c == counter and hit:
            vals.extend(v)
    return vals[sl]


def main() -> int:
    tag = sys.argv[1]
    prof = Path(sys.argv[2]) if len(sys.argv) > 2 else ROOT / "gpurun_out" / "r06prof"
    commit = sys.argv[3] if len(sys.argv) > 3 else None
    out = ROOT / "profiles"
    out.mkdir(exist_ok=True)
    if (prof / "kernel_stats.csv").exists():
        shutil.copy(prof / "kernel_stats.csv", out / f"{tag}_kernel_stats.csv")
    bench = bench_line(prof / "bench_profiled.log") if (prof / "bench_profiled.log").exists() else None
    if bench:
        (out / f"{tag}_bench.json").write_text(json.dumps(bench, indent=1) + "\n")
    pm_bench = bench_line(prof / "p1.log") if (prof / "p1.log").exists() else None
    ref = bench or pm_bench
    data = pmc([prof / f"p{i}.csv" for i in (1, 2, 3, 4)])
    # (label, kernel-name substring, algorithmic bytes per launch, dispatches
    # to average: the PMC bench runs --warmup 1 --steps 2; a leg's first call
    # may run the form-unknown instantiation, which has its own name)
    targets = []
    # (label, kernel-name match, algorithmic bytes per launch, dispatches,
    #  read parts [(bytes, calibration pattern)])
    if ref:
        n = ref["config"]["spans_per_gpu"]
        nt = ref["config"]["traces_per_gpu"]
        targets.append(("headline edge_agg <pair, direct stats, unique-id scan>",
                        "edge_agg_kernel<1, 1, true, 0>", ref["roofline"]["bytes_per_launch"],
                        slice(0, 2), [(24 * n + 8 * (nt + 1), "stream8")]))
        if "trace_structure" in ref:
            ts = ref["trace_structure"]
            targets.append(("trace structure", "trace_struct_kernel<true>", ts["bytes_per_launch"],
                            slice(None), [(26 * n, "stream8")]))
        if "tt_width" in ref:
            tw = ref["tt_width"]
            # (the first call's form probe, a compact-form launch of 16
            # workgroups over the first 2^19 spans, has the other form's name)
            targets.append(("TrainTicket width edge_agg <pair histogram, wide stats>",
                            "edge_agg_kernel<1, 3, true, 0>", tw["bytes_per_launch"],
                            slice(0, 3), [(tw["bytes_per_launch"], "stream8")]))
        if "long_traces" in ref:
            targets.append(("LONG chunk walk edge_agg <compact, direct stats, wide scan | id hash>",
                            r"re:edge_agg_kernel<2, 1, true, [034]>", None, slice(1, 4), None))
            targets.append(("LONG long-trace resolve", "edge_big_resolve_kernel", None, slice(1, 4),
                            None))
            targets.append(("LONG long-trace record", "edge_big_record_kernel<2, 1>", None,
                            slice(1, 4), None))
        if "pagerank" in ref:
            p = ref["pagerank"]
            nn, ne = p["nodes"], p["edges"]
            it = p["iters_per_solve"]
            targets.append(("PageRank persistent solve (100 iterations)", "ppr_persistent_kernel",
                            p["bytes_per_iter"] * it, slice(1, None),
                            [((4 * (nn + 1) + 8 * ne) * it, "stream8"),
                             (8 * ne * it, "gather8_far")]))
            for key in ("batched", "batched_k16"):
                if key in p:
                    kb = p[key]["vectors"]
                    targets.append((f"PageRank persistent batch ({kb} vectors, 100 iterations)",
                                    f"ppr_batch_persistent_kernel<{kb},",
                                    (4 * (nn + 1) + 8 * ne + 16 * nn * kb) * it, slice(1, None),
                                    [((4 * (nn + 1) + 8 * ne) * it, "stream8"),
                                     (8 * kb * ne * it, "gather16_win")]))
        if "ewma" in ref:
            e = ref["ewma"]
            samples = e["steps_per_chunk"] * e["S"]
            l = e["W"] * 64 // math.gcd(e["W"], 64)
            seg = max(l, 16384 // l * l)
            segs = -(-e["steps_per_chunk"] // seg)
            alg = (4 * samples + 4 * samples // e["W"] + 40 * e["S"]) / segs
            targets.append(("EWMA/z time segment (config-4 chunk / segments)", "ewma_zt_kernel",
                            alg, slice(None), [(4 * samples / segs, "stream16")]))
        if "ungrouped" in ref:
            nu = ref["ungrouped"]["spans"]
            targets += [
                ("grouping: level-A counts", "bk_count_a_kernel", 8 * nu, slice(None),
                 [(8 * nu, "stream8")]),
                ("grouping: level-A record scatter", "bk_scatter_a_kernel", 72 * nu, slice(None),
                 [(32 * nu, "stream8")]),
                ("grouping: level-B counts", "bk_count_b_kernel", 8 * nu, slice(None),
                 [(8 * nu, "stream8")]),
                ("grouping: level-B pair scatter (LDS-atomic ranks)", "bk_scatter_b_fast_kernel",
                 16 * nu, slice(None), [(8 * nu, "stream8")]),
                ("ungrouped: join buckets -> edge records (pairs, gathers, records)",
                 "bk_join_kernel", 48 * nu, slice(None),
                 [(8 * nu, "stream8"), (32 * nu, "gather32_win")]),
                ("fused ungrouped: edge records -> table", "edge_rec_kernel", 8 * nu, slice(None),
                 [(8 * nu, "stream8")])]
    kernels = {}
    for label, match, alg, sl, parts in targets:
        fetch = select(data, match, "FETCH_SIZE", sl)
        write = select(data, match, "WRITE_SIZE", sl)
        if not fetch:
            continue
        f_b = sum(fetch) / len(fetch) * 1024 * 2
        w_b = sum(write) / len(write) * 1024 if write else 0.0
        k = {"kernel": match, "launches": len(fetch), "read_bytes_per_launch": f_b,
             "write_bytes_per_launch": w_b, "hbm_bytes_per_launch": f_b + w_b,
             "algorithmic_bytes_per_launch": alg,
             "traffic_over_algorithmic": (f_b + w_b) / alg if alg else None}
        if parts:
            exp = expected_fetch(parts)
            k["calibration"] = {"read_parts": [{"bytes": b, "pattern": pt,
                                                "fetch_per_byte": CALIB[pt]["fetch_over_true"]}
                                               for b, pt in parts],
                                "expected_fetch_size_bytes": exp,
                                "measured_fetch_size_bytes": f_b / 2,
                                "calibrated_ratio": (f_b / 2) / exp if exp else None}
        sq = {}
        for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
                  "SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_BUSY_CYCLES",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_INSTS_VMEM_RD",
                  "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INST_CYCLES_VMEM_RD",
                  "GRBM_GUI_ACTIVE"):
            v = select(data, match, c, sl)
            if v:
                sq[c] = sum(v) / len(v)
        if sq.get("SQ_WAVE_CYCLES"):
            sq["wait_any_frac"] = sq.get("SQ_WAIT_ANY", 0.0) / sq["SQ_WAVE_CYCLES"]
        if sq.get("SQ_ACTIVE_INST_LDS"):
            sq["lds_bank_conflict_frac"] = sq.get("SQ_LDS_BANK_CONFLICT", 0.0) / sq["SQ_ACTIVE_INST_LDS"]
        if sq:
            k["sq"] = sq
        kernels[label] = k
    # the LONG leg's three kernels together against the leg's algorithmic bytes
    # (24 B/span + 8 B/trace, every span read once: the long-trace pass's
    # second reads of listed spans are the pass's overhead)
    parts = [v for k, v in kernels.items() if k.startswith("LONG ")]
    if ref and "long_traces" in ref and len(parts) == 3:
        tot = sum(v["hbm_bytes_per_launch"] for v in parts)
        alg = ref["long_traces"]["bytes_per_launch"]
        kernels["LONG leg (chunk walk + resolve + record)"] = {
            "kernels": [v["kernel"] for v in parts], "hbm_bytes_per_launch": tot,
            "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": tot / alg}
    if kernels:
        (out / f"{tag}_pmc.json").write_text(json.dumps(
            {"round": tag, "commit": commit, "correction": CORR, "pmc_bench": "bench.py --steps 2 --warmup 1 "
             "--no-cpu-baseline --legs trace_structure,ungrouped,tt_width,long_traces,pagerank,"
             "ewma --ewma-chunks 1 (one process per counter pass)", "kernels": kernels},
            indent=1) + "\n")
        print(json.dumps(kernels, indent=1))
        hl = next((v for k, v in kernels.items() if k.startswith("headline")), None)
        if hl and ref:
            d = dict(hl, round=tag, commit=commit, n_spans=ref["config"]["spans_per_gpu"],
                     correction=CORR)
            (out / "edge_agg_pmc.json").write_text(json.dumps(d, indent=1) + "\n")
    # the headline kernel's own dispatches in the bench process's trace: the
    # first warmup call runs the form-unknown instantiation <1, 1, true, 1>;
    # then warmup - 1 + steps dispatches of <1, 1, true, 0> (later legs do not
    # run that instantiation)
    trace = prof / "kernel_trace.csv"
    if bench and trace.exists():
        rows = []
        per_kernel: dict = {}
        with open(trace) as f:
            for r in csv.DictReader(f):
                ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
                per_kernel.setdefault(r["Kernel_Name"].split("(")[0], []).append(ms)
                if "edge_agg_kernel<1, 1, true, 0>" in r["Kernel_Name"]:
                    rows.append((int(r["Start_Timestamp"]), ms))
        rows.sort()
        k = bench["warmup"] - 1 + bench["steps"]
        timed = [ms for _, ms in rows[:k]][bench["warmup"] - 1:]
        if timed:
            hk = {"round": tag, "kernel": "edge_agg_kernel<1, 1, true, 0> (SN width: pair "
                  "histogram, direct stats, unique-id scan)",
                  "dispatches": len(timed), "rocprof_avg_ms": sum(timed) / len(timed),
                  "rocprof_min_ms": min(timed), "rocprof_max_ms": max(timed),
                  "bench_hipevent_kernel_ms": bench["roofline"]["kernel_ms"],
                  "bench_ms_per_step": bench["ms_per_step"],
                  "bytes_per_launch": bench["roofline"]["bytes_per_launch"],
                  "line_frac": bench["roofline"]["frac"],
                  "note": "bench line and dispatch times from the same profiled process"}
            hk["frac_from_rocprof_avg"] = hk["bytes_per_launch"] / (hk["rocprof_avg_ms"] * 1e-3) / 8e12
            hk["frac_rel_diff"] = hk["frac_from_rocprof_avg"] / hk["line_frac"] - 1.0
            hk["avg_le_ms_per_step"] = hk["rocprof_avg_ms"] <= hk["bench_ms_per_step"]
            (out / f"{tag}_headline_kernel.json").write_text(json.dumps(hk, indent=1) + "\n")
            print(json.dumps(hk, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
