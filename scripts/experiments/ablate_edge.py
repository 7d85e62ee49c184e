#!/usr/bin/env python3
"""Time the edge-aggregation kernel of the shipped library and of the
experiment-only ablation builds (csrc/build/variants/libanomod_abl*.so:
1 = no stats atomics, 2 = no histogram, 4 = no parent scan, 7 = all three
off) on the same synthetic workload.  Each library runs in its own process."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
PKG = ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"


def one(traces: int, steps: int):
    sys.path.insert(0, str(PKG))
    import numpy as np

    import anomod
    from anomod import _lib as L

    with anomod.Context(0) as ctx:
        topo = os.environ.get("ABL_TOPO", "SN")
        sp = ctx.generate(anomod.SynthSpec(topo, seed=20251103, p_orphan_ppm=100), traces)
        for _ in range(2):
            ctx.edge_aggregate(sp, with_hist=False)
        ms = []
        for _ in range(steps):
            ctx.edge_aggregate(sp, with_hist=False)
            ms.append(ctx.stage_ms(L.STAGE_EDGE_AGG))
        n = sp.n_spans
        print(json.dumps({"lib": os.environ.get("ANOMOD_LIB", "main"), "spans": n,
                          "kernel_ms": float(np.median(ms)), "min_ms": float(np.min(ms)),
                          "gspans_per_s": n / np.median(ms) / 1e6,
                          "GBps": (24 * n + 8 * traces) / np.median(ms) / 1e6}), flush=True)


def main():
    traces = int(os.environ.get("ABL_TRACES", 1 << 26))
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        one(traces, 7)
        return
    libs = [None] + sorted(str(p) for p in (PKG / "csrc/build/variants").glob(os.environ.get("ABL_GLOB", "libanomod_*.so")))
    print("libs:", [Path(l).name if l else "main" for l in libs], flush=True)
    for lib in libs * int(os.environ.get("ABL_ROUNDS", 1)):
        env = dict(os.environ)
        if lib:
            env["ANOMOD_LIB"] = lib
        r = subprocess.run([sys.executable, __file__, "--one"], env=env, timeout=300)
        print(f"rc={r.returncode} lib={Path(lib).name if lib else 'main'}", flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
