#!/usr/bin/env python3
"""Where features() -> rank() spends a config-2 experiment (host profile,
cProfile, 10 experiments after warm-up); prints the top functions by
cumulative time.

  python scripts/r06/profile_features.py"""
import cProfile
import pstats
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]

import anomod  # noqa: E402
import bench  # noqa: E402

with anomod.Context(0) as ctx:
    exps = [anomod.load_experiment(anomod.SynthSpec("TT", seed=20251103 + i, fault_service=f),
                                   n_traces=650, series_per_service=130, name=f"tt_{f or 'normal'}")
            for i, f in enumerate(bench.TT_FAULTS)]
    base = anomod.features(exps[0], ctx)
    for e in exps[1:3]:
        anomod.rank(anomod.features(e, ctx, baseline=base), ctx=ctx)
    pr = cProfile.Profile()
    pr.enable()
    for e in exps[1:11]:
        anomod.rank(anomod.features(e, ctx, baseline=base), ctx=ctx)
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(28)
