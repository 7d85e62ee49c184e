#!/usr/bin/env python3
"""cProfile of bench.py's BASELINE config-2 leg (13 TrainTicket experiments
through features() -> rank()): where the per-experiment host time goes."""
import cProfile
import pstats
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]
import anomod  # noqa: E402
import bench  # noqa: E402

with anomod.Context(0) as ctx:
    bench.tt_config2(ctx)
    pr = cProfile.Profile()
    pr.enable()
    r = bench.tt_config2(ctx)
    pr.disable()
    print(r, flush=True)
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)
