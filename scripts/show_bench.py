#!/usr/bin/env python3
"""Compact view of a bench line: python scripts/show_bench.py <log>"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"value {d['value'] / 1e9:.1f} G spans/s  ms/step {d['ms_per_step']:.3f}  "
      f"kernel {d['roofline']['kernel_ms']:.3f} ms  frac {d['roofline']['frac']:.3f}")
for k, v in d.items():
    if isinstance(v, dict) and k not in ("config", "roofline", "cpu_baseline"):
        keep = {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()
                if kk in ("kernel_ms", "frac", "step_ms", "group_ms", "edge_ms", "group_frac",
                          "iters_per_s", "ms_per_experiment", "top3_hit_rate", "samples_per_s")}
        print(f"  {k}: {keep}")
