#!/usr/bin/env python3
"""Compact view of gpurun_out/grp_*_<tag>.log (scripts/gpu_group_iter.sh)."""
import json
import sys
from pathlib import Path

tag = sys.argv[1]
out = Path(__file__).resolve().parents[1] / "gpurun_out"
t = out / f"grp_tests_{tag}.log"
if t.exists():
    lines = t.read_text().splitlines()
    print("\n".join(l for l in lines if "FAIL" in l or "Error" in l)[-2000:])
    print(lines[-1] if lines else "(empty)")
for name in ("time", "time27", "timeLONG", "timeTT"):
    f = out / f"grp_{name}_{tag}.log"
    if not f.exists():
        continue
    try:
        d = json.loads(f.read_text().strip().splitlines()[-1])
    except Exception:
        print(name, "unparsed:", f.read_text()[-300:])
        continue
    print(name, d["spans"], {k: v for k, v in d.items() if "group_ms" in k or "info" in k})
