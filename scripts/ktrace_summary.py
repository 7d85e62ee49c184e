#!/usr/bin/env python3
"""Per-dispatch durations from a rocprofv3 kernel_trace.csv, in dispatch
order: name, grid, ms.  python scripts/ktrace_summary.py trace.csv [filter]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    m = re.search(r"::(\w+_kernel(?:<[^>]*>)?)\(", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"][:40]
    if flt and flt not in name:
        continue
    ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(f"{name[:44]:44s} grid {int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):>9} "
          f"x{r['Grid_Size_Y']:>3} {ms:9.3f} ms")
