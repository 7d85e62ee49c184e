#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter CSVs: kernel, counter,
mean per dispatch, dispatches.  python scripts/pmc_table.py a.csv [b.csv ...] [--filter X]"""
import csv
import re
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
flt = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--filter=")), "")
acc = defaultdict(list)
for path in args:
    for r in csv.DictReader(open(path)):
        m = re.search(r"::(\w+_kernel(?:<[^>]*>)?)\(", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        if flt and flt not in name:
            continue
        acc[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k[:40]:40s} {c:24s} {sum(v) / len(v):18.1f}  x{len(v)}")
