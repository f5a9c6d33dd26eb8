#!/usr/bin/env python3
"""One sort step of a rocprofv3 kernel trace: every kernel with the idle gap before it (dev tool).
   timeline.py run_kernel_trace.csv [marker-substring]  (default marker: bin_sort)"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
mark = sys.argv[2] if len(sys.argv) > 2 else "bin_sort"
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
a, b = idx[-2] + 1, idx[-1]
prev = int(rows[a - 1]["End_Timestamp"])
t0, gaps = prev, 0
for r in rows[a:b + 2]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gaps += s - prev
    print(f"gap {(s - prev) / 1e3:8.1f}us  dur {(e - s) / 1e3:8.1f}us  at {(s - t0) / 1e3:8.1f}  {r['Kernel_Name'][:64]}")
    prev = e
print(f"step {(prev - t0) / 1e3:.1f} us, idle gaps {gaps / 1e3:.1f} us")
