#!/usr/bin/env python3
"""Prints a rocprofv3 kernel_stats.csv as ms per call and per sort (dev tool)."""
import csv
import sys

path, sorts = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = 0.0
for r in csv.DictReader(open(path)):
    per = float(r["TotalDurationNs"]) / 1e6 / sorts
    tot += per
    print(f"{r['Name'][:78]:78s} {r['Calls']:>5} {float(r['AverageNs']) / 1e6:8.3f} ms/call {per:8.3f} ms/sort")
print(f"{'total':78s} {'':5} {'':8}          {tot:8.3f} ms/sort")
