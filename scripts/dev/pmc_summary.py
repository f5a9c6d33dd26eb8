#!/usr/bin/env python3
"""Per-kernel counter values from the rocprofv3 databases of pmc_sub.sh (dev tool).
Prints, per kernel (filtered by the arguments), every counter summed over the dispatches of one
run, divided by the number of dispatches (per launch)."""
import collections
import glob
import sqlite3
import sys

vals = collections.defaultdict(dict)
for db in sorted(glob.glob("gpurun_out/pmc*/**/*.db", recursive=True)):
    c = sqlite3.connect(db)
    q = ("select kernel_name, counter_name, sum(value), count(distinct dispatch_id) from counters_collection "
         "group by kernel_name, counter_name")
    for k, cn, v, nd in c.execute(q):
        vals[k.split("(")[0][-48:]][cn] = v / max(nd, 1)
want = sys.argv[1:] or None
for k, d in vals.items():
    if want and not any(w in k for w in want):
        continue
    print(f"== {k}")
    for cn, v in sorted(d.items()):
        print(f"   {cn:28s} {v:16.5g}")
