#!/usr/bin/env python3
"""Per-kernel average of every counter in a rocprofv3 counter_collection.csv."""
import collections, csv, sys
for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void dsort::", "")[:48]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        n = len(disp[k])
        print(f"{k:48s} n={n} " + " ".join(f"{c}={x / n:.3g}" for c, x in sorted(v.items())))
