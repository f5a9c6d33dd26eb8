#!/usr/bin/env python3
"""Per-kernel counters (per launch) of g_pmc_ab.sh, side by side per variant (dev tool)."""
import collections, glob, re, sqlite3, sys
vals = collections.defaultdict(lambda: collections.defaultdict(dict))
for db in sorted(glob.glob("gpurun_out/pmc_*_[0-9]/**/*.db", recursive=True)):
    v = re.match(r"gpurun_out/pmc_(.+)_\d/", db).group(1)
    c = sqlite3.connect(db)
    q = ("select kernel_name, counter_name, sum(value), count(distinct dispatch_id) from counters_collection "
         "group by kernel_name, counter_name")
    for k, cn, val, nd in c.execute(q):
        vals[k.split("(")[0][-48:]][cn][v] = val / max(nd, 1)
want = sys.argv[1:]
for k, d in vals.items():
    if want and not any(w in k for w in want):
        continue
    vs = sorted({v for cn in d for v in d[cn]})
    print(f"== {k}   " + "  ".join(f"{v:>14s}" for v in vs))
    for cn in sorted(d):
        print(f"   {cn:24s} " + "  ".join(f"{d[cn].get(v, float('nan')):14.5g}" for v in vs))
