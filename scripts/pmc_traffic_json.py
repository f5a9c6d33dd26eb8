#!/usr/bin/env python3
"""profiles/r1_pmc_traffic.json from two rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE runs of
scripts/pmc.sh over scripts/kdriver.py at 2^30 uniform int32):
   pmc_traffic_json.py <fetch counter_collection.csv> <write counter_collection.csv> [note] [passes]
Per-launch bytes: FETCH_SIZE (KB) x 2 (MI355X_MICROARCH.md HBM section: wide streaming reads
report half their bytes) + WRITE_SIZE (KB)."""
import collections
import csv
import json
import sys

NAMES = {"block_sort_w_kernel": "block_sort_w_kernel", "mergew_kernel": "mergew_kernel",
         "partk_kernel": "partk_kernel", "bucket_hist_kernel": "bucket_hist_kernel",
         "bucket_scatter": "bucket_scatter"}


def per_kernel(path, counter):
    tot, disp = collections.defaultdict(float), collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        for key in NAMES:
            if key in r["Kernel_Name"]:
                tot[key] += float(r["Counter_Value"])
                disp[key].add(r["Dispatch_Id"])
    return {k: (tot[k] / len(disp[k]) * 1024, len(disp[k]), tot[k] * 1024) for k in tot}


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
out = {
    "source": "rocprofv3 --pmc, separate FETCH_SIZE / WRITE_SIZE passes (scripts/pmc.sh), 2^30 "
              "uniform int32, scripts/kdriver.py; converted by scripts/pmc_traffic_json.py",
    "units": "bytes per launch",
    "calibration": "FETCH_SIZE x2 (MI355X_MICROARCH.md HBM section: half of wide streaming reads; "
                   "block_sort_w_kernel reads exactly 4 B/key with 16-B loads and reports half of "
                   "4.29 GB, confirming the factor); WRITE_SIZE as reported. "
                   + (sys.argv[3] if len(sys.argv) > 3 else ""),
    "kernels": {},
}
# a merge pass may be several launches (one per kernel fan-in): per-pass bytes = all merge
# launches / (sorts x passes), sorts = tile-sort launches
passes = int(sys.argv[4]) if len(sys.argv) > 4 else 0
sorts = fetch.get("block_sort_w_kernel", (0, 0, 0))[1]
for k in NAMES:
    if k in fetch and k in write:
        f, n, ft = fetch[k]
        wb, _, wt = write[k]
        out["kernels"][k] = {"launches": n, "fetch_bytes": 2 * f, "write_bytes": wb,
                             "traffic_bytes": 2 * f + wb}
        if k == "mergew_kernel" and passes and sorts:
            out["kernels"][k]["traffic_bytes_per_pass"] = (2 * ft + wt) / (sorts * passes)
json.dump(out, sys.stdout, indent=1)
print()
