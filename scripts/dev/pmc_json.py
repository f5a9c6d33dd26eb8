#!/usr/bin/env python3
"""profiles/r<N>_pmc_traffic.json from the rocprofv3 databases of scripts/gpu_profile_r<N>.sh: per
kernel and launch (and per sort: all its launches in one sort), HBM traffic = (2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB (FETCH_SIZE doubled: the
gfx950 correction of MI355X_MICROARCH.md § HBM), for the 2^30 int32 sort; the int64 Zipf sort's
figures under "int64".   pmc_json.py OUT.json [TAG32 TAG64]   (default tags i32_ i64_)"""
import glob
import json
import sqlite3
import sys


def per_launch(tag):
    out, nlaunch = {}, {}
    for db in sorted(glob.glob(f"gpurun_out/{tag}pmc*/**/*.db", recursive=True)):
        c = sqlite3.connect(db)
        q = ("select kernel_name, counter_name, sum(value), count(distinct dispatch_id) from counters_collection "
             "group by kernel_name, counter_name")
        for k, cn, v, nd in c.execute(q):
            name = k.split("(")[0].replace("void ", "").split("::")[-1]
            out.setdefault(name, {})[cn] = v / max(nd, 1)
            if cn == "WRITE_SIZE":
                nlaunch[name] = nd
    # sorts in the profiled run: launches of the first level's slot-map kernel (once per sort)
    sorts = max([nd for k, nd in nlaunch.items() if k.startswith("bucket_slotmap_kernel")] or [1])
    res = {}
    for k, d in out.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            per = int((2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024)
            # (per sort: kernels launched more than once per sort -- the tile sort's two parts since
            # round 5, the nested sorts' tile sorts -- count every launch)
            rec = {"fetch_kib": d["FETCH_SIZE"], "write_kib": d["WRITE_SIZE"],
                   "traffic_bytes_per_launch": per, "launches_per_sort": nlaunch.get(k, 1) / sorts,
                   "traffic_bytes_per_sort": int(per * nlaunch.get(k, 1) / sorts)}
            for extra in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS",
                          "SQ_LDS_IDX_ACTIVE", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY",
                          "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VMEM_WR", "SQ_INSTS_VMEM_RD",
                          "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum", "TCC_EA0_RDREQ_sum"):
                if extra in d:
                    rec[extra] = d[extra]
            res[k] = rec
    return res


t32 = sys.argv[2] if len(sys.argv) > 2 else "i32_"
t64 = sys.argv[3] if len(sys.argv) > 3 else "i64_"
import hashlib  # noqa: E402
import os  # noqa: E402

# the build the counters were taken on (bench.py uses the table as measured only for this build)
LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                   "distributed-sorting-with-fault-tolerance_amd", "lib", "libdsort.so")
# (round 5: the profiling script records the sha256 of the library it ran ON THE BOX in
# gpurun_out/pmc_lib_sha256.txt; the local file is only the fallback)
SHA_BOX = os.path.join("gpurun_out", "pmc_lib_sha256.txt")
sha = open(SHA_BOX).read().split()[0] if os.path.exists(SHA_BOX) else hashlib.sha256(open(LIB, "rb").read()).hexdigest()
doc = {"source": "rocprofv3 --pmc (separate passes, scripts/dev/pmc_sub.sh) over scripts/dev/ktime.py --reps 1, "
                 "2^30 keys; converted by scripts/dev/pmc_json.py",
       "lib_sha256": sha, "lib_sha256_from": "the box" if os.path.exists(SHA_BOX) else "the local build",
       "keys": 1 << 30, "key_bytes": 4, "dist": "uniform", "kernels": per_launch(t32),
       "int64": {"keys": 1 << 30, "key_bytes": 8, "dist": "zipf", "kernels": per_launch(t64)}}
json.dump(doc, open(sys.argv[1] if len(sys.argv) > 1 else "profiles/r2_pmc_traffic.json", "w"), indent=1)
for t, ks in (("int32", doc["kernels"]), ("int64", doc["int64"]["kernels"])):
    for k, r in ks.items():
        print(f"{t} {k:34s} {r['traffic_bytes_per_sort'] / 1e9:8.3f} GB per sort ({r['launches_per_sort']:g} launches)")
