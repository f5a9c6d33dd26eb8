#!/usr/bin/env python3
"""A/B helper for compile-time variants (DSORT_LIB=build_variants/<v>/libdsort.so): per-stage device
times of the fastest of `reps` sorts, then a bit-exact check against torch.sort."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd"))
import torch  # noqa: E402
import dsort  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--keys", type=lambda s: int(eval(s, {}, {})), default=1 << 30)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--dtype", choices=["i32", "i64"], default="i32")
ap.add_argument("--dist", choices=["uniform", "zipf"], default="uniform")
a = ap.parse_args()
tag = os.environ.get("DSORT_LIB")
tag = os.path.basename(os.path.dirname(tag)) if tag else "default"
ctx = dsort.Context(0)
t = torch.empty(a.keys, dtype=torch.int32 if a.dtype == "i32" else torch.int64, device="cuda")
if a.dist == "zipf":
    ctx.gen_zipf_i64(t, 0x5EED2026)
else:
    ctx.gen_uniform(t, 0x5EED2026)
o = torch.empty_like(t)
rows = []
for _ in range(a.reps):
    ctx.sort_dev(t, o)
    rows.append(ctx.stats())
best = min(rows, key=lambda r: r["total_ms"])
ok = torch.equal(o, torch.sort(t).values)
print(f"{tag:>10s} {a.dtype} {a.dist} n={a.keys}: total {best['total_ms']:.3f}  hist {best['bucket_hist_ms']:.3f}  "
      f"scatter {best['bucket_scatter_ms']:.3f} (min {min(r['bucket_scatter_ms'] for r in rows):.3f})  "
      f"sub {best['sub_partition_ms']:.3f}  tile {best['tile_sort_kernel_ms']:.3f}  exact={ok}", flush=True)
if not ok:
    sys.exit(1)
