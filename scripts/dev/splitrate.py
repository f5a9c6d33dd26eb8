#!/usr/bin/env python3
"""Over-tile sub-bucket rate of the default sort (dev tool): sorts 2^30 uniform int32 keys for
`--seeds` seeds and prints each sort's sub_split_subbuckets, merge passes and device time.
   splitrate.py [--seeds K] [--keys N] [--opt name=value ...]   (DSORT_LIB selects a build)"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd"))
import torch  # noqa: E402
import dsort  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--keys", type=lambda s: int(eval(s, {}, {})), default=1 << 30)
ap.add_argument("--seeds", type=int, default=10)
ap.add_argument("--opt", action="append", default=[])
a = ap.parse_args()
ctx = dsort.Context(0)
for kv in a.opt:
    k, v = kv.split("=")
    ctx.set_option(k, int(eval(v, {}, {})))
t = torch.empty(a.keys, dtype=torch.int32, device="cuda")
o = torch.empty_like(t)
splits = 0
for sd in range(a.seeds):
    ctx.gen_uniform(t, 0x1000 + sd)
    ctx.sort_dev(t, o)
    st = ctx.stats()
    splits += st["sub_split_subbuckets"]
    print(f"seed {sd}: split {st['sub_split_subbuckets']} passes {st['merge_passes']} "
          f"fallback {st['sub_scatter_fallback']} total {st['total_ms']:.3f} ms", flush=True)
print(f"split sub-buckets: {splits} in {a.seeds} sorts")
