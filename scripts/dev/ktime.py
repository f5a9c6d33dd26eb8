#!/usr/bin/env python3
"""Kernel timing without verification (for ablation variants via DSORT_LIB): sorts N uniform
int32 keys `reps` times and prints the per-stage device times of the fastest call."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd"))
import torch  # noqa: E402
import dsort  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--keys", type=lambda s: int(eval(s, {}, {})), default=1 << 30)
ap.add_argument("--reps", type=int, default=4)
ap.add_argument("--dtype", choices=["i32", "i64"], default="i32")
ap.add_argument("--dist", choices=["uniform", "zipf", "sorted", "reverse", "equal", "few", "byte", "ref100", "mixed"],
                default="uniform")
ap.add_argument("--opt", action="append", default=[], help="dsort option name=value (repeatable)")
a = ap.parse_args()
tag = os.environ.get("DSORT_LIB")
tag = os.path.basename(os.path.dirname(tag)) if tag else "default"
tag = f"{tag} {a.dtype} {a.dist}"
ctx = dsort.Context(0)
for kv in a.opt:
    k, v = kv.split("=")
    ctx.set_option(k, int(eval(v, {}, {})))
    tag += f" {k}={v}"
t = torch.empty(a.keys, dtype=torch.int32 if a.dtype == "i32" else torch.int64, device="cuda")
if a.dist == "zipf":
    ctx.gen_zipf_i64(t, 0x5EED2026)
else:
    ctx.gen_uniform(t, 0x5EED2026)
    if a.dist == "sorted":
        t.copy_(torch.sort(t)[0])
    elif a.dist == "reverse":
        t.copy_(torch.sort(t, descending=True)[0])
    elif a.dist == "equal":
        t.fill_(12345)
    elif a.dist == "few":  # 16 distinct keys spread over the whole range
        t.copy_((t & 15) * (1 << 27) - (1 << 30))
    elif a.dist == "byte":  # 256 distinct small keys
        t.copy_(t & 255)
    elif a.dist == "ref100":  # the reference's input.txt shape: keys in [1, 100]
        t.copy_((t & 0x7FFFFFFF) % 100 + 1)
    elif a.dist == "mixed":  # half the keys in [1, 100] (input.txt's shape), half uniform, interleaved at random
        t.copy_(torch.where((t & 1) == 1, ((t >> 1) & 0x7FFFFFFF) % 100 + 1, t))
o = torch.empty_like(t)
best = None
for _ in range(a.reps):
    ctx.sort_dev(t, o)
    st = ctx.stats()
    if best is None or st["total_ms"] < best["total_ms"]:
        best = st
torch.cuda.synchronize()
n = max(best["merge_kernel_launches"], 1)
print(f"{tag:>24s}: total {best['total_ms']:.3f} ms  hist {best['bucket_hist_ms']:.3f}  "
      f"scatter {best['bucket_scatter_ms']:.3f}  sub {best['sub_partition_ms']:.3f}  "
      f"tile {best['tile_sort_kernel_ms']:.3f}  partition {best['partition_ms']:.3f}  "
      f"merge-kernel avg {best['merge_kernel_ms'] / n:.3f} ms x{best['merge_kernel_launches']}  "
      f"passes {best['merge_passes']}", flush=True)
