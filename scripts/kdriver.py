#!/usr/bin/env python3
"""Minimal driver for counter collection: sorts N keys (device-resident) a few times."""
import argparse, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd"))
import torch  # noqa: E402
import dsort  # noqa: E402
ap = argparse.ArgumentParser()
ap.add_argument("--keys", type=lambda s: int(eval(s)), default=1 << 28)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--dtype", default="i32")
a = ap.parse_args()
ctx = dsort.Context(0)
t = torch.empty(a.keys, dtype=torch.int32 if a.dtype == "i32" else torch.int64, device="cuda")
ctx.gen_uniform(t, 0x5EED2026)
o = torch.empty_like(t)
for _ in range(a.reps):
    ctx.sort_dev(t, o)
torch.cuda.synchronize()
print("ok", ctx.stats())
