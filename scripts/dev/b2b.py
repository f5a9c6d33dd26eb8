#!/usr/bin/env python3
"""Back-to-back sorts as in bench.py's timed loop (no read-back between them), for a kernel-trace
timeline of one step with its idle gaps (scripts/dev/timeline.py).  b2b.py [--keys N] [--steps K]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd"))
import torch  # noqa: E402
import dsort  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--keys", type=lambda s: int(eval(s, {}, {})), default=1 << 30)
ap.add_argument("--steps", type=int, default=6)
ap.add_argument("--dtype", choices=["i32", "i64"], default="i32")
ap.add_argument("--dist", choices=["uniform", "zipf"], default="uniform")
ap.add_argument("--timing", type=int, default=1, help="DSORT_OPT_STAGE_TIMING (0: no stage events)")
ap.add_argument("--opt", action="append", default=[], help="dsort option name=value (repeatable)")
a = ap.parse_args()
ctx = dsort.Context(0)
for kv in a.opt:
    k, v = kv.split("=")
    ctx.set_option(k, int(v))
if a.timing != 1:
    ctx.set_option("stage_timing", a.timing)
t = torch.empty(a.keys, dtype=torch.int32 if a.dtype == "i32" else torch.int64, device="cuda")
if a.dist == "zipf":
    ctx.gen_zipf_i64(t, 0x5EED2026)
else:
    ctx.gen_uniform(t, 0x5EED2026)
o = torch.empty_like(t)
ctx.sort_dev(t, o)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.steps):
    ctx.sort_dev(t, o)
torch.cuda.synchronize()
print(f"{a.steps} back-to-back sorts: {1e3 * (time.perf_counter() - t0) / a.steps:.3f} ms per step", flush=True)
