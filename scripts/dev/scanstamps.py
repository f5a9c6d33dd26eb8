#!/usr/bin/env python3
"""Phase cycles of sb_scan_kernel<true> (the last launch) from a DSORT_STAMPS + DSORT_SCAN_STAMPS
build (DSORT_LIB=...), thread 0's view, averaged over workgroups (buckets): scanstamps.py i32|i64;
dev tool."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd"))
import torch  # noqa: E402
import dsort  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else "i32"
n = 1 << 30
ctx = dsort.Context(0)
t = torch.empty(n, dtype=torch.int32 if dt == "i32" else torch.int64, device="cuda")
if dt == "i64":
    ctx.gen_zipf_i64(t, 0x5EED2026)
else:
    ctx.gen_uniform(t, 0x5EED2026)
o = torch.empty_like(t)
ctx.sort_dev(t, o)
ctx.sort_dev(t, o)
torch.cuda.synchronize()
buf = np.zeros((1 << 18) * 8, dtype=np.uint64)
fn = ctx.lib.dsort_debug_sbstamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert fn(buf.ctypes.data, buf.nbytes) == 0
S = buf.reshape(-1, 8)[:1024].astype(np.float64)
S = S[S[:, :7].sum(axis=1) > 0]
names = ["sums + scan", "starts", "tile ends (search)", "chain (thread 0)", "tiles + scan", "tile records",
         "piece tables"]
tot = S[:, :7].sum(axis=1)
print(f"{dt}: workgroups {len(S)}  cycles per workgroup: mean {tot.mean():.0f}")
for k, nm in enumerate(names):
    print(f"  {nm:20s} {S[:, k].mean():10.0f}  {100 * S[:, k].mean() / tot.mean():5.1f} %")
