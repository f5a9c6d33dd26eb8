#!/usr/bin/env python3
"""Phase cycle sums of the line scatter from a DSORT_STAMPS build (DSORT_LIB=...): per workgroup
(wave 0's view), averaged over workgroups; dev tool.   bkstamps.py [i32|i64z|mixed|few]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd"))
import torch  # noqa: E402
import dsort  # noqa: E402

n = 1 << 30
ctx = dsort.Context(0)
if len(sys.argv) > 1 and sys.argv[1] == "i64z":
    t = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx.gen_zipf_i64(t, 0x5EED2026)
else:
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.gen_uniform(t, 0x5EED2026)
    if len(sys.argv) > 1 and sys.argv[1] == "mixed":  # half [1, 100], half uniform (the refined slot)
        t.copy_(torch.where((t & 1) == 1, ((t >> 1) & 0x7FFFFFFF) % 100 + 1, t))
    elif len(sys.argv) > 1 and sys.argv[1] == "few":  # 16 distinct keys over the range
        t.copy_((t & 15) * (1 << 27) - (1 << 30))
o = torch.empty_like(t)
ctx.sort_dev(t, o)
ctx.sort_dev(t, o)
torch.cuda.synchronize()
buf = np.zeros(8192 * 16, dtype=np.uint64)
fn = ctx.lib.dsort_debug_bkstamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert fn(buf.ctypes.data, buf.nbytes) == 0
S = buf.reshape(-1, 16).astype(np.float64)
S = S[S[:, :8].sum(axis=1) > 0]
names = ["barrier A wait", "scan | B", "owner starts, line map | C", "keys to LDS | D",
         "lines (HBM writes) | E (+ the last sub-tile's tail)", "carry", "keys in (load wait) + slots",
         "classify + rank"]
tot = S[:, :8].sum(axis=1)
print(f"workgroups {len(S)}  cycles per workgroup: mean {tot.mean():.0f}")
for k, nm in enumerate(names):
    print(f"  {nm:48s} {S[:, k].mean():12.0f}  {100 * S[:, k].mean() / tot.mean():5.1f} %")
