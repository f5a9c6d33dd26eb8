#!/usr/bin/env python3
"""Phase timeline of the last mergew launch from a DSORT_STAMPS build (DSORT_LIB=...):
per tile, s_memtime deltas between phase stamps for wave 0 and wave 15 (median / p90)."""
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
t = torch.empty(n, dtype=torch.int32, device="cuda")
ctx.gen_uniform(t, 0x5EED2026)
o = torch.empty_like(t)
ctx.sort_dev(t, o)
ctx.sort_dev(t, o)
torch.cuda.synchronize()
st = ctx.stats()
tiles = 70912 if len(sys.argv) < 2 else int(sys.argv[1])
buf = np.zeros((1 << 17) * 32, dtype=np.uint64)
fn = ctx.lib.dsort_debug_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert fn(buf.ctypes.data, buf.nbytes) == 0
S = buf.reshape(-1, 32)[:tiles].astype(np.int64)
names = ["setup", "chunktab", "staging", "stage-bar", "L0 merge", "L0 store", "L1 merge", "L1 store",
         "L2 merge", "L2 store", "L3 merge", "L3 store"]
print(f"merge kernel avg {st['merge_kernel_ms'] / max(st['merge_kernel_launches'], 1):.3f} ms")
for wv, off in (("wave0", 0), ("wave15", 16)):
    d = np.diff(S[:, off:off + 13], axis=1)
    tot = S[:, off + 12] - S[:, off]
    print(f"{wv}: tile total median {np.median(tot):.0f} cyc p90 {np.percentile(tot, 90):.0f}")
    for k, nm in enumerate(names):
        print(f"   {nm:10s} median {np.median(d[:, k]):8.0f}  p90 {np.percentile(d[:, k], 90):8.0f}")
