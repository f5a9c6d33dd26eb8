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

# Concurrency of the staging phase among all workgroups, on the s_memrealtime stamps (100 MHz,
# comparable across CUs; slots 13 tile start, 14 staging start, 15 staging end, 29 tile end):
# if workgroups are phase-locked, staging overlaps in bursts.
R = S[:, [13, 14, 15, 29]]
R = R[R[:, 3] > R[:, 3].max() - 200000]  # tiles of the last launch (< 2 ms before its end)
t0 = R[:, 0].min()
grid = np.arange(t0, R[:, 3].max(), 2)
stg = np.zeros(grid.size, np.int32)
live = np.zeros(grid.size, np.int32)
for s0, a, b, e in R:
    stg[np.searchsorted(grid, a):np.searchsorted(grid, b)] += 1
    live[np.searchsorted(grid, s0):np.searchsorted(grid, e)] += 1
mid = slice(grid.size // 10, grid.size * 9 // 10)
print(f"span {(R[:, 3].max() - t0) / 100:.0f} us; live WGs mean {live[mid].mean():.1f}; staging WGs "
      f"mean {stg[mid].mean():.1f} p10 {np.percentile(stg[mid], 10):.0f} p50 "
      f"{np.percentile(stg[mid], 50):.0f} p90 {np.percentile(stg[mid], 90):.0f} max {stg[mid].max()}")
print(f"staging median {np.median(R[:, 2] - R[:, 1]) * 10:.0f} ns, tile median "
      f"{np.median(R[:, 3] - R[:, 0]) * 10:.0f} ns")
tl = np.arange(grid.size // 3, grid.size // 3 + 60 * 50, 50)  # 60 samples, 1 us apart
print("staging WGs every 1 us:", " ".join(str(stg[i]) for i in tl))
print("live WGs every 1 us:   ", " ".join(str(live[i]) for i in tl))
