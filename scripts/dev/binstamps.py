#!/usr/bin/env python3
"""Phase timeline of the bin sort (bin_sort_kernel<T, true>) from a DSORT_STAMPS build
(DSORT_LIB=build_variants/stamps/libdsort.so): per tile, s_memtime deltas between the phase stamps
of wave 0 and wave 15 (median / p90).  Stamp slots: 0 start, 1 gathered, 2 range, 3 counted,
4 starts, 5 placed, 6 window pass 1, 7 pass 2 (+3 if any), 8 before out, 9 done."""
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
if len(sys.argv) > 1 and sys.argv[1] == "i64z":  # (binstamps.py i64z: 2^30 Zipf int64, config C4)
    t = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx.gen_zipf_i64(t, 0x5EED2026)
else:
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.gen_uniform(t, 0x5EED2026)
o = torch.empty_like(t)
ctx.sort_dev(t, o)
ctx.sort_dev(t, o)
torch.cuda.synchronize()
st = ctx.stats()
buf = np.zeros((1 << 17) * 32, dtype=np.uint64)
fn = ctx.lib.dsort_debug_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert fn(buf.ctypes.data, buf.nbytes) == 0
S = buf.reshape(-1, 32).astype(np.int64)
S = S[(S[:, 0] > 0) & (S[:, 9] > S[:, 0])]
names = ["gather", "range", "count", "starts", "place", "win1", "win2", "win3?", "out"]
print(f"tile sort kernel {st['tile_sort_kernel_ms']:.3f} ms, {S.shape[0]} tiles stamped")
for wv, off in (("wave0", 0), ("wave15", 16)):
    d = np.diff(S[:, off:off + 10], axis=1)
    tot = S[:, off + 9] - S[:, off]
    print(f"{wv}: tile total median {np.median(tot):.0f} cyc p90 {np.percentile(tot, 90):.0f}")
    for k, nm in enumerate(names):
        print(f"   {nm:8s} median {np.median(d[:, k]):8.0f}  p90 {np.percentile(d[:, k], 90):8.0f}  "
              f"mean share {d[:, k].mean() / tot.mean():.3f}")
