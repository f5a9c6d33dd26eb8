#!/usr/bin/env python3
"""Phase cycles of parse_kernel (the last launch) from a DSORT_STAMPS build (DSORT_LIB=...), thread 0's
view, over tiles: txstamps.py [keys]; dev tool."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd"))
import torch  # noqa: E402
import dsort  # noqa: E402

n = int(eval(sys.argv[1])) if len(sys.argv) > 1 else 1 << 26
ctx = dsort.Context(0)
keys = torch.empty(n, dtype=torch.int32, device="cuda")
ctx.gen_uniform(keys, 7)
ctx.sort_dev(keys)
text = torch.empty(12 * n, dtype=torch.uint8, device="cuda")
back = torch.empty(n, dtype=torch.int32, device="cuda")
ln = ctx.format_text(keys, text)
ctx.parse_text(text, ln, back)
ctx.parse_text(text, ln, back)
torch.cuda.synchronize()
buf = np.zeros((1 << 18) * 8, dtype=np.uint64)
fn = ctx.lib.dsort_debug_txstamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert fn(buf.ctypes.data, buf.nbytes) == 0
S = buf.reshape(-1, 8)[:, :4].astype(np.float64)
S = S[S.sum(axis=1) > 0]
names = ["tile offset load", "staging", "starts + scan", "tokens + stores"]
tot = S.sum(axis=1)
print(f"parse tiles {len(S)}  cycles per tile: mean {tot.mean():.0f} median {np.median(tot):.0f}")
for k, nm in enumerate(names):
    print(f"  {nm:20s} mean {S[:, k].mean():10.0f} median {np.median(S[:, k]):10.0f}  {100 * S[:, k].mean() / tot.mean():5.1f} %")
