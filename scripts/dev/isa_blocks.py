#!/usr/bin/env python3
"""Basic-block instruction-class counts of one kernel in a hipcc -S listing:
   isa_blocks.py wave.s <symbol-substring>"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(sys.argv[2]) + r"\S*:", l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))


def cls(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_waitcnt", "s_barrier", "s_cbranch", "s_branch", "s_nop", "s_sleep", "s_memtime")):
        return op.split("_")[1]
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "gmem"
    return op


tot = collections.Counter()
blk, cnt, first = "entry", collections.Counter(), start
for i in range(start + 1, end):
    t = lines[i].strip().split()
    if not t or t[0].startswith((";", ".")) and not t[0].startswith(".LBB"):
        continue
    if t[0].endswith(":"):
        if cnt:
            print(f"{blk:14s} L{first - start:<6d} " + " ".join(f"{k}={v}" for k, v in sorted(cnt.items())))
        blk, cnt, first = t[0][:-1], collections.Counter(), i
        continue
    c = cls(t[0])
    cnt[c] += 1
    tot[c] += 1
    if c in ("cbranch", "branch"):
        cnt["->" + t[-1]] += 1
print(f"{blk:14s} L{first - start:<6d} " + " ".join(f"{k}={v}" for k, v in sorted(cnt.items())))
print("TOTAL", dict(tot))
