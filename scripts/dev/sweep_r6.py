#!/usr/bin/env python3
"""Randomised correctness sweep of round 6's changes against torch.sort on the GPU (dev tool, not a
test): duplicate-heavy inputs of many shapes (one-key slots spread by the index hash, pure buckets
dropped and filled, the refined slot), both key widths, several seeds and sizes; then the bucket
exchange at one RCCL rank with C3's bucket geometry (compacted partition, piece tables before the
tile count, the per-vector-slot gather).  Prints one line per case and a summary; exit status 1 on
any mismatch.   sweep_r6.py [--quick]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd"))
import torch  # noqa: E402

import dsort  # noqa: E402

quick = "--quick" in sys.argv
ctx = dsort.Context(0)
bad = 0
cases = 0


def make(n, dt, dist, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    t = torch.empty(n, dtype=dt, device="cuda")
    if dist.startswith("k"):  # k distinct keys spread over the range
        k = int(dist[1:])
        vals = torch.randint(-(1 << 30), 1 << 30, (k,), device="cuda", generator=g).to(dt)
        t.copy_(vals[torch.randint(0, k, (n,), device="cuda", generator=g)])
    elif dist == "zipf":
        t64 = torch.empty(n, dtype=torch.int64, device="cuda")
        ctx.gen_zipf_i64(t64, seed)
        t.copy_(t64 if dt == torch.int64 else (t64 >> 33).to(torch.int32))
    elif dist == "mixed":  # half [1, 100], half uniform
        ctx.gen_uniform(t, seed)
        small = torch.randint(1, 101, (n,), device="cuda", generator=g).to(dt)
        t.copy_(torch.where((t & 1) == 1, t, small))
    elif dist == "heavy":  # one key at 40 %, the rest uniform
        ctx.gen_uniform(t, seed)
        t.copy_(torch.where(torch.rand(n, device="cuda", generator=g) < 0.4, torch.full_like(t, 12345), t))
    elif dist == "sortedfew":  # sorted input of 64 keys
        vals = torch.randint(-1000, 1000, (n,), device="cuda", generator=g).to(dt) // 31
        t.copy_(torch.sort(vals)[0])
    else:
        ctx.gen_uniform(t, seed)
    return t


def check(name, t, out):
    global bad, cases
    cases += 1
    ok = torch.equal(out, torch.sort(t)[0])
    if not ok:
        bad += 1
    print(f"{'ok ' if ok else 'BAD'} {name}", flush=True)


dists = ["k2", "k3", "k17", "k100", "k1000", "zipf", "mixed", "heavy", "sortedfew", "uniform"]
sizes = [(1 << 25) + 4097, (1 << 26) + 3] if quick else [(1 << 25) + 4097, (1 << 26) + 3, (1 << 28) + 11]
seeds = [1, 2] if quick else [1, 2, 3]
for dt in (torch.int32, torch.int64):
    for n in sizes:
        for dist in dists:
            for seed in seeds:
                t = make(n, dt, dist, seed)
                out = torch.empty_like(t)
                ctx.sort_dev(t, out)
                torch.cuda.synchronize()
                check(f"sort {str(dt)[6:]} n={n} {dist} seed={seed} map={ctx.stats()['first_level_map']}", t, out)
                del t, out
        torch.cuda.empty_cache()

# the bucket exchange at one RCCL rank with C3's geometry (128 buckets of ~4M keys at 2^29; here
# 2^27 keys over 32 buckets: 4M-key buckets, 16384-key tiles)
ctx.comm_init(1, 0, dsort.Context.unique_id())
try:
    for dt in (torch.int32, torch.int64):
        for dist in (["uniform", "k17", "zipf", "heavy"] if not quick else ["uniform", "zipf"]):
            n = (1 << 27) + 5
            t = make(n, dt, dist, 7)
            with ctx.options(buckets=32):
                ptr, nout = ctx.sample_sort_dev(t)
                ctx.synchronize()
            out = torch.empty_like(t)
            ctx.check(ctx.lib.dsort_copy_d2d(ctx.h, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ptr),
                                             out.element_size() * n))
            torch.cuda.synchronize()
            st = ctx.stats()
            check(f"bucket exchange {str(dt)[6:]} n={n} {dist} tile={st['tile_keys']} pending={st['pending_frees']}",
                  t, out if nout == n else out[:0])
            del t, out
            torch.cuda.empty_cache()
finally:
    ctx.comm_destroy()
print(f"{cases} cases, {bad} mismatches")
sys.exit(1 if bad else 0)
