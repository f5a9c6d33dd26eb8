#!/usr/bin/env python3
"""One rank of config C3 (2^32 uniform int32 over 8 GPUs) measured on one MI355X.

A rank of the sample sort (dsort_api.hip sample_sort) does, in order:
  1. the local sort of its 2^29-key chunk (the worker's merge_sort, client.c:166) -- here
     dsort_sort_dev_copy_i32 on 2^29 keys;
  2. the sample all-gather, splitters and cut search (tiny);
  3. the key all-to-all over xGMI: 7/8 of its keys leave, as many arrive;
  4. the merge of the P = 8 received runs (the gather + merge_chunks of server.c:414-415 and
     500-515) -- here dsort_merge_dev_i32 of 8 sorted runs of 2^26 keys that cover one rank's key
     range (1/8 of the int32 range, as uniform input gives every rank).

Steps 1 and 4 run here for real (HIP events on the calls' stream, averaged over --steps), the
merge is checked bit-exact against torch.sort, and step 3 is PROJECTED from the xGMI peak
(7 links x 153 GB/s, MI355X_MICROARCH.md).  Prints one JSON line.

    python scripts/c3_rank.py [--steps 10] [--rank-keys 2**29] [--ranks 8] [--exchange-frac 1.0]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd"))

HBM = 8000.0
XGMI_LINK = 153.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rank-keys", type=lambda s: int(eval(s, {}, {})), default=1 << 29)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--rank", type=int, default=3, help="which rank's key range the received runs cover")
    ap.add_argument("--no-check", action="store_true")
    args = ap.parse_args()

    import torch

    import dsort

    ctx = dsort.Context(0)
    n, P = args.rank_keys, args.ranks
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731  (torch's current stream = the calls' stream)

    # ---- 1. the local sort of one rank's chunk
    chunk = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.gen_uniform(chunk, 0x5EED2026, args.rank * n)
    sorted_chunk = torch.empty_like(chunk)
    for _ in range(args.warmup):
        ctx.sort_dev(chunk, sorted_chunk)
    torch.cuda.synchronize()
    e0, e1 = ev(), ev()
    e0.record()
    for _ in range(args.steps):
        ctx.sort_dev(chunk, sorted_chunk)
    e1.record()
    torch.cuda.synchronize()
    sort_ms = e0.elapsed_time(e1) / args.steps
    st = ctx.stats()
    del chunk, sorted_chunk

    # ---- 4. the receive merge: P sorted runs of n/P keys inside rank `rank`'s key range
    m = n // P
    recv = torch.empty(P * m, dtype=torch.int32, device="cuda")
    ctx.gen_uniform(recv, 0x5EED2026 ^ 0xC3, 0)
    span = (1 << 32) // P
    lo = -(1 << 31) + args.rank * span
    # key = lo + (u mod span): one rank's range under uniform input (span is a power of two)
    r64 = recv.to(torch.int64) & (span - 1)
    recv.copy_((r64 + lo).to(torch.int32))
    del r64
    for s in range(P):
        seg = recv[s * m:(s + 1) * m]
        ctx.sort_dev(seg)
    out = torch.empty_like(recv)
    lens = [m] * P
    for _ in range(args.warmup):
        ctx.merge_dev(recv, lens, out)
    torch.cuda.synchronize()
    e0, e1 = ev(), ev()
    e0.record()
    for _ in range(args.steps):
        ctx.merge_dev(recv, lens, out)
    e1.record()
    torch.cuda.synchronize()
    merge_ms = e0.elapsed_time(e1) / args.steps
    # per-kernel: one more instrumented merge (the mergew kernel alone, HIP events around it)
    ctx.merge_dev(recv, lens, out)
    mst = ctx.stats()
    exact = None
    if not args.no_check:
        exact = bool(torch.equal(out, torch.sort(recv).values))
    nb = 2 * 4 * P * m
    # ---- 3. projected exchange: (P-1)/P of the rank's keys over P-1 links
    x_bytes = 4 * n * (P - 1) / P
    x_ms = x_bytes / ((P - 1) * XGMI_LINK * 1e9) * 1e3
    total = sort_ms + x_ms + merge_ms
    res = {
        "what": f"one rank of C3: local sort of {n} int32 keys + merge of {P} received runs of {m}",
        "sort_ms": round(sort_ms, 4),
        "sort_stages_ms": {k: round(st[k], 4) for k in ("bucket_hist_ms", "bucket_scatter_ms", "sub_partition_ms",
                                                          "tile_sort_kernel_ms", "total_ms")},
        "merge_ms": round(merge_ms, 4),
        "mergew_kernel_ms": round(mst["merge_kernel_ms"], 4),
        "merge_passes": mst["merge_passes"],
        "merge_frac_hbm": round(nb / (merge_ms * 1e-3) / 1e9 / HBM, 4),
        "mergew_frac_hbm": round(nb / (mst["merge_kernel_ms"] * 1e-3) / 1e9 / HBM, 4) if mst["merge_kernel_ms"] else None,
        "merge_bit_exact_vs_torch_sort": exact,
        "projection": {
            "label": "PROJECTION (exchange not run: one GPU); xGMI at peak",
            "exchange_bytes": int(x_bytes), "exchange_ms_at_peak": round(x_ms, 4),
            "rank_ms": round(total, 4),
            "job_keys_per_s": P * n / (total * 1e-3),
            "single_pass_bound_frac": round(2 * 4 * n / (total * 1e-3) / 1e9 / HBM, 4),
        },
    }
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
