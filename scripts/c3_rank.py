#!/usr/bin/env python3
"""One rank of config C3 (2^32 uniform int32 over 8 GPUs) measured on one MI355X.

Two designs of a rank's work, both run here for real (HIP events on the calls' stream, averaged
over --steps), the key exchange over xGMI PROJECTED from the link peak (7 links x 153 GB/s,
MI355X_MICROARCH.md):

  sort_then_merge   (round 1-3) the local sort of the rank's 2^29 keys (client.c:166's role), the
                    exchange, then the merge of the P = 8 received sorted runs of 2^26 keys (the
                    gather + merge_chunks of server.c:414-415 / 500-515) -- dsort_sort_dev_copy_i32 and
                    dsort_merge_dev_i32 on one rank's key range, the merge checked against torch.sort;
  bucket_exchange   (round 4, the default) the first partition level of the UNSORTED keys by global
                    splitters, the exchange of buckets, the second level + tile sort of the received
                    pieces -- dsort_sample_sort_dev_i32 on ONE rank (RCCL, world 1) with C3's bucket
                    size (DSORT_OPT_BUCKETS = 128: 4M-key buckets, as 1024 global buckets give each of 8
                    ranks at 2^32 keys); the exchange there is a self copy, the projection adds the xGMI
                    transfer of the 7/8 that would leave.

    python scripts/c3_rank.py [--steps 10] [--rank-keys 2**29] [--ranks 8] [--no-check]
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
    ap.add_argument("--c3-buckets", type=int, default=128, help="global buckets of the one-rank bucket exchange")
    ap.add_argument("--only-bx", action="store_true", help="skip the sort-then-merge design (profiling)")
    ap.add_argument("--opt", action="append", default=[], help="extra dsort option name=value for the bucket "
                                                               "exchange (repeatable)")
    args = ap.parse_args()

    import torch

    import dsort

    ctx = dsort.Context(0)
    n, P = args.rank_keys, args.ranks
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731  (torch's current stream = the calls' stream)

    # ---- A. sort-then-merge: the local sort of one rank's chunk
    chunk = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.gen_uniform(chunk, 0x5EED2026, args.rank * n)
    sort_ms = merge_ms = 0.0
    st, mst, exact, nb = {}, {}, None, 1
    if not args.only_bx:
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
        del sorted_chunk

        # the receive merge: P sorted runs of n/P keys inside rank `rank`'s key range
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
            ctx.sort_dev(recv[s * m:(s + 1) * m])
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
        ctx.merge_dev(recv, lens, out)  # one more, instrumented: the merge kernel alone (HIP events)
        mst = ctx.stats()
        exact = None
        if not args.no_check:
            exact = bool(torch.equal(out, torch.sort(recv).values))
        del recv, out
        torch.cuda.empty_cache()
        nb = 2 * 4 * P * m

    # ---- B. bucket exchange on one rank with C3's bucket size
    ctx.comm_init(1, 0, dsort.Context.unique_id())
    acc = {}
    extra = {kv.split("=")[0]: int(eval(kv.split("=")[1], {}, {})) for kv in args.opt}
    with ctx.options(buckets=args.c3_buckets, **extra):
        for _ in range(args.warmup):
            ctx.sample_sort_dev(chunk)
        ctx.synchronize()
        e0, e1 = ev(), ev()
        e0.record()
        for _ in range(args.steps):
            ptr, nout = ctx.sample_sort_dev(chunk)
        e1.record()
        torch.cuda.synchronize()
        bx_ms = e0.elapsed_time(e1) / args.steps
        for _ in range(args.steps):
            ctx.sample_sort_dev(chunk)
            sx = ctx.stats()
            for k in ("bucket_hist_ms", "bucket_scatter_ms", "sub_partition_ms", "tile_sort_kernel_ms",
                      "exchange_ms", "alltoall_ms", "final_merge_ms", "total_ms"):
                acc[k] = acc.get(k, 0.0) + sx[k] / args.steps
        bx_path = sx["exchange_path"]
        bx_ok = None
        if not args.no_check:
            import ctypes
            # the context-owned slice into a tensor (a device copy), compared on the device
            res_t = torch.empty(nout, dtype=torch.int32, device="cuda")
            ctx.check(ctx.lib.dsort_copy_d2d(ctx.h, ctypes.c_void_p(res_t.data_ptr()), ctypes.c_void_p(ptr), 4 * nout))
            bx_ok = bool(nout == n and torch.equal(res_t, torch.sort(chunk).values))
            del res_t
    ctx.comm_destroy()
    del chunk

    # ---- projections: + the key all-to-all over xGMI, (P-1)/P of the rank's keys over P-1 links
    x_bytes = 4 * n * (P - 1) / P
    x_ms = x_bytes / ((P - 1) * XGMI_LINK * 1e9) * 1e3
    t_a = sort_ms + x_ms + merge_ms
    t_b = bx_ms + x_ms
    proj = lambda t: {"rank_ms": round(t, 4), "job_keys_per_s": P * n / (t * 1e-3),  # noqa: E731
                      "single_pass_bound_frac": round(2 * 4 * n / (t * 1e-3) / 1e9 / HBM, 4)}
    res = {
        "what": f"one rank of C3: {n} int32 keys, {P} ranks",
        "sort_then_merge": {
            "sort_ms": round(sort_ms, 4),
            "sort_stages_ms": {k: round(st.get(k, 0.0), 4) for k in ("bucket_hist_ms", "bucket_scatter_ms",
                                                                      "sub_partition_ms", "tile_sort_kernel_ms", "total_ms")},
            "merge_ms": round(merge_ms, 4),
            "mergew_kernel_ms": round(mst.get("merge_kernel_ms", 0.0), 4),
            "merge_passes": mst.get("merge_passes"),
            "merge_frac_hbm": round(nb / (merge_ms * 1e-3) / 1e9 / HBM, 4) if merge_ms else None,
            "mergew_frac_hbm": round(nb / (mst["merge_kernel_ms"] * 1e-3) / 1e9 / HBM, 4) if mst.get("merge_kernel_ms") else None,
            "merge_bit_exact_vs_torch_sort": exact,
        },
        "bucket_exchange": {
            "buckets": args.c3_buckets, "exchange_path": bx_path,
            "sample_sort_ms": round(bx_ms, 4), "stages_ms": {k: round(v, 4) for k, v in acc.items()},
            "bit_exact_vs_torch_sort": bx_ok,
        },
        "projection": {
            "label": "PROJECTION: the exchange is not run on one GPU; xGMI at the link peak",
            "exchange_bytes": int(x_bytes), "exchange_ms_at_peak": round(x_ms, 4),
            # (a leg this run skipped -- --only-bx -- has no projection: null, not a figure built on 0 ms)
            "sort_then_merge": proj(t_a) if not args.only_bx else None, "bucket_exchange": proj(t_b),
        },
    }
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
