#!/usr/bin/env python3
"""Benchmark of the MI355X sort path (BASELINE.json metric: sorted keys/sec, int32, 2^30 keys).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--keys N_TOTAL] [--dtype i32|i64]
                    [--dist uniform|zipf] [--no-cpu-baseline]

One step = one full sort of the synthetic batch with the input already resident in HBM:
  N = 1: dsort_sort_dev_copy (tile sort + merge-path passes) of all keys on one GPU.
  N > 1: launched by torch.distributed.run, one process per GPU; every rank holds an equal
         contiguous chunk (server.c:185-216 partitioning) and the step is the sample sort
         (local sort + splitters + RCCL all-to-all over xGMI + merge of the received runs).
         The total key count stays fixed (strong scaling), as the metric is quoted on 2^30 keys.
The sorted output is verified outside the timed region (ascending + multiset fingerprint).

Prints ONE JSON line on rank 0 (contract in the task statement) with two extra objects:
  roofline      live HIP-event timing of the dominant kernel (the merge-path merge kernel) and
                its algorithmic bytes (2*w bytes per key per launch) against 8 TB/s;
  cpu_baseline  the reference's own algorithm (client.c merge_sort on 4 threads + server.c
                merge_chunks, compiled from the reference sources into oracle/_ref) on a bounded
                sample, timed on this host's cores.
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd")
sys.path.insert(0, PKG)

import torch  # noqa: E402  (before dsort: one HIP runtime)
import dsort  # noqa: E402

SEED = 0x5EED2026
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--keys", type=lambda s: int(eval(s, {}, {})), default=1 << 30,
                    help="total keys (e.g. 2**30)")
    ap.add_argument("--dtype", choices=["i32", "i64"], default="i32")
    ap.add_argument("--dist", choices=["uniform", "zipf"], default="uniform")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-keys", type=lambda s: int(eval(s, {}, {})), default=1 << 25)
    ap.add_argument("--kill-rank", type=int, default=None,
                    help="BASELINE config C5: fault-tolerance run (launch WITHOUT torchrun: the master "
                         "spawns one worker per GPU); this worker dies mid-sort")
    ap.add_argument("--kill-after-pass", type=int, default=1,
                    help="the dying worker SIGKILLs itself after this merge pass of its local sort")
    ap.add_argument("--reassign", choices=["first-live", "next-live"], default="first-live")
    ap.add_argument("--codec", action="store_true",
                    help="time the GPU text codec (output.txt format + %%d parse) on --keys sorted keys")
    return ap.parse_args()


# ------------------------------------------------------------------------- CPU baseline
def cpu_baseline(sample_keys):
    """The reference algorithm on the host: 4 worker threads each run the reference's
    merge_sort (client.c:166) on an equal contiguous chunk (server.c:185-216), then the
    reference's merge_chunks (server.c:481, linear argmin 4-way merge + output.txt text write).
    Uses oracle/_ref (reference compiled from its sources); falls back to the oracle restatement
    (kind "port") when that build is absent."""
    ref_dir = os.path.join(REPO, "oracle", "_ref")
    workers = 4
    keys = np.empty(sample_keys, np.int32)
    orc_path = os.path.join(REPO, "oracle", "liboracle.so")
    orc = ctypes.CDLL(orc_path)
    orc.oracle_gen_uniform_i32.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p]
    orc.oracle_gen_uniform_i32(SEED, 0, sample_keys, keys.ctypes.data)
    sz = [sample_keys // workers + (1 if i < sample_keys % workers else 0) for i in range(workers)]
    offs = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.int64)
    chunks = [keys[o:o + s].copy() for o, s in zip(offs, sz)]
    kind = "reference"
    try:
        cl = ctypes.CDLL(os.path.join(ref_dir, "libref_client.so"))
        sv = ctypes.CDLL(os.path.join(ref_dir, "libref_server.so"))
        cl.merge_sort.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        sv.merge_chunks.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        sort_fn = lambda c: cl.merge_sort(c.ctypes.data, 0, c.size - 1)  # noqa: E731

        def merge_fn(cs, total):
            ptrs = (ctypes.c_void_p * workers)(*[c.ctypes.data for c in cs])
            lens = (ctypes.c_int * workers)(*[c.size for c in cs])
            sv.merge_chunks(workers, ptrs, lens, total)
    except OSError:
        kind = "port"
        orc.oracle_merge_sort_i32.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        orc.oracle_merge_chunks_i32.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        orc.oracle_format_i32.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        orc.oracle_format_i32.restype = ctypes.c_long
        sort_fn = lambda c: orc.oracle_merge_sort_i32(c.ctypes.data, c.size)  # noqa: E731

        def merge_fn(cs, total):
            ptrs = (ctypes.c_void_p * workers)(*[c.ctypes.data for c in cs])
            lens = (ctypes.c_size_t * workers)(*[c.size for c in cs])
            out = np.zeros(total, np.int32)
            orc.oracle_merge_chunks_i32(workers, ptrs, lens, out.ctypes.data)
            buf = ctypes.create_string_buffer(12 * total + 1)
            n = orc.oracle_format_i32(out.ctypes.data, total, buf, len(buf))
            with open("output.txt", "wb") as f:
                f.write(buf.raw[:n])

    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        try:
            t0 = time.perf_counter()
            th = [threading.Thread(target=sort_fn, args=(c,)) for c in chunks]  # ctypes drops the GIL
            for t in th:
                t.start()
            for t in th:
                t.join()
            t1 = time.perf_counter()
            merge_fn(chunks, sample_keys)
            t2 = time.perf_counter()
        finally:
            os.chdir(cwd)
    ok = all(np.all(c[:-1] <= c[1:]) for c in chunks)
    return {
        "value": sample_keys / (t2 - t0), "unit": "sorted keys/s", "cores": workers, "kind": kind,
        "sample": (f"{sample_keys} uniform int32 keys (seed {SEED:#x}); 4 threads x reference merge_sort "
                   f"on equal chunks ({t1 - t0:.2f} s) + reference merge_chunks incl. output.txt "
                   f"text write ({t2 - t1:.2f} s); host nproc={os.cpu_count()}; chunks sorted={ok}"),
    }


def pmc_traffic(kernel, n, w):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/r1_pmc_traffic.json: FETCH_SIZE x2 + WRITE_SIZE, see its calibration note), scaled
    to this run's key count; None when the file is absent or was measured on another key width."""
    path = os.path.join(REPO, "profiles", "r1_pmc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f)["kernels"][kernel]
    except (OSError, KeyError, ValueError):
        return None
    if w != 4:
        return None
    return round(rec.get("traffic_bytes_per_pass", rec["traffic_bytes"]) * n / (1 << 30))


# ------------------------------------------------------------------------- GPU runs
def make_input(ctx, n, first, dtype, dist):
    tdt = torch.int32 if dtype == "i32" else torch.int64
    t = torch.empty(max(n, 1), dtype=tdt, device="cuda")[:n]
    if dist == "zipf":
        if dtype != "i64":
            raise SystemExit("zipf is defined for int64 keys (BASELINE config 4)")
        ctx.gen_zipf_i64(t, SEED, first)
    else:
        ctx.gen_uniform(t, SEED, first)
    torch.cuda.synchronize()
    return t


def run_single(args):
    ctx = dsort.Context(0)
    n = args.keys
    w = 4 if args.dtype == "i32" else 8
    t_in = make_input(ctx, n, 0, args.dtype, args.dist)
    out = torch.empty_like(t_in)
    fp_in = ctx.fingerprint(t_in)
    for _ in range(args.warmup):
        ctx.sort_dev(t_in, out)
    torch.cuda.synchronize()
    if args.warmup == 0:  # still verify once, outside the timed region
        ctx.sort_dev(t_in, out)
        torch.cuda.synchronize()
    ok = ctx.descents(out) == 0 and ctx.fingerprint(out) == fp_in
    if not ok:
        raise SystemExit("bench: sorted output failed verification")
    torch.cuda.synchronize()
    kms, klaunch, bms, tot = 0.0, 0, 0.0, 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.sort_dev(t_in, out)
        st = ctx.stats()  # reads the HIP events of this step (syncs the stream)
        kms += st["merge_kernel_ms"]
        klaunch += st["merge_kernel_launches"]
        bms += st["block_sort_ms"]
        tot += st["total_ms"]
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    stats = ctx.stats()
    ctx.close()
    return elapsed, {"kernel_ms": kms, "launches": klaunch, "block_ms": bms, "device_ms": tot,
                     "passes": stats["merge_passes"], "tile": stats["tile_keys"], "w": w, "n_gpu": n}


def run_multi(args):
    """One rank per GPU (torch.distributed.run): gloo for control, RCCL (inside libdsort) for
    the key exchange.  Strong scaling: the 2^30 keys are split into equal contiguous chunks."""
    import torch.distributed as dist
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    torch.cuda.set_device(local)
    dist.init_process_group("gloo")
    ctx = dsort.Context(local)
    uid = [dsort.Context.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    ctx.comm_init(world, rank, uid[0])
    n = args.keys
    sz = n // world + (1 if rank < n % world else 0)          # server.c:185-216 partition rule
    first = rank * (n // world) + min(rank, n % world)
    t_in = make_input(ctx, sz, first, args.dtype, args.dist)
    w = 4 if args.dtype == "i32" else 8
    in_fp = ctx.fingerprint(t_in)
    for _ in range(max(args.warmup, 1)):
        ptr, nout = ctx.sample_sort_dev(t_in)
    ctx.synchronize()
    # verification outside the timed region: local order, global multiset, rank boundaries
    sfx = args.dtype
    c, fs, fx = dsort.U64(), dsort.U64(), dsort.U64()
    ctx.check(getattr(ctx.lib, f"dsort_count_descents_{sfx}")(ctx.h, ptr, nout, ctypes.byref(c)))
    ctx.check(getattr(ctx.lib, f"dsort_fingerprint_{sfx}")(ctx.h, ptr, nout, ctypes.byref(fs), ctypes.byref(fx)))
    ends = np.zeros(2, np.int64)
    if nout:
        hb = np.zeros(1, np.int64 if sfx == "i64" else np.int32)
        ctx.copy_d2h(hb, ptr, hb.itemsize)
        ends[0] = hb[0]
        ctx.copy_d2h(hb, ptr + (nout - 1) * hb.itemsize, hb.itemsize)
        ends[1] = hb[0]
    M = 0xFFFFFFFFFFFFFFFF
    info = torch.tensor([c.value, nout, ends[0], ends[1]], dtype=torch.int64)
    allinfo = [torch.zeros_like(info) for _ in range(world)]
    dist.all_gather(allinfo, info)
    fps = [None] * world
    dist.all_gather_object(fps, (in_fp[0], in_fp[1], fs.value, fx.value))
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    ex, fm = 0.0, 0.0
    for _ in range(args.steps):
        ptr, nout = ctx.sample_sort_dev(t_in)
        st = ctx.stats()  # synchronizes this rank's stream
        ex += st["exchange_ms"]
        fm += st["final_merge_ms"]
    torch.cuda.synchronize()
    dist.barrier()
    t1 = time.perf_counter()
    el = torch.tensor([t1 - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    A = torch.stack(allinfo)
    ok = bool((A[:, 0] == 0).all()) and int(A[:, 1].sum()) == n
    ok &= sum(f[0] for f in fps) & M == sum(f[2] for f in fps) & M
    x_in = x_out = 0
    for f in fps:
        x_in ^= f[1]
        x_out ^= f[3]
    ok &= x_in == x_out
    for r in range(world - 1):
        if A[r, 1] > 0 and A[r + 1, 1] > 0:
            ok &= bool(A[r, 3] <= A[r + 1, 2])
    # the local sort's merge-pass kernel on this rank's chunk (HIP events per launch), outside the
    # timed region: the roofline line of the multi-GPU run
    t_loc = torch.empty_like(t_in)
    ctx.sort_dev(t_in, t_loc)
    lst = ctx.stats()
    del t_loc
    ctx.comm_destroy()
    ctx.close()
    return rank, world, float(el.item()), ok, {"exchange_ms": ex, "final_merge_ms": fm, "w": w,
                                                "n_gpu": sz, "local_kernel_ms": lst["merge_kernel_ms"],
                                                "local_launches": lst["merge_kernel_launches"],
                                                "local_passes": lst["merge_passes"]}


def run_fault(args):
    """BASELINE config C5 through ftsort.Master (server.c's role): a fault-free run, then a run in
    which worker `--kill-rank` dies after merge pass `--kill-after-pass` of its local sort; the
    survivors detect it, rebuild the communicator and sort the dead chunk from its replica."""
    import ftsort

    ndev = torch.cuda.device_count()
    share = args.gpus > ndev  # one GPU box: the workers share it and exchange through gloo
    devices = [0] * args.gpus if share else list(range(args.gpus))
    transport = "host" if share or args.gpus == 1 else "rccl"
    r = ftsort.fault_run(args.gpus, args.keys, args.kill_rank, args.kill_after_pass,
                         "i32" if args.dtype == "i32" else "i64", args.dist, transport, devices, args.reassign)
    if not r["ok"]:
        raise SystemExit(f"bench: fault run failed verification: {json.dumps(r)}")
    free, fault = r["fault_free"], r["fault"]
    out = {"metric": "recovery time after one GPU worker failure mid-sort (BASELINE config C5)",
           "value": round(r["recovery_ms"], 3), "unit": "ms", "n_gpus": args.gpus, "higher_is_better": False,
           "dtype": "int32" if args.dtype == "i32" else "int64", "data": f"synthetic {args.dist} keys",
           "config": {"workload": f"sample sort of {args.keys} keys over {args.gpus} workers, worker "
                                  f"{args.kill_rank} killed after merge pass {args.kill_after_pass}",
                      "transport": transport, "reassign": args.reassign, "devices": devices},
           "fault_free_ms": round(free["t_end_ms"], 3), "fault_ms": round(fault["t_end_ms"], 3),
           "fault_free_keys_per_s": args.keys / (free["t_end_ms"] * 1e-3),
           "fault_keys_per_s": args.keys / (fault["t_end_ms"] * 1e-3),
           "fault_seen_by_master_ms": fault["t_fault_seen_ms"],
           "survivors_notified_ms": fault["t_survivors_notified_ms"],
           "plan": fault["plan"], "slices": fault["slices"], "verified": True}
    print(json.dumps(out), flush=True)


def run_codec(args):
    """the reference's text I/O on the GPU.  Formats `--keys` sorted uniform int32
    keys to output.txt bytes (server.c:517-519) and parses them back (server.c:179/213's %d
    tokens), each timed over `--steps` calls with the data resident in HBM; verifies the round
    trip.  The CPU leg times the oracle's single-threaded codec on a 2^24-key sample."""
    ctx = dsort.Context(0)
    n = args.keys
    keys = make_input(ctx, n, 0, "i32", "uniform")
    ctx.sort_dev(keys)
    text = torch.empty(12 * n, dtype=torch.uint8, device="cuda")
    back = torch.empty(n, dtype=torch.int32, device="cuda")
    for _ in range(args.warmup):
        ln = ctx.format_text(keys, text)
        ctx.parse_text(text, ln, back)
    torch.cuda.synchronize()
    res = {}
    for name, fn in (("format", lambda: ctx.format_text(keys, text)),
                     ("parse", lambda: ctx.parse_text(text, ln, back))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            r = fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        if name == "format":
            ln = r
        res[name] = ms
    if not (ctx.parse_text(text, ln, back) == n and torch.equal(back, keys)):
        raise SystemExit("bench: codec round trip failed")
    moved = 4 * n + ln  # algorithmic bytes of either direction: the keys plus the text
    out = {"metric": "output.txt format keys/sec (GPU text codec, SURVEY 8f.1)", "unit": "keys/s",
           "value": n / (res["format"] * 1e-3), "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
           "higher_is_better": True, "dtype": "int32", "data": "synthetic uniform keys, sorted",
           "config": {"workload": f"{n} sorted int32 keys <-> {ln} bytes of %d\\n text", "keys": n,
                      "text_bytes": ln},
           "format_ms": round(res["format"], 4), "parse_ms": round(res["parse"], 4),
           "parse_keys_per_s": n / (res["parse"] * 1e-3),
           "roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                        "format_achieved": round(moved / (res["format"] * 1e-3) / 1e9, 1),
                        "parse_achieved": round(moved / (res["parse"] * 1e-3) / 1e9, 1),
                        "format_frac": round(moved / (res["format"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "parse_frac": round(moved / (res["parse"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "algorithmic_bytes": moved}}
    if not args.no_cpu_baseline:
        orc = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
        orc.oracle_format_i32.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        orc.oracle_format_i32.restype = ctypes.c_long
        orc.oracle_parse_i32.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        orc.oracle_parse_i32.restype = ctypes.c_long
        m = min(n, 1 << 24)
        sample = keys[:m].cpu().numpy()
        buf = np.empty(12 * m, np.uint8)
        t0 = time.perf_counter()
        L = orc.oracle_format_i32(sample.ctypes.data, m, buf.ctypes.data, buf.size)
        t1 = time.perf_counter()
        dst = np.empty(m, np.int32)
        c = orc.oracle_parse_i32(buf.ctypes.data, L, dst.ctypes.data, m)
        t2 = time.perf_counter()
        assert c == m and np.array_equal(dst, sample)
        out["cpu_baseline"] = {"value": m / (t1 - t0), "unit": "keys/s (format)", "cores": 1, "kind": "port",
                               "parse_keys_per_s": m / (t2 - t1),
                               "sample": f"{m} sorted uniform int32 keys, oracle_format_i32 / oracle_parse_i32 "
                                         "(single thread)"}
    print(json.dumps(out), flush=True)
    ctx.close()


def main():
    args = parse()
    if args.codec:
        run_codec(args)
        return
    if args.kill_rank is not None:
        if "WORLD_SIZE" in os.environ:
            raise SystemExit("--kill-rank runs its own master and workers: launch it without torchrun")
        run_fault(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world and world != 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    metric = "sorted keys/sec (int32, 2^30 keys)" if args.dtype == "i32" else "sorted keys/sec (int64)"
    result = {"metric": metric, "unit": "keys/s", "n_gpus": args.gpus, "steps": args.steps,
              "warmup": args.warmup, "higher_is_better": True, "scaling": "strong",
              "vs_baseline": None, "dtype": "int32" if args.dtype == "i32" else "int64",
              "data": f"synthetic {args.dist} keys, splitmix64(seed={SEED:#x} + global index)"}
    if world == 1 and args.gpus == 1:
        elapsed, k = run_single(args)
        n = args.keys
        step_ms = 1000.0 * elapsed / args.steps
        result.update({"value": n * args.steps / elapsed, "ms_per_step": step_ms})
        # one merge pass = one read + one write of every key; a pass of the bucketed int32 sort
        # is one launch per kernel fan-in among its buckets, so time is summed per pass
        npass = k["passes"] * args.steps
        avg_launch_ms = k["kernel_ms"] / max(npass, 1)
        bytes_per_launch = 2 * k["w"] * n
        achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9 if k["launches"] and npass else 0.0
        cfg = "C2-style" if args.dtype == "i32" else "C4-style"
        result["config"] = {"workload": f"{cfg} single-GPU sort of {n} {args.dist} {result['dtype']} keys "
                                        f"(BASELINE metric size); tile {k['tile']} keys, {k['passes']} merge passes",
                            "keys": n, "parallelism": "1 GPU"}
        result["roofline"] = {
            "bound": "hbm", "kernel": "mergew_kernel (k-way merge pass)" if args.dtype == "i32"
            else "mergek_kernel (k-way merge pass, LDS merge path)", "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic("mergew_kernel", n, k["w"]), "avg_pass_ms": round(avg_launch_ms, 4),
            "algorithmic_bytes_per_pass": bytes_per_launch,
            "launches_per_pass": round(k["launches"] / max(npass, 1), 2),
            "partition_and_tile_sort_ms": round(k["block_ms"] / args.steps, 3),
            "whole_sort_single_pass_bound_frac": round(2 * k["w"] * n / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        }
        if not args.no_cpu_baseline and args.dtype == "i32":
            result["cpu_baseline"] = cpu_baseline(args.cpu_sample_keys)
        print(json.dumps(result), flush=True)
    else:
        rank, world, elapsed, ok, k = run_multi(args)
        if rank == 0:
            if not ok:
                raise SystemExit("bench: distributed output failed verification")
            n = args.keys
            step_ms = 1000.0 * elapsed / args.steps
            result.update({"value": n * args.steps / elapsed, "ms_per_step": step_ms})
            result["config"] = {"workload": f"sample sort of {n} {args.dist} {result['dtype']} keys over {world} GPUs "
                                            "(equal chunks, RCCL all-to-all)", "keys": n,
                                "parallelism": f"sample-sort x{world}"}
            nl = k["local_passes"] if k["local_launches"] else 0  # launches of one pass are summed
            avg = k["local_kernel_ms"] / nl if nl else 0.0
            bpl = 2 * k["w"] * k["n_gpu"]  # one read + one write of the rank's chunk per launch
            ach = bpl / (avg * 1e-3) / 1e9 if nl and avg > 0 else None
            result["roofline"] = {"bound": "hbm", "kernel": "mergew_kernel (rank 0 local sort, per GPU)",
                                  "achieved": round(ach, 1) if ach else None, "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
                                  "traffic": pmc_traffic("mergew_kernel", k["n_gpu"], k["w"]),
                                  "avg_pass_ms": round(avg, 4), "algorithmic_bytes_per_pass": bpl,
                                  "rank0_exchange_ms": round(k["exchange_ms"] / args.steps, 3),
                                  "rank0_final_merge_ms": round(k["final_merge_ms"] / args.steps, 3),
                                  "whole_sort_single_pass_bound_frac": round(
                                      2 * k["w"] * n / (step_ms * 1e-3) / 1e9 / (HBM_PEAK_GBS * world), 4)}
            print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
