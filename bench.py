#!/usr/bin/env python3
"""Benchmark of the MI355X sort path (BASELINE.json metric: sorted keys/sec, int32, 2^30 keys,
at 1/2/4/8 GPUs, with the HBM / xGMI roofline fraction).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--keys N_TOTAL] [--dtype i32|i64]
                    [--dist uniform|zipf] [--path single|samplesort] [--no-cpu-baseline]

One step = one full sort of the synthetic batch, input already resident in HBM:
  single      (default at N = 1) dsort_sort_dev_copy: partition, tile sort and merge-path passes
              of all keys on one GPU;
  samplesort  (default at N > 1; --path samplesort forces it at N = 1) one process per GPU, every
              rank holding an equal contiguous chunk (server.c:185-216), the step being the sample
              sort: local sort + splitters + RCCL all-to-all over xGMI + merge of the received runs
              (replaces the gather at server.c:414-415).  The total key count stays fixed (strong
              scaling: the metric is quoted on 2^30 keys); --keys 2**32 is config C3.
Ranks: `python bench.py --gpus N` spawns the N rank processes itself (subprocess, before any GPU
call, rendezvous on 127.0.0.1); under torch.distributed.run it is one of them.  --gpus must equal
the number of rank processes, and N GPUs must be visible.
The sorted output is verified outside the timed region (ascending + multiset fingerprint + rank
boundaries).

Rank 0 prints ONE JSON line with two extra objects:
  roofline      live HIP-event timing of every kernel of the sort (first-level histogram and
                scatter, second-level partition, tile sort: algorithmic bytes = 1 or 2 x key
                bytes per key) against 8 TB/s; `kernel` is the slowest of them (at N > 1 the
                slowest stage of any rank's local sort); `all_kernels_frac` = the committed PMC
                bytes of the whole sort over its device time; at N > 1 the key
                exchange's bytes over xGMI against (N-1) links x 153 GB/s;
  cpu_baseline  the reference's own algorithm (client.c merge_sort on 4 threads + server.c
                merge_chunks, compiled from the reference sources into oracle/_ref) on a bounded
                sample, plus the reference's TCP server + 4 clients on input.txt (config C1),
                timed on this host's cores.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd")
sys.path.insert(0, PKG)

SEED = 0x5EED2026
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
XGMI_LINK_GBS = 153.0   # one xGMI link (7 per MI355X, one to every peer of an 8-GPU node)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--keys", type=lambda s: int(eval(s, {}, {})), default=1 << 30,
                    help="total keys over all GPUs (e.g. 2**30)")
    ap.add_argument("--dtype", choices=["i32", "i64"], default="i32")
    ap.add_argument("--dist", choices=["uniform", "zipf"], default="uniform")
    ap.add_argument("--path", choices=["auto", "single", "samplesort"], default="auto")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-keys", type=lambda s: int(eval(s, {}, {})), default=1 << 27)
    ap.add_argument("--kill-rank", type=int, default=None,
                    help="BASELINE config C5: fault-tolerance run (launch WITHOUT torchrun: the master "
                         "spawns one worker per GPU); this worker dies mid-sort")
    ap.add_argument("--kill-after-stage", dest="kill_after_stage", type=int, default=0,
                    help="the dying worker SIGKILLs itself after this stage of its local sort "
                         "(DSORT_OPT_KILL_AFTER_STAGE; >= 2^25 keys per worker: 0 first-level partition, "
                         "1 second-level partition, 2 tile sort); an unreachable stage is an error")
    ap.add_argument("--kill-stage", choices=["sort", "exchange"], default="sort",
                    help="C5: die in the local sort (after --kill-after-stage) or inside the key exchange")
    ap.add_argument("--reassign", choices=["first-live", "next-live"], default="first-live")
    ap.add_argument("--codec", action="store_true",
                    help="time the GPU text codec (output.txt format + %%d parse) on --keys sorted keys")
    ap.add_argument("--legs", default="all",
                    help="sample-sort runs only (N > 1, or --path samplesort): extra legs after the metric's "
                         "timed region, comma-separated from c3,c4,c5 ('all', default; 'none' to skip)")
    ap.add_argument("--no-legs", dest="legs", action="store_const", const="none")
    ap.add_argument("--leg-timeout", type=float, default=180.0,
                    help="exchange deadline of a sort leg in seconds (the C5 leg gets 2x)")
    ap.add_argument("--launcher-selftest", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# ------------------------------------------------------------------------- rank launcher
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_envs(n, port, base=None, store=None):
    """The environment of each of n rank processes (torch.distributed.run's variables).  `store`:
    a file for the ranks' rendezvous (DSORT_BENCH_STORE), which then needs no TCP port: a port
    chosen here and bound later by rank 0 can be taken in between (a multi-rank test hung on that
    in round 4)."""
    base = dict(os.environ if base is None else base)
    out = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                 HSA_ENABLE_IPC_MODE_LEGACY="0")
        if store:
            e["DSORT_BENCH_STORE"] = store
        out.append(e)
    return out


def init_group(dist, rank, world):
    """The ranks' gloo group: a file rendezvous when this script spawned them, else torchrun's
    MASTER_ADDR/MASTER_PORT (env://)."""
    store = os.environ.get("DSORT_BENCH_STORE")
    if store:
        dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)


def launch_ranks(n, argv, check_devices=True, timeout_s=1800):
    """Spawns n copies of this script as ranks 0..n-1 (children, never exec; no GPU call in this
    process: torch.cuda.device_count() does not initialise the GPU on this image).  Returns the
    first non-zero exit code, else 0; a failing rank takes the others down."""
    if check_devices:
        import torch

        ndev = torch.cuda.device_count()
        if n > ndev:
            print(f"bench: --gpus {n} needs {n} visible GPUs (one rank per GPU), found {ndev}",
                  file=sys.stderr, flush=True)
            return 2
    tmpd = tempfile.mkdtemp(prefix="dsort_bench_")
    envs = rank_envs(n, free_port(), store=os.path.join(tmpd, "store"))
    procs = [subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=e) for e in envs]
    rc, t_end = 0, time.time() + timeout_s
    try:
        while any(p.poll() is None for p in procs):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad or time.time() > t_end:
                rc = bad[0] if bad else 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
        import shutil

        shutil.rmtree(tmpd, ignore_errors=True)
    if rc == 0:
        rc = next((p.returncode for p in procs if p.returncode), 0)
    return rc


def launcher_selftest():
    """--launcher-selftest: one line per rank with the plumbing it received (CPU test)."""
    line = json.dumps({"rank": int(os.environ["RANK"]), "world": int(os.environ["WORLD_SIZE"]),
                       "local_rank": int(os.environ["LOCAL_RANK"]), "master": os.environ["MASTER_ADDR"],
                       "port": int(os.environ["MASTER_PORT"])}) + "\n"
    os.write(1, line.encode())  # one write per line: the ranks share the parent's stdout


# ------------------------------------------------------------------------- CPU baseline
def host_info():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        usable = os.cpu_count()
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": usable}


def reference_tcp_c1(reps=5, timeout=60.0):
    """Config C1 on the reference itself: oracle/_ref/server + 4 oracle/_ref/client processes on
    127.0.0.1 (server.c:120-157 accepts exactly 4), the reference's input.txt (10 000 keys,
    tests/golden/ref_input.txt) sorted `reps` times in one session; wall time from the file name
    on the server's stdin to its "Sorting completed" line (server.c:265-270).  None when the
    reference build is absent."""
    ref = os.path.join(REPO, "oracle", "_ref")
    server, client = os.path.join(ref, "server"), os.path.join(ref, "client")
    src = os.path.join(REPO, "tests", "golden", "ref_input.txt")
    if not (os.path.exists(server) and os.path.exists(client) and os.path.exists(src)):
        return None
    with tempfile.TemporaryDirectory() as d:
        port = free_port()
        with open(os.path.join(d, "server.conf"), "w") as f:
            f.write(f"SERVER_PORT={port}\n")
        with open(os.path.join(d, "client.conf"), "w") as f:
            f.write(f"SERVER_IP=127.0.0.1\nSERVER_PORT={port}\n")
        with open(src, "rb") as fi, open(os.path.join(d, "input.txt"), "wb") as fo:
            fo.write(fi.read())
        # the server's stdout on a pseudo-terminal: printf is then line-buffered, as on the
        # reference's console, so every line is seen when it is printed.  Boxes without pty
        # devices fall back to watching output.txt: merge_chunks() writes it whole and closes it
        # (server.c:484-523) just before the "Sorting completed" line.
        import pty

        try:
            mfd, sfd = pty.openpty()
        except OSError:
            return _reference_tcp_c1_filepoll(d, server, client, reps, timeout)
        srv = subprocess.Popen([server, "server.conf"], cwd=d, stdin=subprocess.PIPE, stdout=sfd,
                               stderr=sfd, bufsize=0)
        os.close(sfd)
        clients = []
        try:
            lines = []

            def reader():
                buf = b""
                while True:
                    try:
                        chunk = os.read(mfd, 1 << 16)
                    except OSError:
                        break
                    if not chunk:
                        break
                    buf += chunk
                    *full, buf = buf.split(b"\n")
                    now = time.perf_counter()
                    lines.extend((now, ln) for ln in full)

            th = threading.Thread(target=reader, daemon=True)
            th.start()
            t0 = time.time()
            while not any(b"waiting for worker" in ln for _, ln in lines):
                if time.time() - t0 > timeout or srv.poll() is not None:
                    return None
                time.sleep(0.01)
            for _ in range(4):
                clients.append(subprocess.Popen([client, "client.conf"], cwd=d, stdout=subprocess.DEVNULL,
                                                stderr=subprocess.DEVNULL))
            while sum(b"connected" in ln.lower() for _, ln in lines) < 4:
                if time.time() - t0 > timeout or srv.poll() is not None:
                    return None
                time.sleep(0.01)
            times = []
            for _ in range(reps):
                seen = sum(b"Sorting completed" in ln for _, ln in lines)
                ts = time.perf_counter()
                srv.stdin.write(b"input.txt\n")
                while sum(b"Sorting completed" in ln for _, ln in lines) <= seen:
                    if time.time() - t0 > timeout or srv.poll() is not None:
                        return None
                    time.sleep(0.0005)
                te = [t for t, ln in lines if b"Sorting completed" in ln][seen]
                times.append(te - ts)
            srv.stdin.write(b"exit\n")
            ok = open(os.path.join(d, "output.txt"), "rb").read() == \
                open(os.path.join(REPO, "tests", "golden", "ref_output.txt"), "rb").read()
        finally:
            for p in clients + [srv]:
                if p.poll() is None:
                    p.kill()
                p.wait()
            os.close(mfd)
    return _c1_result(times, ok, "pty")


def _reference_tcp_c1_filepoll(d, server, client, reps, timeout):
    """reference_tcp_c1 without a pty: the server's stdout is discarded; each file's end is the
    moment output.txt (removed before the file name is sent) reaches the reference output's full
    size.  The first file also waits for the 4 clients to connect, so only the median is fair."""
    want = open(os.path.join(REPO, "tests", "golden", "ref_output.txt"), "rb").read()
    outp = os.path.join(d, "output.txt")
    srv = subprocess.Popen([server, "server.conf"], cwd=d, stdin=subprocess.PIPE, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL, bufsize=0)
    clients = []
    try:
        time.sleep(0.3)
        for _ in range(4):
            clients.append(subprocess.Popen([client, "client.conf"], cwd=d, stdout=subprocess.DEVNULL,
                                            stderr=subprocess.DEVNULL))
        t0 = time.time()
        times = []
        for _ in range(reps):
            if os.path.exists(outp):
                os.remove(outp)
            ts = time.perf_counter()
            srv.stdin.write(b"input.txt\n")
            while not (os.path.exists(outp) and os.path.getsize(outp) >= len(want)):
                if time.time() - t0 > timeout or srv.poll() is not None:
                    return None
                time.sleep(0.0002)
            times.append(time.perf_counter() - ts)
        time.sleep(0.05)
        ok = open(outp, "rb").read() == want
        srv.stdin.write(b"exit\n")
    finally:
        for p in clients + [srv]:
            if p.poll() is None:
                p.kill()
            p.wait()
    return _c1_result(times, ok, "output-file poll (no pty)")


def _c1_result(times, ok, mode):
    med = sorted(times)[len(times) // 2]
    return {"keys": 10000, "files": len(times), "first_file_ms": round(1e3 * times[0], 3),
            "median_file_ms": round(1e3 * med, 3), "keys_per_s_median": 10000 / med,
            "output_matches_reference_output_txt": ok, "timing": mode}


def cpu_baseline(sample_keys, target_keys):
    """The reference algorithm on the host: 4 worker threads each run the reference's
    merge_sort (client.c:166) on an equal contiguous chunk (server.c:185-216), then the
    reference's merge_chunks (server.c:481, linear argmin 4-way merge + output.txt text write).
    Uses oracle/_ref (reference compiled from its sources); falls back to the oracle restatement
    (kind "port") when that build is absent.  Also times the reference's TCP path on input.txt
    (config C1)."""
    ref_dir = os.path.join(REPO, "oracle", "_ref")
    workers = 4
    keys = np.empty(sample_keys, np.int32)
    orc = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
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
    # merge_sort is n log n per chunk, merge_chunks linear: the sample's time scaled to the metric size
    import math
    scale_sort = (target_keys / sample_keys) * math.log2(target_keys / workers) / math.log2(sample_keys / workers)
    est = (t1 - t0) * scale_sort + (t2 - t1) * target_keys / sample_keys
    hi = host_info()
    return {
        "value": sample_keys / (t2 - t0), "unit": "sorted keys/s", "cores": workers, "kind": kind,
        "sample": (f"{sample_keys} uniform int32 keys (seed {SEED:#x}); 4 threads x reference merge_sort "
                   f"on equal chunks ({t1 - t0:.2f} s) + reference merge_chunks incl. output.txt "
                   f"text write ({t2 - t1:.2f} s); chunks sorted={ok}; host {hi['cpu_model']}, "
                   f"nproc={hi['nproc']}, usable={hi['affinity_cpus']}"),
        "host": hi,
        "scaled_to_metric": {"keys": target_keys, "est_seconds": round(est, 2),
                             "est_keys_per_s": target_keys / est,
                             "rule": "sort time x (N/n) x log2(N/4)/log2(n/4) + merge time x N/n"},
        "c1_reference_tcp": reference_tcp_c1(),
    }


# The kernels of the default (bucketed) sort, as rocprofv3 names them, per key width: the stage
# they run (dsort_stats field of their HIP-event time) and their algorithmic bytes per key
# (w = key bytes): the histogram reads every key once, the other three read and write every key
# (the second level and the tile sort only the keys outside single-key buckets).
STAGE_KERNELS = {
    # (round 5: the first level's kernels carry the adaptive-map flag; uniform int32 keys take the
    # fixed map, int64 has one map kind; the scatter's last flag is the sorted-runs instance, which
    # uniform and Zipf keys do not take)
    4: [("bucket_hist_kernel<int, false>", "bucket_hist_ms", 1, "n"),
        ("bucket_scatter_lines_kernel<int, false, false, false>", "bucket_scatter_ms", 2, "n"),
        ("sb_local_kernel<int>", "sub_partition_ms", 2, "tile_sort_keys"),
        ("bin_sort_kernel<int, true, 8>", "tile_sort_kernel_ms", 2, "tile_sort_keys")],
    8: [("bucket_hist_kernel<long, false>", "bucket_hist_ms", 1, "n"),
        ("bucket_scatter_lines_kernel<long, {ids}, false, false>", "bucket_scatter_ms", 2, "n"),
        ("sb_local_kernel<long>", "sub_partition_ms", 2, "tile_sort_keys"),
        ("bin_sort_kernel<long, true, 8>", "tile_sort_kernel_ms", 2, "tile_sort_keys")],
}
# the generator and runtime copies are not part of the sort
NOT_SORT = ("gen_uniform", "gen_zipf", "__amd_rocclr", "fingerprint", "descents")
PMC_FILES = ("r6_pmc_traffic.json", "r5_pmc_traffic.json", "r4_pmc_traffic.json", "r3_pmc_traffic.json", "r2_pmc_traffic.json")


def lib_sha256():
    """sha256 of the libdsort.so this run loads: the PMC tables record the build they measured."""
    import hashlib

    import dsort
    try:
        with open(dsort.LIB_PATH, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def _pmc_doc(w, dist="uniform"):
    """The newest committed rocprofv3 PMC traffic table for key width w (bytes per launch:
    FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md), or None.  `match`
    says whether it was measured on this very library build and key distribution (an
    older table is only an estimate for a newer build)."""
    for name in PMC_FILES:
        path = os.path.join(REPO, "profiles", name)
        try:
            with open(path) as f:
                top = json.load(f)
        except (OSError, ValueError):
            continue
        doc = top
        if w != doc.get("key_bytes", 4) and "int64" in doc:
            doc = dict(doc["int64"])
        if w == doc.get("key_bytes", 4):
            doc["file"] = "profiles/" + name
            sha = top.get("lib_sha256")
            doc["match"] = bool(sha) and sha == lib_sha256() and doc.get("dist", "uniform") == dist
            return doc
    return None


def pmc_traffic(kernel, n, w, dist="uniform"):
    """HBM bytes per sort of `kernel` (all its launches) from the newest PMC table, scaled to this run's key count;
    None when absent, measured on another key width, or on another build / distribution."""
    doc = _pmc_doc(w, dist)
    if not doc or not doc["match"] or kernel not in doc["kernels"]:
        return None
    rec = doc["kernels"][kernel]
    # (per sort when the table has it: the stage times span all of a kernel's launches in a sort)
    return round(rec.get("traffic_bytes_per_sort", rec["traffic_bytes_per_launch"]) * n / doc.get("keys", 1 << 30))


def pmc_sort_bytes(n, w, dist="uniform"):
    """HBM bytes of one whole sort: every kernel of the PMC table but the generator / copies, and
    whether the table was measured on this build and distribution."""
    doc = _pmc_doc(w, dist)
    if not doc:
        return None, None, False
    tot = sum(r.get("traffic_bytes_per_sort", r["traffic_bytes_per_launch"]) for k, r in doc["kernels"].items()
              if not k.startswith(NOT_SORT))
    return round(tot * n / doc.get("keys", 1 << 30)), doc["file"], doc["match"]


# ------------------------------------------------------------------------- GPU runs
def make_input(ctx, n, first, dtype, dist):
    import torch

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
    import torch

    import dsort

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
    # the timed steps run back to back (a sort returns while its last kernels run; nothing is read
    # back in between) with no stage events (DSORT_OPT_STAGE_TIMING = 0: each event costs the GPU a
    # few us between two kernels), then as many steps again, each with its HIP events and followed
    # by a read of them, give the per-stage device times of the roofline (outside the timed region)
    ctx.set_option("stage_timing", 0)
    ctx.sort_dev(t_in, out)  # (untimed: the first sort of this mode)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.sort_dev(t_in, out)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ctx.set_option("stage_timing", 1)
    acc = {k: 0.0 for k in ("merge_kernel_ms", "block_sort_ms", "total_ms", "tile_sort_kernel_ms", "partition_ms",
                            "bucket_hist_ms", "bucket_scatter_ms", "sub_partition_ms")}
    npass, tkeys = 0, 0
    for _ in range(args.steps):
        ctx.sort_dev(t_in, out)
        st = ctx.stats()  # reads the HIP events of this step (syncs the stream)
        for k in acc:
            acc[k] += st[k]
        npass += st["merge_passes"]
        tkeys += st["tile_sort_keys"]
    torch.cuda.synchronize()
    stats = ctx.stats()
    ctx.close()
    # for context, not a baseline of the metric: the same keys through torch.sort (rocPRIM's radix
    # sort of this image's PyTorch), outside the timed region
    lib_ms = None
    try:
        del out
        torch.cuda.empty_cache()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.sort(t_in)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(3):
            torch.sort(t_in)
        e1.record()
        torch.cuda.synchronize()
        lib_ms = e0.elapsed_time(e1) / 3
    except RuntimeError:  # (out of memory on a smaller device: no comparison)
        lib_ms = None
    k = {key: v / max(args.steps, 1) for key, v in acc.items()}  # per step
    k["torch_sort_ms"] = lib_ms
    k.update({"passes": stats["merge_passes"], "npass": npass, "tile": stats["tile_keys"], "w": w,
              "tile_sort_keys": tkeys // max(args.steps, 1), "n": n})
    return t1 - t0, k


def _sync_ok(dist, flag):
    """Every rank's status after a phase of a measurement: the minimum over ranks (gloo), so every
    rank leaves a failed phase together instead of pairing different collectives."""
    import torch

    t = torch.tensor([1 if flag else 0], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def measure_samplesort(ctx, dist, rank, world, n, dtype, distname, steps, warmup, strict=True):
    """One sample-sort workload on the ranks' communicator: n keys in all, split into equal
    contiguous chunks (server.c:185-216), `warmup` untimed sorts, verification (local order, global
    multiset fingerprint, rank boundaries), `steps` timed sorts back to back between two barriers
    (no stage events), then `steps` instrumented sorts for the per-stage device times.  Returns
    (elapsed_max_over_ranks, verified, per_rank table (PR_* columns), key bytes, error).  strict:
    a library error raises (the metric line); else every rank returns it (an extra leg)."""
    import torch

    import dsort

    sz = n // world + (1 if rank < n % world else 0)          # server.c:185-216 partition rule
    first = rank * (n // world) + min(rank, n % world)
    w = 4 if dtype == "i32" else 8
    err = None

    def guarded(fn):
        nonlocal err
        try:
            fn()
            return True
        except dsort.DsortError as e:
            if strict:
                raise
            err = f"rank {rank}: {e}"
            return False

    st_in = {}

    def prepare():
        st_in["t"] = make_input(ctx, sz, first, dtype, distname)
        st_in["fp"] = ctx.fingerprint(st_in["t"])
        for _ in range(max(warmup, 1)):
            st_in["res"] = ctx.sample_sort_dev(st_in["t"])
        ctx.synchronize()

    if not _sync_ok(dist, guarded(prepare)):
        return None, False, None, w, err or "a peer failed"
    t_in, in_fp = st_in["t"], st_in["fp"]
    ptr, nout = st_in["res"]
    # verification outside the timed region: local order, global multiset, rank boundaries
    c, fs, fx = dsort.U64(), dsort.U64(), dsort.U64()
    ctx.check(getattr(ctx.lib, f"dsort_count_descents_{dtype}")(ctx.h, ptr, nout, ctypes.byref(c)))
    ctx.check(getattr(ctx.lib, f"dsort_fingerprint_{dtype}")(ctx.h, ptr, nout, ctypes.byref(fs), ctypes.byref(fx)))
    ends = np.zeros(2, np.int64)
    if nout:
        hb = np.zeros(1, np.int64 if dtype == "i64" else np.int32)
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
    ctx.set_option("stage_timing", 0)  # (no stage events in the timed steps, as at N = 1)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()

    def timed_steps():
        for _ in range(steps):
            ctx.sample_sort_dev(t_in)
        torch.cuda.synchronize()

    ok_t = guarded(timed_steps)
    dist.barrier()
    t1 = time.perf_counter()
    ctx.set_option("stage_timing", 1)
    if not _sync_ok(dist, ok_t):
        return None, False, None, w, err or "a peer failed"
    el = torch.tensor([t1 - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    # per-stage device times from as many instrumented steps again (outside the timed region)
    timed = ("exchange_ms", "alltoall_ms", "final_merge_ms", "merge_kernel_ms", "tile_sort_kernel_ms",
             "bucket_hist_ms", "bucket_scatter_ms", "sub_partition_ms", "total_ms")
    acc = {k: 0.0 for k in timed}
    acc.update({"merge_kernel_launches": 0, "merge_passes": 0, "sent": 0, "tile_sort_keys": 0, "exchange_path": 0})

    def instrumented():
        for _ in range(steps):
            ctx.sample_sort_dev(t_in)
            st = ctx.stats()  # synchronizes this rank's stream
            for k in timed:
                acc[k] += st[k]
            acc["tile_sort_keys"] += st["tile_sort_keys"]
            acc["merge_kernel_launches"] += st["merge_kernel_launches"]
            acc["merge_passes"] += st["merge_passes"]
            acc["sent"] += st["keys_sent"]
            acc["exchange_path"] = st["exchange_path"]
        torch.cuda.synchronize()

    if not _sync_ok(dist, guarded(instrumented)):
        return None, False, None, w, err or "a peer failed"
    # per-rank figures of the roofline, gathered (rank 0 reports the slowest rank)
    st_n = max(steps, 1)
    mine = torch.tensor([acc["tile_sort_kernel_ms"] / st_n, acc["alltoall_ms"] / st_n, acc["exchange_ms"] / st_n,
                         acc["final_merge_ms"] / st_n, acc["sent"] / st_n, sz,
                         acc["bucket_hist_ms"] / st_n, acc["bucket_scatter_ms"] / st_n,
                         acc["sub_partition_ms"] / st_n, acc["tile_sort_keys"] / st_n, acc["exchange_path"],
                         acc["total_ms"] / st_n],
                        dtype=torch.float64)
    everyone = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(everyone, mine)
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
    del t_in, st_in
    torch.cuda.empty_cache()
    return float(el.item()), ok, torch.stack(everyone).numpy(), w, None


# The extra legs of a multi-GPU run (the driver issues one `bench.py --gpus N` per N,
# so the other multi-GPU configs ride on it, after the metric's timed region): BASELINE configs
# C3 (2^32 int32 over 8 GPUs; at N < 8 the same 2^29 keys per GPU), C4 (2^30 Zipf int64 over N)
# and C5 (the C3 size with worker min(3, N-1) killed after its first partition level; through the
# C master, in a child process).  Each leg: 3 timed steps after 1 warmup, an exchange deadline.
LEG_NAMES = ("c3", "c4", "c5")


def leg_plan(world):
    c3_keys = 1 << 32 if world == 8 else (1 << 29) * world
    # (C3's bucket geometry at any N: 1024 global buckets over 8 ranks = 128 buckets of 4M keys per
    # rank; below 8 GPUs the same 128 per rank are forced -- DSORT_OPT_BUCKETS is the global count)
    return {"c3": {"keys": c3_keys, "dtype": "i32", "dist": "uniform", "buckets": 128 * world},
            "c4": {"keys": 1 << 30, "dtype": "i64", "dist": "zipf"},
            # (one GPU: two workers sharing it over the master's relay, a plumbing check at 2^26 keys)
            "c5": ({"keys": c3_keys, "workers": world, "kill_rank": min(3, world - 1), "transport": "rccl"}
                   if world > 1 else {"keys": 1 << 26, "workers": 2, "kill_rank": 1, "transport": "relay"})}


def legs_wanted(args):
    if args.legs in ("", "none"):
        return []
    want = LEG_NAMES if args.legs == "all" else tuple(x for x in args.legs.split(",") if x)
    bad = [x for x in want if x not in LEG_NAMES]
    if bad:
        raise SystemExit(f"bench: unknown --legs {bad} (choose from {LEG_NAMES})")
    return list(want)


def leg_summary(name, spec, world, steps, res):
    """The report of one sort leg (C3 / C4) from measure_samplesort's result, or its error."""
    elapsed, ok, per_rank, w, err = res
    out = {"config": {"c3": "C3", "c4": "C4"}[name], "keys": spec["keys"], "dtype": "int32" if w == 4 else "int64",
           "dist": spec["dist"], "n_gpus": world, "steps": steps}
    if err or elapsed is None:
        out.update({"verified": False, "error": err or "failed"})
        return out
    ns = argparse.Namespace(keys=spec["keys"], steps=steps, warmup=1, dtype=spec["dtype"], dist=spec["dist"],
                            no_cpu_baseline=True)
    full = summarize_multi(ns, world, elapsed, per_rank, w)
    out.update({"verified": bool(ok), "value": full["value"], "unit": "keys/s", "ms_per_step": full["ms_per_step"],
                "workload": full["config"]["workload"], "roofline": full["roofline"]})
    return out


def run_c5_leg(spec, dtype="i32", timeout_s=900):
    """C5 in a child process (bench.py --kill-rank, which runs the C master and its workers): this
    process may have touched the GPU, so the master is started as a child, never exec'd.  The
    master keeps the chunk replicas in POSIX shared memory (/dev/shm): a node whose /dev/shm cannot
    hold them skips the leg with that reason instead of failing the workers mid-run."""
    import shutil

    need = spec["keys"] * (4 if dtype == "i32" else 8)
    try:
        free = shutil.disk_usage("/dev/shm").free
    except OSError:
        free = None
    if free is not None and free < need + (need >> 3):
        return {"config": "C5", "verified": False,
                "error": f"skipped: /dev/shm has {free} bytes free, the replicas need {need}"}
    cmd = [sys.executable, "-u", os.path.abspath(__file__), "--kill-rank", str(spec["kill_rank"]),
           "--gpus", str(spec["workers"]), "--keys", str(spec["keys"]), "--dtype", dtype, "--kill-after-stage", "0"]
    t0 = time.perf_counter()
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"config": "C5", "verified": False, "error": f"timed out after {timeout_s} s"}
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"config": "C5", "verified": False, "error": f"rc {p.returncode}: {(p.stderr or p.stdout)[-600:]}"}
    r = json.loads(lines[-1])
    r["workload_config"] = r.pop("config", None)
    r.update({"config": "C5", "wall_s": round(time.perf_counter() - t0, 1), "transport": spec["transport"]})
    return r


def run_multi(args, rank, world):
    """One rank per GPU: gloo for control, RCCL (inside libdsort) for the key exchange.  Strong
    scaling: the --keys total is split into equal contiguous chunks (server.c:185-216).  Then the
    extra legs (--legs), which do not touch the metric's numbers."""
    import torch
    import torch.distributed as dist

    import dsort

    local = int(os.environ.get("LOCAL_RANK", rank))
    torch.cuda.set_device(local)
    if world == 1 and "MASTER_PORT" not in os.environ:  # --path samplesort, one GPU, no launcher
        os.environ.setdefault("DSORT_BENCH_STORE", os.path.join(tempfile.mkdtemp(prefix="dsort_bench_"), "store"))
    init_group(dist, rank, world)
    ctx = dsort.Context(local)
    uid = [dsort.Context.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    ctx.comm_init(world, rank, uid[0])
    elapsed, ok, per_rank, w, _ = measure_samplesort(ctx, dist, rank, world, args.keys, args.dtype, args.dist,
                                                     args.steps, args.warmup)
    legs = {}
    plan = leg_plan(world)
    for name in legs_wanted(args):
        if name == "c5":
            continue
        spec = plan[name]
        ctx.set_option("comm_timeout_ms", int(args.leg_timeout * 1000))  # (a stuck exchange ends the leg)
        ctx.set_option("buckets", spec.get("buckets", -1))
        t0 = time.perf_counter()
        res = measure_samplesort(ctx, dist, rank, world, spec["keys"], spec["dtype"], spec["dist"], 3, 1, strict=False)
        ctx.set_option("buckets", -1)
        legs[name] = leg_summary(name, spec, world, 3, res)
        legs[name]["wall_s"] = round(time.perf_counter() - t0, 2)
        if res[4]:  # (the communicator may be gone: no further sort leg)
            break
    ctx.set_option("comm_timeout_ms", 0)
    try:
        ctx.comm_destroy()
    except dsort.DsortError:
        pass
    ctx.close()
    torch.cuda.empty_cache()
    dist.barrier()
    if "c5" in legs_wanted(args) and rank == 0:
        # (the other ranks hold no sort memory now and wait at the barrier below)
        legs["c5"] = run_c5_leg(plan["c5"], timeout_s=int(args.leg_timeout * 2))
    dist.barrier()
    dist.destroy_process_group()
    return elapsed, ok, per_rank, w, legs


def result_header(args, world):
    metric = "sorted keys/sec (int32, 2^30 keys)" if args.dtype == "i32" else "sorted keys/sec (int64)"
    return {"metric": metric, "unit": "keys/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "int32" if args.dtype == "i32" else "int64",
            "data": f"synthetic {args.dist} keys, splitmix64(seed={SEED:#x} + global index)"}


def stage_roofline(k, w, n, dist="uniform", drop_pure=False):
    """Per-stage HIP-event times of the sort's kernels (the average launch of each over the timed
    steps) against their algorithmic bytes, and the slowest of them.  drop_pure: the first-level
    scatter writes only the keys outside single-key buckets (round 5: the one-GPU sort, whose second
    level fills those with their key; round 6: the bucket exchange too, whose owners fill them) --
    it reads n keys and writes tile_sort_keys (for a rank of the bucket exchange: its received
    non-pure keys, the same share of its keys in expectation, exact on one GPU)."""
    stages = []
    for kernel, field, per_key, keys_field in STAGE_KERNELS[w]:
        # (int64: the scatter variant that reads the histogram's bucket ids runs on skewed keys --
        # the slot map chooses on the device; the bench's Zipf input takes it, uniform keys do not)
        kernel = kernel.format(ids="true" if dist == "zipf" else "false")
        ms = k.get(field, 0.0)
        if ms <= 0:
            continue
        nb = per_key * w * k[keys_field]
        if drop_pure and field == "bucket_scatter_ms":
            nb = w * (k[keys_field] + k["tile_sort_keys"])
        ach = nb / (ms * 1e-3) / 1e9
        stages.append({"kernel": kernel, "avg_launch_ms": round(ms, 4), "algorithmic_bytes_per_launch": nb,
                       "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                       "traffic": pmc_traffic(kernel, n, w, dist)})
    return stages


def report_single(args, elapsed, k):
    result = result_header(args, 1)
    n = args.keys
    step_ms = 1000.0 * elapsed / args.steps
    result.update({"value": n * args.steps / elapsed, "ms_per_step": step_ms})
    cfg = "C2-style" if args.dtype == "i32" else "C4-style"
    result["config"] = {"workload": f"{cfg} single-GPU sort of {n} {args.dist} {result['dtype']} keys "
                                    f"(BASELINE metric size); tile {k['tile']} keys, {k['passes']} merge passes",
                        "keys": n, "parallelism": "1 GPU"}
    w = k["w"]
    stages = stage_roofline(k, w, n, args.dist, drop_pure=True)
    if stages:  # the bucketed path: the dominant kernel is the slowest stage
        dom = max(stages, key=lambda r: r["avg_launch_ms"])
    else:  # below 2^25 keys: tile sort + merge passes
        tile_ms = k["tile_sort_kernel_ms"]
        nb = 2 * w * k["tile_sort_keys"]
        ach = nb / (tile_ms * 1e-3) / 1e9 if tile_ms > 0 else 0.0
        dom = {"kernel": STAGE_KERNELS[w][3][0], "avg_launch_ms": round(tile_ms, 4),
               "algorithmic_bytes_per_launch": nb, "achieved": round(ach, 1),
               "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(STAGE_KERNELS[w][3][0], n, w, args.dist)}
    roof = {"bound": "hbm", "kernel": dom["kernel"], "achieved": dom["achieved"], "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": dom["frac"], "traffic": dom["traffic"],
            "avg_launch_ms": dom["avg_launch_ms"], "algorithmic_bytes_per_launch": dom["algorithmic_bytes_per_launch"],
            "timing": "HIP events around each kernel launch on the sort's stream, averaged over the timed steps",
            "stages": stages, "tile_sort_keys": k["tile_sort_keys"],
            "partition_ms": round(k["partition_ms"], 3), "device_ms": round(k["total_ms"], 3),
            "merge_passes": k["npass"] // max(args.steps, 1), "merge_kernel_ms": round(k["merge_kernel_ms"], 4),
            "whole_sort_single_pass_bound_frac": round(2 * w * n / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    # SURVEY.md §8d primary: every sort kernel's PMC bytes over the sort's device time
    pb, src, match = pmc_sort_bytes(n, w, args.dist)
    if pb and k["total_ms"] > 0:
        # (a table measured on another build or distribution gives an estimate only, so labelled)
        key = "all_kernels_frac" if match else "all_kernels_frac_estimate"
        roof[key] = round(pb / (k["total_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        roof["all_kernels"] = {"pmc_bytes_per_sort": pb, "device_ms": round(k["total_ms"], 3), "pmc_source": src,
                               "pmc_measured_on_this_build": match,
                               "rule": "sum of FETCH_SIZE x2 + WRITE_SIZE over the sort's kernels / device time "
                                       "of the sort (HIP events, first splitter kernel to last tile) / 8 TB/s"}
    result["roofline"] = roof
    if k.get("torch_sort_ms"):
        result["gpu_library_reference"] = {
            "what": "torch.sort of the same resident keys on the same GPU (rocPRIM radix sort of (key, int64 "
                    "index) pairs -- torch.sort always returns the indices too, so it moves 3x (int32) / 2x "
                    "(int64) the bytes of a keys-only sort: not like for like); for context, outside the "
                    "timed region",
            "ms": round(k["torch_sort_ms"], 3), "keys_per_s": n / (k["torch_sort_ms"] * 1e-3),
            "speedup_of_value": round(k["torch_sort_ms"] / step_ms, 3)}
    if not args.no_cpu_baseline and args.dtype == "i32":
        result["cpu_baseline"] = cpu_baseline(args.cpu_sample_keys, n)
    print(json.dumps(result), flush=True)


# columns of run_multi's per-rank rows (report_multi)
PR_TILE, PR_A2A, PR_EXCH, PR_FINAL, PR_SENT, PR_KEYS, PR_HIST, PR_SCAT, PR_SUB, PR_TKEYS, PR_PATH, PR_TOTAL = range(12)


def multi_all_kernels(per_rank, w, world, dist):
    """SURVEY.md §8d's primary figure at N > 1: every rank's sort kernels' HBM bytes (the PMC table
    of the one-GPU sort, bytes per key scaled to the rank's keys: a rank runs the same kernels on its
    chunk and on the keys it receives) plus the exchange's own HBM traffic (the bytes a rank ships
    are read once and written once at the receiver), over the slowest rank's device time, against
    the aggregate HBM peak (N x 8 TB/s).  None when there is no PMC table of this key width, or for
    skewed keys: the one-GPU out-of-place sort drops the keys of single-key buckets in
    its scatter, the bucket exchange writes every key, so the one-GPU table would misstate them."""
    if dist != "uniform":
        return None
    tot, src, match = 0, None, True
    for r in range(world):
        pb, src, m = pmc_sort_bytes(int(per_rank[r, PR_KEYS]), w, dist)
        if pb is None:
            return None
        match &= bool(m)  # (measured only when every rank's figure is)
        tot += pb + 2 * w * int(per_rank[r, PR_SENT])
    dev = float(per_rank[:, PR_TOTAL].max())
    if dev <= 0:
        return None
    frac = round(tot / (dev * 1e-3) / 1e9 / (HBM_PEAK_GBS * world), 4)
    return {"frac": frac, "measured": bool(match),
            "detail": {"pmc_bytes_all_ranks": int(tot), "device_ms_slowest_rank": round(dev, 3), "pmc_source": src,
                       "pmc_measured_on_this_build": bool(match),
                       "rule": "sum over ranks of (PMC bytes per key of the one-GPU sort's kernels x the rank's keys "
                               "+ 2 x key bytes shipped) / slowest rank's device time / (N x 8 TB/s)"}}


def report_multi(args, world, elapsed, per_rank, w, legs=None):
    result = summarize_multi(args, world, elapsed, per_rank, w)
    if legs:
        result["legs"] = legs
    if not args.no_cpu_baseline and args.dtype == "i32":
        # the reference's CPU path beside the N-GPU number (rank 0, after the timed region and the
        # other ranks' exit): the same leg as N = 1
        result["cpu_baseline"] = cpu_baseline(args.cpu_sample_keys, args.keys)
    print(json.dumps(result), flush=True)


def summarize_multi(args, world, elapsed, per_rank, w):
    result = result_header(args, world)
    n = args.keys
    step_ms = 1000.0 * elapsed / args.steps
    result.update({"value": n * args.steps / elapsed, "ms_per_step": step_ms})
    bx = int(per_rank[0, 10]) == 1
    how = ("bucket exchange: global splitters, first partition level of the unsorted chunk, RCCL all-to-all of "
           "buckets over xGMI, second level + tile sort of the received buckets" if bx else
           "local sort, splitters, RCCL all-to-all over xGMI, merge of the received runs")
    result["config"] = {"workload": f"sample sort of {n} {args.dist} {result['dtype']} keys over {world} GPUs "
                                    f"(equal contiguous chunks; {how})",
                        "keys": n, "keys_per_gpu": n // world, "parallelism": f"samplesort x{world}",
                        "exchange_path": "bucket exchange" if bx else "sort + merge"}
    # the local sort's stages on every rank (HIP events); the dominant kernel is the slowest stage
    # of the slowest rank
    best = None
    for r in range(world):
        kr = {"tile_sort_kernel_ms": float(per_rank[r, 0]), "bucket_hist_ms": float(per_rank[r, 6]),
              "bucket_scatter_ms": float(per_rank[r, 7]), "sub_partition_ms": float(per_rank[r, 8]),
              "n": float(per_rank[r, 5]), "tile_sort_keys": float(per_rank[r, 9])}
        for st in stage_roofline(kr, w, int(kr["n"]), args.dist, drop_pure=True):
            if best is None or st["avg_launch_ms"] > best[1]["avg_launch_ms"]:
                best = (r, st)
    if best is None:  # below 2^25 keys per rank: the tile sort
        slow = int(np.argmax(per_rank[:, 0]))
        tile_ms, n_gpu = float(per_rank[slow, 0]), float(per_rank[slow, 5])
        bpl = 2 * w * n_gpu
        ach = bpl / (tile_ms * 1e-3) / 1e9 if tile_ms > 0 else 0.0
        best = (slow, {"kernel": STAGE_KERNELS[w][3][0], "avg_launch_ms": round(tile_ms, 4),
                       "algorithmic_bytes_per_launch": int(bpl), "achieved": round(ach, 1),
                       "frac": round(ach / HBM_PEAK_GBS, 4),
                       "traffic": pmc_traffic(STAGE_KERNELS[w][3][0], int(n_gpu), w, args.dist)})
    rk, dom = best
    roof = {"bound": "hbm", "kernel": dom["kernel"] + f" (local sort, rank {rk}: the slowest stage of any rank)",
            "achieved": dom["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": dom["frac"],
            "traffic": dom["traffic"], "avg_launch_ms": dom["avg_launch_ms"],
            "algorithmic_bytes_per_launch": int(dom["algorithmic_bytes_per_launch"]),
            "whole_sort_single_pass_bound_frac": round(
                2 * w * n / (step_ms * 1e-3) / 1e9 / (HBM_PEAK_GBS * world), 4)}
    if world > 1:
        # the all-to-all: every GPU ships w * N_g * (P-1)/P bytes to its P-1 peers, one xGMI link
        # each; the slowest rank's transfer time against (P-1) links x 153 GB/s
        sent = per_rank[:, 4] * w
        a2a = per_rank[:, 1]
        r = int(np.argmax(a2a))
        xg = sent[r] / (a2a[r] * 1e-3) / 1e9 if a2a[r] > 0 else None
        peak = (world - 1) * XGMI_LINK_GBS
        roof["xgmi"] = {"achieved": round(xg, 1) if xg else None, "peak": peak, "unit": "GB/s",
                        "frac": round(xg / peak, 4) if xg else None,
                        "algorithmic_bytes_per_gpu": int(w * (n // world) * (world - 1) / world),
                        "measured_bytes_slowest_rank": int(sent[r]),
                        "alltoall_ms": round(float(a2a[r]), 4),
                        "exchange_stage_ms": round(float(per_rank[:, 2].max()), 4),
                        ("received_buckets_sort_ms" if bx else "final_merge_ms"): round(float(per_rank[:, 3].max()), 4)}
    ak = multi_all_kernels(per_rank, w, world, args.dist)
    if ak:
        # (measured when the PMC table was taken on this very build and key distribution; else an estimate)
        roof["all_kernels_frac" if ak["measured"] else "all_kernels_frac_estimate"] = ak["frac"]
        roof["all_kernels"] = ak["detail"]
    roof["device_ms_per_rank"] = [round(float(x), 3) for x in per_rank[:, PR_TOTAL]]
    result["roofline"] = roof
    return result


def run_fault(args):
    """BASELINE config C5 through the C master (dsort_master --mode samplesort, server.c's role,
    driven by ftsort.fault_run): a fault-free run, then a run in which worker `--kill-rank` dies in
    its local sort (after stage --kill-after-stage) or inside the key exchange; the master
    sees it (socket EOF / exit / heartbeat), reassigns its chunk from the pinned replica by the
    reference's rule, and the survivors abort the communicator, rebuild it and finish."""
    import ftsort

    ndev = _device_count()
    share = args.gpus > ndev  # one GPU box: the workers share it and exchange through the master
    devices = "share" if share else list(range(args.gpus))
    transport = "relay" if share else "rccl"
    r = ftsort.fault_run(args.gpus, args.keys, args.kill_rank, args.kill_after_stage,
                         "i32" if args.dtype == "i32" else "i64", args.dist, transport, devices, args.reassign,
                         stage=args.kill_stage)
    if not r["ok"]:
        raise SystemExit(f"bench: fault run failed verification: {json.dumps(r)}")
    free, fault = r["fault_free"], r["fault"]
    out = {"metric": "recovery time after one GPU worker failure mid-sort (BASELINE config C5)",
           "value": round(r["recovery_ms"], 3), "unit": "ms", "n_gpus": args.gpus, "higher_is_better": False,
           "dtype": "int32" if args.dtype == "i32" else "int64", "data": f"synthetic {args.dist} keys",
           "config": {"workload": f"sample sort of {args.keys} keys over {args.gpus} workers, worker "
                                  f"{args.kill_rank} killed in the {args.kill_stage} stage",
                      "transport": transport, "reassign": args.reassign, "devices": devices},
           "fault_free_ms": round(free["t_end_ms"], 3), "fault_ms": round(fault["t_end_ms"], 3),
           "fault_free_keys_per_s": args.keys / (free["t_end_ms"] * 1e-3),
           "fault_keys_per_s": args.keys / (fault["t_end_ms"] * 1e-3),
           "fault_seen_by_master_ms": fault["t_fault_seen_ms"],
           "survivors_notified_ms": fault["t_survivors_notified_ms"],
           "rebuild_ms": fault["t_rebuild_ms"], "owners": fault["owners"], "slices": fault["slices"],
           "verified": True}
    print(json.dumps(out), flush=True)


def _device_count():
    import torch

    return torch.cuda.device_count()  # does not initialise the GPU on this image


def run_codec(args):
    """the reference's text I/O on the GPU.  Formats `--keys` sorted uniform int32
    keys to output.txt bytes (server.c:517-519) and parses them back (server.c:179/213's %d
    tokens), each timed over `--steps` calls with the data resident in HBM; verifies the round
    trip.  The CPU leg times the oracle's single-threaded codec on a 2^24-key sample."""
    import torch

    import dsort

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


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.kill_rank is not None:
        if "WORLD_SIZE" in os.environ:
            raise SystemExit("--kill-rank runs its own master and workers: launch it without torchrun")
        run_fault(args)
        return 0
    if args.codec:
        run_codec(args)
        return 0
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, argv, check_devices=not args.launcher_selftest)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.launcher_selftest:
        launcher_selftest()
        return 0
    if args.gpus != world:
        raise SystemExit(f"bench: --gpus {args.gpus} but {world} rank process(es) (WORLD_SIZE); "
                         "they must match (one rank per GPU)")
    path = args.path if args.path != "auto" else ("single" if world == 1 else "samplesort")
    if path == "single":
        if world != 1:
            raise SystemExit("bench: --path single runs on one GPU")
        elapsed, k = run_single(args)
        report_single(args, elapsed, k)
        return 0
    elapsed, ok, per_rank, w, legs = run_multi(args, rank, world)
    if rank == 0:
        if not ok:
            raise SystemExit("bench: distributed output failed verification")
        report_multi(args, world, elapsed, per_rank, w, legs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
