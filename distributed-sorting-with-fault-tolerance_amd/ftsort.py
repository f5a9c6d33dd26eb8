"""ftsort -- fault-tolerant multi-GPU sample sort (BASELINE config C5).

The reference's fault tolerance lives in its master (server.c:297-477):

  * the master holds every chunk (server.c:185-216);
  * a worker whose send/recv fails is marked dead (server.c:358-365, 421-427);
  * its chunk is re-sent to the first live worker after a 100 ms pause (server.c:368-391,
    430-446);
  * the sorted chunk still lands in the chunk's own result slot (server.c:415).

This module keeps that rule for the GPU path.

Master (server.c's role; this process, no GPU work):
  * hosts the control store (torch.distributed.TCPStore) and spawns one worker process per GPU;
  * keeps a replica of every chunk in host shared memory (/dev/shm), the analogue of server.c's
    chunks[];
  * detects a worker's death by waitpid, or a hung worker by a stale heartbeat (which it then
    kills);
  * publishes the recovery plan: the dead ranks, the survivors, and who takes which dead chunk.
    The rule is "first-live", the first live rank in index order as in server.c:368-384, or
    "next-live", the next live rank after the dead one.

Worker (client.c's role; one process per GPU):
  * sorts its chunk with libdsort (block sort + merge passes);
  * runs the sample-sort exchange (RCCL all-to-all, or the host transport when ranks share a GPU);
  * merges the key range it owns.

After a fault, the survivors:
  1. abort the communicator and build a new one over the survivors;
  2. the assignee loads the dead chunk from its replica, sorts it and merges it into its own run;
  3. all survivors run the exchange over P-1 ranks.

The output is the concatenation of the survivors' slices in their new rank order.

Timing: every phase time is taken against one "go" timestamp the master publishes. For a fault
run, recovery time = (fault run end) - (fault-free run end); the end is the slowest worker's.
"""
import ctypes
import json
import os
import signal
import subprocess
import sys
import tempfile
import threading
import time
from datetime import timedelta

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SEED = 0x5EED2026


def chunk_range(n_total, world, rank):
    """Equal contiguous chunks, the remainder on the lowest ranks (server.c:185-216)."""
    q, r = divmod(n_total, world)
    return q + (1 if rank < r else 0), rank * q + min(rank, r)


def reassign(dead, world, rule="first-live"):
    """Survivor that takes each dead rank's chunk.
    first-live: the first live rank in index order (server.c:368-384 scans is_alive from 0);
    next-live: the next live rank after the dead one (cyclic), which spreads several failures."""
    live = [r for r in range(world) if r not in dead]
    if not live:
        raise RuntimeError("no live worker left (server.c:387-389 gives up the same way)")
    out = {}
    for d in sorted(dead):
        if rule == "first-live":
            out[d] = live[0]
        elif rule == "next-live":
            out[d] = next((r for r in live if r > d), live[0])
        else:
            raise ValueError(f"unknown reassignment rule {rule!r}")
    return out


def replica_path(job, rank):
    return f"/dev/shm/dsort-{job}-chunk{rank}.bin"


# ------------------------------------------------------------------------------------ worker
class _Comm:
    """The sample sort's communicator for one epoch: RCCL over `ranks` (one GPU per rank), or the
    host transport over a gloo group built from the store (ranks sharing a GPU)."""

    def __init__(self, ctx, store, transport, epoch, ranks, me, timeout_s=30.0):
        import torch.distributed as tdist

        import dsort

        self.ctx = ctx
        self.world = len(ranks)
        self.rank = ranks.index(me)
        self.transport = transport
        if transport == "rccl":
            key = f"uid/{epoch}"
            if self.rank == 0:
                store.set(key, dsort.Context.unique_id())
            uid = store.get(key)
            ctx.comm_init(self.world, self.rank, bytes(uid))
        else:
            pg = tdist.ProcessGroupGloo(tdist.PrefixStore(f"pg{epoch}/", store), self.rank, self.world,
                                        timedelta(seconds=timeout_s))
            self.pg = pg
            ctx.comm_init_transport(self.world, self.rank, dsort.torch_dist_transport(self.world, pg))

    def abort(self):
        self.ctx.comm_abort()


def _dev_checks(ctx, ptr, n, sfx):
    import dsort

    c, fs, fx = dsort.U64(), dsort.U64(), dsort.U64()
    first = last = 0
    if n:
        ctx.check(getattr(ctx.lib, f"dsort_count_descents_{sfx}")(ctx.h, ptr, n, ctypes.byref(c)))
        ctx.check(getattr(ctx.lib, f"dsort_fingerprint_{sfx}")(ctx.h, ptr, n, ctypes.byref(fs), ctypes.byref(fx)))
        hb = np.zeros(1, np.int64 if sfx == "i64" else np.int32)
        ctx.copy_d2h(hb, ptr, hb.itemsize)
        first = int(hb[0])
        ctx.copy_d2h(hb, ptr + (n - 1) * hb.itemsize, hb.itemsize)
        last = int(hb[0])
    return {"descents": c.value, "fp_sum": fs.value, "fp_xor": fx.value, "first": first, "last": last}


def worker_main(rank, world, port, n_total, dtype, dist, transport, device, job, kill_after_pass):
    """One GPU worker (client.c's role).  Reports through the store; returns nothing."""
    import torch
    import torch.distributed as tdist

    import dsort

    store = tdist.TCPStore("127.0.0.1", port, None, False, timedelta(seconds=120))
    torch.cuda.set_device(device)
    ctx = dsort.Context(device)
    sfx = dtype
    tdt = torch.int32 if dtype == "i32" else torch.int64
    sz, first = chunk_range(n_total, world, rank)
    chunk = torch.empty(max(sz, 1), dtype=tdt, device="cuda")[:sz]
    if dist == "zipf":
        ctx.gen_zipf_i64(chunk, SEED, first)
    else:
        ctx.gen_uniform(chunk, SEED, first)
    fp_in = ctx.fingerprint(chunk) if sz else (0, 0)
    chunk.cpu().numpy().tofile(replica_path(job, rank))  # the master's copy of chunk `rank`
    comm = _Comm(ctx, store, transport, 0, list(range(world)), rank)
    torch.cuda.synchronize()

    stop = threading.Event()

    def heartbeat():
        while not stop.is_set():
            store.set(f"hb/{rank}", str(time.time()))
            stop.wait(0.05)

    threading.Thread(target=heartbeat, daemon=True).start()
    store.set(f"ready/{rank}", json.dumps({"fp_sum": fp_in[0], "fp_xor": fp_in[1], "n": sz}))
    store.wait(["go"])
    t_go = float(store.get("go"))

    # ---- local sort (the fault, if injected, strikes inside this call: after merge pass k)
    if kill_after_pass is not None:
        os.environ["DSORT_INJECT_KILL_AFTER_PASS"] = str(kill_after_pass)
    run = torch.empty_like(chunk)
    if sz:
        ctx.sort_dev(chunk, run)
    torch.cuda.synchronize()
    t_sorted = time.time()
    os.environ.pop("DSORT_INJECT_KILL_AFTER_PASS", None)
    store.set(f"sorted/0/{rank}", "1")

    # ---- wait for every worker's run, or for the master's recovery plan
    keys = [f"sorted/0/{r}" for r in range(world)]
    plan = None
    while True:
        if store.check(["plan/1"]):
            plan = json.loads(store.get("plan/1"))
            break
        if store.check(keys):
            break
        time.sleep(0.0002)
    t_detect = None
    if plan is None:
        try:
            ptr, nout = ctx.sample_merge_dev(run)
            torch.cuda.synchronize()
        except dsort.DsortError:
            # a worker died inside the exchange: the master publishes a plan
            store.wait(["plan/1"])
            plan = json.loads(store.get("plan/1"))
    if plan is not None:
        t_detect = time.time()
        comm.abort()
        survivors = plan["survivors"]
        comm = _Comm(ctx, store, transport, 1, survivors, rank)
        for d, a in plan["assign"].items():
            if a != rank:
                continue
            dsz, _ = chunk_range(n_total, world, int(d))
            host = np.fromfile(replica_path(job, int(d)), dtype=np.int32 if dtype == "i32" else np.int64)
            assert host.size == dsz
            extra = torch.from_numpy(host).to("cuda")
            both = torch.empty(run.numel() + dsz, dtype=tdt, device="cuda")
            both[:run.numel()].copy_(run)
            if dsz:
                ctx.sort_dev(extra, both[run.numel():])
            merged = torch.empty_like(both)
            ctx.merge_dev(both, [run.numel(), dsz], merged)
            run = merged
        torch.cuda.synchronize()
        ptr, nout = ctx.sample_merge_dev(run)
        torch.cuda.synchronize()
    t_done = time.time()
    res = {"rank": rank, "new_rank": comm.rank, "n_out": nout, "t_sorted": t_sorted - t_go,
           "t_detect": (t_detect - t_go) if t_detect else None, "t_done": t_done - t_go,
           "run_keys": int(run.numel())}
    res.update(_dev_checks(ctx, ptr, nout, sfx))
    store.set(f"res/{rank}", json.dumps(res))
    store.wait(["exit"])
    stop.set()
    try:
        ctx.comm_destroy()
    except dsort.DsortError:
        pass
    ctx.close()


# ------------------------------------------------------------------------------------ master
class Master:
    """server.c's role for the GPU workers: spawn, watch, reassign, verify."""

    def __init__(self, nworkers, n_total, dtype="i32", dist="uniform", transport="rccl", devices=None,
                 rule="first-live", heartbeat_timeout=5.0, log_dir=None, worker_cmd=None):
        self.world = nworkers
        self.n = n_total
        self.dtype = dtype
        self.dist = dist
        self.transport = transport
        self.devices = devices if devices is not None else list(range(nworkers))
        self.rule = rule
        self.hb_timeout = heartbeat_timeout
        self.log_dir = log_dir or tempfile.mkdtemp(prefix="dsort-ft-")
        # the worker program (argv prefix); tests substitute a CPU test double here
        self.worker_cmd = worker_cmd or [sys.executable, "-u", os.path.abspath(__file__), "worker"]

    def run(self, kill_rank=None, kill_after_pass=None, timeout_s=300.0):
        import torch.distributed as tdist

        job = f"{os.getpid()}-{int(time.time() * 1e6) % 10**9}"
        store = tdist.TCPStore("127.0.0.1", 0, None, True, timedelta(seconds=120), wait_for_workers=False)
        port = store.port
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        env.pop("DSORT_INJECT_KILL_AFTER_PASS", None)
        procs, logs = [], []
        for r in range(self.world):
            kp = kill_after_pass if r == kill_rank else None
            log = open(os.path.join(self.log_dir, f"worker{r}.log"), "w")
            cmd = self.worker_cmd + [str(r), str(self.world), str(port),
                   str(self.n), self.dtype, self.dist, self.transport, str(self.devices[r]), job,
                   "none" if kp is None else str(kp)]
            procs.append(subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT))
            logs.append(log)
        t_limit = time.time() + timeout_s
        try:
            return self._supervise(store, procs, job, kill_rank, t_limit)
        finally:
            try:
                store.set("exit", "1")
            except Exception:
                pass
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            for lg in logs:
                lg.close()
            for r in range(self.world):
                try:
                    os.unlink(replica_path(job, r))
                except OSError:
                    pass

    def _dead(self, store, procs, dead):
        """Workers that exited without reporting, or whose heartbeat is stale (then killed)."""
        now = time.time()
        out = set()
        for r, p in enumerate(procs):
            if r in dead:
                continue
            if p.poll() is not None and not store.check([f"res/{r}"]):
                out.add(r)
            elif store.check([f"hb/{r}"]) and now - float(store.get(f"hb/{r}")) > self.hb_timeout:
                p.send_signal(signal.SIGKILL)  # fence the hung worker before its chunk moves
                out.add(r)
        return out

    def _supervise(self, store, procs, job, kill_rank, t_limit):
        ready = [f"ready/{r}" for r in range(self.world)]
        while not store.check(ready):
            if any(p.poll() is not None for p in procs):
                raise RuntimeError(f"a worker exited during start-up; logs in {self.log_dir}")
            if time.time() > t_limit:
                raise TimeoutError("workers did not start")
            time.sleep(0.01)
        inputs = [json.loads(store.get(k)) for k in ready]
        t_go = time.time()
        store.set("go", repr(t_go))
        dead, t_fault = set(), None
        plan = None
        while True:
            newly = self._dead(store, procs, dead)
            if newly:
                if plan is not None:
                    raise RuntimeError("a second failure during recovery is not handled")
                t_fault = time.time() - t_go
                dead |= newly
                survivors = [r for r in range(self.world) if r not in dead]
                assign = reassign(dead, self.world, self.rule)
                plan = {"dead": sorted(dead), "survivors": survivors,
                        "assign": {str(d): a for d, a in assign.items()}}
                store.set("plan/1", json.dumps(plan))
            live = [r for r in range(self.world) if r not in dead]
            if store.check([f"res/{r}" for r in live]):
                break
            if time.time() > t_limit:
                raise TimeoutError(f"sort did not finish; logs in {self.log_dir}")
            time.sleep(0.0005)
        res = [json.loads(store.get(f"res/{r}")) for r in live]
        res.sort(key=lambda x: x["new_rank"])
        m = (1 << 64) - 1
        ok = all(x["descents"] == 0 for x in res)
        ok &= sum(x["n_out"] for x in res) == self.n
        ok &= sum(i["fp_sum"] for i in inputs) & m == sum(x["fp_sum"] for x in res) & m
        xi = xo = 0
        for i in inputs:
            xi ^= i["fp_xor"]
        for x in res:
            xo ^= x["fp_xor"]
        ok &= xi == xo
        nz = [x for x in res if x["n_out"]]
        ok &= all(a["last"] <= b["first"] for a, b in zip(nz, nz[1:]))
        detect = [x["t_detect"] for x in res if x["t_detect"] is not None]
        return {
            "ok": bool(ok), "world": self.world, "n": self.n, "dead": sorted(dead), "plan": plan,
            "t_end_ms": 1e3 * max(x["t_done"] for x in res),
            "t_local_sort_ms": 1e3 * max(x["t_sorted"] for x in res),
            "t_fault_seen_ms": None if t_fault is None else 1e3 * t_fault,
            "t_survivors_notified_ms": 1e3 * min(detect) if detect else None,
            "slices": [x["n_out"] for x in res],
        }


def fault_run(nworkers, n_total, kill_rank, kill_after_pass, dtype="i32", dist="uniform", transport="rccl",
              devices=None, rule="first-live"):
    """A fault-free run then a run with `kill_rank` dying after merge pass `kill_after_pass` of its
    local sort; returns both reports and the recovery time (BASELINE config C5)."""
    m = Master(nworkers, n_total, dtype, dist, transport, devices, rule)
    free = m.run()
    fault = m.run(kill_rank=kill_rank, kill_after_pass=kill_after_pass)
    return {"fault_free": free, "fault": fault, "recovery_ms": fault["t_end_ms"] - free["t_end_ms"],
            "ok": free["ok"] and fault["ok"] and fault["dead"] == [kill_rank]}


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "worker":
    sys.path.insert(0, HERE)
    a = sys.argv[2:]
    worker_main(int(a[0]), int(a[1]), int(a[2]), int(a[3]), a[4], a[5], a[6], int(a[7]), a[8],
                None if a[9] == "none" else int(a[9]))
