"""ftsort -- Python harness of the fault-tolerant multi-GPU sample sort (BASELINE config C5).

The product is C: `dsort_master --mode samplesort` (host/ss_master.c, server.c's role: owns the
chunk replicas in pinned shared memory, spawns one `dsort_worker --mode samplesort` per GPU, ships
the RCCL unique id over its TCP control socket, supervises, reassigns a dead worker's chunk by the
reference's rule, server.c:368-384) and the workers (host/ss_worker.c, client.c's role).  This
module only runs that binary and reads its JSON line, for bench.py (--kill-rank) and the tests.
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
MASTER = os.path.join(HERE, "bin", "dsort_master")


def chunk_range(n_total, world, rank):
    """Equal contiguous chunks, the remainder on the lowest ranks (server.c:185-216)."""
    q, r = divmod(n_total, world)
    return q + (1 if rank < r else 0), rank * q + min(rank, r)


def reassign(dead, world, rule="first-live"):
    """Survivor that takes each dead rank's chunk (the C master's rule, for test expectations).
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


def run_master(nworkers, n_total, dtype="i32", dist="uniform", transport="rccl", devices=None,
               rule="first-live", kill_rank=None, kill_stage="sort", kill_after_stage=0,
               kill_exchange_stage=2, output=None, timeout_s=600, extra=(), env=None, kill_in_recovery=None):
    """One run of the C master; returns its JSON report (plus 'stderr_tail')."""
    cmd = [MASTER, "--mode", "samplesort", "--gpus", str(nworkers), "--keys", str(n_total),
           "--dtype", dtype, "--dist", dist, "--transport", transport, "--reassign", rule]
    if devices is not None:
        cmd += ["--devices", devices if isinstance(devices, str) else ",".join(str(d) for d in devices)]
    if kill_rank is not None:
        cmd += ["--kill-rank", str(kill_rank), "--kill-stage", kill_stage]
        cmd += ["--kill-after-stage", str(kill_after_stage)] if kill_stage == "sort" else \
               ["--kill-exchange-stage", str(kill_exchange_stage)]
    if kill_in_recovery is not None:
        cmd += ["--kill-in-recovery", str(kill_in_recovery)]
    if output:
        cmd += ["--output", output]
    cmd += list(extra)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s,
                       env=dict(os.environ if env is None else env, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"ss_result"')]
    if not lines:
        raise RuntimeError(f"dsort_master gave no report (rc {p.returncode}):\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}")
    rep = json.loads(lines[-1])
    rep["stderr_tail"] = p.stderr[-2000:]
    rep["stdout_tail"] = p.stdout[-2000:]
    return rep


def fault_run(nworkers, n_total, kill_rank, kill_after_stage, dtype="i32", dist="uniform", transport="rccl",
              devices=None, rule="first-live", stage="sort", kill_exchange_stage=2):
    """A fault-free run, then a run with `kill_rank` dying in its local sort (after stage
    `kill_after_stage`, dsort.h DSORT_OPT_KILL_AFTER_STAGE) or inside the exchange; recovery time =
    the difference of the two ends
    (each the slowest survivor's DONE at the master, from GO)."""
    free = run_master(nworkers, n_total, dtype, dist, transport, devices, rule)
    fault = run_master(nworkers, n_total, dtype, dist, transport, devices, rule, kill_rank=kill_rank,
                       kill_stage=stage, kill_after_stage=kill_after_stage, kill_exchange_stage=kill_exchange_stage)
    return {"fault_free": free, "fault": fault, "recovery_ms": fault["t_end_ms"] - free["t_end_ms"],
            "ok": free["ok"] and fault["ok"] and fault["dead"] == [kill_rank]}
