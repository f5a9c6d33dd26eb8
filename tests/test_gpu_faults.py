"""Fault machinery of the library on the MI355X (pytest -m gpu):

  * the kill points of a local sort (DSORT_OPT_KILL_AFTER_STAGE, dsort.h): every stage of the
    bucketed path (>= 2^25 keys: first-level partition, second-level partition, tile sort) and of
    the merge path really SIGKILLs the process after that stage, and a stage the sort never reaches
    is an error (DSORT_ESTAGE), not a silent fault-free run -- the reference's fault moment is "any
    time the socket fails" (server.c:358-395, 421-449);
  * the RCCL communicator's abort and rebuild (the survivor path of server.c:421-449 in the
    multi-GPU design): a non-blocking communicator is built, sorts, is aborted from a second thread
    (ncclCommAbort), and a fresh one (new unique id, ncclCommInitRankConfig) sorts again -- at one
    rank, the size of this box."""
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

from conftest import PKG, REPO

sys.path.insert(0, PKG)
pytestmark = pytest.mark.gpu
SEED = 0x5EED2026

_KILL_CHILD = r"""
import sys
sys.path.insert(0, {pkg!r})
import torch
import dsort
n, w, stage = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
ctx = dsort.Context(0)
t = torch.empty(n, dtype=torch.int32 if w == 4 else torch.int64, device="cuda")
ctx.gen_uniform(t, {seed}, 0)
out = torch.empty_like(t)
torch.cuda.synchronize()
print("stages", ctx.sort_stages(n, w), flush=True)
ctx.set_option("kill_after_stage", stage)
try:
    ctx.sort_dev(t, out)
    torch.cuda.synchronize()
    print("returned ok", flush=True)
except dsort.DsortError as e:
    print("error", e, flush=True)
    sys.exit(3)
"""


def _kill_child(n, w, stage):
    code = _KILL_CHILD.format(pkg=PKG, seed=SEED)
    return subprocess.run([sys.executable, "-c", code, str(n), str(w), str(stage)], capture_output=True, text=True,
                          timeout=120, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


@pytest.mark.parametrize("n,w,stage", [(1 << 25, 4, 0), (1 << 25, 4, 1), (1 << 25, 4, 2), (1 << 25, 8, 1),
                                       (1 << 20, 4, 0), (1 << 20, 4, 2)])
def test_kill_point_fires(n, w, stage):
    p = _kill_child(n, w, stage)
    assert p.returncode == -9, p.stdout + p.stderr  # SIGKILL, after the stage finished
    assert "returned ok" not in p.stdout


@pytest.mark.parametrize("n,w,stage", [(1 << 25, 4, 3), (1 << 20, 4, 3), (1, 4, 0)])
def test_unreachable_kill_point_is_an_error(n, w, stage):
    p = _kill_child(n, w, stage)
    assert p.returncode == 3 and "ESTAGE" in p.stdout and "stages" in p.stdout, p.stdout + p.stderr


def _sorted_slice_ok(ctx, ptr, nout, fp_in):
    import ctypes

    import dsort
    c, fs, fx = dsort.U64(), dsort.U64(), dsort.U64()
    ctx.check(ctx.lib.dsort_count_descents_i32(ctx.h, ptr, nout, ctypes.byref(c)))
    ctx.check(ctx.lib.dsort_fingerprint_i32(ctx.h, ptr, nout, ctypes.byref(fs), ctypes.byref(fx)))
    return c.value == 0 and (fs.value, fx.value) == fp_in


def test_rccl_abort_and_rebuild_one_rank(gpu_ctx):
    """dsort_comm_init (non-blocking RCCL) -> sample sort -> dsort_comm_abort from a second thread
    while a sample sort runs -> the communicator is gone (DSORT_ECOMM) -> dsort_comm_init with a new
    unique id -> sample sort again (dsort_api.hip: abort_comm_locked, exch_wait, dsort_comm_init)."""
    import torch

    import dsort
    ctx = gpu_ctx
    n = 1 << 26
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.gen_uniform(t, SEED, 0)
    fp_in = ctx.fingerprint(t)
    ctx.comm_init(1, 0, dsort.Context.unique_id())
    ptr, nout = ctx.sample_sort_dev(t)
    ctx.synchronize()
    assert nout == n and _sorted_slice_ok(ctx, ptr, nout, fp_in)
    res = {}

    def run():
        try:
            res["ok"] = ctx.sample_sort_dev(t)
            ctx.synchronize()
        except dsort.DsortError as e:
            res["err"] = str(e)

    th = threading.Thread(target=run)
    th.start()
    time.sleep(0.003)
    ctx.comm_abort()  # another thread: raises the flag (exchange running) or aborts the idle comm
    th.join(60)
    assert not th.is_alive()
    assert "ok" in res or "ECOMM" in res["err"], res
    # the communicator is gone either way (an abort that came after the exchange is taken by the
    # next call)
    with pytest.raises(dsort.DsortError, match="ECOMM"):
        ctx.sample_sort_dev(t)
    ctx.comm_init(1, 0, dsort.Context.unique_id())  # a fresh ncclCommInitRankConfig
    ptr, nout = ctx.sample_sort_dev(t)
    ctx.synchronize()
    assert nout == n and _sorted_slice_ok(ctx, ptr, nout, fp_in)
    # idle abort (ncclCommAbort on a live communicator), then re-init once more, then destroy
    ctx.comm_abort()
    ctx.comm_init(1, 0, dsort.Context.unique_id())
    ptr, nout = ctx.sample_sort_dev(t)
    ctx.synchronize()
    assert _sorted_slice_ok(ctx, ptr, nout, fp_in)
    ctx.comm_destroy()
    del t
    torch.cuda.empty_cache()


def test_rccl_abort_frees_a_survivor_blocked_in_the_exchange(gpu_ctx):
    """The survivor side of server.c:421-449 in the multi-GPU design, deterministic: with
    DSORT_OPT_TEST_HOLD_EXCHANGE the sample sort's wait for the key all-to-all reports "not done"
    (as when a peer died before sending), so the call is parked inside exch_wait's poll loop.
    dsort_comm_abort from another thread must free it: the call returns DSORT_ECOMM (never "ok"),
    ncclCommAbort has run under the communicator lock, and a fresh communicator sorts again."""
    import torch

    import dsort
    ctx = gpu_ctx
    n = (1 << 25) + 333
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.gen_uniform(t, SEED, 7)
    fp_in = ctx.fingerprint(t)
    ctx.comm_init(1, 0, dsort.Context.unique_id())
    res = {}

    def run():
        try:
            res["ok"] = ctx.sample_sort_dev(t)
            ctx.synchronize()
        except dsort.DsortError as e:
            res["err"] = str(e)

    with ctx.options(test_hold_exchange=1, comm_timeout_ms=60000):
        th = threading.Thread(target=run)
        th.start()
        time.sleep(0.5)
        assert th.is_alive(), res  # parked in the exchange, not finished
        t0 = time.perf_counter()
        ctx.comm_abort()
        th.join(30)
        freed_ms = 1e3 * (time.perf_counter() - t0)
    assert not th.is_alive()
    assert "err" in res and "ECOMM" in res["err"] and "dsort_comm_abort" in res["err"], res
    assert freed_ms < 1000, freed_ms
    with pytest.raises(dsort.DsortError, match="ECOMM"):  # the communicator is gone
        ctx.sample_sort_dev(t)
    ctx.comm_init(1, 0, dsort.Context.unique_id())
    ptr, nout = ctx.sample_sort_dev(t)
    ctx.synchronize()
    assert nout == n and _sorted_slice_ok(ctx, ptr, nout, fp_in)
    ctx.comm_destroy()
    del t
    torch.cuda.empty_cache()


def test_held_exchange_times_out_at_the_deadline(gpu_ctx):
    """The same parked wait with nobody aborting: DSORT_OPT_COMM_TIMEOUT_MS ends it with
    DSORT_ETIMEOUT and aborts the communicator (a hung peer, not a dead one)."""
    import torch

    import dsort
    ctx = gpu_ctx
    t = torch.empty(1 << 20, dtype=torch.int32, device="cuda")
    ctx.gen_uniform(t, SEED, 0)
    ctx.comm_init(1, 0, dsort.Context.unique_id())
    with ctx.options(test_hold_exchange=1, comm_timeout_ms=300):
        t0 = time.perf_counter()
        with pytest.raises(dsort.DsortError, match="ETIMEOUT"):
            ctx.sample_sort_dev(t)
        assert time.perf_counter() - t0 < 10
    with pytest.raises(dsort.DsortError, match="ECOMM"):
        ctx.sample_sort_dev(t)
    ctx.comm_destroy()


def test_faulted_exchanges_release_replaced_arenas(gpu_ctx):
    """the arenas the second level replaces while the keys are in flight (their release
    deferred: a device-wide synchronize could hang on a dead peer's stream) are freed once no kernel
    can touch them -- also when the exchange fails (dsort_api.hip sample_sort_bx: the abort, the
    sort stream's drain, then flush_later).  Three bucket exchanges of growing size, each ending in
    DSORT_ETIMEOUT at the held final wait for the all-to-all, after the second level has grown its
    arenas (a failure inside the waves takes the same release, round 5): every one
    returns with nothing pending (dsort_stats.pending_frees), the larger ones having deferred some
    (deferred_frees: the path is exercised), and a good sort follows."""
    import torch

    import dsort
    ctx = gpu_ctx
    sizes = [(1 << 24) + 11, (1 << 26) + 13, (1 << 27) + 17]
    t = torch.empty(sizes[-1], dtype=torch.int32, device="cuda")
    ctx.gen_uniform(t, SEED, 5)
    fp = ctx.fingerprint(t)
    deferred = []
    for n in sizes:
        ctx.comm_init(1, 0, dsort.Context.unique_id())
        # (a deadline the second level meets: the sort times out in the held final wait, after both
        # waves ran and grew their arenas)
        with ctx.options(test_hold_exchange=1, comm_timeout_ms=3000):
            with pytest.raises(dsort.DsortError, match="ETIMEOUT.*key all-to-all"):
                ctx.sample_sort_dev(t[:n])
        st = ctx.stats()
        assert st["pending_frees"] == 0, st
        deferred.append(st["deferred_frees"])
        ctx.comm_destroy()
    assert sum(deferred[1:]) > 0, deferred  # (the grown second-level arenas)
    ctx.comm_init(1, 0, dsort.Context.unique_id())
    try:
        ptr, nout = ctx.sample_sort_dev(t)
        ctx.synchronize()
        assert nout == sizes[-1] and _sorted_slice_ok(ctx, ptr, nout, fp)
        assert ctx.stats()["pending_frees"] == 0
    finally:
        ctx.comm_destroy()
    del t
    torch.cuda.empty_cache()


def test_c_master_rccl_one_gpu_with_comm_deadline():
    """dsort_master --mode samplesort over RCCL on this box's one GPU with an exchange deadline
    (DSORT_OPT_COMM_TIMEOUT_MS: every polled wait of the exchange and the communicator set-up)."""
    import ftsort
    r = ftsort.run_master(1, (1 << 25) + 7, transport="rccl", devices=[0], timeout_s=180,
                          extra=["--comm-timeout-ms", "60000"])
    assert r["ok"], r
    assert r["transport"] == "rccl" and r["epochs"] == 1 and r["slices"] == [(1 << 25) + 7]


def test_c3_rank_layout_one_rccl_rank_bit_exact(gpu_ctx):
    """One rank of config C3 (2^32 int32 over 8 GPUs) on this box's one GPU, the layout of
    scripts/c3_rank.py: 2^29 keys (rank 3's chunk of the global synthetic input), the bucket
    exchange over one RCCL rank with DSORT_OPT_BUCKETS = 128 -- 4M-key buckets, as 1024 global
    buckets give each of 8 ranks -- so the second level takes its large-bucket geometry (16384-key
    tiles).  The rank's slice equals torch.sort of its keys element for element (the rank-local
    part of server.c:414-415 + 500-515's replacement)."""
    import ctypes

    import torch

    import dsort
    ctx = gpu_ctx
    n = 1 << 29
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.gen_uniform(t, SEED, 3 * n)
    ctx.comm_init(1, 0, dsort.Context.unique_id())
    try:
        # (the wave fence: this rank's own wave-1 buckets, read in place from the partition buffer,
        # are fingerprinted across wave 0's second level and tile sort -- round 6)
        with ctx.options(buckets=128, test_wave_fence=1):
            ptr, nout = ctx.sample_sort_dev(t)
            ctx.synchronize()
        st = ctx.stats()
        assert nout == n and st["exchange_path"] == 1 and st["tile_keys"] == 16384, st
        assert st["fence_ranges"] == 1, st
        out = torch.empty_like(t)
        ctx.check(ctx.lib.dsort_copy_d2d(ctx.h, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ptr), 4 * n))
        torch.cuda.synchronize()
        assert torch.equal(out, torch.sort(t).values)
    finally:
        ctx.comm_destroy()
    del t, out
    torch.cuda.empty_cache()
