"""The host transport's collective sequence under a rank failure, CPU only (gloo, world size 3).

Round 4's multi-rank GPU test hung once.  The library's host-transport
sample sort runs a fixed sequence of collectives; every one after the first now has a status gate
in front of it and every wait is bounded by the exchange deadline (csrc/dsort_tx.h).
tests/tx/tx_harness.cpp runs that very TxSeq/TxGuard code with the bucket exchange's sequence on
the CPU through the same Python transport the GPU tests use (dsort.torch_dist_transport), and
(round 6) the first collective has a gate in front of it too:
  * a rank failing locally right before the key all-to-all (or any other collective) makes every
    rank return at once: the failed one its own error, the peers DSORT_ECOMM naming it -- the
    survivor side of server.c:421-449, where a peer's failure surfaces as an error;
  * a rank that hangs there makes its peers return DSORT_ETIMEOUT at the deadline, not block.
"""
import ctypes
import json
import os
import subprocess
import sys
import time

import pytest
import torch.multiprocessing as mp

from conftest import PKG, REPO

HARNESS_SRC = os.path.join(REPO, "tests", "tx", "tx_harness.cpp")
HARNESS_DIR = os.path.join(REPO, "tests", "tx", "build")
EHIP, ECOMM, ETIMEOUT = -3, -4, -6


def build_harness():
    os.makedirs(HARNESS_DIR, exist_ok=True)
    out = os.path.join(HARNESS_DIR, "libtxharness.so")
    deps = [HARNESS_SRC, os.path.join(PKG, "csrc", "dsort_tx.h"), os.path.join(REPO, "include", "dsort.h")]
    if not os.path.exists(out) or any(os.path.getmtime(d) > os.path.getmtime(out) for d in deps):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-shared", "-fPIC",
                               "-I" + os.path.join(REPO, "include"), "-I" + os.path.join(PKG, "csrc"),
                               "-o", out, HARNESS_SRC])
    return out


def _rank(rank, world, store, so, fail_rank, fail_at, hang_ms, timeout_ms, outdir, rerun):
    import datetime

    import torch.distributed as dist

    sys.path.insert(0, PKG)
    import dsort

    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=30))
    lib = ctypes.CDLL(so)
    lib.txh_deadline_ms.restype = ctypes.c_int64
    lib.txh_run.argtypes = [ctypes.POINTER(dsort.Transport), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                            ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_char_p, ctypes.c_size_t,
                            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    t = dsort.torch_dist_transport(world, deadline_fn=lib.txh_deadline_ms)
    msg = ctypes.create_string_buffer(512)
    peer, ncoll = ctypes.c_int(-2), ctypes.c_int(-2)
    t0 = time.monotonic()
    rc = lib.txh_run(ctypes.byref(t), world, rank, 2, fail_rank, fail_at, hang_ms, timeout_ms, msg, len(msg),
                     ctypes.byref(peer), ctypes.byref(ncoll))
    el = time.monotonic() - t0
    res = {"rc": rc, "msg": msg.value.decode(), "peer": peer.value, "ncoll": ncoll.value, "s": el,
           "poisoned": getattr(t, "poisoned", None)}
    if rerun and rank != fail_rank:
        # a second sequence on the same transport, no failure injected: after a timeout the
        # transport is poisoned and must refuse at once (a stale gloo op could pair)
        t0 = time.monotonic()
        rc2 = lib.txh_run(ctypes.byref(t), world, rank, 2, -1, -1, 0, 20_000, msg, len(msg),
                          ctypes.byref(peer), ctypes.byref(ncoll))
        res.update(rc2=rc2, msg2=msg.value.decode(), s2=time.monotonic() - t0)
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    os._exit(0)  # (a timed-out gloo op may still be pending: leave without waiting for it)


def run(tmp_path, fail_rank=-1, fail_at=-1, hang_ms=0, timeout_ms=20_000, world=3, rerun=False):
    so = build_harness()
    mp.spawn(_rank, args=(world, str(tmp_path / "store"), so, fail_rank, fail_at, hang_ms, timeout_ms, str(tmp_path),
                          rerun), nprocs=world, join=True)
    return [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]


def test_sequence_runs_clean(tmp_path):
    res = run(tmp_path)
    assert all(r["rc"] == 0 and r["ncoll"] == 5 for r in res), res


# collective 3 = the key all-to-all of wave 0 (0 counts, 1 samples, 2 bucket starts, 4 wave 1);
# 0 = before the very first collective (the presorted entry's staging failing)
@pytest.mark.parametrize("fail_at", [3, 0, 1, 4])
def test_local_failure_fails_every_rank_at_the_next_gate(tmp_path, fail_at):
    res = run(tmp_path, fail_rank=1, fail_at=fail_at)
    assert res[1]["rc"] == EHIP and "injected" in res[1]["msg"], res[1]
    for r in (0, 2):
        assert res[r]["rc"] == ECOMM, res[r]
        assert res[r]["peer"] == 1 and "rank 1 failed locally" in res[r]["msg"], res[r]
        assert res[r]["ncoll"] == fail_at, res[r]  # nobody entered the collective rank 1 skipped
    assert max(r["s"] for r in res) < 10, res  # returned at the gate, far inside the 20 s deadline


def test_hung_rank_times_out_its_peers_at_the_deadline(tmp_path):
    res = run(tmp_path, fail_rank=1, fail_at=3, hang_ms=6000, timeout_ms=1500)
    for r in (0, 2):
        assert res[r]["rc"] == ETIMEOUT, res[r]
        assert res[r]["s"] < 5, res[r]  # the 1.5 s deadline, not gloo's 30 s timeout
    assert res[1]["rc"] in (ETIMEOUT, ECOMM), res[1]  # woke up past the deadline


def test_transport_is_poisoned_after_a_timeout(tmp_path):
    res = run(tmp_path, fail_rank=1, fail_at=3, hang_ms=6000, timeout_ms=1500, rerun=True)
    for r in (0, 2):
        assert res[r]["rc"] == ETIMEOUT and res[r]["poisoned"], res[r]
        # the next sort on the same group fails at its first gate, without touching gloo
        assert res[r]["rc2"] == ECOMM and "callback returned -4" in res[r]["msg2"], res[r]
        assert res[r]["s2"] < 1.0, res[r]
