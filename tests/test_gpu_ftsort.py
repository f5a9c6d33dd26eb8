"""Fault-tolerant multi-GPU sample sort (BASELINE config C5) on the 1-GPU box: the workers share
cuda:0, so they exchange through the host transport (gloo); one worker SIGKILLs itself in the
middle of its local sort (after merge pass 0, DSORT_INJECT_KILL_AFTER_PASS) and the survivors
must still produce the sorted input, with the dead worker's chunk reassigned as in
server.c:368-391.  Verified bit-exactly through order, multiset fingerprint and slice
boundaries (ftsort.Master), and against numpy for the survivors' concatenation."""
import os
import sys

import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd"))
pytestmark = pytest.mark.gpu


def _master(world, n, rule="first-live"):
    import ftsort

    return ftsort.Master(world, n, transport="host", devices=[0] * world, rule=rule)


def test_fault_free_run_sorts():
    r = _master(3, 1_500_007).run()
    assert r["ok"], r
    assert r["dead"] == [] and r["plan"] is None


@pytest.mark.parametrize("rule,kill", [("first-live", 2), ("next-live", 1), ("first-live", 0)])
def test_worker_killed_mid_sort_is_recovered(rule, kill):
    n = 1 << 22  # 2^20 keys per worker: 64 tiles, two merge passes; the kill follows pass 0
    r = _master(4, n, rule).run(kill_rank=kill, kill_after_pass=0)
    assert r["ok"], r
    assert r["dead"] == [kill]
    import ftsort

    assert r["plan"]["assign"] == {str(kill): ftsort.reassign({kill}, 4, rule)[kill]}
    assert len(r["slices"]) == 3 and sum(r["slices"]) == n
    assert r["t_fault_seen_ms"] is not None and r["t_survivors_notified_ms"] is not None
