"""The fault-tolerance master (ftsort.Master, server.c's role) on CPU: worker processes are the
numpy test double tests/double/ft_worker.py speaking the same control-store protocol, so failure
detection (exit and stale heartbeat), the recovery plan, the reassignment rule of server.c:368-384
and the end-to-end verification run without a GPU."""
import os
import sys

import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "distributed-sorting-with-fault-tolerance_amd"))
import ftsort  # noqa: E402

DOUBLE = [sys.executable, "-u", os.path.join(REPO, "tests", "double", "ft_worker.py")]


def test_reassign_rules():
    assert ftsort.reassign({3}, 8) == {3: 0}                      # first live (server.c:368)
    assert ftsort.reassign({0}, 8) == {0: 1}
    assert ftsort.reassign({3}, 8, "next-live") == {3: 4}
    assert ftsort.reassign({7}, 8, "next-live") == {7: 0}
    assert ftsort.reassign({0, 1}, 3, "next-live") == {0: 2, 1: 2}
    with pytest.raises(RuntimeError):
        ftsort.reassign({0, 1}, 2)


def test_chunk_range_is_the_reference_partition():
    sizes = [ftsort.chunk_range(10002, 4, r) for r in range(4)]  # server.c:185-216
    assert [s for s, _ in sizes] == [2501, 2501, 2500, 2500]
    assert [f for _, f in sizes] == [0, 2501, 5002, 7502]


def _master(world, n, rule="first-live", hb=5.0):
    return ftsort.Master(world, n, transport="host", devices=[0] * world, rule=rule, heartbeat_timeout=hb,
                         worker_cmd=DOUBLE)


def test_fault_free_protocol():
    r = _master(3, 30_001).run()
    assert r["ok"] and r["dead"] == [] and sum(r["slices"]) == 30_001


@pytest.mark.parametrize("kill,rule", [(1, "first-live"), (0, "first-live"), (2, "next-live")])
def test_dead_worker_chunk_is_reassigned(kill, rule):
    r = _master(4, 40_003, rule).run(kill_rank=kill, kill_after_pass=0)
    assert r["ok"], r
    assert r["dead"] == [kill]
    assert r["plan"]["assign"] == {str(kill): ftsort.reassign({kill}, 4, rule)[kill]}
    assert len(r["slices"]) == 3


def test_hung_worker_is_fenced_by_heartbeat():
    m = _master(3, 9_001, hb=0.5)
    r = m.run(kill_rank=2, kill_after_pass="hang")
    assert r["ok"] and r["dead"] == [2]
