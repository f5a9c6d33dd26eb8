"""The multi-GPU sample sort driven from C (dsort_master --mode samplesort, host/ss_master.c and
host/ss_worker.c) on CPU: the master and its worker processes run against the C-ABI TEST DOUBLE
(tests/double, oracle inside) with the relay transport (exchanges through the master), so the
control protocol, the master-held chunk replicas in shared memory, the supervision, the
reassignment rules (server.c:368-384) and the recovery epoch are exercised here; the same binaries
run with the real libdsort.so in tests/test_gpu_samplesort_c.py.  Output is checked bit-exactly
against numpy on the same synthetic keys (the oracle's generator = the library's)."""
import json
import os
import subprocess

import numpy as np
import pytest

from cluster import build_double
from conftest import PKG

MASTER = os.path.join(PKG, "bin", "dsort_master")
pytestmark = pytest.mark.skipif(not os.path.exists(MASTER), reason="build first")
SEED = 0x5EED2026


@pytest.fixture(scope="module")
def libdir():
    return build_double()


def run_master(libdir, tmp_path, *args, timeout=120):
    env = dict(os.environ, LD_LIBRARY_PATH=libdir + ":" + os.environ.get("LD_LIBRARY_PATH", ""))
    p = subprocess.run([MASTER, "--mode", "samplesort", "--transport", "relay", "--devices", "share", *args],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=timeout)
    line = [ln for ln in p.stdout.splitlines() if ln.startswith('{"ss_result"')]
    assert line, p.stdout[-3000:] + p.stderr[-3000:]
    return json.loads(line[-1]), p


def expected(oracle, n, dt=np.int32):
    return np.sort(oracle.gen_uniform(SEED, 0, n, dt))


@pytest.mark.parametrize("world,n", [(1, 1000), (2, 100_003), (3, 65_537), (4, 3)])
def test_fault_free(libdir, tmp_path, oracle, world, n):
    out = tmp_path / "out.txt"
    r, p = run_master(libdir, tmp_path, "--gpus", str(world), "--keys", str(n), "--output", str(out))
    assert r["ok"], p.stdout + p.stderr
    assert r["dead"] == [] and r["epochs"] == 1 and sum(r["slices"]) == n
    assert out.read_bytes() == b"".join(b"%d\n" % int(k) for k in expected(oracle, n))


def test_int64_keys(libdir, tmp_path, oracle):
    out = tmp_path / "out.bin"
    r, p = run_master(libdir, tmp_path, "--gpus", "3", "--keys", "50001", "--dtype", "i64", "--output", str(out))
    assert r["ok"], p.stdout + p.stderr
    got = np.fromfile(out, np.int64)
    assert np.array_equal(got, expected(oracle, 50001, np.int64))


@pytest.mark.parametrize("rule,kill,owner", [("first-live", 2, 0), ("first-live", 0, 1), ("next-live", 1, 2),
                                             ("next-live", 3, 0)])
@pytest.mark.parametrize("stage", ["sort", "exchange1", "exchange2"])
def test_worker_killed_is_recovered(libdir, tmp_path, oracle, rule, kill, owner, stage):
    """A worker dies in its local sort or inside the exchange (after the sample all-gather, or with
    the counts exchanged and the keys about to move); the master reassigns its chunk by the rule,
    the survivors rebuild and the output is still the sorted input."""
    n = 40_009
    out = tmp_path / "out.txt"
    extra = ["--kill-stage", "sort"] if stage == "sort" else ["--kill-stage", "exchange", "--kill-exchange-stage",
                                                              stage[-1]]
    r, p = run_master(libdir, tmp_path, "--gpus", "4", "--keys", str(n), "--kill-rank", str(kill), *extra,
                      "--reassign", rule, "--output", str(out))
    assert r["ok"], p.stdout + p.stderr
    assert r["dead"] == [kill] and r["survivors"] == 3 and r["epochs"] == 2
    assert r["owners"][kill] == owner
    assert r["t_fault_seen_ms"] >= 0 and r["t_survivors_notified_ms"] >= r["t_fault_seen_ms"]
    assert out.read_bytes() == b"".join(b"%d\n" % int(k) for k in expected(oracle, n))


@pytest.mark.parametrize("kstage", [0, 1, 2])
def test_worker_killed_at_every_sort_stage(libdir, tmp_path, oracle, kstage):
    """The library's three kill points of a bucketed local sort (first-level partition, second-level
    partition, tile sort; dsort.h DSORT_OPT_KILL_AFTER_STAGE), each a real stage of the double's sort."""
    n = 30_011
    out = tmp_path / "out.txt"
    r, p = run_master(libdir, tmp_path, "--gpus", "3", "--keys", str(n), "--kill-rank", "1", "--kill-stage", "sort",
                      "--kill-after-stage", str(kstage), "--output", str(out))
    assert r["ok"], p.stdout + p.stderr
    assert r["dead"] == [1] and r["epochs"] == 2 and sum(r["slices"]) == n
    assert out.read_bytes() == b"".join(b"%d\n" % int(k) for k in expected(oracle, n))


def test_unreachable_kill_stage_is_an_error(libdir, tmp_path):
    """A kill stage the victim's sort never reaches is refused up front (no silent fault-free run)."""
    env = dict(os.environ, LD_LIBRARY_PATH=libdir + ":" + os.environ.get("LD_LIBRARY_PATH", ""))
    p = subprocess.run([MASTER, "--mode", "samplesort", "--transport", "relay", "--devices", "share", "--gpus", "3",
                        "--keys", "3000", "--kill-rank", "2", "--kill-after-stage", "3"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=60)
    assert p.returncode == 2 and "has 3 stages" in p.stderr, p.stderr


@pytest.mark.parametrize("first_stage", [["--kill-stage", "sort", "--kill-after-stage", "1"],
                                         ["--kill-stage", "exchange", "--kill-exchange-stage", "2"]])
def test_second_failure_during_recovery(libdir, tmp_path, oracle, first_stage):
    """Worker 1 dies; worker 3 dies as soon as it receives the recovery plan, while the other
    survivors rebuild: they must take the next plan (no hang on the first recovery epoch's
    communicator) and the output is still the sorted input (ss_worker.c:437)."""
    n = 50_021
    out = tmp_path / "out.txt"
    r, p = run_master(libdir, tmp_path, "--gpus", "4", "--keys", str(n), "--kill-rank", "1", *first_stage,
                      "--kill-in-recovery", "3", "--output", str(out))
    assert r["ok"], p.stdout + p.stderr
    assert sorted(r["dead"]) == [1, 3] and r["survivors"] == 2 and r["epochs"] == 3
    assert out.read_bytes() == b"".join(b"%d\n" % int(k) for k in expected(oracle, n))


def test_input_file_kat(libdir, tmp_path):
    """The reference's input.txt through the C sample sort: output.txt byte-identical to the
    reference's own output.txt (SURVEY.md §4 KAT)."""
    from conftest import GOLDEN
    out = tmp_path / "output.txt"
    r, p = run_master(libdir, tmp_path, "--gpus", "3", "--input", os.path.join(GOLDEN, "ref_input.txt"),
                      "--output", str(out))
    assert r["ok"], p.stdout + p.stderr
    assert out.read_bytes() == open(os.path.join(GOLDEN, "ref_output.txt"), "rb").read()


def test_all_workers_dead_fails_cleanly(libdir, tmp_path):
    r, p = run_master(libdir, tmp_path, "--gpus", "1", "--keys", "1000", "--kill-rank", "0")
    assert not r["ok"] and p.returncode != 0


def test_hung_worker_is_fenced_not_its_peers(libdir, tmp_path, oracle):
    """A worker that hangs (SIGSTOP after its local sort: its heartbeat stops, its socket stays
    open) with an exchange deadline and a long heartbeat timeout: every peer's exchange times out
    and reports a failed DONE.  The master must fence the silent worker, not the peers that
    reported (the 1 s fencing of failed reporters used to kill every survivor), then
    finish over the survivors."""
    n = 30_011
    out = tmp_path / "out.txt"
    r, p = run_master(libdir, tmp_path, "--gpus", "3", "--keys", str(n), "--hang-rank", "1",
                      "--comm-timeout-ms", "1500", "--timeout-ms", "60000", "--output", str(out), timeout=90)
    assert r["ok"], p.stdout + p.stderr
    assert r["dead"] == [1] and r["survivors"] == 2 and r["epochs"] == 2, r
    assert "silent" in p.stderr and "fenced" in p.stderr
    assert out.read_bytes() == b"".join(b"%d\n" % int(k) for k in expected(oracle, n))
