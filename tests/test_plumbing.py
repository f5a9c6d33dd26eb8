"""Master/worker plumbing on CPU: reference wire protocol (v0) interop in both directions, the
length-prefixed v1 protocol, and the fault-tolerance paths.

The build's master/worker run here against the C-ABI TEST DOUBLE (tests/double, CPU, oracle
inside) because this container has no GPU; the same scenarios run with the real libdsort.so on
the MI355X box in tests/test_gpu_plumbing.py.
"""
import os
import shutil

import numpy as np
import pytest

from cluster import Session, build_double
from conftest import GOLDEN, REF_BUILD, PKG

INT_MIN, INT_MAX = -(2**31), 2**31 - 1
HAVE_REF = os.path.exists(os.path.join(REF_BUILD, "server")) and os.path.exists(os.path.join(REF_BUILD, "client"))
HAVE_BIN = os.path.exists(os.path.join(PKG, "bin", "dsort_master"))
pytestmark = pytest.mark.skipif(not HAVE_BIN, reason="build first (make -C distributed-sorting-with-fault-tolerance_amd)")


@pytest.fixture(scope="module")
def libdir():
    return build_double()


def ref_files(d):
    shutil.copy(os.path.join(GOLDEN, "ref_input.txt"), os.path.join(d, "input.txt"))
    return open(os.path.join(GOLDEN, "ref_output.txt"), "rb").read()


def write_keys(path, keys):
    with open(path, "wb") as f:
        f.write(b"\n".join(str(int(k)).encode() for k in keys))


def expected_text(keys):
    return b"".join(b"%d\n" % int(k) for k in np.sort(np.asarray(keys, np.int64)))


def test_kat_ours_v0(tmp_path, libdir):
    exp = ref_files(tmp_path)
    s = Session(tmp_path, lib_dir=libdir)
    assert s.sort_files(["input.txt"]) == 0, s.master_log()
    assert s.output() == exp
    assert "Sorting completed for file input.txt" in s.master_log()


@pytest.mark.parametrize("proto", ["v0", "v1"])
def test_kat_three_workers(tmp_path, libdir, proto):
    """BASELINE config C1 as written (1 server + 3 clients): the build's worker count is a flag;
    the reference (MAX_WORKERS = 4, server.c:11) would block in accept."""
    exp = ref_files(tmp_path)
    s = Session(tmp_path, workers=3, lib_dir=libdir, proto=proto)
    assert s.sort_files(["input.txt"]) == 0, s.master_log()
    assert s.output() == exp
    assert "workers=3 alive=3" in s.master_log()


@pytest.mark.skipif(not HAVE_REF, reason="reference not built")
def test_interop_our_master_reference_clients(tmp_path, libdir):
    exp = ref_files(tmp_path)
    s = Session(tmp_path, worker_kinds=["ref"] * 4, lib_dir=libdir)
    assert s.sort_files(["input.txt"]) == 0
    assert s.output() == exp


@pytest.mark.skipif(not HAVE_REF, reason="reference not built")
def test_interop_reference_server_our_workers(tmp_path, libdir):
    exp = ref_files(tmp_path)
    s = Session(tmp_path, master="ref", lib_dir=libdir)
    s.sort_files(["input.txt"])
    assert s.output() == exp


@pytest.mark.skipif(not HAVE_REF, reason="reference not built")
def test_interop_mixed_workers_golden(tmp_path, libdir):
    keys = np.load(os.path.join(GOLDEN, "uniform_16383.in.npy"))
    write_keys(tmp_path / "in.txt", keys)
    s = Session(tmp_path, worker_kinds=["ours", "ref", "ours", "ref"], lib_dir=libdir)
    assert s.sort_files(["in.txt"]) == 0
    assert s.output() == expected_text(keys)


def test_multiple_files_one_session(tmp_path, libdir):
    rng = np.random.default_rng(1)
    files = []
    for i, n in enumerate([0, 1, 3, 5000, 40000]):
        k = rng.integers(-(2**31), 2**31 - 1, n).astype(np.int64)
        k[k == -1] = 5
        write_keys(tmp_path / f"f{i}.txt", k)
        files.append((f"f{i}.txt", k))
    s = Session(tmp_path, lib_dir=libdir)
    outs = []
    # one file per session call would lose output.txt between files: run sequentially with
    # distinct output names by re-running the master per file is the reference's behaviour too
    assert s.sort_files([f for f, _ in files]) == 0
    log = s.master_log()
    assert log.count("Sorting completed") == len(files)
    # output.txt holds the LAST file (the reference overwrites it per file, server.c:484)
    assert s.output() == expected_text(files[-1][1])
    del outs


def test_v1_full_key_range(tmp_path, libdir):
    """v1 carries -1 and INT_MAX, which the reference cannot (SURVEY.md §8a (1),(2))."""
    rng = np.random.default_rng(2)
    k = rng.integers(INT_MIN, INT_MAX, 30000, endpoint=True)
    k[:10] = [-1, -1, INT_MAX, INT_MIN, 0, INT_MAX, -1, 7, 7, INT_MIN]
    write_keys(tmp_path / "in.txt", k)
    s = Session(tmp_path, proto="v1", lib_dir=libdir)
    assert s.sort_files(["in.txt"]) == 0
    assert s.output() == expected_text(k)


def test_v0_rejects_minus_one(tmp_path, libdir):
    write_keys(tmp_path / "in.txt", [3, -1, 2])
    s = Session(tmp_path, lib_dir=libdir)
    s.sort_files(["in.txt"])
    assert "end marker" in s.master_log()
    assert not os.path.exists(tmp_path / "output.txt")


def test_fault_worker_exits_before_reply(tmp_path, libdir):
    """Recv-fault path (server.c:421): worker 3 dies holding chunk 3."""
    exp = ref_files(tmp_path)
    wa = [[], [], ["--fault", "exit-before-reply:1"], []]
    s = Session(tmp_path, worker_args=wa, lib_dir=libdir)
    assert s.sort_files(["input.txt"]) == 0
    assert s.output() == exp
    log = s.master_log()
    assert "Worker 3 failed on chunk 3" in log and "Reassigning chunk 3 to worker node 1" in log
    assert "reassignments=1" in log and "alive=3" in log


def test_fault_worker_dies_after_connect(tmp_path, libdir):
    """Send-fault path (server.c:358)."""
    exp = ref_files(tmp_path)
    wa = [[], ["--fault", "exit-on-connect"], [], []]
    s = Session(tmp_path, worker_args=wa, lib_dir=libdir)
    assert s.sort_files(["input.txt"]) == 0
    assert s.output() == exp
    assert "Reassigning chunk 2 to worker node 1" in s.master_log()


def test_fault_two_workers_least_loaded(tmp_path, libdir):
    exp = ref_files(tmp_path)
    wa = [["--fault", "exit-before-reply:1"], [], ["--fault", "exit-before-reply:1"], []]
    s = Session(tmp_path, worker_args=wa, master_args=["--reassign", "least-loaded"], lib_dir=libdir)
    assert s.sort_files(["input.txt"]) == 0
    assert s.output() == exp
    assert "alive=2" in s.master_log()


def test_fault_hung_worker_timeout_v1(tmp_path, libdir):
    """A worker that stays connected but never answers: the reference hangs forever (SURVEY.md
    §5); the build's --timeout detects it and reassigns."""
    exp = ref_files(tmp_path)
    wa = [[], [], [], ["--fault", "hang-before-reply:1"]]
    s = Session(tmp_path, proto="v1", worker_args=wa, master_args=["--timeout", "1", "--retry-delay-ms", "10"],
                lib_dir=libdir)
    for w in s.workers[3:]:
        pass
    rc = s.sort_files(["input.txt"], timeout=60)
    assert rc == 0
    assert s.output() == exp
    log = s.master_log()
    assert "Worker 4 failed on chunk 4 (timeout" in log


def test_all_workers_dead(tmp_path, libdir):
    ref_files(tmp_path)
    wa = [["--fault", "exit-before-reply:1"]] * 2
    s = Session(tmp_path, workers=2, worker_args=wa, lib_dir=libdir)
    s.sort_files(["input.txt"])
    assert "Sorting failed for file input.txt" in s.master_log()
    assert not os.path.exists(tmp_path / "output.txt")


def test_master_refuses_without_gpu(tmp_path, libdir, monkeypatch):
    """No CPU fallback: when dsort_init reports no device the master exits with an error."""
    monkeypatch.setenv("DSORT_DOUBLE_NO_GPU", "1")
    with pytest.raises(RuntimeError):
        Session(tmp_path, lib_dir=libdir)
