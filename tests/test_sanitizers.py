"""The C host (master and worker, both modes) under ThreadSanitizer and AddressSanitizer on CPU,
against the C-ABI test double (SURVEY.md §5 asks for it: the reference races on is_alive[] at
server.c:361, 369, 424, 431).  Builds `make sanitize SAN=thread|address` (host code only; the GPU
library is not involved) and runs the pthreaded TCP master with fault injection (a worker exits
before replying, reassignment) and the sample-sort master/worker with kills in the sort and in the
exchange; any sanitizer report fails the test."""
import os
import shutil
import subprocess

import pytest

from cluster import Session, build_double
from conftest import GOLDEN, PKG

SAN_REPORT = ("WARNING: ThreadSanitizer", "ERROR: AddressSanitizer", "ERROR: LeakSanitizer")


@pytest.fixture(scope="module")
def libdir():
    return build_double()


def build(kind, libdir):
    subprocess.check_call(["make", "-s", "-C", PKG, "sanitize", f"SAN={kind}", f"DOUBLE_DIR={libdir}"],
                          stdout=subprocess.DEVNULL)
    return os.path.join(PKG, "build", f"san-{kind}")


def san_env(libdir):
    return dict(os.environ, LD_LIBRARY_PATH=libdir, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
                ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")


@pytest.mark.parametrize("kind", ["thread", "address"])
def test_tcp_master_with_reassignment(tmp_path, libdir, kind):
    bdir = build(kind, libdir)
    shutil.copy(os.path.join(GOLDEN, "ref_input.txt"), os.path.join(tmp_path, "input.txt"))
    s = Session(tmp_path, workers=4, proto="v1", lib_dir=libdir, bin_dir=bdir, env=san_env(libdir),
                worker_args=[[], ["--fault", "exit-before-reply:1"], [], []],
                master_args=["--retry-delay-ms", "10", "--reassign", "least-loaded"])
    assert s.sort_files(["input.txt", "input.txt"]) == 0, s.master_log()
    log = s.master_log() + "".join(open(os.path.join(tmp_path, f"worker{i}.log")).read() for i in range(1, 5))
    assert not any(m in log for m in SAN_REPORT), log[-4000:]
    assert s.output() == open(os.path.join(GOLDEN, "ref_output.txt"), "rb").read()


@pytest.mark.parametrize("kind", ["thread", "address"])
@pytest.mark.parametrize("stage", [["--kill-stage", "sort"], ["--kill-stage", "exchange", "--kill-exchange-stage", "1"],
                                   ["--kill-stage", "exchange", "--kill-exchange-stage", "2"]])
def test_samplesort_master_worker(tmp_path, libdir, kind, stage):
    bdir = build(kind, libdir)
    p = subprocess.run([os.path.join(bdir, "dsort_master"), "--mode", "samplesort", "--transport", "relay",
                        "--devices", "share", "--gpus", "4", "--keys", "50000", "--kill-rank", "2", *stage,
                        "--worker", os.path.join(bdir, "dsort_worker")],
                       cwd=tmp_path, env=san_env(libdir), capture_output=True, text=True, timeout=300)
    out = p.stdout + p.stderr
    assert not any(m in out for m in SAN_REPORT), out[-4000:]
    assert p.returncode == 0 and '"ok": true' in p.stdout, out[-3000:]
