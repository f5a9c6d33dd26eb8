"""The reference's end-to-end configuration C1 on the MI355X box with the REAL libdsort.so:
1 master (GPU merge) + 4 GPU workers on 127.0.0.1, all on device 0 (5 processes).  Checks the
reference's output.txt bit for bit, interop with the reference's client, and a worker fault."""
import os
import shutil

import numpy as np
import pytest

from cluster import Session
from conftest import GOLDEN, REF_BUILD

pytestmark = pytest.mark.gpu
HAVE_REF = os.path.exists(os.path.join(REF_BUILD, "client"))


def ref_files(d):
    shutil.copy(os.path.join(GOLDEN, "ref_input.txt"), os.path.join(d, "input.txt"))
    return open(os.path.join(GOLDEN, "ref_output.txt"), "rb").read()


def test_c1_kat_gpu_workers(tmp_path):
    exp = ref_files(tmp_path)
    s = Session(tmp_path)
    assert s.sort_files(["input.txt"], timeout=100) == 0, s.master_log()
    assert s.output() == exp
    print(s.master_log().splitlines()[-2])


@pytest.mark.parametrize("proto", ["v0", "v1"])
def test_c1_three_gpu_workers(tmp_path, proto):
    """BASELINE config C1 as written: 1 server + 3 client processes (the reference hard-codes 4,
    server.c:11; the build takes --workers).  Chunks of 3334/3333/3333 keys; output.txt bytes
    identical to the reference's."""
    exp = ref_files(tmp_path)
    s = Session(tmp_path, workers=3, proto=proto)
    assert s.sort_files(["input.txt"], timeout=100) == 0, s.master_log()
    assert s.output() == exp
    assert "workers=3 alive=3" in s.master_log()


def test_c1_three_gpu_workers_one_fails(tmp_path):
    exp = ref_files(tmp_path)
    s = Session(tmp_path, workers=3, worker_args=[[], ["--fault", "exit-before-reply:1"], []])
    assert s.sort_files(["input.txt"], timeout=100) == 0, s.master_log()
    assert s.output() == exp
    assert "Reassigning chunk 2 to worker node 1" in s.master_log()


@pytest.mark.skipif(not HAVE_REF, reason="reference not built")
def test_c1_gpu_master_reference_clients(tmp_path):
    exp = ref_files(tmp_path)
    s = Session(tmp_path, worker_kinds=["ref"] * 4)
    assert s.sort_files(["input.txt"], timeout=100) == 0
    assert s.output() == exp


def test_c1_gpu_worker_fault(tmp_path):
    exp = ref_files(tmp_path)
    wa = [[], [], ["--fault", "exit-before-reply:1"], []]
    s = Session(tmp_path, worker_args=wa)
    assert s.sort_files(["input.txt"], timeout=100) == 0
    assert s.output() == exp
    assert "Reassigning chunk 3 to worker node 1" in s.master_log()


def test_v1_large_file_gpu(tmp_path):
    rng = np.random.default_rng(9)
    k = rng.integers(-(2**31), 2**31, 2_000_000, dtype=np.int64)
    with open(tmp_path / "big.txt", "wb") as f:
        f.write(b" ".join(str(int(x)).encode() for x in k))
    s = Session(tmp_path, proto="v1")
    assert s.sort_files(["big.txt"], timeout=100) == 0, s.master_log()
    got = np.array(s.output().split(), dtype=np.int64)
    assert np.array_equal(got, np.sort(k))
