"""Sample sort with several ranks.  On the 1-GPU box all ranks share cuda:0, which RCCL refuses
("invalid usage": one GPU per rank), so these ranks run the SAME libdsort sample sort with the
exchanges through the host transport (gloo); the RCCL exchange itself is exercised with one rank
here and with one rank per GPU by the driver's multi-GPU bench.  Checks: the concatenation of the
rank slices equals numpy.sort of the whole synthetic input (bit-exact), slices are balanced."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from cluster import free_port
from conftest import REPO

pytestmark = pytest.mark.gpu
DRIVER = os.path.join(REPO, "tests", "mp_samplesort.py")


def run_ranks(tmp_path, world, n, dtype="i32", dist="uniform", transport="host"):
    port = free_port()
    out = str(tmp_path / "ss")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, DRIVER, str(r), str(world), str(port), str(n), dtype, dist, out,
                               transport],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(world)]
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace"))
    for p, lg in zip(procs, logs):
        assert p.returncode == 0, lg[-3000:]
    ins = np.concatenate([np.load(out + f".in{r}.npy") for r in range(world)])
    outs = [np.load(out + f".out{r}.npy") for r in range(world)]
    meta = [json.load(open(out + f".rank{r}.json")) for r in range(world)]
    return ins, outs, meta


@pytest.mark.parametrize("world", [1, 2, 4])
def test_sample_sort_ranks_share_gpu(tmp_path, world):
    n = 3_000_017
    ins, outs, meta = run_ranks(tmp_path, world, n)
    assert ins.size == n
    assert np.array_equal(np.concatenate(outs), np.sort(ins))
    sizes = [o.size for o in outs]
    assert max(sizes) <= 1.25 * n / world + 1024, sizes


def test_sample_sort_zipf_i64(tmp_path):
    n = 2_000_003
    ins, outs, meta = run_ranks(tmp_path, 2, n, "i64", "zipf")
    assert np.array_equal(np.concatenate(outs), np.sort(ins))
    sizes = [o.size for o in outs]
    assert max(sizes) <= 1.3 * n / 2, sizes  # the heavy key is split across ranks


def test_sample_sort_rccl_single_rank(tmp_path):
    ins, outs, meta = run_ranks(tmp_path, 1, 1_000_003, transport="rccl")
    assert np.array_equal(np.concatenate(outs), np.sort(ins))


def test_rccl_refuses_shared_gpu_with_clear_error(tmp_path):
    with pytest.raises(AssertionError, match="one GPU per rank"):
        run_ranks(tmp_path, 2, 1000, transport="rccl")


def test_sample_sort_tiny_and_empty_ranks(tmp_path):
    ins, outs, meta = run_ranks(tmp_path, 4, 3)  # rank 3 holds no key
    assert np.array_equal(np.concatenate(outs), np.sort(ins))
