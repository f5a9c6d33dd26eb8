"""Multi-rank sweep of the bucket exchange with pure buckets kept home (dev tool, pytest file outside
tests/: `python -m pytest scripts/dev/mp_sweep_r6.py -q`, GPU box): ranks sharing the GPU over the
host transport, duplicate-heavy inputs and bucket counts that put few or many splitters on a key, each
checked element for element against numpy's sort of the whole input, under the wave fence."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
from test_gpu_multirank import run_ranks  # noqa: E402


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("dtype,dist", [("i32", "few"), ("i64", "few"), ("i64", "zipf"), ("i32", "ref100"),
                                        ("i32", "mixed"), ("i32", "seq")])
@pytest.mark.parametrize("buckets", [0, 48, 384])
def test_exchange_sweep(tmp_path, world, dtype, dist, buckets):
    n = world * (1 << 22) + 777
    opts = {"test_wave_fence": 1}
    if buckets:
        opts["buckets"] = buckets
    ins, outs, meta = run_ranks(tmp_path, world, n, dtype, dist, opts={"all": opts})
    assert all(m["stats"]["exchange_path"] == 1 for m in meta)
    assert np.array_equal(np.concatenate(outs), np.sort(ins))
