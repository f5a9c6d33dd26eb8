"""Pins the oracle (CPU restatement) to the reference.  CPU only.

* the reference's own known-answer pair input.txt -> output.txt;
* golden vectors produced by the reference binaries built from source (tests/golden/make_golden.py);
* when oracle/_ref exists (built from /root/reference by `make -C oracle ref`), direct
  comparison with the reference's merge_sort (client.c:166) and merge_chunks (server.c:481).
"""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, REF_BUILD

CASES = json.load(open(os.path.join(GOLDEN, "cases.json")))
INT_MIN, INT_MAX = -(2**31), 2**31 - 1


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_reference_kat_input_output(oracle):
    raw = open(os.path.join(GOLDEN, "ref_input.txt"), "rb").read()
    exp = open(os.path.join(GOLDEN, "ref_output.txt"), "rb").read()
    assert sha(raw) == CASES["ref_input_sha256"]
    assert sha(exp) == CASES["ref_output_sha256"]
    keys = oracle.parse(raw)
    assert keys.size == 10000
    out = oracle.reference_sort(keys, workers=4)
    assert oracle.format(out) == exp


@pytest.mark.parametrize("case", CASES["e2e"], ids=lambda c: c["name"])
def test_golden_e2e(oracle, case):
    keys = np.load(os.path.join(GOLDEN, case["name"] + ".in.npy"))
    exp = np.load(os.path.join(GOLDEN, case["name"] + ".out.npy"))
    text = b"\n".join(str(int(k)).encode() for k in keys)
    assert sha(text) == case["input_sha256"]
    got = oracle.reference_sort(keys, workers=4)
    assert np.array_equal(got, exp)
    assert sha(oracle.format(got)) == case["output_sha256"]


@pytest.mark.parametrize("case", CASES["merge_chunks"], ids=lambda c: c["name"])
def test_golden_merge_chunks(oracle, case):
    z = np.load(os.path.join(GOLDEN, case["name"] + ".npz"))
    runs = [z[f"arr_{i}"] for i in range(case["k"])]
    got = oracle.merge_chunks(runs)
    w = case["written_prefix"]
    assert got[:w].tolist() == case["reference_output_prefix"]
    if w == case["total"]:
        assert np.array_equal(oracle.merge_runs(runs), got)


@pytest.mark.parametrize("case", CASES["merge_sort"], ids=lambda c: c["name"])
def test_golden_merge_sort(oracle, case):
    a = np.load(os.path.join(GOLDEN, case["name"] + ".in.npy"))
    exp = np.load(os.path.join(GOLDEN, case["name"] + ".out.npy"))
    assert np.array_equal(oracle.merge_sort(a), exp)


def test_intmax_quirk_documented(oracle):
    # the reference loses INT_MAX keys in merge_chunks; the oracle reproduces it,
    # the full-range merge keeps them.
    runs = [np.array([1, INT_MAX, INT_MAX], np.int32), np.array([-5, 2], np.int32),
            np.array([0], np.int32), np.array([INT_MAX], np.int32)]
    quirk = oracle.merge_chunks(runs, fill=123)
    assert quirk.tolist() == [-5, 0, 1, 2, 123, 123, 123]
    assert oracle.merge_runs(runs).tolist() == [-5, 0, 1, 2, INT_MAX, INT_MAX, INT_MAX]


def test_partition_rule(oracle):
    for n, w in [(10000, 4), (10001, 4), (3, 4), (0, 4), (17, 8)]:
        sz, of = oracle.partition(n, w)
        assert sz.sum() == n
        assert all(int(sz[i]) == n // w + (1 if i < n % w else 0) for i in range(w))
        assert np.array_equal(of, np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint64))


def test_generators_and_fingerprint(oracle):
    a = oracle.gen_uniform(0x5EED2026, 0, 1000)
    b = oracle.gen_uniform(0x5EED2026, 500, 500)
    assert np.array_equal(a[500:], b)
    sm = [oracle.lib.oracle_splitmix64(0x5EED2026 + i) >> 32 for i in range(4)]
    assert a[:4].astype(np.uint32).tolist() == sm
    fp1 = oracle.fingerprint(a)
    fp2 = oracle.fingerprint(np.random.default_rng(1).permutation(a))
    assert fp1 == fp2
    a2 = a.copy()
    a2[7] += 1
    assert oracle.fingerprint(a2) != fp1


def test_text_codec_roundtrip(oracle):
    rng = np.random.default_rng(3)
    a = rng.integers(INT_MIN, INT_MAX + 1, 5000, dtype=np.int64).astype(np.int32)
    a[:3] = [INT_MIN, INT_MAX, -1]
    txt = oracle.format(a)
    assert txt == b"".join(b"%d\n" % int(x) for x in a)
    assert np.array_equal(oracle.parse(txt), a)
    assert np.array_equal(oracle.parse(b"  1 -2\n\t3  "), np.array([1, -2, 3], np.int32))
    with pytest.raises(ValueError):
        oracle.parse(b"1 x 2")


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_BUILD, "libref_client.so")),
                    reason="reference not built (make -C oracle ref)")
@pytest.mark.parametrize("n", [0, 1, 2, 3, 1000, 65536, 1 << 18])
def test_against_reference_merge_sort(oracle, n):
    lib = ctypes.CDLL(os.path.join(REF_BUILD, "libref_client.so"))
    lib.merge_sort.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(n)
    a = rng.integers(INT_MIN, INT_MAX + 1, n, dtype=np.int64).astype(np.int32)
    ref = a.copy()
    lib.merge_sort(ref.ctypes.data, 0, n - 1)
    assert np.array_equal(oracle.merge_sort(a), ref)


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_BUILD, "libref_server.so")),
                    reason="reference not built (make -C oracle ref)")
def test_against_reference_merge_chunks(oracle, tmp_path):
    lib = ctypes.CDLL(os.path.join(REF_BUILD, "libref_server.so"))
    lib.merge_chunks.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    rng = np.random.default_rng(5)
    for k in (1, 2, 4, 7):
        runs = [np.sort(rng.integers(INT_MIN, INT_MAX, rng.integers(0, 3000))).astype(np.int32)
                for _ in range(k)]
        ptrs = (ctypes.c_void_p * k)(*[r.ctypes.data for r in runs])
        sizes = (ctypes.c_int * k)(*[r.size for r in runs])
        total = sum(r.size for r in runs)
        cwd = os.getcwd()
        os.chdir(tmp_path)
        try:
            lib.merge_chunks(k, ptrs, sizes, total)
            ref = np.array([int(x) for x in open("output.txt", "rb").read().split()], np.int32)
        finally:
            os.chdir(cwd)
        assert np.array_equal(oracle.merge_chunks(runs), ref)
