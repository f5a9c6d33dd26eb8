#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ from the REFERENCE ITSELF.

Run in the build container only (needs /root/reference and `make -C oracle ref`):

    python tests/golden/make_golden.py

What it does:
  * end-to-end cases: for each synthetic input it starts the reference `server`
    (oracle/_ref/server, built from /root/reference/server.c) and 4 reference `client`
    processes on 127.0.0.1, feeds the file name on the server's stdin (server.c:160-168), and
    keeps the `output.txt` the server writes (server.c:481-524).  Inputs respect the domain in
    which the reference is well defined: no -1 key (in-band sentinel,
    client.c:113), no INT_MAX key (server.c:501), at most 4096 keys per chunk (server.c:193).
  * merge_chunks cases: calls the reference merge_chunks() (server.c:481, compiled into
    oracle/_ref/libref_server.so with main renamed) on hand-made runs, including the INT_MAX
    case that shows the reference's lost-key quirk.
  * merge_sort cases: calls the reference merge_sort() (client.c:166) on full-range data
    (-1 and INT_MAX allowed at function level).

Outputs: <name>.in.npy / <name>.out.npy (int32), cases.json (sizes, sha256 of the input text
and of the reference's output.txt bytes).  The reference's own input.txt / output.txt are
copied verbatim as data (ref_input.txt / ref_output.txt).
"""
import ctypes
import hashlib
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_BUILD = os.path.join(REPO, "oracle", "_ref")
REF_SRC = "/root/reference"
INT_MIN, INT_MAX = -(2**31), 2**31 - 1


def sha(b):
    return hashlib.sha256(b).hexdigest()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_reference(text, workers=4, timeout=60):
    """Run reference server + `workers` clients on `text`; return output.txt bytes."""
    with tempfile.TemporaryDirectory() as d:
        port = free_port()
        with open(os.path.join(d, "server.conf"), "w") as f:
            f.write(f"SERVER_PORT={port}\n")
        with open(os.path.join(d, "client.conf"), "w") as f:
            f.write(f"SERVER_IP=127.0.0.1\nSERVER_PORT={port}\n")
        with open(os.path.join(d, "in.txt"), "wb") as f:
            f.write(text)
        srv = subprocess.Popen([os.path.join(REF_BUILD, "server"), "server.conf"], cwd=d,
                               stdin=subprocess.PIPE, stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL)
        time.sleep(0.2)
        clients = [subprocess.Popen([os.path.join(REF_BUILD, "client"), "client.conf"], cwd=d,
                                    stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
                   for _ in range(workers)]
        srv.stdin.write(b"in.txt\nexit\n")
        srv.stdin.close()
        try:
            srv.wait(timeout=timeout)
        finally:
            for c in clients:
                try:
                    c.wait(timeout=5)
                except subprocess.TimeoutExpired:
                    c.kill()
            if srv.poll() is None:
                srv.kill()
        with open(os.path.join(d, "output.txt"), "rb") as f:
            return f.read()


def to_text(keys, sep=b"\n"):
    return sep.join(str(int(k)).encode() for k in keys)


def e2e_cases(rng):
    lo, hi = INT_MIN, INT_MAX - 1  # INT_MAX excluded (server.c:501)

    def uni(n):
        a = rng.integers(lo, hi + 1, size=n, dtype=np.int64)
        a[a == -1] = -2  # -1 is the wire sentinel (client.c:113)
        return a.astype(np.int32)

    cases = []
    for n in (1, 3, 4, 5, 1023, 1024, 1025, 4096, 16383, 16384):
        cases.append((f"uniform_{n}", uni(n)))
    cases.append(("allequal_1025", np.full(1025, 7, np.int32)))
    cases.append(("sorted_16384", np.sort(uni(16384))))
    cases.append(("reverse_16383", np.sort(uni(16383))[::-1].copy()))
    cases.append(("fewdistinct_4096", rng.choice(np.array([-5, 0, 3, INT_MIN, INT_MAX - 1], np.int32), 4096)))
    cases.append(("fewdistinct_16384", rng.choice(np.array([-3, -2, 0, 1, 2, 3], np.int32), 16384)))
    cases.append(("small_1_100_10000", rng.integers(1, 101, 10000).astype(np.int32)))
    cases.append(("negative_9999", (-rng.integers(2, 1000, 9999)).astype(np.int32)))
    return cases


def main():
    if not os.path.exists(os.path.join(REF_BUILD, "server")):
        sys.exit("build the reference first: make -C oracle ref")
    rng = np.random.default_rng(20261015)
    meta = {"generator": "tests/golden/make_golden.py", "reference": REF_SRC,
            "e2e": [], "merge_chunks": [], "merge_sort": []}

    # the reference's own known-answer pair, kept as data
    shutil.copyfile(os.path.join(REF_SRC, "input.txt"), os.path.join(HERE, "ref_input.txt"))
    shutil.copyfile(os.path.join(REF_SRC, "output.txt"), os.path.join(HERE, "ref_output.txt"))
    raw = open(os.path.join(HERE, "ref_input.txt"), "rb").read()
    out = run_reference(raw)
    exp = open(os.path.join(HERE, "ref_output.txt"), "rb").read()
    assert out == exp, "reference did not reproduce its own output.txt"
    meta["ref_input_sha256"] = sha(raw)
    meta["ref_output_sha256"] = sha(exp)

    for name, keys in e2e_cases(rng):
        text = to_text(keys)
        out = run_reference(text)
        got = np.array([int(x) for x in out.split()], dtype=np.int32)
        assert got.size == keys.size and np.array_equal(got, np.sort(keys)), name
        np.save(os.path.join(HERE, f"{name}.in.npy"), keys)
        np.save(os.path.join(HERE, f"{name}.out.npy"), got)
        meta["e2e"].append({"name": name, "n": int(keys.size), "input_sep": "\\n",
                            "input_sha256": sha(text), "output_sha256": sha(out)})
        print("e2e", name, keys.size)

    # merge_chunks(int num_chunks, int *chunks[], int chunk_sizes[], int total_size)
    lib = ctypes.CDLL(os.path.join(REF_BUILD, "libref_server.so"))
    lib.merge_chunks.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.POINTER(ctypes.c_int)),
                                 ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    mc_cases = [
        ("mc_k4_unequal", [np.sort(rng.integers(-1000, 1000, n)).astype(np.int32) for n in (7, 0, 13, 1)]),
        ("mc_k1", [np.sort(rng.integers(-50, 50, 33)).astype(np.int32)]),
        ("mc_k8_dups", [np.sort(rng.integers(0, 4, n)).astype(np.int32) for n in (5, 9, 0, 2, 17, 3, 3, 1)]),
        ("mc_k3_extremes", [np.array([INT_MIN, -1, 0], np.int32), np.array([INT_MIN, INT_MIN], np.int32),
                            np.array([-1, INT_MAX - 1], np.int32)]),
        ("mc_k4_intmax_quirk", [np.array([1, INT_MAX, INT_MAX], np.int32), np.array([-5, 2], np.int32),
                                np.array([0], np.int32), np.array([INT_MAX], np.int32)]),
    ]
    cwd = os.getcwd()
    for name, runs in mc_cases:
        with tempfile.TemporaryDirectory() as d:
            os.chdir(d)
            try:
                k = len(runs)
                arrs = [np.ascontiguousarray(r, dtype=np.int32) for r in runs]
                ptrs = (ctypes.POINTER(ctypes.c_int) * k)(
                    *[a.ctypes.data_as(ctypes.POINTER(ctypes.c_int)) for a in arrs])
                sizes = (ctypes.c_int * k)(*[a.size for a in arrs])
                total = sum(a.size for a in arrs)
                lib.merge_chunks(k, ptrs, sizes, total)
                out = open("output.txt", "rb").read()
            finally:
                os.chdir(cwd)
        vals = [int(x) for x in out.split()]
        n_written = total - sum(int((a == INT_MAX).sum()) for a in arrs)
        np.savez(os.path.join(HERE, f"{name}.npz"), *arrs)
        meta["merge_chunks"].append({"name": name, "k": len(arrs), "total": total,
                                     "written_prefix": n_written,
                                     "reference_output_prefix": vals[:n_written]})
        print("merge_chunks", name, vals)

    lib2 = ctypes.CDLL(os.path.join(REF_BUILD, "libref_client.so"))
    lib2.merge_sort.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int]
    for name, n in (("ms_full_range_5000", 5000), ("ms_2", 2), ("ms_0", 0)):
        a = rng.integers(INT_MIN, INT_MAX + 1, n, dtype=np.int64).astype(np.int32)
        if n >= 2:
            a[0], a[1] = -1, INT_MAX
        b = a.copy()
        lib2.merge_sort(b.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), 0, n - 1)
        np.save(os.path.join(HERE, f"{name}.in.npy"), a)
        np.save(os.path.join(HERE, f"{name}.out.npy"), b)
        meta["merge_sort"].append({"name": name, "n": n})
        print("merge_sort", name, n)

    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
