"""GPU parity of the worker sort and the master merge against the oracle and the reference's
golden vectors.  Runs on the MI355X box only (pytest -m gpu).  Every call goes through the C ABI
(libdsort.so); the oracle is only the checker."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

CASES = json.load(open(os.path.join(GOLDEN, "cases.json")))
INT_MIN, INT_MAX = -(2**31), 2**31 - 1
I64_MIN, I64_MAX = -(2**63), 2**63 - 1
TILE32, TILE64 = 8192, 4096
WTILE = 8192  # int32 tile of the wave-register tile sort (dsort_wave.hip; merge tiles: 16384)


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_reference_kat_output_txt(gpu_ctx, oracle):
    """input.txt -> 4 equal chunks -> GPU worker sort each -> GPU merge -> output.txt bytes."""
    raw = open(os.path.join(GOLDEN, "ref_input.txt"), "rb").read()
    exp = open(os.path.join(GOLDEN, "ref_output.txt"), "rb").read()
    keys = oracle.parse(raw)
    sz, of = oracle.partition(keys.size, 4)
    chunks = [keys[int(o):int(o) + int(s)].copy() for s, o in zip(sz, of)]
    for c in chunks:
        gpu_ctx.sort(c)
    merged = gpu_ctx.merge(chunks)
    assert oracle.format(merged) == exp
    assert sha(oracle.format(merged)) == CASES["ref_output_sha256"]


@pytest.mark.parametrize("case", CASES["e2e"], ids=lambda c: c["name"])
def test_golden_e2e_whole_and_chunked(gpu_ctx, oracle, case):
    keys = np.load(os.path.join(GOLDEN, case["name"] + ".in.npy"))
    exp = np.load(os.path.join(GOLDEN, case["name"] + ".out.npy"))
    whole = gpu_ctx.sort(keys.copy())
    assert np.array_equal(whole, exp)
    sz, of = oracle.partition(keys.size, 4)
    chunks = [gpu_ctx.sort(keys[int(o):int(o) + int(s)].copy()) for s, o in zip(sz, of)]
    merged = gpu_ctx.merge(chunks)
    assert np.array_equal(merged, exp)
    assert sha(oracle.format(merged)) == case["output_sha256"]


@pytest.mark.parametrize("case", [c for c in CASES["merge_chunks"] if c["written_prefix"] == c["total"]],
                         ids=lambda c: c["name"])
def test_golden_merge_chunks(gpu_ctx, case):
    z = np.load(os.path.join(GOLDEN, case["name"] + ".npz"))
    runs = [z[f"arr_{i}"] for i in range(case["k"])]
    assert gpu_ctx.merge(runs).tolist() == case["reference_output_prefix"]


def test_merge_keeps_intmax(gpu_ctx, oracle):
    """Documented divergence from the reference: INT_MAX keys are kept."""
    runs = [np.array([1, INT_MAX, INT_MAX], np.int32), np.array([-5, 2], np.int32),
            np.array([0], np.int32), np.array([INT_MAX], np.int32)]
    assert gpu_ctx.merge(runs).tolist() == oracle.merge_runs(runs).tolist()


@pytest.mark.parametrize("case", CASES["merge_sort"], ids=lambda c: c["name"])
def test_golden_merge_sort(gpu_ctx, case):
    a = np.load(os.path.join(GOLDEN, case["name"] + ".in.npy"))
    exp = np.load(os.path.join(GOLDEN, case["name"] + ".out.npy"))
    assert np.array_equal(gpu_ctx.sort(a.copy()), exp)


SIZES = [0, 1, 2, 3, 15, 16, 17, 511, 1023, 1024, 1025, 4096, TILE32 - 1, TILE32, TILE32 + 1, 2 * TILE32,
         3 * TILE32 + 5, 5 * TILE32 - 7, WTILE - 1, WTILE + 1, 2 * WTILE - 1, 17 * TILE32 + 123, 100003,
         17 * WTILE + 1, 1 << 20, (1 << 20) + 3333]


def _dist(rng, kind, n, dt):
    info = np.iinfo(dt)
    if kind == "uniform":
        return rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
    if kind == "equal":
        return np.full(n, -1, dt)
    if kind == "sorted":
        return np.sort(rng.integers(info.min, info.max, n, dtype=dt, endpoint=True))
    if kind == "reverse":
        return np.sort(rng.integers(info.min, info.max, n, dtype=dt, endpoint=True))[::-1].copy()
    if kind == "few":
        return rng.choice(np.array([info.min, -1, 0, 1, info.max], dt), n)
    if kind == "extremes":
        a = rng.integers(-3, 3, n).astype(dt)
        a[::3] = info.max
        a[1::5] = info.min
        return a
    raise ValueError(kind)


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("kind", ["uniform", "equal", "sorted", "reverse", "few", "extremes"])
def test_sort_i32_vs_oracle(gpu_ctx, oracle, n, kind):
    rng = np.random.default_rng(n * 7 + len(kind))
    a = _dist(rng, kind, n, np.int32)
    exp = oracle.merge_sort(a) if n <= 200000 else np.sort(a, kind="stable")
    got = gpu_ctx.sort(a.copy())
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("n", [0, 1, 5, TILE64 - 1, TILE64, TILE64 + 1, 9 * TILE64 + 77, 300001])
@pytest.mark.parametrize("kind", ["uniform", "few", "extremes", "reverse"])
def test_sort_i64_vs_oracle(gpu_ctx, oracle, n, kind):
    rng = np.random.default_rng(n * 13 + len(kind))
    a = _dist(rng, kind, n, np.int64)
    exp = oracle.merge_sort(a) if n <= 200000 else np.sort(a, kind="stable")
    assert np.array_equal(gpu_ctx.sort(a.copy()), exp)


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 8, 9, 16, 33])
def test_merge_k_runs_vs_oracle(gpu_ctx, oracle, k):
    rng = np.random.default_rng(k)
    lens = rng.integers(0, 3 * TILE32, k)
    lens[0] = 0 if k > 2 else lens[0]
    runs = [np.sort(rng.integers(-1000, 1000, int(m))).astype(np.int32) for m in lens]
    exp = oracle.merge_runs(runs)
    assert np.array_equal(gpu_ctx.merge(runs), exp)
    runs64 = [np.sort(rng.integers(I64_MIN, I64_MAX, int(m), endpoint=True)) for m in lens]
    assert np.array_equal(gpu_ctx.merge(runs64), oracle.merge_runs(runs64, np.int64))


def test_merge_all_empty(gpu_ctx):
    assert gpu_ctx.merge([np.zeros(0, np.int32)] * 3).size == 0


def test_device_sort_inplace_and_copy(gpu_ctx, oracle):
    import torch
    n = 3 * TILE32 * 64 + 99
    a = oracle.gen_uniform(0x5EED2026, 0, n)
    t = torch.from_numpy(a).cuda()
    out = torch.empty_like(t)
    gpu_ctx.sort_dev(t, out)
    assert np.array_equal(t.cpu().numpy(), a)  # input untouched
    assert np.array_equal(out.cpu().numpy(), np.sort(a))
    gpu_ctx.sort_dev(t)
    assert np.array_equal(t.cpu().numpy(), np.sort(a))


def test_gpu_generator_matches_oracle(gpu_ctx, oracle):
    import torch
    t = torch.empty(100000, dtype=torch.int32, device="cuda")
    gpu_ctx.gen_uniform(t, 0x5EED2026, 12345)
    assert np.array_equal(t.cpu().numpy(), oracle.gen_uniform(0x5EED2026, 12345, 100000))
    t64 = torch.empty(50000, dtype=torch.int64, device="cuda")
    gpu_ctx.gen_uniform(t64, 7, 3)
    assert np.array_equal(t64.cpu().numpy(), oracle.gen_uniform(7, 3, 50000, np.int64))


def test_gpu_fingerprint_matches_oracle(gpu_ctx, oracle):
    import torch
    a = oracle.gen_uniform(11, 0, 1 << 20)
    t = torch.from_numpy(a).cuda()
    assert gpu_ctx.fingerprint(t) == oracle.fingerprint(a)
    b = np.random.default_rng(2).integers(I64_MIN, I64_MAX, 70001, dtype=np.int64)
    assert gpu_ctx.fingerprint(torch.from_numpy(b).cuda()) == oracle.fingerprint(b)
    s = torch.from_numpy(np.sort(a)).cuda()
    assert gpu_ctx.descents(s) == 0
    assert gpu_ctx.descents(t) == int((a[1:] < a[:-1]).sum())


@pytest.mark.parametrize("n,dt,dist", [(1 << 28, "i32", "uniform"), ((1 << 26) + 12345, "i64", "uniform"),
                                       (1 << 30, "i32", "uniform"), (1 << 30, "i64", "zipf")])
def test_full_size_properties(gpu_ctx, n, dt, dist):
    """At BASELINE sizes the oracle is too slow: check size-independent properties on the GPU --
    the output is ascending and is the same multiset as the input (fingerprint).  2^28 int32 is
    config C2; 2^30 int32 is the metric's size with the default 1024-bucket skewed layout; 2^30
    Zipf int64 is config C4 on one GPU."""
    import torch
    tdt = torch.int32 if dt == "i32" else torch.int64
    t = torch.empty(n, dtype=tdt, device="cuda")
    if dist == "zipf":
        gpu_ctx.gen_zipf_i64(t, 0x5EED2026, 0)
    else:
        gpu_ctx.gen_uniform(t, 0x5EED2026, 0)
    fp_in = gpu_ctx.fingerprint(t)
    out = torch.empty_like(t)
    gpu_ctx.sort_dev(t, out)
    assert gpu_ctx.descents(out) == 0
    assert gpu_ctx.fingerprint(out) == fp_in
    del t, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n,dt,dist", [(1 << 28, "i32", "uniform"), (1 << 30, "i32", "uniform"),
                                       (1 << 30, "i64", "zipf")])
def test_full_size_bit_exact_vs_torch_sort(gpu_ctx, n, dt, dist):
    """north_star asks for bit-exact output at the metric's sizes: the default (bucketed) path of
    dsort_sort_dev_copy compared element for element with torch.sort (rocPRIM's radix sort -- an
    independent implementation) on config C2 (2^28 int32), the metric size (2^30 int32) and
    config C4 on one GPU (2^30 Zipf int64).  The fingerprint test above stays as well."""
    import torch
    tdt = torch.int32 if dt == "i32" else torch.int64
    t = torch.empty(n, dtype=tdt, device="cuda")
    if dist == "zipf":
        gpu_ctx.gen_zipf_i64(t, 0x5EED2026, 0)
    else:
        gpu_ctx.gen_uniform(t, 0x5EED2026, 0)
    out = torch.empty_like(t)
    gpu_ctx.sort_dev(t, out)
    torch.cuda.synchronize()
    assert gpu_ctx.stats()["merge_passes"] == 0  # the two-level partition path, no merge pass
    ref = torch.sort(t).values
    assert torch.equal(out, ref)
    del t, out, ref
    torch.cuda.empty_cache()


def test_zipf_i64_sort(gpu_ctx):
    import torch
    n = (1 << 24) + 17
    t = torch.empty(n, dtype=torch.int64, device="cuda")
    gpu_ctx.gen_zipf_i64(t, 0x5EED2026)
    host = t.cpu().numpy()
    top = np.unique(host[: 1 << 20], return_counts=True)[1].max() / (1 << 20)
    assert top > 0.05  # heavy hitter present
    out = torch.empty_like(t)
    gpu_ctx.sort_dev(t, out)
    assert np.array_equal(out.cpu().numpy(), np.sort(host))


@pytest.mark.parametrize("k", [2, 7, 17, 32])
def test_merge_unbalanced_runs_i32(gpu_ctx, oracle, k):
    """One long run among tiny ones: pairs of every size, windows per pair from 1 to many, partial
    windows and empty segments in the same merge tile (dsort_wave.hip, mergew_kernel)."""
    rng = np.random.default_rng(1000 + k)
    lens = [int(x) for x in rng.integers(0, 60, k)]
    lens[k // 2] = 5 * WTILE + 333
    runs = [np.sort(rng.integers(INT_MIN, INT_MAX, m, dtype=np.int64, endpoint=True)).astype(np.int32)
            for m in lens]
    assert np.array_equal(gpu_ctx.merge(runs), oracle.merge_runs(runs))


@pytest.mark.parametrize("k", [31, 32, 64, 65])
def test_merge_many_random_runs_i32(gpu_ctx, oracle, k):
    rng = np.random.default_rng(77 + k)
    lens = rng.integers(0, 40000, k)
    runs = [np.sort(rng.integers(-50, 50, int(m))).astype(np.int32) for m in lens]  # many duplicates
    assert np.array_equal(gpu_ctx.merge(runs), oracle.merge_runs(runs))


def test_heavy_duplicates_i32(gpu_ctx):
    """Zipf-like int32 keys: the tile cuts fall inside runs of one key (partk's exact tie cut)."""
    rng = np.random.default_rng(5)
    n = (1 << 23) + 99
    a = np.minimum(rng.zipf(1.3, n), 2**31 - 1).astype(np.int64)
    a = (a * 2654435761) % (2**32) - 2**31
    a = a.astype(np.int32)
    assert np.unique(a[: 1 << 16], return_counts=True)[1].max() > (1 << 16) // 5
    assert np.array_equal(gpu_ctx.sort(a.copy()), np.sort(a))


@pytest.mark.parametrize("n", [16 * WTILE + 1, 256 * WTILE + 12345])
def test_sort_i32_pass_boundaries(gpu_ctx, n):
    """Tile counts just past one and two merge passes of fan-in 16."""
    import torch
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu_ctx.gen_uniform(t, 99, 0)
    host = t.cpu().numpy()
    out = torch.empty_like(t)
    gpu_ctx.sort_dev(t, out)
    assert np.array_equal(out.cpu().numpy(), np.sort(host))


def test_back_to_back_sorts_on_two_streams(gpu_ctx):
    """A sort returns while its last kernels still run, and the context's arenas are shared: a
    following sort on another stream must wait for it on the device (order_begin/order_end in
    dsort_wave.hip).  Two bucketed sorts issued back to back on two streams, then checked."""
    import torch
    n = (1 << 25) + 4097
    a = torch.empty(n, dtype=torch.int32, device="cuda")
    b = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu_ctx.gen_uniform(a, 11)
    gpu_ctx.gen_uniform(b, 12)
    torch.cuda.synchronize()
    oa, ob = torch.empty_like(a), torch.empty_like(b)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(2):
        with torch.cuda.stream(s1):
            gpu_ctx.sort_dev(a, oa)
        with torch.cuda.stream(s2):
            gpu_ctx.sort_dev(b, ob)
    torch.cuda.synchronize()
    assert torch.equal(oa, torch.sort(a)[0])
    assert torch.equal(ob, torch.sort(b)[0])


def test_stage_timing_off_sorts_the_same_and_records_nothing(gpu_ctx):
    """DSORT_OPT_STAGE_TIMING = 0 (bench.py's timed steps): the sort records no stage events -- its
    *_ms statistics read 0 -- and its output is the same as with them; switched back on, the next
    sort's statistics are measured again."""
    import torch
    n = (1 << 25) + 123
    a = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu_ctx.gen_uniform(a, 21)
    o = torch.empty_like(a)
    exp = torch.sort(a)[0]
    with gpu_ctx.options(stage_timing=0):
        assert gpu_ctx.get_option("stage_timing") == 0
        gpu_ctx.sort_dev(a, o)
        torch.cuda.synchronize()
        st = gpu_ctx.stats()
    assert torch.equal(o, exp)
    assert st["total_ms"] == 0 and st["tile_sort_kernel_ms"] == 0 and st["bucket_scatter_ms"] == 0, st
    o.zero_()
    gpu_ctx.sort_dev(a, o)
    torch.cuda.synchronize()
    st = gpu_ctx.stats()
    assert torch.equal(o, exp)
    assert st["total_ms"] > 0 and st["tile_sort_kernel_ms"] > 0 and st["bucket_scatter_ms"] > 0, st


def test_c3_receive_merge_8_runs_bit_exact(gpu_ctx):
    """Config C3's per-rank receive merge (dsort_api.hip sample_sort step 8: the gather + merge of
    server.c:414-415 / 500-515): 8 sorted runs of 2^26 int32 keys inside one rank's key range
    (1/8 of the int32 range, as uniform input gives every rank) merged by dsort_merge_dev_i32,
    compared element for element with torch.sort."""
    import torch
    P, m = 8, 1 << 26
    recv = torch.empty(P * m, dtype=torch.int32, device="cuda")
    gpu_ctx.gen_uniform(recv, 0x5EED2026 ^ 0xC3, 0)
    span = (1 << 32) // P
    r64 = recv.to(torch.int64) & (span - 1)
    recv.copy_((r64 - (1 << 31) + 3 * span).to(torch.int32))
    del r64
    for s in range(P):
        gpu_ctx.sort_dev(recv[s * m:(s + 1) * m])
    out = torch.empty_like(recv)
    gpu_ctx.merge_dev(recv, [m] * P, out)
    torch.cuda.synchronize()
    assert torch.equal(out, torch.sort(recv).values)
    del recv, out
    torch.cuda.empty_cache()


def _shaped_i32(gpu_ctx, n, dist):
    import torch
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu_ctx.gen_uniform(t, 0x5EED2026, 0)
    if dist == "ref100":  # the shape of the reference's input.txt: keys in [1, 100]
        t.copy_((t & 0x7FFFFFFF) % 100 + 1)
    elif dist == "byte":  # 256 small keys
        t.copy_(t & 255)
    elif dist == "signed100":  # 100 keys around zero (the sign flip of the slot map)
        t.copy_((t & 0x7FFFFFFF) % 100 - 50)
    elif dist == "narrow16":  # 2^16 distinct keys across zero
        t.copy_((t & 0xFFFF) - 30000)
    elif dist == "mixed":  # half uniform, half in [1, 100]: no map separates the small keys
        t.copy_(torch.where((t & 1) == 1, t, (t & 0x7FFFFFFF) % 100 + 1))
    elif dist == "mixed_signed":  # half uniform, half in [-50, 50): the small keys in two fixed slots
        t.copy_(torch.where((t & 1) == 1, t, (t & 0x7FFFFFFF) % 100 - 50))
    elif dist == "cluster":  # half uniform, half distinct keys of [0, 2^20): one slot of many distinct keys
        t.copy_(torch.where((t & 1) == 1, t, (t >> 1) & 0xFFFFF))
    return t


@pytest.mark.parametrize("dist,want_map", [("ref100", 1), ("byte", 1), ("signed100", 1), ("narrow16", 1),
                                           ("mixed", 3), ("mixed_signed", 3), ("cluster", 3), ("uniform", 0)])
def test_small_key_ranges_adaptive_map_bit_exact(gpu_ctx, dist, want_map):
    """int32 keys from a narrow range (the reference's input.txt holds 10 000 keys in [1, 100]): the
    fixed 11-bit slot map of the first partition level puts every splitter into one slot; the slot
    map kernel then switches to the adaptive map (linear over the splitters' range, one-key slots;
    DESIGN.md §3.3), reported as first_level_map.  Round 6: small keys mixed half and half with
    uniform ones (no map separates them) keep the fixed map with its most crowded slot refined by a
    second table (first_level_map 3): [1, 100] (one-key sub-slots), [-50, 50) (across two fixed
    slots, one refined), 2^20 distinct small keys (sub-slots of distinct splitters).  2^28 keys
    (config C2's size) against torch.sort, element for element."""
    import torch
    n = 1 << 28
    t = _shaped_i32(gpu_ctx, n, dist)
    out = torch.empty_like(t)
    gpu_ctx.sort_dev(t, out)
    torch.cuda.synchronize()
    st = gpu_ctx.stats()
    if want_map is not None:
        assert st["first_level_map"] == want_map, st
    assert torch.equal(out, torch.sort(t).values)
    del t, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n", [(1 << 25) + 77, 3 * (1 << 25) - 5])
def test_small_key_ranges_other_sizes(gpu_ctx, n):
    """The adaptive map at other bucket counts (32 and 96 buckets), odd sizes."""
    import torch
    for dist in ("ref100", "byte"):
        t = _shaped_i32(gpu_ctx, n, dist)
        out = torch.empty_like(t)
        gpu_ctx.sort_dev(t, out)
        torch.cuda.synchronize()
        assert gpu_ctx.stats()["first_level_map"] == 1
        assert torch.equal(out, torch.sort(t).values)
