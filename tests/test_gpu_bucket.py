"""The bucketed sort against numpy on the MI355X: the sample-splitter partition (dsort_bucket.h,
dsort_sub.h), then either the second partition level + tile packing (default: no merge pass) or,
with DSORT_OPT_SUB_KEYS = 0, the tile sort and k-way merge passes inside every bucket.  The option
DSORT_OPT_BUCKETS forces a bucket count at any size, so small inputs exercise the same kernels as
the 2^30-key bench: empty buckets and sub-buckets, single-tile buckets, unaligned tiles, heavy
duplicates split across buckets and sub-buckets by the (key, position) composite, oversized
sub-buckets (merged afterwards)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

INT_MIN, INT_MAX = -(2**31), 2**31 - 1
TILE = 8192  # int32 tile of the tile sort (dsort_wave.hip WG<int32_t>)


def _keys(rng, kind, n):
    if kind == "uniform":
        return rng.integers(INT_MIN, INT_MAX, n, endpoint=True).astype(np.int32)
    if kind == "equal":
        return np.full(n, 7, np.int32)
    if kind == "few":
        return (rng.integers(0, 4, n) * 1000 - 1500).astype(np.int32)
    if kind == "sorted":
        return np.sort(rng.integers(INT_MIN, INT_MAX, n, endpoint=True).astype(np.int32))
    if kind == "reverse":
        return np.sort(rng.integers(INT_MIN, INT_MAX, n, endpoint=True).astype(np.int32))[::-1].copy()
    if kind == "extremes":
        return rng.choice(np.array([INT_MIN, INT_MIN + 1, -1, 0, 1, INT_MAX - 1, INT_MAX], np.int32), n)
    if kind == "narrow":  # every key inside one radix slot of the bucket lookup
        return rng.integers(1000, 1064, n).astype(np.int32)
    raise ValueError(kind)


def _sort(ctx, a, inplace):
    import torch
    t = torch.from_numpy(a).cuda()
    if inplace:
        ctx.sort_dev(t)
        out = t
    else:
        out = torch.empty_like(t)
        ctx.sort_dev(t, out)
        assert np.array_equal(t.cpu().numpy(), a)  # the input is left alone
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("kind", ["uniform", "equal", "few", "sorted", "reverse", "extremes", "narrow"])
@pytest.mark.parametrize("B,n", [(2, 100_003), (3, 17), (7, 3 * TILE + 5), (33, 1_000_003),
                                 (64, 4 * TILE), (1024, 500_000)])
@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("mode", ["local", "scatter", "merge"])
def test_bucketed_sort_vs_numpy(gpu_ctx, kind, B, n, inplace, mode):
    """Every second-level path: local partition + gathering tile sort (default), scatter to
    sub-buckets, and round 1's merge passes inside the buckets."""
    a = _keys(np.random.default_rng(B * 131 + n), kind, n)
    opts = {"local": dict(), "scatter": dict(sub_gather=0), "merge": dict(sub_keys=0)}[mode]
    with gpu_ctx.options(buckets=B, **opts):
        assert np.array_equal(_sort(gpu_ctx, a, inplace), np.sort(a))


@pytest.mark.parametrize("tiles,passes", [(200, 2), (300, 3)])
def test_bucketed_sort_multi_pass_buckets(gpu_ctx, tiles, passes):
    """Few buckets of many tiles: more than 16 (256) runs per bucket -> 2 (3) merge passes on the
    merge path; the sub-bucket path needs none (its 1024 sub-buckets per bucket are still below a
    tile)."""
    a = _keys(np.random.default_rng(tiles), "uniform", 2 * tiles * TILE + 777)
    with gpu_ctx.options(buckets=2, sub_keys=0):
        assert np.array_equal(_sort(gpu_ctx, a, False), np.sort(a))
        assert gpu_ctx.stats()["merge_passes"] == passes
    with gpu_ctx.options(buckets=2):
        assert np.array_equal(_sort(gpu_ctx, a, False), np.sort(a))
        # The sub-bucket path stays on the local partition.  A sub-bucket above a tile (a sampling
        # outlier, about 1 % of the sorts of this case) is cut by chunks into tiles whose outputs
        # are merged: one small merge for that sub-bucket alone, never the scatter path.
        st = gpu_ctx.stats()
        assert st["sub_scatter_fallback"] == 0
        assert st["merge_passes"] == (1 if st["sub_split_subbuckets"] else 0)


@pytest.mark.parametrize("dtype", ["i32", "i64"])
@pytest.mark.parametrize("B", [3, 9])
def test_bucketed_sort_mixed_fanin(gpu_ctx, dtype, B):
    """Buckets whose mean size sits at a power-of-two run count (64 int32 tiles, 256 int64
    tiles), so the sampling spread puts some buckets above it and some below: a pass mixes
    per-bucket fan-ins (one launch per kernel fan-in).  It must sort exactly (keys: a dense
    duplicate-heavy cluster plus the full int range)."""
    import torch
    rng = np.random.default_rng(B * 7 + 3)
    n = B * 64 * TILE + 333
    dense = rng.integers(-1000, 1000, n // 2)
    tail = rng.integers(INT_MIN, INT_MAX, n - n // 2, endpoint=True)
    a = rng.permutation(np.concatenate([dense, tail])).astype(np.int32 if dtype == "i32" else np.int64)
    t = torch.from_numpy(a).cuda()
    out = torch.empty_like(t)
    with gpu_ctx.options(buckets=B, sub_keys=0):
        gpu_ctx.sort_dev(t, out)
        torch.cuda.synchronize()
        assert gpu_ctx.stats()["merge_passes"] >= 1
    assert np.array_equal(out.cpu().numpy(), np.sort(a))


def test_forced_buckets_small_input_matches_unforced(gpu_ctx):
    """with a forced bucket count the splitter samples used to be sorted by the
    bucketed int64 sort in place over its own arena.  The nested sample sort now never buckets:
    a forced-B sort equals the default path and numpy."""
    import torch
    rng = np.random.default_rng(11)
    for kind in ("uniform", "few", "equal"):
        a = _keys(rng, kind, 1 << 21)
        t = torch.from_numpy(a).cuda()
        o1, o2 = torch.empty_like(t), torch.empty_like(t)
        with gpu_ctx.options(buckets=1024):
            gpu_ctx.sort_dev(t, o1)
        gpu_ctx.sort_dev(t, o2)
        torch.cuda.synchronize()
        assert torch.equal(o1, o2)
        assert np.array_equal(o1.cpu().numpy(), np.sort(a))


@pytest.mark.parametrize("dtype", ["i32", "i64"])
@pytest.mark.parametrize("kind", ["uniform", "few", "zipfish"])
@pytest.mark.parametrize("sub_keys,os,merged", [(-1, -1, False), (300, 1, None), (40_000, 4, True)])
def test_sub_buckets(gpu_ctx, dtype, kind, sub_keys, os, merged):
    """Second partition level: default sub-buckets (no merge pass), tiny ones with one sample each
    (crowded slot tables, many empty sub-buckets), and ones larger than a tile (every sub-bucket
    is tile-sorted in pieces and merged: merge_passes >= 1).  Duplicate-heavy keys split over
    sub-buckets by (key, position)."""
    import torch
    B = 16
    n = B * 40 * TILE + 101
    rng = np.random.default_rng(len(kind) * 10 + os)
    if kind == "zipfish":
        a = (rng.zipf(1.3, n) % 100_003) * 7919 - 40_000_000
    elif kind == "few":
        a = rng.integers(0, 4, n) * 1000 - 1500
    else:
        a = rng.integers(INT_MIN, INT_MAX, n, endpoint=True)
    a = a.astype(np.int32 if dtype == "i32" else np.int64)
    t = torch.from_numpy(a).cuda()
    out = torch.empty_like(t)
    with gpu_ctx.options(buckets=B, sub_keys=sub_keys, sub_oversample=os):
        gpu_ctx.sort_dev(t, out)
        torch.cuda.synchronize()
        passes = gpu_ctx.stats()["merge_passes"]
    assert np.array_equal(out.cpu().numpy(), np.sort(a))
    if merged and dtype == "i64" and kind == "few":
        # (int64 one-key slots put every copy of a key in its inner buckets, DSORT_ONEKEY_HASH: with 4
        # keys of ~4 splitters each every bucket is pure or empty, and none reaches the second level)
        merged = False
    if merged is not None:
        assert (passes >= 1) == merged


def test_bucketed_default_at_2p26_matches_regular_path(gpu_ctx):
    """Default bucket count at 2^26 (64 buckets) and buckets=0 (regular passes): same output, no
    descents, same multiset."""
    import torch
    n = 1 << 26
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu_ctx.gen_uniform(t, 0x5EED2026)
    fp = gpu_ctx.fingerprint(t)
    o1, o2 = torch.empty_like(t), torch.empty_like(t)
    gpu_ctx.sort_dev(t, o1)
    assert gpu_ctx.stats()["merge_passes"] == 0  # 64 buckets of ~2^20 keys, sub-buckets in tiles
    with gpu_ctx.options(buckets=0):
        gpu_ctx.sort_dev(t, o2)
    torch.cuda.synchronize()
    assert gpu_ctx.descents(o1) == 0 and gpu_ctx.fingerprint(o1) == fp
    assert torch.equal(o1, o2)


I64_MIN, I64_MAX = -(2**63), 2**63 - 1


def _keys64(rng, kind, n):
    if kind == "uniform":
        return rng.integers(I64_MIN, I64_MAX, n, endpoint=True, dtype=np.int64)
    if kind == "equal":
        return np.full(n, -5, np.int64)
    if kind == "few":
        return rng.integers(0, 3, n).astype(np.int64) * (1 << 40) - (1 << 41)
    if kind == "extremes":
        return rng.choice(np.array([I64_MIN, I64_MIN + 1, -1, 0, 1, I64_MAX - 1, I64_MAX], np.int64), n)
    if kind == "small":  # all keys inside one lookup slot (top 12 bits equal)
        return rng.integers(0, 1 << 20, n).astype(np.int64)
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["uniform", "equal", "few", "extremes", "small"])
@pytest.mark.parametrize("B,n", [(2, 50_001), (5, 4096 * 3 + 1), (64, 1_000_003), (1024, 300_000)])
@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("mode", ["local", "scatter"])
def test_bucketed_sort_i64_vs_numpy(gpu_ctx, kind, B, n, inplace, mode):
    a = _keys64(np.random.default_rng(B * 7 + n), kind, n)
    with gpu_ctx.options(buckets=B, sub_gather=1 if mode == "local" else 0):
        assert np.array_equal(_sort(gpu_ctx, a, inplace), np.sort(a))


def test_bucketed_zipf_i64_2p26(gpu_ctx):
    """Default bucket count on the BASELINE config-4 distribution (heavy duplicates): sorted,
    same multiset, identical to the regular passes."""
    import torch
    n = 1 << 26
    t = torch.empty(n, dtype=torch.int64, device="cuda")
    gpu_ctx.gen_zipf_i64(t, 0x5EED2026)
    fp = gpu_ctx.fingerprint(t)
    o1, o2 = torch.empty_like(t), torch.empty_like(t)
    gpu_ctx.sort_dev(t, o1)
    with gpu_ctx.options(buckets=0):
        gpu_ctx.sort_dev(t, o2)
    torch.cuda.synchronize()
    assert gpu_ctx.descents(o1) == 0 and gpu_ctx.fingerprint(o1) == fp
    assert torch.equal(o1, o2)


@pytest.mark.parametrize("dtype", ["i32", "i64"])
@pytest.mark.parametrize("shift_in,shift_out", [(1, 3), (3, 0), (0, 5), (2, 2)])
@pytest.mark.parametrize("B,n", [(5, 300_001), (700, 2_000_003)])
def test_bucketed_sort_unaligned_views(gpu_ctx, dtype, shift_in, shift_out, B, n):
    """Input and output tensors that start at element offsets (not 16-byte aligned): the 16-byte
    loads of the tile sort and the line-aligned bucket scatter must not assume aligned caller
    buffers."""
    import torch
    rng = np.random.default_rng(B + shift_in * 7 + shift_out)
    a = _keys(rng, "uniform", n) if dtype == "i32" else _keys64(rng, "uniform", n)
    tdt = torch.int32 if dtype == "i32" else torch.int64
    src = torch.empty(n + 8, dtype=tdt, device="cuda")
    dst = torch.full((n + 8,), 77, dtype=tdt, device="cuda")
    src[shift_in:shift_in + n] = torch.from_numpy(a).cuda()
    with gpu_ctx.options(buckets=B):
        gpu_ctx.sort_dev(src[shift_in:shift_in + n], dst[shift_out:shift_out + n])
        torch.cuda.synchronize()
    d = dst.cpu().numpy()
    assert np.array_equal(d[shift_out:shift_out + n], np.sort(a))
    assert (d[:shift_out] == 77).all() and (d[shift_out + n:] == 77).all()  # nothing written outside
    assert np.array_equal(src[shift_in:shift_in + n].cpu().numpy(), a)


@pytest.mark.parametrize("dtype", ["i32", "i64"])
@pytest.mark.parametrize("shift", [1, 2, 3])
def test_bucketed_sort_unaligned_view_in_place(gpu_ctx, dtype, shift):
    import torch
    n = 1_500_007
    rng = np.random.default_rng(shift)
    a = _keys(rng, "few", n) if dtype == "i32" else _keys64(rng, "few", n)
    tdt = torch.int32 if dtype == "i32" else torch.int64
    buf = torch.full((n + 8,), 5, dtype=tdt, device="cuda")
    buf[shift:shift + n] = torch.from_numpy(a).cuda()
    with gpu_ctx.options(buckets=37):
        gpu_ctx.sort_dev(buf[shift:shift + n])
        torch.cuda.synchronize()
    d = buf.cpu().numpy()
    assert np.array_equal(d[shift:shift + n], np.sort(a))
    assert (d[:shift] == 5).all() and (d[shift + n:] == 5).all()


@pytest.mark.parametrize("dtype", [np.int32, np.int64])
@pytest.mark.parametrize("mode", ["local", "scatter"])
@pytest.mark.parametrize("n", [1 << 22, (1 << 22) + 12345])
def test_pure_buckets_heavy_keys(gpu_ctx, dtype, mode, n):
    """Heavy keys filling whole buckets: a bucket between two splitters of the same key holds only
    that key and is copied to the output as it lies (no sub-buckets, no tiles); the buckets around
    it (the heavy key plus its neighbours) take the normal path.  Runs of pure buckets next to each
    other and a pure bucket next to the first and the last bucket."""
    rng = np.random.default_rng(n + (7 if dtype == np.int64 else 0))
    info = np.iinfo(dtype)
    a = rng.integers(info.min, info.max, n, endpoint=True, dtype=dtype)
    r = rng.random(n)
    a[r < 0.40] = dtype(7)
    a[(r >= 0.40) & (r < 0.55)] = dtype(-3)
    a[(r >= 0.55) & (r < 0.60)] = info.max
    a[(r >= 0.60) & (r < 0.63)] = info.min
    opts = {"local": dict(), "scatter": dict(sub_gather=0)}[mode]
    with gpu_ctx.options(buckets=256, **opts):
        assert np.array_equal(_sort(gpu_ctx, a, False), np.sort(a))


@pytest.mark.parametrize("dtype", [np.int32, np.int64])
@pytest.mark.parametrize("mode", ["local", "scatter"])
@pytest.mark.parametrize("n", [1 << 22, (1 << 22) + 999])
def test_one_key_slots_skewed(gpu_ctx, dtype, mode, n):
    """Skewed small keys (a Zipf head) with the type's extremes: the int64 lookups switch to the
    log slot map, every heavy key gets a one-key slot whose copies are split over its run of
    buckets -- int32 by index (the outer two exactly as the composite order), int64 by a hash of
    the index over the inner ones (DSORT_ONEKEY_HASH) -- and the tail and the extremes share wide
    slots (dsort_bucket.h BkMap, bucket_fast, bucket_onekey)."""
    rng = np.random.default_rng(n + (11 if dtype == np.int64 else 0))
    info = np.iinfo(dtype)
    a = np.minimum(rng.zipf(1.3, n), 1 << 20).astype(dtype)
    r = rng.random(n)
    a[r < 0.01] = info.max
    a[(r >= 0.01) & (r < 0.02)] = info.min
    a[(r >= 0.02) & (r < 0.05)] = rng.integers(info.min, info.max, int(((r >= 0.02) & (r < 0.05)).sum()),
                                               dtype=dtype)
    opts = {"local": dict(), "scatter": dict(sub_gather=0)}[mode]
    with gpu_ctx.options(buckets=512, **opts):
        assert np.array_equal(_sort(gpu_ctx, a, False), np.sort(a))


@pytest.mark.parametrize("dtype", ["i32", "i64"])
@pytest.mark.parametrize("kind", ["uniform", "sorted", "few"])
@pytest.mark.parametrize("sub_keys", [20_000, 60_000])
def test_oversized_subbuckets_split_on_local_path(gpu_ctx, dtype, kind, sub_keys):
    """Sub-buckets forced above a tile (DSORT_OPT_SUB_KEYS > TILE) on the default local path: each
    one is cut by chunks into tiles (sb_scan_kernel<true>, split_tiles) and their outputs merged.
    Deterministic: every non-trivial sub-bucket is split, the sort never leaves the local path, and
    the output is exact."""
    import torch
    B = 4
    n = B * 48 * TILE + 4097
    rng = np.random.default_rng(sub_keys + len(kind))
    if dtype == "i32":
        a = _keys(rng, kind if kind != "few" else "few", n)
    else:
        a = _keys64(rng, {"uniform": "uniform", "sorted": "uniform", "few": "few"}[kind], n)
        if kind == "sorted":
            a = np.sort(a)
    t = torch.from_numpy(a).cuda()
    out = torch.empty_like(t)
    with gpu_ctx.options(buckets=B, sub_keys=sub_keys):
        gpu_ctx.sort_dev(t, out)
        torch.cuda.synchronize()
        st = gpu_ctx.stats()
    assert np.array_equal(out.cpu().numpy(), np.sort(a))
    assert st["sub_scatter_fallback"] == 0
    if kind != "few":  # (few distinct keys: most buckets hold one key and skip the second level)
        assert st["sub_split_subbuckets"] > 0 and st["merge_passes"] >= 1


@pytest.mark.parametrize("kind", ["uniform", "sorted", "few"])
def test_large_buckets_take_16k_tiles(gpu_ctx, kind):
    """int32 buckets above 2M keys (C3's 4M-key buckets per rank) are tile-sorted on 16384-key
    tiles with sub-buckets of an eighth of a tile (sub_sort): exact output, the tile size in the
    stats, no over-tile split and no scatter fallback on uniform keys."""
    import torch
    n = (1 << 23) + 777  # two buckets of about 4.2M keys
    a = _keys(np.random.default_rng(23 + len(kind)), kind, n)
    t = torch.from_numpy(a).cuda()
    out = torch.empty_like(t)
    with gpu_ctx.options(buckets=2):
        gpu_ctx.sort_dev(t, out)
        torch.cuda.synchronize()
        st = gpu_ctx.stats()
    assert np.array_equal(out.cpu().numpy(), np.sort(a))
    assert st["sub_scatter_fallback"] == 0
    if kind == "uniform":
        assert st["tile_keys"] == 2 * TILE and st["sub_split_subbuckets"] == 0


@pytest.mark.parametrize("dtype", [np.int32, np.int64])
@pytest.mark.parametrize("kind", ["sorted", "reverse", "noisy", "sawtooth", "sorted_dups"])
@pytest.mark.parametrize("mode", ["local", "scatter"])
def test_runs_hint_inputs(gpu_ctx, dtype, kind, mode):
    """Presorted inputs turn on the runs hint (BkMap.hot, from the splitters' input indices): the
    histogram, the scatter and the second level's sub-bucket counts (sb_local_kernel) then count a
    wave's run of one (sub-)bucket with one atomic (bk::bucket_bump).  The hint is only a hint, so
    inputs that set it but break the runs (1 % of the keys moved, sorted blocks in falling order,
    long runs of equal keys) must sort exactly too."""
    rng = np.random.default_rng(len(kind) * 17 + (5 if dtype == np.int64 else 0))
    info = np.iinfo(dtype)
    n = (1 << 21) + 333
    if kind == "sorted_dups":
        a = np.sort(rng.integers(-40, 40, n)).astype(dtype)
    else:
        a = np.sort(rng.integers(info.min, info.max, n, dtype=dtype, endpoint=True))
    if kind == "reverse":
        a = a[::-1].copy()
    elif kind == "noisy":
        i = rng.integers(0, n, n // 100)
        a[i] = rng.integers(info.min, info.max, i.size, dtype=dtype, endpoint=True)
    elif kind == "sawtooth":  # ascending blocks of 2^17 keys, the blocks in descending order
        blocks = [a[s:s + (1 << 17)] for s in range(0, n, 1 << 17)]
        a = np.concatenate(blocks[::-1])
    opts = {"local": dict(), "scatter": dict(sub_gather=0)}[mode]
    with gpu_ctx.options(buckets=256, **opts):
        assert np.array_equal(_sort(gpu_ctx, a, False), np.sort(a))


@pytest.mark.parametrize("order", ["random", "sorted", "reverse"])
@pytest.mark.parametrize("mode", ["local", "scatter"])
@pytest.mark.parametrize("B", [256, 1024])
def test_int32_one_key_slots(gpu_ctx, order, mode, B):
    """int32 one-key slots (bucket_onekey through the packed entry's field 3 in the scatter and
    the histogram's flag, BkMap.one): 16 distinct keys spread over the whole range each own a
    slot of the fixed 11-bit map and a run of buckets; two keys that share a slot, the type's
    extremes and a thin uniform tail keep the searched and the plain slots busy in the same sort."""
    rng = np.random.default_rng(B + len(order) * 3 + len(mode))
    n = (1 << 22) + 4097
    heavy = (np.arange(16, dtype=np.int64) * (1 << 28) - (1 << 31) + 12345).astype(np.int32)
    a = rng.choice(heavy, n)
    r = rng.random(n)
    a[r < 0.05] = 77  # two keys in one slot (77 and 78)
    a[(r >= 0.05) & (r < 0.08)] = 78
    a[(r >= 0.08) & (r < 0.09)] = INT_MIN
    a[(r >= 0.09) & (r < 0.10)] = INT_MAX
    tail = r >= 0.97
    a[tail] = rng.integers(INT_MIN, INT_MAX, int(tail.sum()), endpoint=True)
    if order != "random":
        a = np.sort(a)
        if order == "reverse":
            a = a[::-1].copy()
    opts = {"local": dict(), "scatter": dict(sub_gather=0)}[mode]
    with gpu_ctx.options(buckets=B, **opts):
        assert np.array_equal(_sort(gpu_ctx, a, False), np.sort(a))


@pytest.mark.parametrize("dtype", ["i32", "i64"])
@pytest.mark.parametrize("kind", ["uniform", "sorted"])
def test_tile_table_overflow_after_early_tile_sort(gpu_ctx, dtype, kind):
    """The local path launches the tile sort of its first (keys / TILE) tiles before the host reads
    the tile count back (sub_sort, tile_sort_early).  DSORT_OPT_TEST_TILE_CAP shrinks the tile
    tables below the tiles the packing makes but above that early part, so the sort finds the
    overflow with the early tile sort in flight and takes the scatter path over the same arena:
    the output is still exact, and the fallback is reported."""
    import torch
    B = 256  # (the piece tables inside the scan, the early launch's condition)
    tile = TILE  # (8192 keys for both widths)
    n = B * 5 * tile + 333
    rng = np.random.default_rng(91 + len(kind))
    a = _keys(rng, kind, n) if dtype == "i32" else _keys64(rng, "uniform", n)
    if dtype == "i64" and kind == "sorted":
        a = np.sort(a)
    t = torch.from_numpy(a).cuda()
    out = torch.empty_like(t)
    early = n // tile
    with gpu_ctx.options(buckets=B, test_tile_cap=early + 8):
        gpu_ctx.sort_dev(t, out)
        torch.cuda.synchronize()
        st = gpu_ctx.stats()
    assert np.array_equal(out.cpu().numpy(), np.sort(a))
    assert st["sub_scatter_fallback"] == 1
    with gpu_ctx.options(buckets=B):
        gpu_ctx.sort_dev(t, out)
        torch.cuda.synchronize()
        st = gpu_ctx.stats()
    assert np.array_equal(out.cpu().numpy(), np.sort(a))
    assert st["sub_scatter_fallback"] == 0


@pytest.mark.parametrize("dtype", ["i32", "i64"])
def test_tile_table_overflow_with_dropped_pure_buckets(gpu_ctx, dtype):
    """the out-of-place first-level scatter drops the keys of pure buckets (one heavy
    key) and the second level fills their output ranges.  When the tile tables overflow, the
    scatter-path retry must fill them itself (it is passed the fill keys) -- half the keys are one
    heavy key here, so about half the output comes from the fill.  DSORT_OPT_TEST_TILE_CAP is set
    just above the early tile sort's part, taken from a first run's tile_sort_keys."""
    import torch
    B = 256
    n = B * 5 * TILE + 333
    rng = np.random.default_rng(4242)
    if dtype == "i32":
        a = _keys(rng, "uniform", n)
        a[rng.random(n) < 0.5] = 123_457
    else:
        a = _keys64(rng, "uniform", n)
        a[rng.random(n) < 0.5] = -(1 << 33) + 5
    t = torch.from_numpy(a).cuda()
    out = torch.empty_like(t)
    with gpu_ctx.options(buckets=B):
        gpu_ctx.sort_dev(t, out)
        torch.cuda.synchronize()
        st = gpu_ctx.stats()
    want = np.sort(a)
    assert np.array_equal(out.cpu().numpy(), want)
    assert st["sub_scatter_fallback"] == 0 and st["tile_sort_keys"] < 0.6 * n, st  # pure buckets skipped
    early = st["tile_sort_keys"] // TILE
    out.fill_(0)
    with gpu_ctx.options(buckets=B, test_tile_cap=early + 8):
        gpu_ctx.sort_dev(t, out)
        torch.cuda.synchronize()
        st = gpu_ctx.stats()
    assert st["sub_scatter_fallback"] == 1, st
    assert np.array_equal(out.cpu().numpy(), want)
