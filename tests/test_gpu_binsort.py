"""The bin sort of a tile (dsort_wave.hip bin_sort_tile) and its fall back to the bitonic tile
sort, against numpy on the MI355X.  Inputs below 2^25 keys are sorted tile by tile (8192 int32 /
8192 int64 keys, then merge passes), so each case below shapes the tiles directly:

- spread keys: every tile takes the bin path;
- a cluster of many distinct keys inside a wide range: one bin holds thousands of different keys,
  the window passes cannot sort it, the check declines the tile and the bitonic sort runs;
- duplicate runs: whole waves share a bin (aggregated atomics), the bins are trivially sorted;
- key_max keys and padding: they are not binned and come out as the tail of the tile;
- key_min and key_max together: the full-range offset arithmetic."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

I32 = np.iinfo(np.int32)
I64 = np.iinfo(np.int64)


def _sort(ctx, a):
    import torch
    t = torch.from_numpy(a).cuda()
    out = torch.empty_like(t)
    ctx.sort_dev(t, out)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _case(kind, n, dt, rng):
    info = np.iinfo(dt)
    if kind == "spread":
        return rng.integers(info.min, info.max, n, endpoint=True, dtype=dt)
    if kind == "cluster":  # 90 % distinct keys in [0, 50000), the rest over the whole range
        a = rng.integers(0, 50_000, n).astype(dt)
        m = rng.random(n) < 0.1
        a[m] = rng.integers(info.min, info.max, int(m.sum()), endpoint=True, dtype=dt)
        return a
    if kind == "runs":  # a few heavy values plus spread keys
        a = rng.integers(info.min, info.max, n, endpoint=True, dtype=dt)
        m = rng.random(n) < 0.7
        a[m] = rng.choice(np.array([-7, 3, 1 << 20, info.max // 3], dtype=dt), int(m.sum()))
        return a
    if kind == "maxheavy":
        a = rng.integers(-1000, 1000, n).astype(dt)
        a[rng.random(n) < 0.4] = info.max
        return a
    if kind == "extremes":
        a = rng.integers(info.min, info.max, n, endpoint=True, dtype=dt)
        a[rng.random(n) < 0.2] = info.min
        a[rng.random(n) < 0.2] = info.max
        return a
    if kind == "two":  # two values far apart: two bins, each a run
        return rng.choice(np.array([info.min + 5, info.max - 5], dtype=dt), n)
    if kind == "narrow_distinct":  # range smaller than the bin count
        return rng.integers(100, 1100, n).astype(dt)
    raise ValueError(kind)


@pytest.mark.parametrize("dtype", [np.int32, np.int64])
@pytest.mark.parametrize("kind", ["spread", "cluster", "runs", "maxheavy", "extremes", "two", "narrow_distinct"])
@pytest.mark.parametrize("n", [1, 17, 8191, 16384, 3 * 16384 + 5, 1 << 20])
def test_binsort_tiles_vs_numpy(gpu_ctx, dtype, kind, n):
    a = _case(kind, n, dtype, np.random.default_rng(n * 7 + len(kind)))
    with gpu_ctx.options(buckets=0):
        assert np.array_equal(_sort(gpu_ctx, a), np.sort(a))


@pytest.mark.parametrize("dtype", [np.int32, np.int64])
@pytest.mark.parametrize("kind", ["cluster", "runs", "maxheavy", "extremes"])
def test_binsort_in_the_bucketed_path(gpu_ctx, dtype, kind):
    """The same shapes through the partition (forced buckets): gathered tiles, the splitter hint
    for duplicate runs, declined tiles re-gathered by the bitonic sort."""
    n = 3_000_017
    a = _case(kind, n, dtype, np.random.default_rng(len(kind)))
    with gpu_ctx.options(buckets=16):
        assert np.array_equal(_sort(gpu_ctx, a), np.sort(a))
