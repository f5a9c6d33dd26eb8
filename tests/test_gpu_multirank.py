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

from conftest import REPO

pytestmark = pytest.mark.gpu
DRIVER = os.path.join(REPO, "tests", "mp_samplesort.py")


def run_ranks(tmp_path, world, n, dtype="i32", dist="uniform", transport="host", opts=None, expect_fail=False):
    store = str(tmp_path / "store")  # (a file rendezvous: no port to lose)
    out = str(tmp_path / "ss")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, DRIVER, str(r), str(world), store, str(n), dtype, dist, out,
                               transport, json.dumps(opts or {})],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(world)]
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            tails = list(logs)
            for q in procs[len(logs):]:
                try:
                    tails.append(q.communicate(timeout=10)[0].decode(errors="replace"))
                except (subprocess.TimeoutExpired, ValueError, OSError):
                    tails.append("(no output)")
            pytest.fail("ranks timed out; their last output:\n" + "\n---\n".join(t[-600:] for t in tails))
        logs.append(o.decode(errors="replace"))
    for p, lg in zip(procs, logs):
        assert p.returncode == 0, lg[-3000:]
    if expect_fail:
        return [json.load(open(out + f".rank{r}.json")) for r in range(world)]
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


@pytest.mark.parametrize("world,dtype,dist", [(1, "i32", "uniform"), (2, "i32", "uniform"), (3, "i32", "uniform"),
                                              (4, "i32", "uniform"), (3, "i32", "seq"), (2, "i32", "rev"),
                                              (3, "i32", "few"), (2, "i64", "uniform"), (3, "i64", "zipf"),
                                              (2, "i64", "few"), (3, "i32", "ref100"), (2, "i32", "mixed")])
def test_bucket_exchange_bit_exact(tmp_path, world, dtype, dist):
    """The bucket exchange (dsort_api.hip sample_sort_bx: global splitters from every rank's
    samples, the first partition level before the exchange, the received pieces finished by the
    second level and the tile sort): ranks sharing the GPU over the host transport, the
    concatenated slices equal numpy's sort of the whole input element for element, for uniform,
    globally sorted / reversed (every rank one key range), few distinct keys (pure buckets filled
    with their key) and Zipf int64 (heavy keys split across ranks).

    The host transport runs the waves in RCCL's order (round 6): wave 1's send ranges are staged
    from the partition buffer after wave 0's second level and tile sort ran on it.  The wave fence
    (DSORT_OPT_TEST_WAVE_FENCE) also fingerprints every range wave 1 still needs -- its sends, the
    rank's own wave-1 buckets, its landing zone -- across wave 0, and would fail the sort naming
    the range wave 0 wrote into."""
    n = world * (1 << 22) + 12_345
    ins, outs, meta = run_ranks(tmp_path, world, n, dtype, dist, opts={"all": {"test_wave_fence": 1}})
    assert ins.size == n
    assert all(m["stats"]["exchange_path"] == 1 for m in meta), [m["stats"]["exchange_path"] for m in meta]
    # (every rank fenced its non-empty wave-1 ranges: at least its own buckets)
    assert all(m["stats"]["fence_ranges"] >= 1 for m in meta), [m["stats"]["fence_ranges"] for m in meta]
    assert np.array_equal(np.concatenate(outs), np.sort(ins))
    if dist in ("uniform", "seq", "rev"):
        sizes = [o.size for o in outs]
        assert max(sizes) <= 1.1 * n / world, sizes


def test_bucket_exchange_pure_buckets_stay_home(tmp_path):
    """Round 6: a global bucket between two splitters of one key (pure) is filled with that key by
    its owner; the first level drops its keys and writes the others at compacted starts, so they
    never cross to another rank.  8 distinct keys over 192 global buckets: every key has ~24
    splitters, nearly every key lies in a pure bucket, and almost nothing is shipped -- against
    about 2/3 of the keys when everything crossed."""
    world = 3
    n = world * (1 << 22) + 12_345
    ins, outs, meta = run_ranks(tmp_path, world, n, "i32", "few", opts={"all": {"buckets": 192, "test_wave_fence": 1}})
    assert all(m["stats"]["exchange_path"] == 1 for m in meta), [m["stats"]["exchange_path"] for m in meta]
    assert np.array_equal(np.concatenate(outs), np.sort(ins))
    sent = sum(m["stats"]["keys_sent"] for m in meta)
    assert sent <= 0.05 * n, sent


def test_small_sample_sort_takes_the_merge_path(tmp_path):
    """Below 2^22 keys per rank the sample sort sorts locally and merges the received runs."""
    ins, outs, meta = run_ranks(tmp_path, 2, 1_000_003)
    assert all(m["stats"]["exchange_path"] == 2 for m in meta)
    assert np.array_equal(np.concatenate(outs), np.sort(ins))


@pytest.mark.parametrize("n,fail_at,presorted", [(3 * (1 << 22) + 12_345, 3, False), (3 * (1 << 22) + 12_345, 1, False),
                                                 (3 * (1 << 22) + 12_345, 4, False), (1_000_003, 3, False),
                                                 (3 * (1 << 22) + 12_345, 0, False), (1_000_003, 0, True),
                                                 (1_000_003, 1, True)])
def test_local_failure_in_the_exchange_fails_every_rank(tmp_path, n, fail_at, presorted):
    """A rank failing locally right before a collective of the host-transport sample sort
    (DSORT_OPT_TEST_FAIL_EXCHANGE; 3 = the key all-to-all of the bucket exchange's first wave, 1 =
    the samples, 4 = the second wave; on the merge path below 2^22 keys per rank, 3 = the keys):
    its peers meet the failure at the next status gate and return DSORT_ECOMM naming it, instead of
    blocking in a collective it never joins (dsort_tx.h; the survivor side of server.c:421-449).
    fail_at 0 (round 6): before the very first collective, which now has a gate too --
    on the bucket exchange (the key counts) and on the presorted fault-recovery entry
    (dsort_sample_merge_dev, whose first collective is the samples)."""
    res = run_ranks(tmp_path, 3, n, opts={"rank_opts": {"1": {"test_fail_exchange": fail_at}}, "presorted": presorted},
                    expect_fail=True)
    assert res[1]["rc"] == -3 and "DSORT_OPT_TEST_FAIL_EXCHANGE" in res[1]["error"], res[1]
    for r in (0, 2):
        assert res[r]["rc"] == -4 and "rank 1 failed locally" in res[r]["error"], res[r]
    assert max(r["s"] for r in res) < 30, res


@pytest.mark.parametrize("world,gather", [(2, 0), (3, 0), (2, 1)])
def test_bucket_exchange_oversized_subbuckets(tmp_path, world, gather):
    """Sub-buckets above a tile (DSORT_OPT_SUB_KEYS forces them) in the bucket exchange, on the
    scatter path (sub_gather = 0) and the local path: their split tiles are merged into a buffer
    of their own.  ADVICE r4: the scatter path merged into its source -- in the bucket exchange the
    partition buffer, which still holds this rank's second-wave buckets (and, over RCCL, buckets
    still being sent) -- and the output of the later wave was wrong."""
    n = world * (1 << 22) + 12_345
    ins, outs, meta = run_ranks(tmp_path, world, n, opts={"all": {"sub_gather": gather, "sub_keys": 20_000,
                                                                  "test_wave_fence": 1}})
    assert all(m["stats"]["exchange_path"] == 1 for m in meta)
    assert all(m["stats"]["fence_ranges"] >= 1 for m in meta), [m["stats"]["fence_ranges"] for m in meta]
    assert any(m["stats"]["sub_split_subbuckets"] > 0 for m in meta), [m["stats"] for m in meta]
    assert np.array_equal(np.concatenate(outs), np.sort(ins))


def test_wave_fence_catches_a_write_into_wave_1(tmp_path):
    """The wave fence is not vacuous: with DSORT_OPT_TEST_WAVE_FENCE = 2 rank 0 flips one key of
    its first fenced wave-1 range between the two fingerprints (as a stray write of wave 0's second
    level would); its sort fails with DSORT_EHIP naming the range, and rank 1 leaves at the next
    status gate with DSORT_ECOMM instead of waiting in the second wave."""
    n = 2 * (1 << 22) + 12_345
    res = run_ranks(tmp_path, 2, n, opts={"rank_opts": {"0": {"test_wave_fence": 2}}}, expect_fail=True)
    assert res[0]["rc"] == -3 and "DSORT_OPT_TEST_WAVE_FENCE" in res[0]["error"], res[0]
    assert "wave-1" in res[0]["error"] or "own wave-1" in res[0]["error"], res[0]
    assert res[1]["rc"] == -4 and "rank 0 failed locally" in res[1]["error"], res[1]
