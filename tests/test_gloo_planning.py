"""The multi-GPU sample sort's host rules across real processes, CPU only (gloo, world 2 and 3):
every rank samples its sorted chunk (dsort_plan_sample_positions), the samples are all-gathered,
every rank derives the same splitters (dsort_plan_splitters_*) and cuts its chunk
(dsort_plan_cuts_*), the pieces travel with all_to_all, and the concatenation of the ranks'
merged slices must be the sorted input.  The local sort and the merge are numpy stand-ins here
(the GPU versions are tested in test_gpu_multirank.py); what is under test is the planning code
the GPU path runs, exercised over a real process group."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG


def _rank(rank, world, store, n_total, dist_kind, outdir):
    sys.path.insert(0, PKG)
    import dsort

    # (a file rendezvous: no TCP port to lose between choosing it and binding it)
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    rng = np.random.default_rng(1234)
    allkeys = (rng.integers(-50, 50, n_total) if dist_kind == "dups" else
               rng.integers(-(2**31), 2**31, n_total)).astype(np.int32)
    if dist_kind == "dups":
        allkeys[::3] = 7  # a heavy hitter spread over every rank
    sz = n_total // world + (1 if rank < n_total % world else 0)
    first = rank * (n_total // world) + min(rank, n_total % world)
    local = np.sort(allkeys[first:first + sz])
    S = 64
    idx = dsort.plan_sample_positions(local.size, S)
    samples = local[idx.astype(np.int64)] if local.size else np.full(S, 2**31 - 1, np.int32)
    g_samples = [torch.zeros(S, dtype=torch.int32) for _ in range(world)]
    dist.all_gather(g_samples, torch.from_numpy(samples))
    g_n = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(g_n, torch.tensor([local.size], dtype=torch.int64))
    all_idx = np.concatenate([dsort.plan_sample_positions(int(g_n[r][0]), S) for r in range(world)])
    sv, sr, si = dsort.plan_splitters(torch.cat(g_samples).numpy(), all_idx, world)
    cuts = dsort.plan_cuts(local, rank, world, sv, sr, si).astype(np.int64)
    scounts = [int(cuts[d + 1] - cuts[d]) for d in range(world)]
    g_counts = [torch.zeros(world, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(g_counts, torch.tensor(scounts, dtype=torch.int64))
    rcounts = [int(g_counts[s_][rank]) for s_ in range(world)]
    out = torch.zeros(sum(rcounts), dtype=torch.int32)
    dist.all_to_all_single(out, torch.from_numpy(local.copy()), output_split_sizes=rcounts,
                           input_split_sizes=scounts)
    mine = np.sort(out.numpy())
    np.save(os.path.join(outdir, f"slice{rank}.npy"), mine)
    np.save(os.path.join(outdir, "all.npy"), allkeys)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,kind", [(2, "uniform"), (2, "dups"), (3, "dups")])
def test_sample_sort_planning_over_gloo(tmp_path, world, kind):
    n = 40_003
    mp.spawn(_rank, args=(world, str(tmp_path / "store"), n, kind, str(tmp_path)), nprocs=world, join=True)
    slices = [np.load(tmp_path / f"slice{r}.npy") for r in range(world)]
    allkeys = np.load(tmp_path / "all.npy")
    assert np.array_equal(np.concatenate(slices), np.sort(allkeys))
    sizes = [x.size for x in slices]
    assert max(sizes) <= 1.2 * n / world + 64, sizes
