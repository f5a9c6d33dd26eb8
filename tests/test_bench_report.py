"""bench.py's N > 1 result line on CPU (no GPU): report_multi fed a synthetic per-rank table (the
rows run_multi gathers from every rank) must carry SURVEY.md §8d in full -- the slowest stage's HBM
roofline, the xGMI figure of the key exchange, the all-kernels fraction (PMC bytes over device
time, labelled measured only on the PMC table's own build) and the reference CPU path beside it
(cpu_baseline, as at N = 1)."""
import json
import os
import sys

import numpy as np

from conftest import REPO


def _per_rank(world, n, w):
    sys.path.insert(0, REPO)
    import bench

    rows = np.zeros((world, 12))
    for r in range(world):
        nk = n // world
        rows[r, bench.PR_TILE] = 0.30 + 0.01 * r
        rows[r, bench.PR_A2A] = 0.9
        rows[r, bench.PR_EXCH] = 1.2
        rows[r, bench.PR_FINAL] = 0.7
        rows[r, bench.PR_SENT] = nk * (world - 1) / world
        rows[r, bench.PR_KEYS] = nk
        rows[r, bench.PR_HIST] = 0.1
        rows[r, bench.PR_SCAT] = 0.35 + 0.01 * r
        rows[r, bench.PR_SUB] = 0.25
        rows[r, bench.PR_TKEYS] = nk
        rows[r, bench.PR_PATH] = 1
        rows[r, bench.PR_TOTAL] = 1.9 + 0.05 * r
    return rows


def test_report_multi_carries_roofline_all_kernels_and_cpu_baseline(capsys):
    sys.path.insert(0, REPO)
    import bench

    world, n = 4, 1 << 30
    args = bench.parse(["--gpus", str(world), "--steps", "5", "--cpu-sample-keys", str(1 << 16)])
    bench.report_multi(args, world, 5 * 2.1e-3, _per_rank(world, n, 4), 4)
    line = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == world and d["unit"] == "keys/s" and abs(d["value"] - n / 2.1e-3) < 1e3
    roof = d["roofline"]
    assert roof["bound"] == "hbm" and 0 < roof["frac"] < 1 and roof["peak"] == 8000.0
    assert "rank 3" in roof["kernel"]  # the slowest stage of the slowest rank
    assert roof["xgmi"]["peak"] == 3 * 153.0 and roof["xgmi"]["frac"] > 0
    key = "all_kernels_frac" if "all_kernels_frac" in roof else "all_kernels_frac_estimate"
    assert 0 < roof[key] < 1, roof
    assert roof["all_kernels"]["device_ms_slowest_rank"] == 2.05
    assert len(roof["device_ms_per_rank"]) == world
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("reference", "port") and cb["cores"] == 4 and cb["value"] > 0
    assert "65536" in cb["sample"]


def test_report_multi_without_cpu_baseline(capsys):
    sys.path.insert(0, REPO)
    import bench

    args = bench.parse(["--gpus", "2", "--no-cpu-baseline"])
    bench.report_multi(args, 2, 10 * 4e-3, _per_rank(2, 1 << 30, 4), 4)
    d = json.loads([ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][-1])
    assert "cpu_baseline" not in d and d["n_gpus"] == 2


def test_stage_roofline_counts_only_the_scatters_written_keys():
    """The one-GPU out-of-place sort's first-level scatter writes only the keys outside single-key
    buckets (round 5: the second level fills those): its algorithmic bytes are n keys read plus
    tile_sort_keys written; the bucket exchange's scatter (drop_pure False) reads and writes all n."""
    sys.path.insert(0, REPO)
    import bench

    n, w, tk = 1 << 30, 8, 507 << 20
    k = {"bucket_hist_ms": 2.2, "bucket_scatter_ms": 3.9, "sub_partition_ms": 2.4, "tile_sort_kernel_ms": 1.7,
         "n": n, "tile_sort_keys": tk}
    one = {s["kernel"].split("<")[0]: s for s in bench.stage_roofline(k, w, n, "zipf", drop_pure=True)}
    multi = {s["kernel"].split("<")[0]: s for s in bench.stage_roofline(k, w, n, "zipf")}
    assert one["bucket_scatter_lines_kernel"]["algorithmic_bytes_per_launch"] == w * (n + tk)
    assert multi["bucket_scatter_lines_kernel"]["algorithmic_bytes_per_launch"] == 2 * w * n
    assert one["bucket_hist_kernel"]["algorithmic_bytes_per_launch"] == w * n
    assert one["bin_sort_kernel"]["algorithmic_bytes_per_launch"] == 2 * w * tk


def test_pmc_sort_bytes_count_every_launch_of_a_kernel():
    """The PMC table's per-sort traffic counts every launch of a kernel in one sort (round 5: the
    tile sort runs in two launches, the first before the host reads the tile count), and the bench
    line's whole-sort bytes and per-stage traffic use it."""
    import bench
    doc = bench._pmc_doc(4, "uniform")
    assert doc is not None
    bs = doc["kernels"]["bin_sort_kernel<int, true, 8>"]
    assert bs["launches_per_sort"] == 2
    assert bs["traffic_bytes_per_sort"] == int(bs["traffic_bytes_per_launch"] * 2)
    pb, _, _ = bench.pmc_sort_bytes(1 << 30, 4, "uniform")
    exp = sum(r["traffic_bytes_per_sort"] for k, r in doc["kernels"].items() if not k.startswith(bench.NOT_SORT))
    assert pb == exp and pb > 3 * 2 * 4 * (1 << 30)  # about 3.7x one read + one write of the keys


def test_multi_line_carries_c3_c4_c5_legs(capsys):
    """the driver's one `bench.py --gpus N` run also measures configs C3, C4 and C5
    after the metric's timed region.  Synthetic per-leg results through leg_summary and a C5 child
    line: the keys are present, verified, and the metric's own value is unchanged by them."""
    sys.path.insert(0, REPO)
    import bench

    world = 8
    plan = bench.leg_plan(world)
    assert plan["c3"]["keys"] == 1 << 32 and plan["c3"]["buckets"] == 1024
    assert plan["c4"] == {"keys": 1 << 30, "dtype": "i64", "dist": "zipf"}
    assert plan["c5"]["kill_rank"] == 3 and plan["c5"]["workers"] == 8 and plan["c5"]["transport"] == "rccl"
    assert bench.leg_plan(2)["c3"]["keys"] == 1 << 30 and bench.leg_plan(2)["c5"]["kill_rank"] == 1
    assert bench.leg_plan(1)["c5"]["transport"] == "relay"  # (one GPU: two workers share it)
    args = bench.parse(["--gpus", str(world), "--steps", "5", "--no-cpu-baseline"])
    assert bench.legs_wanted(args) == ["c3", "c4", "c5"]
    assert bench.legs_wanted(bench.parse(["--no-legs"])) == []
    assert bench.legs_wanted(bench.parse(["--legs", "c4"])) == ["c4"]
    c3 = bench.leg_summary("c3", plan["c3"], world, 3, (3 * 6.0e-3, True, _per_rank(world, 1 << 32, 4), 4, None))
    c4 = bench.leg_summary("c4", plan["c4"], world, 3, (3 * 2.0e-3, True, _per_rank(world, 1 << 30, 8), 8, None))
    bad = bench.leg_summary("c4", plan["c4"], world, 3, (None, False, None, 8, "rank 2: ETIMEOUT"))
    c5 = {"config": "C5", "value": 812.5, "unit": "ms", "verified": True, "transport": "rccl"}
    bench.report_multi(args, world, 5 * 2.1e-3, _per_rank(world, 1 << 30, 4), 4, {"c3": c3, "c4": c4, "c5": c5})
    d = json.loads([ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][-1])
    assert abs(d["value"] - (1 << 30) / 2.1e-3) < 1e3  # the metric's value is the metric's own
    legs = d["legs"]
    assert legs["c3"]["config"] == "C3" and legs["c3"]["verified"] and legs["c3"]["keys"] == 1 << 32
    assert abs(legs["c3"]["value"] - (1 << 32) / 6.0e-3) < 1e3 and legs["c3"]["dtype"] == "int32"
    assert "xgmi" in legs["c3"]["roofline"] and legs["c3"]["roofline"]["frac"] > 0  # (synthetic stage times)
    key = "all_kernels_frac" if "all_kernels_frac" in legs["c3"]["roofline"] else "all_kernels_frac_estimate"
    assert key in legs["c3"]["roofline"]
    assert legs["c4"]["dtype"] == "int64" and legs["c4"]["dist"] == "zipf" and legs["c4"]["verified"]
    # (skewed keys: no all-kernels figure scaled from the one-GPU table)
    assert "all_kernels_frac" not in legs["c4"]["roofline"] and "all_kernels_frac_estimate" not in legs["c4"]["roofline"]
    assert legs["c5"]["verified"] and legs["c5"]["unit"] == "ms"
    assert bad["verified"] is False and "ETIMEOUT" in bad["error"]
