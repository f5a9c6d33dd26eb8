"""bench.py's rank launcher on CPU (no GPU call): `python bench.py --gpus N` spawns N rank
processes with torch.distributed.run's variables (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*), each rank
must see its own rank and the same rendezvous; --gpus must match WORLD_SIZE under torchrun; and a
request for more GPUs than visible fails with a clear message and a non-zero exit."""
import json
import os
import subprocess
import sys

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def test_launcher_spawns_ranks_with_plumbing():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launcher-selftest"], capture_output=True,
                       text=True, timeout=300, env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    assert p.returncode == 0, p.stderr
    ranks = sorted((json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")), key=lambda d: d["rank"])
    assert [d["rank"] for d in ranks] == [0, 1, 2]
    assert all(d["world"] == 3 and d["local_rank"] == d["rank"] and d["master"] == "127.0.0.1" for d in ranks)
    assert len({d["port"] for d in ranks}) == 1


def test_gpus_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    p = subprocess.run([sys.executable, BENCH, "--gpus", "4"], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode != 0 and "must match" in p.stderr


def test_more_gpus_than_visible_fails_clearly():
    env = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    p = subprocess.run([sys.executable, BENCH, "--gpus", "64", "--steps", "1"], capture_output=True, text=True,
                       timeout=300, env=env)
    assert p.returncode == 2
    assert "needs 64 visible GPUs" in p.stderr


def test_rank_env_builder():
    sys.path.insert(0, REPO)
    import bench

    envs = bench.rank_envs(4, 12345, base={"X": "1"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_PORT"] == "12345" and e["X"] == "1" for e in envs)
    assert all(e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" for e in envs)
