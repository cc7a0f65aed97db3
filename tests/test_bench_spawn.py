"""bench.py's multi-GPU plumbing on the CPU (no HIP call): `--gpus N` run directly spawns N rank
processes itself, the ranks rendezvous over gloo on 127.0.0.1, each builds its own config-5 shard
(ports seeded 1000 + rank, frames 0x5EED ^ rank), and rank 0 prints one line carrying the
max-over-ranks reduction. Under torchrun, a --gpus that disagrees with WORLD_SIZE is refused."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run", "--frames", "2048"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == n and line["baseline_config"] == 5 and line["scaling"] == "weak"
    ranks = line["per_rank"]
    assert [p["rank"] for p in ranks] == list(range(n))
    assert [p["local_rank"] for p in ranks] == list(range(n))
    assert all(p["workload"].endswith("4096ports-zipf0.99") and p["frames"] == 2048 for p in ranks)
    assert len({p["digest"] for p in ranks}) == n          # independent shards
    assert line["max_wall"] == float(n)                     # MAX over ranks (rank r reports 1 + r)


def test_single_gpu_default_is_config2():
    r = _run(["--dry-run", "--frames", "1024"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["baseline_config"] == 2


def test_strong_scaling_shards():
    r = _run(["--gpus", "2", "--dry-run", "--strong-total", "5000", "--config", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["scaling"] == "strong"
    assert [p["frames"] for p in line["per_rank"]] == [2500, 2500]


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "4", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
