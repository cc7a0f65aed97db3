"""bench.py's multi-GPU plumbing on the CPU (no HIP call): `--gpus N` run directly spawns N rank
processes itself, the ranks rendezvous over gloo on 127.0.0.1, each builds its own shard of the
headline workload (config 2, frames 0x5EED ^ rank) and of the `scale` workload (config 5, ports
seeded 1000 + rank), and rank 0 prints one line carrying the max-over-ranks reduction. The same
two workloads at every N, N = 1 included, so per-N values compare one workload. Under torchrun,
a --gpus that disagrees with WORLD_SIZE is refused."""
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
    assert line["n_gpus"] == n and line["baseline_config"] == 2 and line["scaling"] == "weak"
    ranks = line["per_rank"]
    assert [p["rank"] for p in ranks] == list(range(n))
    assert [p["local_rank"] for p in ranks] == list(range(n))
    assert all(p["workload"] == "2048-64B-1port" and p["frames"] == 2048 for p in ranks)
    assert all(p["scale_workload"] == "2048-64B-4096ports-zipf0.99" and p["scale_frames"] == 2048
               for p in ranks)
    assert len({p["digest"] for p in ranks}) == n          # independent shards
    assert len({p["scale_digest"] for p in ranks}) == n
    assert line["max_wall"] == float(n)                     # MAX over ranks (rank r reports 1 + r)


def test_same_workloads_at_one_and_two_gpus():
    """N = 1 and N = 2 measure the same headline and scale workloads (rank 0's shards equal)."""
    one = _run(["--gpus", "1", "--dry-run", "--frames", "1024"])
    two = _run(["--gpus", "2", "--dry-run", "--frames", "1024"])
    assert one.returncode == 0 and two.returncode == 0, (one.stderr[-1000:], two.stderr[-1000:])
    l1 = json.loads(one.stdout.strip().splitlines()[-1])
    l2 = json.loads(two.stdout.strip().splitlines()[-1])
    assert l1["n_gpus"] == 1 and l1["baseline_config"] == l2["baseline_config"] == 2
    r1, r2 = l1["per_rank"][0], l2["per_rank"][0]
    for k in ("workload", "frames", "digest", "scale_workload", "scale_frames", "scale_digest"):
        assert r1[k] == r2[k], k


def test_strong_scaling_shards():
    r = _run(["--gpus", "2", "--dry-run", "--strong-total", "5000", "--config", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["scaling"] == "strong"
    assert [p["frames"] for p in line["per_rank"]] == [2500, 2500]


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "4", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
