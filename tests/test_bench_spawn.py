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


SMALL = ["--frames", "2048", "--strong-piece", "1024"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [2, 3, 8])
def test_gpus_n_spawns_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run"] + SMALL, timeout=280)
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
    # strong: the ranks' pieces tile the one 8-piece batch in order
    assert sum((p["strong_pieces"] for p in ranks), []) == list(range(8))
    assert sum(p["strong_frames"] for p in ranks) == 8 * 1024


@pytest.mark.timeout(400)
def test_strong_batch_same_at_one_two_and_eight_gpus():
    """The strong-scaling object measures ONE 8-piece batch at every N: the pieces cut back out of
    each rank's part (bytes, lengths, rebased offsets) are the same pieces in the same order at
    N = 1, 2 and 8, and at N = 8 each rank's part is config 5's shard of that rank (the weak
    point of the curve)."""
    lines = {}
    for n in (1, 2, 8):
        r = _run(["--gpus", str(n), "--dry-run"] + SMALL, timeout=280)
        assert r.returncode == 0, r.stderr[-2000:]
        lines[n] = json.loads(r.stdout.strip().splitlines()[-1])
    pieces = {n: sum((p["strong_piece_digests"] for p in l["per_rank"]), []) for n, l in lines.items()}
    assert len(pieces[1]) == 8 and len(set(pieces[1])) == 8
    assert pieces[1] == pieces[2] == pieces[8]
    one = lines[1]["per_rank"][0]
    assert one["strong_frames"] == 8 * 1024 and one["strong_pieces"] == list(range(8))
    assert one["strong_workload"].startswith("8192-64B-4096ports-zipf0.99")
    for p in lines[8]["per_rank"]:
        assert p["strong_frames"] == 1024
    # --frames 2048 vs --strong-piece 1024: a piece is config 5 at 1024 frames, seeded by its index
    r = _run(["--gpus", "8", "--dry-run", "--frames", "1024", "--strong-piece", "1024"], timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    for p in json.loads(r.stdout.strip().splitlines()[-1])["per_rank"]:
        assert p["strong_piece_digests"] == [p["scale_digest_rebased"]]


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
    r = _run(["--gpus", "2", "--dry-run", "--strong-total", "5000", "--config", "2", "--no-strong"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["scaling"] == "strong"
    assert [p["frames"] for p in line["per_rank"]] == [2500, 2500]


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "4", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
