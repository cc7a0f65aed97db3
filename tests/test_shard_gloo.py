"""N>1 path on CPU: two gloo ranks each take a contiguous shard of one batch,
classify it (the oracle stands in for the GPU, which this container lacks), and rank 0 merges the
per-shard lanes in shard order. The merge must equal the single-batch result exactly; the timing
reduction bench.py uses (all_reduce MAX) is exercised too."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import oracle as O
    from udpdk_amd import frames as F, shard as S
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = F.config_batch(5, n=20000)          # Zipf-0.99 over 4096 ports
    b = w.batch
    a, e = S.shard_range(b.n, world, rank)
    bt = O.bindtable_from_lists(w.port_lists())
    meta, loff, pkt, cnt = O.rx(bt, b.frames, b.frames_bytes, b.offset[a:e], b.length[a:e], None,
                                w.n_sockets)
    parts = [None] * world
    dist.all_gather_object(parts, (loff, pkt, a, meta, cnt))
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        goff, gpkt = S.merge_lanes([(p[0], p[1], p[2]) for p in parts], w.n_sockets)
        wm, wl, wp, wc = O.rx(bt, b.frames, b.frames_bytes, b.offset, b.length, None, w.n_sockets)
        ok = (np.array_equal(goff, wl) and np.array_equal(gpkt, wp)
              and np.array_equal(np.concatenate([p[3] for p in parts]), wm)
              and np.array_equal(sum(p[4] for p in parts), wc) and t.item() == float(world))
        q.put(ok)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_shards_merge_to_single_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert ok
    assert all(p.exitcode == 0 for p in procs)


def test_shard_range_covers_batch():
    from udpdk_amd import shard as S
    for n in [0, 1, 7, 1000, 1 << 20]:
        for world in [1, 2, 3, 8]:
            rs = [S.shard_range(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
