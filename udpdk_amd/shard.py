"""Multi-GPU sharding of frame batches.

Frame batches are embarrassingly parallel: shard s of S takes a contiguous run of frames, every
GPU holds a replica of the ~0.3 MB bind snapshot, and no collective touches the data path. The
per-shard lanes concatenated in shard order are the global lanes, because each shard's kernel is
stable and shards are contiguous; :func:`merge_lanes` does that on the host.
"""
from __future__ import annotations

import numpy as np


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    per = (n + world - 1) // world
    a = min(n, rank * per)
    return a, min(n, a + per)


def merge_lanes(parts: list[tuple[np.ndarray, np.ndarray, int]], n_lanes: int):
    """parts: [(lane_off[n_lanes+1], lane_pkt[D], first_frame_index)] in shard order.
    Returns global (lane_off, lane_pkt) with frame indices rebased to the whole batch."""
    counts = np.zeros(n_lanes, np.int64)
    for off, _, _ in parts:
        counts += np.diff(off.astype(np.int64))
    goff = np.zeros(n_lanes + 1, np.int64)
    goff[1:] = np.cumsum(counts)
    out = np.zeros(int(goff[-1]), np.uint32)
    cursor = goff[:-1].copy()
    for off, pkt, base in parts:
        off = off.astype(np.int64)
        for lane in np.nonzero(np.diff(off))[0]:
            seg = pkt[off[lane]:off[lane + 1]].astype(np.int64) + base
            out[cursor[lane]:cursor[lane] + len(seg)] = seg
            cursor[lane] += len(seg)
    return goff.astype(np.uint32), out
