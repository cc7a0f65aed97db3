"""CPU checks of the receive-side scaling restatement (f4): the Toeplitz hash against the
published RSS verification vectors (tests/golden/rss_vectors.json), the redirection table and the
per-queue lists, and the library's default configuration (host-only call)."""
import json
import os
import socket

import numpy as np

import oracle as O
from udpdk_amd import abi, frames as F

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "rss_vectors.json")))
KEY = bytes.fromhex(G["key"])


def test_toeplitz_verification_vectors():
    for v in G["ipv4"]:
        a = socket.inet_aton(v["src"]) + socket.inet_aton(v["dst"])
        p = v["sport"].to_bytes(2, "big") + v["dport"].to_bytes(2, "big")
        assert O.toeplitz(KEY, a) == int(v["ipv4"], 16)
        assert O.toeplitz(KEY, a + p) == int(v["ipv4_l4"], 16)


def test_default_conf():
    cf = abi.rss_conf(8)
    assert bytes(cf.key) == KEY and cf.hash_types == 3 and cf.n_queues == 8
    assert cf.reta_size == 128 and [cf.reta[i] for i in range(128)] == [i % 8 for i in range(128)]


def test_rss_lists_partition_in_order():
    b = F.mixed_batch(3, 3000, [10001, 10002], [9, 20000], ["172.31.100.1", "172.31.100.9"])
    reta = np.arange(128) % 5
    h, qo, qp = O.rss(KEY, 3, reta, 5, b.frames, b.frames_bytes, b.offset, b.length)
    assert qo[-1] == b.n and sorted(qp.tolist()) == list(range(b.n))
    for q in range(5):
        seg = qp[qo[q]:qo[q + 1]]
        assert np.all(np.diff(seg.astype(np.int64)) > 0)                # arrival order
        assert np.all(reta[h[seg] & 127] == q)
    # frames the gate rejects hash to 0 and go to reta[0]
    assert np.any(h == 0)
