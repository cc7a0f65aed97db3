"""Writes the golden fixtures under tests/golden/.

Sources (no fixture here is produced by the code it checks):
  * tx_vectors.json   — header bytes of udpdk_sendto as emitted by the reference's own
                        udpdk_syscall.c compiled during the survey,
                        with config.ini values (config.ini:9-14). Transcribed, not recomputed.
  * checksum_vectors.json — published RFC 1071 examples: RFC 1071 §3 numeric example and the
                        widely used IPv4 header example (checksum 0xb861).
  * rx_probes.json    — RX behaviours the survey observed by running the reference's
                        reassemble(), as scenarios with the
                        expected verdict / deliveries.
  * rx_mixed.npz      — REGRESSION ONLY: a seeded mixed batch with the oracle's outputs at the
                        time of writing, to detect drift of the oracle itself.
Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

CONFIG = {"src_mac": "6805ca95f8ec", "dst_mac": "6805ca95fa64", "src_ip": "172.31.100.2"}

# SURVEY.md §8.G, bytes as printed there (Ethernet | IPv4 | UDP, spaces removed)
TX_VECTORS = [
    {"id": "V1", "desc": "s0 bound ANY:10000 -> 172.31.100.1:10001 len=64",
     "setup": [["socket"], ["bind", 0, "0.0.0.0", 10000]],
     "send": {"sock": 0, "dst": "172.31.100.1", "port": 10001, "len": 64}, "pkt_len": 106,
     "hdr": "6805ca95fa646805ca95f8ec0800" "4500005c000000004011" "5a4f" "ac1f6402ac1f6401"
            "2710271100480000"},
    {"id": "V2", "desc": "s1 bound 10.1.2.3:5353 -> 172.31.100.1:10001 len=1458",
     "setup": [["socket"], ["socket"], ["bind", 0, "0.0.0.0", 10000], ["bind", 1, "10.1.2.3", 5353]],
     "send": {"sock": 1, "dst": "172.31.100.1", "port": 10001, "len": 1458}, "pkt_len": 1500,
     "hdr": "6805ca95fa646805ca95f8ec0800" "450005ce000000004011" "58fb" "0a010203ac1f6401"
            "14e9271105ba0000"},
    {"id": "V3", "desc": "s0 -> 172.31.190.80:10001 len=64 (raw sum 0xffff, rte_ipv4_cksum keeps it)",
     "setup": [["socket"], ["bind", 0, "0.0.0.0", 10000]],
     "send": {"sock": 0, "dst": "172.31.190.80", "port": 10001, "len": 64}, "pkt_len": 106,
     "hdr": "6805ca95fa646805ca95f8ec0800" "4500005c000000004011" "ffff" "ac1f6402ac1fbe50"
            "2710271100480000"},
    {"id": "V4", "desc": "s2 unbound, auto-bind -> raw src port 0",
     "setup": [["socket"], ["socket"], ["socket"], ["bind", 0, "0.0.0.0", 10000],
               ["bind", 1, "10.1.2.3", 5353]],
     "send": {"sock": 2, "dst": "172.31.100.1", "port": 10001, "len": 8}, "pkt_len": 50,
     "hdr": "6805ca95fa646805ca95f8ec0800" "45000024000000004011" "5a87" "ac1f6402ac1f6401"
            "0000271100100000"},
    {"id": "V5", "desc": "s3 unbound, second auto-bind -> raw src port 1 (host order 256)",
     "setup": [["socket"], ["socket"], ["socket"], ["socket"], ["bind", 0, "0.0.0.0", 10000],
               ["bind", 1, "10.1.2.3", 5353], ["autobind", 2]],
     "send": {"sock": 3, "dst": "172.31.100.1", "port": 10001, "len": 8}, "pkt_len": 50,
     "hdr": "6805ca95fa646805ca95f8ec0800" "45000024000000004011" "5a87" "ac1f6402ac1f6401"
            "0100271100100000"},
]

CHECKSUM_VECTORS = [
    # RFC 1071 §3: sum of 00 01 f2 03 f4 f5 f6 f7 (network order) = 0xddf2, checksum 0x220d
    {"id": "rfc1071-s3", "bytes": "0001f203f4f5f6f7", "sum_be": 0xDDF2, "cksum_be": 0x220D},
    # IPv4 header example (checksum field b861)
    {"id": "ipv4-b861", "bytes": "450000730000400040110000c0a80001c0a800c7", "cksum_be": 0xB861},
]

RX_PROBES = [
    {"id": "ptype-ipv4-ethertype-ipv6", "ref": "SURVEY §8 a2 [probe]",
     "ptype": 0x211, "ethertype": 0x86DD, "expect_verdict": "DELIVERED"},
    {"id": "ptype-0-ethertype-ipv4", "ref": "SURVEY §8 a2 [probe]",
     "ptype": 0x0, "ethertype": 0x0800, "expect_verdict": "NOT_IPV4"},
    {"id": "df-only-not-fragment", "ref": "SURVEY §8 a3 [probe]", "frag": 0x4000,
     "expect_verdict": "DELIVERED"},
    {"id": "mf-is-fragment", "ref": "SURVEY §8 a3", "frag": 0x2000, "expect_verdict": "FRAG"},
    {"id": "offset-is-fragment", "ref": "SURVEY §8 a3", "frag": 0x0010, "expect_verdict": "FRAG"},
    {"id": "not-udp", "ref": "SURVEY §8 a4", "proto": 6, "expect_verdict": "NOT_UDP"},
    {"id": "reuseport-fanout-order", "ref": "SURVEY §8 a6 [probe]",
     "binds": [[5, "10.0.0.7", 15], [6, "10.0.0.7", 15]], "dst_ip": "10.0.0.7",
     "expect_verdict": "DELIVERED", "expect_deliveries": [5, 6]},
    {"id": "any-head-swallows-specific", "ref": "SURVEY §8 a6 / Q3",
     "binds": [[1, "0.0.0.0", 0], [2, "10.0.0.7", 2]], "dst_ip": "10.0.0.7",
     "expect_verdict": "DELIVERED", "expect_deliveries": [1]},
    {"id": "specific-no-match", "ref": "SURVEY §8 a6 (poller.c:406-411)",
     "binds": [[3, "10.0.0.9", 0]], "dst_ip": "10.0.0.7", "expect_verdict": "NO_MATCH",
     "expect_deliveries": []},
    {"id": "no-bind", "ref": "SURVEY §8 a6 (poller.c:376-380)", "binds": [], "dst_ip": "10.0.0.7",
     "expect_verdict": "NO_BIND", "expect_deliveries": []},
]

ALIAS_PROBES = [  # SURVEY §8 a7 [probe]: sockets 0..N-1 on distinct ports, (uint8_t) slot aliasing
    {"n_sockets": 300, "aliased": 44},
    {"n_sockets": 1024, "aliased": 768},
]

SOCKOPT_PROBES = [  # SURVEY §8 Q4 [probe]: REUSEPORT (15) sets every bit of REUSEADDR (2)
    {"set": "SO_REUSEPORT", "so_options": 15, "get_SO_REUSEADDR": 1, "get_SO_REUSEPORT": 1},
    {"set": "SO_REUSEADDR", "so_options": 2, "get_SO_REUSEADDR": 1, "get_SO_REUSEPORT": 1},
]


def main():
    with open(os.path.join(HERE, "tx_vectors.json"), "w") as f:
        json.dump({"config": CONFIG, "vectors": TX_VECTORS}, f, indent=1)
    with open(os.path.join(HERE, "checksum_vectors.json"), "w") as f:
        json.dump(CHECKSUM_VECTORS, f, indent=1)
    with open(os.path.join(HERE, "rx_probes.json"), "w") as f:
        json.dump({"frames": RX_PROBES, "alias": ALIAS_PROBES, "sockopt": SOCKOPT_PROBES}, f, indent=1)

    # regression fixture from the oracle (not a pin)
    import oracle as O
    from udpdk_amd import frames as F
    from udpdk_amd.abi import raw_ip, raw_port
    ports = [10001, 10002, 10003]
    lists = {raw_port(10001): [(0, 0, 0)],
             raw_port(10002): [(raw_ip("172.31.100.1"), 1, 1), (raw_ip("172.31.100.1"), 2, 1)],
             raw_port(10003): [(raw_ip("172.31.100.9"), 3, 0)]}
    b = F.mixed_batch(7, 600, ports, [9999, 20000], ["172.31.100.1", "172.31.100.9"], with_ptype=True)
    bt = O.bindtable_from_lists(lists)
    meta, loff, pkt, cnt = O.rx(bt, b.frames, b.frames_bytes, b.offset, b.length, b.ptype, 4)
    np.savez_compressed(os.path.join(HERE, "rx_mixed.npz"), frames=b.frames[:b.frames_bytes],
                        offset=b.offset, length=b.length, ptype=b.ptype, meta=meta, lane_off=loff,
                        lane_pkt=pkt, counters=cnt,
                        lists=np.array([[p, ip, s, r] for p, l in lists.items() for ip, s, r in l],
                                       np.uint32))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
