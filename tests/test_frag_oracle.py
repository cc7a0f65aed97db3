"""CPU checks of the TX fragmentation restatement (oracle_tx_fragment, the poller's
udpdk_poller.c:461-501 + DPDK 20.05 rte_ipv4_fragment_packet) and of the span helper the GPU
path's callers use. DPDK is not in the container and the reference holds no fragment vectors, so
the fragment bytes are pinned by restatement only ("parity unpinned" beyond the properties below:
an independent pure-Python restatement of one case, reassembly round trips, header checksums)."""
import numpy as np
import pytest

import oracle as O
from udpdk_amd import abi

SRC_MAC = bytes.fromhex("6805ca95f8ec")
DST_MAC = bytes.fromhex("6805ca95fa64")
SRC_IP = abi.raw_ip("172.31.100.2")
DST_IP = abi.raw_ip("172.31.100.1")


def _sum16(b):
    s = sum(b[i] | (b[i + 1] << 8) for i in range(0, len(b), 2))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def _frame(L, seed=0):
    pay = bytes((i * 13 + seed) & 0xFF for i in range(L))
    return O.tx_frame(SRC_MAC, DST_MAC, SRC_IP, 1, 0, abi.raw_port(10000), DST_IP,
                      abi.raw_port(10001), pay), pay


@pytest.mark.parametrize("mtu", [1500, 1020, 68])
@pytest.mark.parametrize("L", [0, 1, 1457, 1458, 1459, 1472, 1473, 2006, 2952, 2953, 9000, 65507])
def test_fragment_round_trip(L, mtu):
    fr, pay = _frame(L, L)
    frags = O.tx_fragment(fr, mtu)
    span = abi.lib().udpdk_gpu_tx_span(L, mtu, None)
    assert sum(len(f) for f in frags) == span
    if len(fr) <= mtu:
        assert frags == [fr]
        return
    fpl = mtu - 20
    assert len(frags) == -(-(L + 8) // fpl)
    ip_payload = bytearray()
    for k, f in enumerate(frags):
        assert f[:14] == fr[:14]
        h = f[14:34]
        assert _sum16(h) == 0xFFFF                              # the NIC-filled checksum verifies
        assert h[0] == 0x45 and h[8] == 64 and h[9] == 17 and h[4:6] == b"\0\0"
        assert h[12:20] == fr[26:34]
        tl = (h[2] << 8) | h[3]
        assert tl == len(f) - 14
        fo = (h[6] << 8) | h[7]
        assert (fo & 0x1FFF) * 8 == len(ip_payload)
        assert bool(fo & 0x2000) == (k + 1 < len(frags)) and not fo & 0x4000
        if k + 1 < len(frags):
            assert tl - 20 == fpl
        ip_payload += f[34:]
    assert bytes(ip_payload) == fr[34:]                         # UDP header + payload


def test_fragment_known_answer_2006():
    """Independent restatement of one case: the largest sendto that fits a 2048 B mbuf
    (RTE_MBUF_DEFAULT_BUF_SIZE data room, udpdk_init.c:78-99) at IPV4_MTU_DEFAULT."""
    fr, pay = _frame(2006)
    frags = O.tx_fragment(fr, 1500)
    assert [len(f) for f in frags] == [1514, 34 + 534]

    def hdr(tl, fo):
        h = bytearray.fromhex("4500") + tl.to_bytes(2, "big") + b"\0\0" + fo.to_bytes(2, "big") + \
            bytes([64, 17, 0, 0]) + fr[26:34]
        ck = (~_sum16(h)) & 0xFFFF
        h[10:12] = ck.to_bytes(2, "little")
        return bytes(h)
    assert frags[0] == fr[:14] + hdr(1500, 0x2000) + fr[34:34 + 1480]
    assert frags[1] == fr[:14] + hdr(554, 185) + fr[34 + 1480:]


def test_span_helper():
    n = abi.C.c_uint32()
    assert abi.lib().udpdk_gpu_tx_span(1458, 1500, abi.C.byref(n)) == 1500 and n.value == 1
    assert abi.lib().udpdk_gpu_tx_span(1459, 1500, abi.C.byref(n)) == 1501 and n.value == 1
    assert abi.lib().udpdk_gpu_tx_span(1473, 1500, abi.C.byref(n)) == 1481 + 68 and n.value == 2
    assert abi.lib().udpdk_gpu_tx_span(65507, 1500, abi.C.byref(n)) == 65515 + 34 * 45 and n.value == 45
    assert abi.lib().udpdk_gpu_tx_span(3000, 0, abi.C.byref(n)) == 3042 and n.value == 1
