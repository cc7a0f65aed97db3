"""The recvfrom restatement (oracle.recv_gather, udpdk_syscall.c:401-488) on hand-built frames:
Ethernet padding trimmed by dgram_len (:459-462), truncation to len (:464-468), raw source
address and port (:446-447). CPU only."""
import numpy as np

import oracle as O


def _frame(payload: bytes, pad_to: int = 0, src=(10, 1, 2, 3), sport=5353):
    ulen = 8 + len(payload)
    f = bytearray(14 + 20 + 8) + payload
    f[12:14] = b"\x08\x00"
    f[14] = 0x45
    f[23] = 17
    f[26:30] = bytes(src)
    f[34:36] = sport.to_bytes(2, "big")
    f[38:40] = ulen.to_bytes(2, "big")
    if len(f) < pad_to:
        f += b"\xee" * (pad_to - len(f))
    return bytes(f)


def _batch(frames):
    off = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint32)
    buf = np.frombuffer(b"".join(frames), np.uint8).copy()
    ln = np.array([len(f) for f in frames], np.uint16)
    return buf, off, ln


def test_padding_trimmed_and_truncation():
    frames = [_frame(b"hello", pad_to=60), _frame(bytes(range(100))), _frame(b"")]
    buf, off, ln = _batch(frames)
    pay, olen, sip, spt = O.recv_gather(buf, off, ln, np.arange(3, dtype=np.uint32), 0, 3, 64)
    assert list(olen) == [5, 64, 0]                      # padding trimmed; truncated to len
    assert bytes(pay[0, :5]) == b"hello"
    assert bytes(pay[1, :64]) == bytes(range(64))
    assert sip[0] == int.from_bytes(bytes((10, 1, 2, 3)), "little")     # raw s_addr
    assert spt[0] == int.from_bytes((5353).to_bytes(2, "big"), "little")  # raw sin_port


def test_range_and_order():
    frames = [_frame(bytes([i]) * (i + 1)) for i in range(6)]
    buf, off, ln = _batch(frames)
    lane = np.array([5, 3, 1, 0], np.uint32)
    pay, olen, _, _ = O.recv_gather(buf, off, ln, lane, 1, 2, 16)
    assert list(olen) == [4, 2]
    assert bytes(pay[0, :4]) == b"\x03" * 4 and bytes(pay[1, :2]) == b"\x01" * 2
