"""The multi-device plan on the CPU (no GPU call): udpdk_shard_plan reads a config file the way
udpdk_init does and returns the device of every RX shard context it would create, in shard order
(one context per GPU, contiguous shards). Eight GPUs give eight contexts on
eight distinct device ordinals."""
import ctypes as C
import errno

import pytest

from udpdk_amd import abi


def _plan(tmp_path, body, max_=16):
    p = tmp_path / "udpdk.ini"
    p.write_text("[port0]\nmac_addr = 68:05:ca:95:f8:ec\nip_addr = 172.31.100.2\n" + body)
    out = (C.c_int * max_)()
    n = abi.lib().udpdk_shard_plan(str(p).encode(), out, max_)
    return n, list(out[:max(0, min(n, max_))])


def test_eight_devices_eight_contexts(tmp_path):
    n, dev = _plan(tmp_path, "[gpu]\ndevices = 0-7\n")
    assert n == 8 and dev == list(range(8)) and len(set(dev)) == 8


@pytest.mark.parametrize("spec,want", [("0-3,5", [0, 1, 2, 3, 5]), ("0,0", [0, 0]), ("6 , 2", [6, 2]),
                                       ("0-1,4-5", [0, 1, 4, 5])])
def test_device_lists(tmp_path, spec, want):
    n, dev = _plan(tmp_path, f"[gpu]\ndevices = {spec}\n")
    assert n == len(want) and dev == want


def test_single_device_and_default(tmp_path):
    assert _plan(tmp_path, "[gpu]\ndevice = 3\n") == (1, [3])
    assert _plan(tmp_path, "[gpu]\nmax_frames = 4096\n") == (1, [0])
    # a devices key in another section is not the GPU plan
    assert _plan(tmp_path, "[dpdk]\ndevices = 0-7\n") == (1, [0])


def test_bad_lists(tmp_path):
    for spec in ("", "x", "3-1", "0-99", "1,,2"):
        n, _ = _plan(tmp_path, f"[gpu]\ndevices = {spec}\n")
        assert n == -errno.EINVAL, spec
    assert abi.lib().udpdk_shard_plan(str(tmp_path / "missing.ini").encode(), None, 0) == -errno.ENOENT


def test_plan_truncates_to_max(tmp_path):
    n, dev = _plan(tmp_path, "[gpu]\ndevices = 0-7\n", max_=3)
    assert n == 8 and dev == [0, 1, 2]


@pytest.mark.parametrize("body,want", [
    # a later single device moves only the main context: the shard list stays (as udpdk_init)
    ("devices = 0-3\ndevice = 5\n", [0, 1, 2, 3]),
    ("device = 5\ndevices = 0-3\n", [0, 1, 2, 3]),
    # a one-entry list is no shard list: one context, on the last device named
    ("devices = 2\n", [2]),
    ("devices = 2\ndevice = 5\n", [5]),
    ("device = 5\ndevices = 2\n", [2]),
])
def test_device_and_devices_key_order(tmp_path, body, want):
    n, dev = _plan(tmp_path, "[gpu]\n" + body)
    assert n == len(want) and dev == want
