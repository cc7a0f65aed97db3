"""The C-ABI library loads and exports every function include/*.h declares (no GPU needed)."""
import os
import re
import subprocess

from udpdk_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"\b(udpdk_[a-z0-9_]+)\s*\(", txt)) - {"udpdk_gpu_ctx"}


def test_headers_match_bindings():
    decl = _declared("udpdk_gpu.h") | _declared("udpdk_api.h")
    assert decl == set(abi.declared_symbols())


def test_library_exports_every_declared_symbol():
    L = abi.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", abi.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    for name in abi.declared_symbols():
        assert name in exported, name
        assert getattr(L, name) is not None


def test_abi_version_and_geometry():
    assert abi.lib().udpdk_gpu_abi_version() == 3
    # tile geometry policy: lanes x tiles bounded, tiles >= 1
    assert abi.geometry(1 << 20, 1) == (1024, 1024)
    assert abi.geometry(1 << 20, 1024) == (1024, 1024)
    t, k = abi.geometry(1 << 22, 4096)
    assert t * k >= 1 << 22 and k * 4096 <= 1 << 21
    assert abi.geometry(0, 1) == (1024, 1)


def test_reference_api_surface_present():
    """The ten reference entry points + udpdk_dump_payload (udpdk_api.symlist:1-11)."""
    ref = ["udpdk_init", "udpdk_interrupt", "udpdk_cleanup", "udpdk_socket", "udpdk_getsockopt",
           "udpdk_setsockopt", "udpdk_bind", "udpdk_sendto", "udpdk_recvfrom", "udpdk_close",
           "udpdk_dump_payload"]
    for r in ref:
        assert r in abi.declared_symbols()


def test_ctx_create_without_gpu_fails_cleanly():
    if abi.device_count() > 0:
        return
    import ctypes as C
    h = C.c_void_p()
    rc = abi.lib().udpdk_gpu_ctx_create(0, 1024, 1, C.byref(h))
    assert rc < 0 and not h.value
