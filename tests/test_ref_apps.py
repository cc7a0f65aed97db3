"""Drop-in check of the reference's only boundary, udpdk_api.h (udpdk/Makefile:72-81,
udpdk_api.symlist:1-11): the reference's own applications, compiled in place from
/root/reference/apps/{pktgen,pingpong}/main.c against include/udpdk_api.h, link against
libudpdk_amd.so with no source change. Nothing is copied out of the reference; the objects go
to a temporary directory. Skipped where the reference is absent (the GPU box)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_APPS = "/root/reference/apps"
LIB_DIR = os.path.join(ROOT, "udpdk_amd")


@pytest.mark.parametrize("app", ["pktgen", "pingpong"])
def test_reference_app_builds_and_links(app, tmp_path):
    src = os.path.join(REF_APPS, app, "main.c")
    if not os.path.exists(src):
        pytest.skip("reference apps not present (GPU box)")
    exe = tmp_path / app
    # the reference's own link line (apps/pktgen/Makefile:19-26) minus DPDK: -pthread for
    # pktgen's stats thread; the app itself is not modified
    cmd = ["gcc", "-O2", "-Wall", "-Wno-pointer-sign", "-I", os.path.join(ROOT, "include"), src,
           "-o", str(exe), "-L", LIB_DIR, "-ludpdk_amd", f"-Wl,-rpath,{LIB_DIR}", "-pthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # every udpdk_* symbol the app references resolves in the library
    und = subprocess.run(["nm", "-u", str(exe)], capture_output=True, text=True, check=True).stdout
    used = {ln.split()[-1] for ln in und.splitlines() if "udpdk_" in ln}
    assert used, "app references no udpdk_ symbol"
    exp = subprocess.run(["nm", "-D", "--defined-only", os.path.join(LIB_DIR, "libudpdk_amd.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in exp.splitlines()}
    assert used <= exported, used - exported


def test_reference_app_starts_and_reports_missing_config(tmp_path):
    """pingpong linked against the library runs: without -c the reference's udpdk_init fails
    (udpdk_args.c:150-155: the config file is mandatory) and the app takes its own exit path
    (apps/pingpong/main.c:204-208 jumps to pingpong_end, which returns 0) instead of crashing."""
    src = os.path.join(REF_APPS, "pingpong", "main.c")
    if not os.path.exists(src):
        pytest.skip("reference apps not present (GPU box)")
    exe = tmp_path / "pingpong"
    subprocess.run(["gcc", "-O2", "-Wno-pointer-sign", "-I", os.path.join(ROOT, "include"), src,
                    "-o", str(exe), "-L", LIB_DIR, "-ludpdk_amd", f"-Wl,-rpath,{LIB_DIR}"],
                   check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60,
                       env={**os.environ, "HIP_VISIBLE_DEVICES": ""})
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "Intialized" not in r.stdout
