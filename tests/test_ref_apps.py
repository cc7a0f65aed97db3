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


# ---- the reference's applications exchanging datagrams through the GPU datapath -------------
# Built in place from /root/reference by oracle/Makefile into oracle/_ref/ (the binaries travel to
# the GPU box; the reference does not). Each process's udpdk_init reads "[gpu] port = udp:..." and
# starts the poller thread on a kernel UDP socket carrying one Ethernet frame per datagram, as the
# reference's udpdk_init forks its poller (udpdk_init.c:293, :362-368).
import signal
import socket as _socket
import time

REF_BIN = os.path.join(ROOT, "oracle", "_ref")


def _free_udp_ports(n):
    socks, ports = [], []
    for _ in range(n):
        s = _socket.socket(_socket.AF_INET, _socket.SOCK_DGRAM)
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def _ini(path, ip, mac, dst_mac, wire, peer):
    path.write_text(f"[dpdk]\nlcores_primary=2\n[port0]\nmac_addr={mac}\nip_addr={ip}\n"
                    f"[port0_dst]\nmac_addr={dst_mac}\n"
                    f"[gpu]\ndevice = 0\nmax_frames = 4096\nmax_lanes = 16\n"
                    f"port = udp:127.0.0.1:{wire}\nport_peer = 127.0.0.1:{peer}\n")


def _udp_bound(port):
    """Whether some process has bound 127.0.0.1:port (the peer's wire is up)."""
    want = f"0100007F:{port:04X}"
    for f in ("/proc/net/udp",):
        with open(f) as fh:
            if any(want in ln.split()[1] for ln in fh.readlines()[1:]):
                return True
    return False


def _start(exe, ini, *args):
    return subprocess.Popen([exe, "-c", str(ini), *args], stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True)


def _stop(p, timeout=60):
    if p.poll() is None:
        p.send_signal(signal.SIGINT)            # the apps' own handler: udpdk_interrupt + exit
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        p.kill()
        out, err = p.communicate()
        raise AssertionError(f"{p.args[0]} did not exit after SIGINT: {out[-500:]} {err[-500:]}")
    return p.returncode, out, err


def _wait_bound(port, proc, secs=90):
    t0 = time.time()
    while not _udp_bound(port):
        assert proc.poll() is None, proc.communicate()
        assert time.time() - t0 < secs, "peer wire never came up"
        time.sleep(0.1)
    time.sleep(1.0)                              # udpdk_init returned: the app binds next


@pytest.mark.gpu
def test_reference_pingpong_exchanges_datagrams(tmp_path):
    """apps/pingpong unchanged: pong (172.31.100.1, ANY:10001) bounces every ping back to the
    sender's address; ping (172.31.100.2, ANY:10000) sends its clock to 172.31.100.1:10001 and
    waits for the echo (apps/pingpong/main.c:80-110, :133-141). Both sides' frames are built by
    the GPU TX kernel and classified / demultiplexed by the GPU RX kernels."""
    exe = os.path.join(REF_BIN, "pingpong")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/pingpong not built (needs /root/reference at build time)")
    w_ping, w_pong = _free_udp_ports(2)
    mac_a, mac_b = "68:05:ca:95:f8:ec", "68:05:ca:95:fa:64"
    _ini(tmp_path / "pong.ini", "172.31.100.1", mac_b, mac_a, w_pong, w_ping)
    _ini(tmp_path / "ping.ini", "172.31.100.2", mac_a, mac_b, w_ping, w_pong)
    pong = _start(exe, tmp_path / "pong.ini", "-f", "pong")
    ping = None
    try:
        _wait_bound(w_pong, pong)
        ping = _start(exe, tmp_path / "ping.ini", "-f", "ping", "-d", "20000")
        time.sleep(6.0)
        rc_ping, out_ping, err_ping = _stop(ping)
        ping = None
        rc_pong, out_pong, err_pong = _stop(pong)
        pong = None
    finally:
        for p in (ping, pong):
            if p is not None and p.poll() is None:
                p.kill()
    assert rc_ping == 0 and rc_pong == 0, (out_ping[-800:], err_ping[-800:], out_pong[-800:], err_pong[-800:])
    assert "App: UDPDK Intialized" in out_ping and "PING mode" in out_ping
    assert "PONG mode" in out_pong
    pongs = [ln for ln in out_ping.splitlines() if ln.startswith("Received pong; delta = ")]
    sent = out_ping.count("Sending ping")
    assert len(pongs) >= 20, out_ping[-800:]
    assert sent - len(pongs) <= 1                 # every ping but the one in flight came back


@pytest.mark.gpu
def test_reference_pktgen_send_and_recv(tmp_path):
    """apps/pktgen unchanged: -f send at 2000 pkt/s with 64 B payloads to 172.31.100.1:10001
    (apps/pktgen/main.c:140-165), -f recv on ANY:10001 (:170-205) counting what arrives; the
    receiver's once-a-second stats line shows the packets, and -d dumps one payload."""
    exe = os.path.join(REF_BIN, "pktgen")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/pktgen not built (needs /root/reference at build time)")
    w_tx, w_rx = _free_udp_ports(2)
    mac_a, mac_b = "68:05:ca:95:f8:ec", "68:05:ca:95:fa:64"
    _ini(tmp_path / "rx.ini", "172.31.100.1", mac_b, mac_a, w_rx, w_tx)
    _ini(tmp_path / "tx.ini", "172.31.100.2", mac_a, mac_b, w_tx, w_rx)
    rx = _start(exe, tmp_path / "rx.ini", "-f", "recv")
    tx = None
    try:
        _wait_bound(w_rx, rx)
        tx = _start(exe, tmp_path / "tx.ini", "-f", "send", "-r", "2000", "-s", "64")
        time.sleep(5.0)
        rc_tx, out_tx, _ = _stop(tx)
        tx = None
        time.sleep(1.5)                            # the receiver's next stats line
        rc_rx, out_rx, err_rx = _stop(rx)
        rx = None
    finally:
        for p in (tx, rx):
            if p is not None and p.poll() is None:
                p.kill()
    assert rc_tx == 0 and rc_rx == 0, (out_tx[-500:], out_rx[-500:], err_rx[-500:])
    import re
    sent = [int(m) for m in re.findall(r"Sent: (\d+) pkts", out_tx)]
    recv = [int(m) for m in re.findall(r"Recv: (\d+) pkts", out_rx)]
    assert sent and recv, (out_tx[-500:], out_rx[-500:])
    assert max(sent) >= 3000
    # the wire is a kernel UDP socket pair on one host: nothing should be lost at 2 kpkt/s
    assert max(recv) >= 0.95 * max(sent), (max(recv), max(sent))
