"""Benchmark: device-resident RX parse + checksum + port demux (BASELINE.json metric).

A step = one udpdk_gpu_rx call over one batch of frames already resident in HBM (single-lane
batches: rx_classify + rx_compact1; otherwise rx_classify + rx_scan + rx_scatter). The timed
region is exactly K steps between a barrier + hipDeviceSynchronize on each side (host wall
clock: `value`); an untimed pass of K steps before it gives the GPU time (two events on the
library stream) and the per-kernel durations (events carried by the kernel dispatches
themselves, hipExtLaunchKernelGGL, so they agree with rocprofv3's kernel trace).

Workload: BASELINE.json configs[1] at every N (1 M synthetic 64 B Eth/IPv4/UDP frames, 1 bound
port, per GPU: weak scaling, no data-path collective), so the driver's per-N values compare one
workload. Beside it, at every N, the `scale` object measures the scaling workload BASELINE.json
configs[4] (config 5) the same way: every rank processes its own independent 4 M x 64 B shard
over 4096 ports, Zipf-0.99 (ports seeded 1000 + rank, frames 0x5EED ^ rank), barrier + max over
ranks, aggregate over all GPUs. Each rank reports its GPU's PCI bus id; with N > 1 they must be
distinct (UDPDK_BENCH_SHARED_DEVICE=1 allows a rehearsal with every rank on one GPU).

`--gpus N` is honoured two ways: under torchrun (WORLD_SIZE set) it must equal WORLD_SIZE; run
directly with N > 1, bench.py spawns N worker processes itself (one per GPU, gloo rendezvous on
127.0.0.1) before anything touches HIP, and prints rank 0's line.

To keep the 256 MiB Infinity Cache from serving the 64 B batch (≈80 MB) out of cache, the timed
loop rotates over enough device copies of the batch that a copy is evicted before its reuse
(> 512 MiB in flight), so every step reads its frames from HBM.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from udpdk_amd import abi, frames as F  # noqa: E402

HBM_PEAK_GBS = 8000.0    # MI355X HBM3E peak, MI355X_MICROARCH.md chip table


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (one process each); default WORLD_SIZE, else 1")
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", type=int, default=None,
                   help="BASELINE.json config number (1..5) of the headline line; default 2")
    p.add_argument("--no-scale", action="store_true", help="skip the config-5 `scale` object")
    p.add_argument("--frames", type=int, default=None, help="override frames per GPU")
    p.add_argument("--strong-total", type=int, default=None,
                   help="strong scaling: this many frames in total, split into contiguous equal "
                        "shards over the ranks (SURVEY.md 8(e): one 32 M batch)")
    p.add_argument("--no-strong", action="store_true",
                   help="skip the `strong` object (one 32 M-frame config-5 batch over the ranks)")
    p.add_argument("--strong-pieces", type=int, default=8,
                   help="`strong`: the batch is this many config-5 shards of --strong-piece frames")
    p.add_argument("--strong-piece", type=int, default=1 << 22, help="frames per strong-batch piece")
    p.add_argument("--rotate-mib", type=int, default=640, help="device bytes cycled by the loop")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extra", action="store_true", help="skip the 1500 B / IMIX side lines")
    p.add_argument("--cpu-seconds", type=float, default=4.0, help="target CPU time per baseline leg")
    p.add_argument("--pipeline", type=int, default=None, choices=(1, 2, 3, 4),
                   help="udpdk_gpu_pipeline_depth: d > 1 overlaps consecutive batches on d streams "
                        "(default: 3 for one socket, 4 when the batch takes the multi-lane path)")
    p.add_argument("--timing-every", type=int, default=16,
                   help="per-kernel timing on every Nth call (dispatch-carried events)")
    p.add_argument("--dry-run", action="store_true",
                   help="no GPU: rendezvous, build each rank's workload, print the plan line")
    return p.parse_args()


def spawn_workers(n: int) -> int:
    """`bench.py --gpus N` without torchrun: start N copies of this script as ranks 0..N-1
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), each on GPU
    LOCAL_RANK. Called before any HIP call in this process, which never touches the GPU. Rank
    0's stdout (the JSON line) is passed through; the exit code is the first failing rank's."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = procs[0].communicate()[0]
    rcs = [procs[0].returncode] + [p.wait() for p in procs[1:]]
    sys.stdout.write(out.decode())
    sys.stdout.flush()
    return next((rc for rc in rcs if rc), 0)


class Rx:
    """Device-resident copies of one batch plus prebuilt ctypes argument blocks."""

    def __init__(self, ctx: abi.GpuContext, w: F.Workload, rotate_bytes: int):
        b = w.batch
        self.ctx, self.w = ctx, w
        self.n = b.n
        self.sum_len = int(b.length.astype(np.int64).sum())
        per_copy = b.frames.nbytes + 10 * b.n
        self.copies = max(1, math.ceil(rotate_bytes / per_copy)) if rotate_bytes else 1
        hs = abi.snapshot_from_lists(w.port_lists(), w.n_sockets)
        ctx.upload_snapshot(hs)
        self._hs = hs
        self.args = []
        for _ in range(self.copies):
            db = abi.rx_upload(ctx, b.frames, b.offset, b.length)
            db.frames_bytes = b.frames_bytes
            out = abi.rx_alloc_out(ctx, b.n, w.n_sockets, b.n)
            bt = abi.RxBatch(db.frames.ptr, db.frames_bytes, db.offset.ptr, db.length.ptr, None, b.n)
            ot = abi.RxOut(out.meta.ptr, out.lane_off.ptr, out.lane_pkt.ptr, out.lane_cap)
            self.args.append((C.byref(bt), C.byref(ot), bt, ot, db, out))
        self.f = abi.lib().udpdk_gpu_rx
        self.h = ctx.handle
        # the single-lane path (one bound socket, no fan-out) compacts with rx_compact1 where
        # the multi-lane path scans and scatters: the third timed kernel id is named by what ran
        self.third = "rx_compact1" if w.n_sockets <= 1 else "rx_scatter"

    def step(self, i: int):
        a = self.args[i % self.copies]
        rc = self.f(self.h, a[0], a[1])
        if rc:
            raise abi.UdpdkError(f"udpdk_gpu_rx rc={rc}")

    def check(self):
        rc, st = abi.rx_stats(self.ctx)
        if rc != 0 or st.counters[abi.V_DELIVERED] != self.n:
            raise abi.UdpdkError(f"bench batch not fully delivered: rc={rc} "
                                 f"delivered={st.counters[abi.V_DELIVERED]} n={self.n}")
        return st

    def classify_bytes(self) -> int:
        # rx_classify algorithmic bytes per launch: every frame byte + u32 offset + u16 length
        # read, u32 verdict written, plus the tile histogram column (lanes x tiles x 4 B); on
        # the single-lane path classify also writes the lane entries (speculative compaction,
        # DESIGN.md §3; every frame of configs 1-3 is delivered)
        t, k = abi.geometry(self.n, self.w.n_sockets)
        spec = 4 * self.n if self.w.n_sockets == 1 else 0
        return self.sum_len + 6 * self.n + 4 * self.n + 4 * self.w.n_sockets * k + spec

    def pipeline_bytes(self) -> int:
        # sum(frame_len) + 8 N (descriptor) + 4 N (verdict) + 4 D (lane entry)
        return self.sum_len + 8 * self.n + 4 * self.n + 4 * self.n + 4 * (self.w.n_sockets + 1)


class HipEvents:
    """Two timing events on the library's stream (libamdhip64 through ctypes): the GPU time of
    the whole timed region, with no per-launch events inside it (an event pair around a single
    launch adds the dispatch latency that back-to-back launches hide)."""

    def __init__(self, ctx: abi.GpuContext):
        self.hip = C.CDLL("libamdhip64.so")
        self.stream = C.c_void_p(abi.lib().udpdk_gpu_stream(ctx.handle))
        self.ev = [C.c_void_p(), C.c_void_p()]
        for e in self.ev:
            if self.hip.hipEventCreate(C.byref(e)) != 0:
                raise RuntimeError("hipEventCreate failed")

    def record(self, i: int):
        if self.hip.hipEventRecord(self.ev[i], self.stream) != 0:
            raise RuntimeError("hipEventRecord failed")

    def elapsed_ms(self) -> float:
        self.hip.hipEventSynchronize(self.ev[1])
        ms = C.c_float()
        if self.hip.hipEventElapsedTime(C.byref(ms), self.ev[0], self.ev[1]) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return float(ms.value)

    def close(self):
        for e in self.ev:
            self.hip.hipEventDestroy(e)


_HIP = None


def device_sync():
    """hipDeviceSynchronize (what torch.cuda.synchronize does): the timed region's brackets.
    The library's own ctx.sync() waits on each pipe's stream in turn and costs ~1 us per step
    more at 20 steps (profiles/r02g_sync_cost.json)."""
    global _HIP
    if _HIP is None:
        _HIP = C.CDLL("libamdhip64.so")
    rc = _HIP.hipDeviceSynchronize()
    if rc:
        raise RuntimeError(f"hipDeviceSynchronize failed: {rc}")


def time_loop(rx: Rx, steps: int, warmup: int, barrier, timing_every: int):
    """`warmup` untimed calls; then, also untimed, the `steps` calls once between two events on
    the library stream (GPU time, with a join so that the other pipes' calls are inside) and with
    the library's per-kernel timing mode (events riding on the kernel dispatches themselves, on
    every `timing_every`-th call). Then the timed region (value): the same number of calls
    between a barrier + device synchronisation on each side (host wall clock) and nothing else
    inside: the join and the event records cost ~30 us per region (profiles/r02g_sync_cost.json)."""
    ctx = rx.ctx
    for i in range(warmup):
        rx.step(i)
    rx.check()
    ev = HipEvents(ctx)
    ctx.timing(timing_every)
    ctx.timing_read()                    # reset accumulators
    ctx.sync()
    ev.record(0)
    for i in range(steps):
        rx.step(warmup + i)
    ctx.join()                           # the other pipes' calls before the closing event
    ev.record(1)
    ctx.sync()
    gpu_ms = ev.elapsed_ms()
    ev.close()
    ms, n = ctx.timing_read() if timing_every else ([0.0] * abi.N_KERNEL_IDS, [0] * abi.N_KERNEL_IDS)
    ctx.timing(0)
    kt = {name: 1e3 * ms[k] / n[k] for k, name in
          enumerate(("rx_classify", "rx_scan", rx.third)) if n[k]}
    # the timed region
    barrier()
    device_sync()
    t0 = time.perf_counter()
    for i in range(steps):
        rx.step(warmup + steps + i)
    device_sync()
    t1 = time.perf_counter()
    barrier()
    st = rx.check()
    return (t1 - t0), gpu_ms / steps, kt, st


def _digest(*arrays) -> str:
    import hashlib
    h = hashlib.blake2b(digest_size=8)
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def host_cores() -> int:
    """CPUs this process may run on (its affinity mask): all online cores unless the host
    partitions them; the count the CPU baseline's "cores" states."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def pci_bus_id(device: int) -> str:
    """hipDeviceGetPCIBusId of a device (the process already uses it): names the physical GPU a
    rank ran on, whatever device numbering its environment gives it."""
    global _HIP
    if _HIP is None:
        _HIP = C.CDLL("libamdhip64.so")
    buf = C.create_string_buffer(64)
    rc = _HIP.hipDeviceGetPCIBusId(buf, 64, device)
    return buf.value.decode() if rc == 0 else f"unknown(rc={rc})"


def effective_cpus() -> int:
    """The CPUs the process can actually use at once: its affinity mask, capped by the cgroup
    CPU quota (the GPU boxes show 256 CPUs in the mask under a 16-CPU quota; threads beyond
    the quota time-slice). The count the CPU baseline's "cores" states."""
    n = host_cores()
    for f in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(f).read().split()[:2]
            if q != "max":
                n = min(n, max(1, math.ceil(int(q) / int(per))))
            return n
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            n = min(n, max(1, math.ceil(q / per)))
    except (OSError, ValueError):
        pass
    return n


def cpu_quota() -> str:
    """The cgroup CPU limit of this process (v2 cpu.max, else v1 cfs quota/period): the share of
    the host cores the affinity mask may not show."""
    for f in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(f).read().split()[:2]
            return "unlimited" if q == "max" else f"{int(q) / int(per):.2f} cpus ({f})"
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return "unlimited" if q < 0 else f"{q / per:.2f} cpus (cgroup v1)"
    except (OSError, ValueError):
        return "unknown"


def oracle_digest(w: F.Workload):
    """64-bit digest of the oracle's verdict words and lanes for workload w (parity mode,
    SURVEY.md §8(d)); compared with the digest of the GPU outputs of the same batch."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    b = w.batch
    wm, wl, wp, _ = O.rx(O.bindtable_from_lists(w.port_lists()), b.frames, b.frames_bytes, b.offset,
                         b.length, None, w.n_sockets)
    return _digest(wm, wl, wp)


def gpu_digest(ctx, out, n: int, n_lanes: int):
    meta = ctx.download(out.meta, np.uint32, n)
    loff = ctx.download(out.lane_off, np.uint32, n_lanes + 1)
    pkt = ctx.download(out.lane_pkt, np.uint32, int(loff[-1]))
    return _digest(meta, loff, pkt)


def cpu_baseline(w: F.Workload, target_s: float, gpu_dig: str | None = None, sweep=True):
    """Oracle (the C restatement, kind "port") on the host cores: every pinned thread runs the
    poller over its own full, NUMA-local copy of the batch with preallocated poller state (one
    independent shard per thread), with the RX checksum verification; a sweep over thread counts
    (1, 16, 32, 64, 128, 256 and every core the process may run on), the best reported as the
    baseline with its thread count. With gpu_dig (digest of the GPU outputs of the measured
    batch) the leg also runs the restatement once on that batch and compares digests (SURVEY.md
    §8(d) "parity mode")."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    b = w.batch
    bt = O.bindtable_from_lists(w.port_lists())
    parity = None
    if gpu_dig is not None:
        parity = {"oracle": oracle_digest(w), "gpu": gpu_dig}
        parity["match"] = parity["oracle"] == parity["gpu"]
    res = {"parity": parity, "sweep": {}}
    cores = host_cores()
    eff = effective_cpus()
    counts = sorted({t for t in (1, 16, 32, 64, 128, 256) if t <= cores} | {cores, eff}) if sweep else [1, cores]

    def leg(th, csum):
        # calibrate reps so the timed leg takes ~target_s (every rep: th x n frames)
        reps, secs = 1, O.rx_parallel(bt, b.frames, b.frames_bytes, b.offset, b.length, w.n_sockets, csum, th, 1)
        if secs < 0:
            raise RuntimeError(f"oracle_rx_parallel failed at {th} threads")
        reps = max(1, int(target_s / max(secs, 1e-6)))
        secs = O.rx_parallel(bt, b.frames, b.frames_bytes, b.offset, b.length, w.n_sockets, csum, th, reps)
        return (th * b.n * reps / secs / 1e6, reps, secs)
    for th in counts:
        res["sweep"][th] = leg(th, True)
    res[(1, False)] = leg(1, False)
    res[(cores, False)] = leg(cores, False)
    res["best"] = max(res["sweep"], key=lambda t: res["sweep"][t][0])
    return res, cores


def config1_line(target_s: float):
    """BASELINE.json configs[0]: apps/pktgen's traffic (64 B UDP payload = 106 B frames,
    apps/pktgen/main.c:53,156; one socket bound ANY:10001, main.c:183-191) through the CPU poller
    path, here the C restatement of reassemble() + flush_rx_queue (the reference needs DPDK,
    absent), on 1 thread and on every host core."""
    w = F.config_batch(1)
    res, cores = cpu_baseline(w, target_s, sweep=False)
    return {"workload": w.name, "kind": "port",
            "one_thread_mpkt_s": round(res["sweep"][1][0], 2),
            "one_thread_no_csum_mpkt_s": round(res[(1, False)][0], 2),
            "all_cores_mpkt_s": round(res["sweep"][cores][0], 2), "cores": cores,
            "gbps_all_cores": round(res["sweep"][cores][0] * 106 / 1e3, 2)}


def auto_depth(w) -> int:
    """Batches in flight for a workload: the single-lane path (classify + compaction) is fastest
    at 3 streams, the multi-lane path (classify + scan + scatter, whose short kernels fill the
    gaps of other batches' classify) at 4 (profiles/r02j_pipeline_depth.json)."""
    return 3 if w.n_sockets <= 1 else 4


def side_config(ctx, cfg: int, steps: int, rotate: int):
    w = F.config_batch(cfg)
    rx = Rx(ctx, w, rotate)
    ctx.pipeline(auto_depth(w))
    wall, gpu_step, _, st = time_loop(rx, steps, 5, lambda: None, 0)
    ctx.pipeline(1)
    wall1, gpu_step1, kt, _ = time_loop(rx, steps, 5, lambda: None, 4)
    cls_gbps = rx.classify_bytes() / (kt.get("rx_classify", 1e3 * gpu_step1) / 1e6) / 1e9
    a0 = rx.args[0]
    dg = gpu_digest(ctx, a0[5], rx.n, w.n_sockets)
    od = oracle_digest(w)
    out = {"workload": w.name, "mpkt_s": round(rx.n * steps / wall / 1e6, 1),
           "gbps_pipeline": round(rx.pipeline_bytes() * steps / wall / 1e9, 1),
           "gpu_us_per_step": round(1e3 * gpu_step, 2),
           "depth1_mpkt_s": round(rx.n * steps / wall1 / 1e6, 1),
           "kernel_us": {k: round(v, 2) for k, v in kt.items()},
           "classify_gbps": round(cls_gbps, 1),
           "frac_hbm_classify": round(cls_gbps / HBM_PEAK_GBS, 4),
           "frac_hbm_pipeline": round(rx.pipeline_bytes() * steps / wall / 1e9 / HBM_PEAK_GBS, 4),
           "parity": {"gpu": dg, "oracle": od, "match": dg == od}}
    for a in rx.args:
        a[4].frames.free(); a[4].offset.free(); a[4].length.free()
        a[5].meta.free(); a[5].lane_off.free(); a[5].lane_pkt.free()
    return out


class SporadicRx:
    """Config 2's single-socket stream where every `period`-th call carries one stray frame (a
    datagram to an unbound port, NO_BIND, at a seeded position): the call's tiles are not all
    full, so its fused completion repairs the lane in the same launch."""

    def __init__(self, ctx, rotate: int, period: int = 9):
        w = F.config_batch(2)
        wd = F.config_batch(2)
        pos = int(np.random.default_rng(99).integers(0, wd.batch.n))
        v = wd.batch.frames[:wd.batch.n * 64].reshape(wd.batch.n, 64)
        v[pos, 36], v[pos, 37] = 0x4E, 0x20                        # dst port 20000
        self.clean, self.drop = Rx(ctx, w, rotate), Rx(ctx, wd, rotate // 4)
        self.period, self.pos, self.n = period, pos, w.batch.n

    def step(self, i: int):
        (self.drop if i % self.period == self.period - 1 else self.clean).step(i)


def sporadic_line(ctx, steps: int, rotate: int):
    """Per-call time of a single-socket stream with a stray frame every 9th call against the
    clean stream (same pipeline depth, same number of calls, GPU events around the calls), and
    the stray call alone at depth 1 against a clean call; parity of the stray call's outputs."""
    sp = SporadicRx(ctx, rotate)
    depth = auto_depth(sp.clean.w)
    steps = max(steps // 9, 2) * 9

    def run(step, k, d):
        ctx.pipeline(d)
        for i in range(18):
            step(i)
        ctx.sync()
        ev = HipEvents(ctx)
        ev.record(0)
        for i in range(k):
            step(18 + i)
        ctx.join()
        ev.record(1)
        ms = ev.elapsed_ms()
        ev.close()
        ctx.pipeline(1)
        return 1e3 * ms / k
    clean_us = run(sp.clean.step, steps, depth)
    spor_us = run(sp.step, steps, depth)
    clean1 = run(sp.clean.step, 36, 1)
    drop1 = run(sp.drop.step, 36, 1)
    dg = gpu_digest(ctx, sp.drop.args[0][5], sp.n, 1)
    od = oracle_digest(sp.drop.w)
    out = {"workload": f"{sp.clean.w.name}, one NO_BIND frame every {sp.period}th call (frame {sp.pos})",
           "pipeline_depth": depth, "calls": steps,
           "clean_us_per_call": round(clean_us, 3), "sporadic_us_per_call": round(spor_us, 3),
           "sporadic_over_clean": round(spor_us / clean_us, 4),
           "depth1_clean_us": round(clean1, 3), "depth1_stray_call_us": round(drop1, 3),
           "parity": {"gpu": dg, "oracle": od, "match": dg == od}}
    for r in (sp.clean, sp.drop):
        for a in r.args:
            a[4].frames.free(); a[4].offset.free(); a[4].length.free()
            a[5].meta.free(); a[5].lane_off.free(); a[5].lane_pkt.free()
    return out


def tx_line(ctx, payload_len: int, n: int, steps: int, mtu: int = 0):
    """udpdk_gpu_tx_build over n datagrams of payload_len bytes (one bound socket, ANY:10000 ->
    172.31.100.1:10001, frames back to back): device-resident TX header build + rte_ipv4_cksum +
    payload copy, GPU time from events around `steps` back-to-back launches. mtu != 0: the
    poller's fragmentation too (udpdk_gpu_tx_build_mtu)."""
    slots = [(0, abi.raw_port(10000), 1)]
    hs = abi.snapshot_from_lists({}, 1, slots=slots)
    ctx.upload_snapshot(hs)
    rng = np.random.default_rng(7)
    pay = rng.integers(0, 256, n * payload_len + 64, dtype=np.uint8)
    pay_off = (np.arange(n, dtype=np.uint64) * payload_len).astype(np.uint32)
    lens = np.full(n, payload_len, np.uint16)
    span = int(abi.lib().udpdk_gpu_tx_span(payload_len, mtu, None))
    frame_off = (np.arange(n, dtype=np.uint64) * span).astype(np.uint32)
    bufs = [ctx.upload(pay), ctx.upload(pay_off), ctx.upload(lens), ctx.upload(np.zeros(n, np.int32)),
            ctx.upload(np.full(n, abi.raw_ip("172.31.100.1"), np.uint32)),
            ctx.upload(np.full(n, abi.raw_port(10001), np.uint16)), ctx.upload(frame_off)]
    cap = n * span + 64
    out = ctx.alloc(cap)
    cfg = abi.TxConfig((C.c_uint8 * 6)(*bytes.fromhex("6805ca95f8ec")),
                       (C.c_uint8 * 6)(*bytes.fromhex("6805ca95fa64")), abi.raw_ip("172.31.100.2"))
    bt = abi.TxBatch(bufs[0].ptr, pay.nbytes, bufs[1].ptr, bufs[2].ptr, bufs[3].ptr, bufs[4].ptr,
                     bufs[5].ptr, n)
    ot = abi.TxOut(out.ptr, cap, bufs[6].ptr)
    f = abi.lib().udpdk_gpu_tx_build_mtu
    args = (ctx.handle, C.byref(cfg), C.byref(bt), C.byref(ot), mtu)
    for _ in range(5):
        abi._check(f(*args), "udpdk_gpu_tx_build")
    ev = HipEvents(ctx)
    ctx.sync()
    ev.record(0)
    for _ in range(steps):
        f(*args)
    ev.record(1)
    ctx.sync()
    us = 1e3 * ev.elapsed_ms() / steps
    ev.close()
    nbytes = n * payload_len + n * span + 12 * n   # payload in, frames out, metadata
    for b in bufs + [out]:
        b.free()
    nf = C.c_uint32()
    abi.lib().udpdk_gpu_tx_span(payload_len, mtu, C.byref(nf))
    what = f"TX {n} x {payload_len + 42} B frames" if nf.value == 1 else \
        f"TX {n} x {payload_len} B datagrams -> {nf.value} fragments at MTU {mtu}"
    return {"workload": what, "mpkt_s": round(n / us, 1),
            "us_per_launch": round(us, 2), "gbps": round(nbytes / us / 1e3, 1),
            "frac_hbm": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4)}


def reasm_line(ctx, n_dgrams: int, payload_len: int, reps: int):
    """udpdk_gpu_rx_reassemble (f2) over a batch of n_dgrams datagrams of payload_len bytes cut
    at MTU 1500 (frames.frag_batch: every datagram its own flow, fragments in order), the table
    at the reference geometry (0x1000 buckets x 16, udpdk_poller.c:130). The call is synchronous
    (collect, two radix sorts, flow processing, completion sort + scan, emit), so the time is
    host wall clock per call. Bytes: fragment frames read + datagram frames written."""
    b = F.frag_batch(n_dgrams, payload_len)
    ctx.upload_snapshot(abi.snapshot_from_lists({abi.raw_port(F.PORT_RECV): [(0, 0, 0)]}, 1))
    abi.frag_table_create(ctx, 0x1000, 16, 1 << 40, 65515)
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(ctx, b.n, 1, b.n)
    abi.rx_run(ctx, db, out)
    rb, _, st = abi.rx_reassemble(ctx, db, out.meta, 0)
    assert st["done"] == n_dgrams, st
    out_bytes = int(rb.frames_bytes)
    t0 = time.perf_counter()
    for r in range(reps):
        rb, _, st = abi.rx_reassemble(ctx, db, out.meta, r + 1)
    us = 1e6 * (time.perf_counter() - t0) / reps
    assert st["done"] == n_dgrams, st
    # the demux of the reassembled datagrams (full UDP checksum over each datagram)
    out2 = abi.rx_alloc_out(ctx, n_dgrams, 1, n_dgrams)
    m2 = abi.rx_run(ctx, rb, out2)[0]
    ok = bool(np.all(abi.meta_verdict(m2) == 0) and np.all(abi.meta_udp(m2) == 1))
    for x in (db.frames, db.offset, db.length, out.meta, out.lane_off, out.lane_pkt, out2.meta,
              out2.lane_off, out2.lane_pkt):
        x.free()
    nbytes = b.frames_bytes + out_bytes
    return {"workload": f"reassembly {n_dgrams} x {payload_len} B datagrams ({b.n // n_dgrams} fragments "
                        f"each, MTU 1500), one batch", "mdgram_s": round(n_dgrams / us, 2),
            "us_per_call": round(us, 1), "gbps": round(nbytes / us / 1e3, 1),
            "frac_hbm": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4), "all_delivered_udp_ok": ok,
            "timing": "host wall clock per synchronous call"}


def reasm_inplace_line(ctx, n_dgrams: int, payload_len: int, reps: int):
    """udpdk_gpu_rx_reassemble_inplace (f2, zero-copy as DPDK chains the fragment mbufs) over the
    same batch as reasm_line: every datagram's fragments are back to back and in order, so the
    first fragment's frame is extended over the second's (its data moves 34 bytes back, the
    header is patched). The call consumes the batch, so each timed call gets the batch restored
    first (outside the timed region); host wall clock per call. Bytes: the later fragments' data
    read + written, the fragment headers read (the flow analysis), the first header patched."""
    b = F.frag_batch(n_dgrams, payload_len)
    ctx.upload_snapshot(abi.snapshot_from_lists({abi.raw_port(F.PORT_RECV): [(0, 0, 0)]}, 1))
    abi.frag_table_create(ctx, 0x1000, 16, 1 << 40, 65515)
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(ctx, b.n, 1, b.n)
    abi.rx_run(ctx, db, out)

    def restore():
        abi._check(abi.lib().udpdk_gpu_h2d(ctx.handle, C.c_void_p(db.frames.ptr), C.c_void_p(b.frames.ctypes.data),
                                           b.frames_bytes), "h2d")
        ctx.sync()
    ts = []
    for r in range(reps + 1):
        restore()
        t0 = time.perf_counter()
        rb, _, st = abi.rx_reassemble(ctx, db, out.meta, r, inplace=True)
        ts.append(time.perf_counter() - t0)
        assert st["done"] == n_dgrams and rb.frames.ptr == db.frames.ptr, st
    us = 1e6 * sum(ts[1:]) / reps
    out2 = abi.rx_alloc_out(ctx, n_dgrams, 1, n_dgrams)
    m2 = abi.rx_run(ctx, rb, out2)[0]
    ok = bool(np.all(abi.meta_verdict(m2) == 0) and np.all(abi.meta_udp(m2) == 1))
    for x in (db.frames, db.offset, db.length, out.meta, out.lane_off, out.lane_pkt, out2.meta,
              out2.lane_off, out2.lane_pkt):
        x.free()
    nf = b.n // n_dgrams
    moved = n_dgrams * (2 * (payload_len + 8 - 1480) + 64 * nf + 20)
    return {"workload": f"in-place reassembly {n_dgrams} x {payload_len} B datagrams ({nf} fragments each, "
                        f"MTU 1500), one batch", "mdgram_s": round(n_dgrams / us, 2),
            "us_per_call": round(us, 1), "bytes_moved_per_call": moved,
            "gbps_moved": round(moved / us / 1e3, 1), "frac_hbm_moved": round(moved / us / 1e3 / HBM_PEAK_GBS, 4),
            "all_delivered_udp_ok": ok,
            "timing": "host wall clock per synchronous call, the batch restored before each"}


def rss_line(ctx, cfg: int, n_queues: int, steps: int):
    """udpdk_gpu_rss (f4) over one batch of config `cfg`: Toeplitz hash, redirection table and
    per-queue lists, GPU time from events around `steps` back-to-back calls. Algorithmic bytes
    per frame: 26 header bytes + 6 descriptor read, 4 hash + 1 queue id written, 1 queue id
    read + 4 list entry written."""
    w = F.config_batch(cfg)
    b = w.batch
    cf = abi.rss_conf(n_queues)
    abi._check(abi.lib().udpdk_gpu_rss_config(ctx.handle, C.byref(cf)), "udpdk_gpu_rss_config")
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    h, qo, qp = ctx.alloc(4 * b.n), ctx.alloc(4 * (n_queues + 1)), ctx.alloc(4 * b.n)
    bt = abi.RxBatch(db.frames.ptr, db.frames_bytes, db.offset.ptr, db.length.ptr, None, b.n)
    ro = abi.RssOut(h.ptr, qo.ptr, qp.ptr)
    f = abi.lib().udpdk_gpu_rss
    for _ in range(3):
        abi._check(f(ctx.handle, C.byref(bt), C.byref(ro)), "udpdk_gpu_rss")
    ev = HipEvents(ctx)
    ctx.sync()
    ev.record(0)
    for _ in range(steps):
        f(ctx.handle, C.byref(bt), C.byref(ro))
    ev.record(1)
    ctx.sync()
    us = 1e3 * ev.elapsed_ms() / steps
    ev.close()
    counts = np.diff(ctx.download(qo, np.uint32, n_queues + 1).astype(np.int64))
    for x in (db.frames, db.offset, db.length, h, qo, qp):
        x.free()
    nbytes = (26 + 6 + 4 + 1 + 1 + 4) * b.n
    return {"workload": f"RSS {w.name} over {n_queues} queues", "mpkt_s": round(b.n / us, 1),
            "us_per_call": round(us, 2), "gbps": round(nbytes / us / 1e3, 1),
            "frac_hbm": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4),
            "queue_min_max": [int(counts.min()), int(counts.max())]}


def gather_line(ctx, cfg: int, steps: int, slot: int = 2048):
    """udpdk_gpu_rx_gather (f1, the batch form of recvfrom) over every delivery of one RX batch
    of config `cfg`: payload slots of `slot` bytes + length + source address per datagram, GPU
    time from events around `steps` back-to-back launches. Bytes per datagram: payload read +
    payload written + 16 header + 4 lane entry + 6 descriptor + 10 outputs. slot=0: packed
    slots, each its frame's payload rounded up to 16 bytes (udpdk_gpu_rx_gather_packed, the
    layout udpdk_poll_rx gathers into), + 4 bytes of slot offset per datagram."""
    w = F.config_batch(cfg)
    b = w.batch
    ctx.upload_snapshot(abi.snapshot_from_lists(w.port_lists(), w.n_sockets))
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(ctx, b.n, w.n_sockets, b.n)
    _, loff, pkt, _, rc = abi.rx_run(ctx, db, out)
    d = int(loff[-1])
    so = None
    if slot:
        g = abi.rx_alloc_gather(ctx, d, slot)
        call = lambda: abi.rx_gather_enqueue(ctx, db, out.lane_pkt, 0, g)
    else:
        pl = b.length[pkt[:d]].astype(np.int64) - 42
        offs = np.concatenate([[0], np.cumsum((np.maximum(pl, 0) + 15) // 16 * 16)])
        so = ctx.upload(offs.astype(np.uint32))
        g = abi.rx_alloc_gather(ctx, d, 16)
        g.payload.free()
        g.payload = ctx.alloc(int(offs[-1]) + 16)
        bt = abi.RxBatch(db.frames.ptr, db.frames_bytes, db.offset.ptr, db.length.ptr, None, b.n)
        gt = abi.RxGather(g.payload.ptr, 16, g.length.ptr, g.src_ip.ptr, g.src_port.ptr)
        call = lambda: abi.lib().udpdk_gpu_rx_gather_packed(ctx.handle, C.byref(bt), C.c_void_p(out.lane_pkt.ptr),
                                                           0, d, C.c_void_p(so.ptr), C.byref(gt))
    for _ in range(3):
        abi._check(call(), "udpdk_gpu_rx_gather")
    ev = HipEvents(ctx)
    ctx.sync()
    ev.record(0)
    for _ in range(steps):
        call()
    ev.record(1)
    ctx.sync()
    us = 1e3 * ev.elapsed_ms() / steps
    ev.close()
    lens = ctx.download(g.length, np.uint32, d)
    nbytes = 2 * int(lens.astype(np.int64).sum()) + (36 if slot else 40) * d
    for x in (db.frames, db.offset, db.length, out.meta, out.lane_off, out.lane_pkt, g.payload,
              g.length, g.src_ip, g.src_port) + ((so,) if so is not None else ()):
        x.free()
    return {"workload": f"gather {w.name}, " + (f"{slot} B slots" if slot else "packed slots (udpdk_poll_rx layout)"),
            "mdgram_s": round(d / us, 1),
            "us_per_launch": round(us, 2), "gbps": round(nbytes / us / 1e3, 1),
            "frac_hbm": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4)}


def end_to_end_async(ctx, cfg: int, reps: int):
    """The same host-resident batch stream through udpdk_gpu_rx_host_async with pipelining depth
    2: batch k's H2D overlaps batch k-1's kernels and D2H (PCIe is full duplex); one
    udpdk_gpu_rx_host_wait at the end. Frames in pinned memory; outputs alternate between two
    pinned sets."""
    w = F.config_batch(cfg)
    b = w.batch
    ctx.upload_snapshot(abi.snapshot_from_lists(w.port_lists(), w.n_sockets))
    L = abi.lib()

    def pinned(nbytes):
        p = C.c_void_p()
        abi._check(L.udpdk_gpu_host_alloc(ctx.handle, max(16, nbytes), C.byref(p)), "host_alloc")
        return p
    held = [pinned(b.frames_bytes)]
    C.memmove(held[0].value, b.frames.ctypes.data, b.frames_bytes)
    outs = []
    for _ in range(2):
        o = (pinned(4 * b.n), pinned(4 * (w.n_sockets + 1)), pinned(4 * b.n), abi.RxStats())
        held += list(o[:3])
        outs.append(o)
    ctx.pipeline(2)

    def run(k):
        o = outs[k % 2]
        abi._check(L.udpdk_gpu_rx_host_async(ctx.handle, held[0].value, b.frames_bytes,
                                             b.offset.ctypes.data, b.length.ctypes.data, None, b.n,
                                             o[0].value, o[1].value, o[2].value, b.n, C.byref(o[3])),
                   "udpdk_gpu_rx_host_async")
    for k in range(2):
        run(k)
    abi._check(L.udpdk_gpu_rx_host_wait(ctx.handle), "udpdk_gpu_rx_host_wait")
    t0 = time.perf_counter()
    for k in range(reps):
        run(k)
    abi._check(L.udpdk_gpu_rx_host_wait(ctx.handle), "udpdk_gpu_rx_host_wait")
    dt = (time.perf_counter() - t0) / reps
    ok = all(int(o[3].deliveries) == b.n for o in outs)
    ctx.pipeline(1)
    for p in held:
        L.udpdk_gpu_host_free(ctx.handle, p)
    return {"workload": w.name, "mpkt_s": round(b.n / dt / 1e6, 1),
            "frame_gbps": round(int(b.length.sum()) / dt / 1e9, 2), "ms_per_batch": round(dt * 1e3, 3),
            "all_delivered": ok,
            "path": "pinned host frames -> H2D -> rx pipeline -> D2H meta+lanes, two pipes overlapped"}


def end_to_end(ctx, cfg: int, reps: int):
    """Host-resident batch through udpdk_gpu_rx_host: frames already in pinned host memory (DPDK
    hugepage mbufs registered with the runtime), H2D of frames + descriptors, the RX pipeline,
    D2H of verdicts and lanes, synchronous per batch. PCIe-inclusive; never the headline value."""
    w = F.config_batch(cfg)
    b = w.batch
    ctx.upload_snapshot(abi.snapshot_from_lists(w.port_lists(), w.n_sockets))
    L = abi.lib()

    def pinned(nbytes, dtype):
        p = C.c_void_p()
        abi._check(L.udpdk_gpu_host_alloc(ctx.handle, max(16, nbytes), C.byref(p)), "host_alloc")
        arr = np.ctypeslib.as_array((C.c_uint8 * max(16, nbytes)).from_address(p.value))
        return p, arr[:nbytes].view(dtype)
    held = []
    pf, fr = pinned(b.frames_bytes, np.uint8); held.append(pf)
    fr[:] = b.frames[:b.frames_bytes]
    po, meta = pinned(4 * b.n, np.uint32); held.append(po)
    pl, loff = pinned(4 * (w.n_sockets + 1), np.uint32); held.append(pl)
    pp, pkt = pinned(4 * b.n, np.uint32); held.append(pp)
    st = abi.RxStats()

    def once():
        abi._check(L.udpdk_gpu_rx_host(ctx.handle, pf.value, b.frames_bytes, b.offset.ctypes.data,
                                       b.length.ctypes.data, None, b.n, po.value, pl.value, pp.value,
                                       b.n, C.byref(st)), "udpdk_gpu_rx_host")
    once()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    dt = (time.perf_counter() - t0) / reps
    for p in held:
        L.udpdk_gpu_host_free(ctx.handle, p)
    return {"workload": w.name, "mpkt_s": round(b.n / dt / 1e6, 1),
            "frame_gbps": round(int(b.length.sum()) / dt / 1e9, 2), "ms_per_batch": round(dt * 1e3, 3),
            "path": "pinned host frames -> H2D -> rx pipeline -> D2H meta+lanes, synchronous"}


def socket_path_lines(specs=((1 << 20, 64, 1024, 5), (1 << 20, 0, 1024, 3), (1 << 20, 1500, 1024, 3),
                             (1 << 13, 65000, 64, 3)),
                      gpu_extra: str = ""):
    """The reference-API path end to end: tools/bin/bench_sock, a C program
    written against include/udpdk_api.h like the reference's apps, times udpdk_poll_rx (frames in
    pinned host memory -> H2D -> GPU classify/demux -> GPU payload gather -> D2H -> ring
    admission) and the recvfrom loop that empties every ring, per 1 M-frame batch over 1024
    sockets (frame size 0 = IMIX). Runs as its own process on the same GPU."""
    import subprocess
    exe = os.path.join(ROOT, "tools", "bin", "bench_sock")
    if not os.path.exists(exe):
        return [{"error": "tools/bin/bench_sock not built"}]
    import tempfile
    out = []
    with tempfile.NamedTemporaryFile("w", suffix=".ini", delete=False) as f:
        f.write("[port0]\nmac_addr = 68:05:ca:95:f8:ec\nip_addr = 172.31.100.1\n"
                "[port0_dst]\nmac_addr = 68:05:ca:95:fa:64\n"
                "[gpu]\ndevice = 0\nmax_frames = 1048576\nmax_lanes = 1024\n" + gpu_extra)
        ini = f.name
    # the 1500 B batch once more polled in one piece ([gpu] poll_chunk_mb = 0): the pipelined
    # poll's gain against its recvfrom cost on the same box
    ini1 = ini + ".onepiece.ini"
    with open(ini1, "w") as f:
        f.write(open(ini).read() + "\n[gpu]\npoll_chunk_mb = 0\n")
    try:
        for spec in list(specs) + [(1 << 20, 1500, 1024, 3, "one_piece")]:
            n, fb, socks, reps = spec[:4]
            tag = spec[4] if len(spec) > 4 else None
            r = subprocess.run([exe, ini1 if tag else ini, str(n), str(fb), str(socks), str(reps)],
                               capture_output=True, text=True, timeout=300)
            if r.returncode:
                out.append({"frames": n, "frame_bytes": fb, "error": r.stderr[-300:]})
            else:
                d = json.loads(r.stdout.strip().splitlines()[-1])
                if tag:
                    d["poll"] = "one piece (poll_chunk_mb = 0)"
                out.append(d)
    finally:
        os.unlink(ini)
        os.unlink(ini1)
    return out


def rank_parity(ctx, rx: Rx, dist) -> dict:
    """Parity of this rank's measured batch (outside the timed region): the digest of the GPU's
    verdict words and lanes for one call against the oracle's for the same frames (SURVEY.md
    §8(d) parity mode), gathered over the ranks so a multi-GPU run verifies every shard."""
    mine = {"gpu": gpu_digest(ctx, rx.args[0][5], rx.n, rx.w.n_sockets), "oracle": oracle_digest(rx.w)}
    mine["match"] = mine["gpu"] == mine["oracle"]
    ranks = [mine]
    if dist is not None:
        ranks = [None] * dist.get_world_size()
        dist.all_gather_object(ranks, mine)
    return {"rank0": mine, "all_ranks_match": all(r["match"] for r in ranks),
            "per_rank_match": [r["match"] for r in ranks]}


def strong_pieces(world: int, rank: int, pieces: int) -> range:
    """The pieces of the one strong-scaling batch rank `rank` of `world` takes: a contiguous run,
    pieces split as evenly as they go (8 pieces: 8 / 4 / 2 / 1 per rank at N = 1 / 2 / 4 / 8)."""
    return range(rank * pieces // world, (rank + 1) * pieces // world)


def strong_workload(world: int, rank: int, pieces: int, piece: int) -> F.Workload:
    """SURVEY.md §8(e)'s strong-scaling batch: ONE batch of pieces x piece 64 B frames (default
    8 x 4 M = 32 M) over 4096 ports, Zipf-0.99, defined as the concatenation of config 5's shards
    0..pieces-1 in order (piece p = config_batch(5, shard=p)), so rank r's contiguous part is built
    from its own pieces alone. At N = 8 every rank's part is config 5's shard: the weak point."""
    parts = [F.config_batch(5, n=piece, shard=p) for p in strong_pieces(world, rank, pieces)]
    if len(parts) == 1:
        w = parts[0]
    else:
        nb = sum(x.batch.frames_bytes for x in parts)
        flat = np.zeros((nb + 255) // 256 * 256 + 256, np.uint8)
        off, ln, pos = [], [], 0
        for x in parts:
            b = x.batch
            flat[pos:pos + b.frames_bytes] = b.frames[:b.frames_bytes]
            off.append(b.offset.astype(np.uint64) + pos)
            ln.append(b.length)
            pos += b.frames_bytes
        w = F.Workload(parts[0].name, F.Batch(flat, np.concatenate(off).astype(np.uint32),
                                              np.concatenate(ln), nb), 4096, 10000)
    total = pieces * piece
    w.name = f"{F._nlabel(total)}-64B-4096ports-zipf0.99 ({pieces} x {F._nlabel(piece)} pieces)"
    return w


def strong_line(ctx, world: int, rank: int, barrier, dist, steps: int, warmup: int, pieces: int, piece: int):
    """Strong scaling: one batch of pieces x piece frames split into contiguous
    parts over the N ranks (no collective: each part's lanes are the batch's lanes for its frames,
    shard.merge_lanes), each rank's part processed as one udpdk_gpu_rx call per step, pipelined;
    the steps bracketed by a barrier + device sync, the MAX wall over ranks; value = the whole
    batch's frames / that time. Fixed total work, so scaling is "strong"."""
    w = strong_workload(world, rank, pieces, piece)
    rx = Rx(ctx, w, 0)
    depth = auto_depth(w)
    ctx.pipeline(depth)
    wall, gpu_step, _, _ = time_loop(rx, steps, warmup, barrier, 0)
    ctx.pipeline(1)
    mine = rx.n * steps / wall / 1e6
    if dist is not None:
        import torch
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    total = pieces * piece
    out = {"workload": w.name, "baseline_config": 5, "scaling": "strong", "n_gpus": world,
           "frames_total": total, "frames_rank0": rx.n, "pieces_rank0": list(strong_pieces(world, rank, pieces)),
           "value": round(total * steps / wall / 1e6, 2), "unit": "Mpkt/s", "steps": steps,
           "ms_per_step": round(1e3 * wall / steps, 5), "pipeline_depth": depth,
           "gbps_pipeline": round(rx.pipeline_bytes() * world * steps / wall / 1e9, 1),
           "rank0_mpkt_s": round(mine, 2), "rank0_gpu_us_per_step": round(1e3 * gpu_step, 3)}
    out["parity"] = rank_parity(ctx, rx, dist)
    for a in rx.args:
        a[4].frames.free(); a[4].offset.free(); a[4].length.free()
        a[5].meta.free(); a[5].lane_off.free(); a[5].lane_pkt.free()
    return out


def scale_line(ctx, world: int, rank: int, barrier, dist, steps: int, warmup: int, rotate: int):
    """The scaling workload (BASELINE.json configs[4], config 5) at this N: each rank its own
    independent 4 M x 64 B shard over 4096 ports, Zipf-0.99 (seed 1000 + rank), pipelined, the K
    steps bracketed by a barrier + device sync on each side, the MAX wall over ranks; value = all
    ranks' frames / that time. The same object at N = 1, 2, 4, 8 gives config 5's curve."""
    w5 = F.config_batch(5, shard=rank)
    rx5 = Rx(ctx, w5, rotate)
    depth = auto_depth(w5)
    ctx.pipeline(depth)
    wall, gpu_step, _, _ = time_loop(rx5, steps, warmup, barrier, 0)
    ctx.pipeline(1)
    mine = rx5.n * steps / wall / 1e6
    if dist is not None:
        import torch
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    total = rx5.n * steps * world
    gbps = rx5.pipeline_bytes() * steps * world / wall / 1e9
    out = {"workload": w5.name, "baseline_config": 5, "n_gpus": world, "frames_per_gpu": rx5.n,
           "value": round(total / wall / 1e6, 2), "unit": "Mpkt/s", "steps": steps,
           "ms_per_step": round(1e3 * wall / steps, 5), "scaling": "weak", "pipeline_depth": depth,
           "gbps_pipeline": round(gbps, 1), "frac_hbm_pipeline_per_gpu": round(gbps / world / HBM_PEAK_GBS, 4),
           "rank0_mpkt_s": round(mine, 2), "rank0_gpu_us_per_step": round(1e3 * gpu_step, 3)}
    out["parity"] = rank_parity(ctx, rx5, dist)
    for a in rx5.args:
        a[4].frames.free(); a[4].offset.free(); a[4].length.free()
        a[5].meta.free(); a[5].lane_off.free(); a[5].lane_pkt.free()
    return out


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        raise SystemExit(spawn_workers(args.gpus))
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.config is None:
        args.config = 2
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # gloo prints its connection notice on stdout: keep stdout for the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(os.open(os.devnull, os.O_WRONLY), 1)
        try:
            dist.init_process_group("gloo")
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    import torch
    if args.dry_run:
        return dry_run(args, world, rank, dist)

    def barrier():
        if dist is not None:
            dist.barrier()

    ndev = abi.device_count()
    if ndev < 1:
        raise SystemExit("bench.py needs a GPU (no HIP device visible)")
    device = local % ndev
    frames = args.frames
    if args.strong_total:
        frames = -(-args.strong_total // world)          # this rank's contiguous shard
    w = F.config_batch(args.config, n=frames, shard=rank)
    strong_n = 0 if (args.no_strong or args.strong_total) else \
        len(strong_pieces(world, rank, args.strong_pieces)) * args.strong_piece
    ctx = abi.GpuContext(device, max_frames=max(w.batch.n, 1 << 22, strong_n), max_lanes=4096)
    rx = Rx(ctx, w, args.rotate_mib << 20)
    # the timed region (value): consecutive batches pipelined over several streams, no events inside
    if args.pipeline is None:
        args.pipeline = auto_depth(w)
    ctx.pipeline(args.pipeline)
    wall, gpu_step, _, st = time_loop(rx, args.steps, args.warmup, barrier, 0)
    # kernel durations for the roofline: the same calls one at a time (depth 1), every
    # --timing-every-th call carrying dispatch events, so each kernel runs without a neighbour
    ctx.pipeline(1)
    k_steps = max(16, args.steps // 2)
    wall1, gpu_step1, kt, _ = time_loop(rx, k_steps, 5, barrier, args.timing_every)
    # one isolated call (a single launch beside the steady state): events around
    # one udpdk_gpu_rx on an idle GPU, on a device copy not touched by the previous calls
    ev1 = HipEvents(ctx)
    ctx.sync()
    ev1.record(0)
    rx.step(k_steps + 5 + rx.copies // 2)
    ev1.record(1)
    ctx.sync()
    single_us = 1e3 * ev1.elapsed_ms()
    ev1.close()
    cls_bytes = rx.classify_bytes()
    mine = {"rank": rank, "device": device, "pci_bus_id": pci_bus_id(device), "frames": rx.n,
            "mpkt_s": round(rx.n * args.steps / wall / 1e6, 2),
            "gbps": round(rx.pipeline_bytes() * args.steps / wall / 1e9, 1),
            "classify_us": round(kt.get("rx_classify", 0.0), 3),
            "classify_gbps": round(cls_bytes / kt["rx_classify"] / 1e3, 1) if kt.get("rx_classify") else None,
            "kernel_us": {k: round(v, 3) for k, v in kt.items()}}
    per_rank = [mine]
    if dist is not None:
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    distinct = len({p["pci_bus_id"] for p in per_rank}) == world
    if world > 1 and not distinct and os.environ.get("UDPDK_BENCH_SHARED_DEVICE") != "1":
        raise SystemExit(f"ranks share a GPU: {[p['pci_bus_id'] for p in per_rank]} "
                         "(set UDPDK_BENCH_SHARED_DEVICE=1 for a one-GPU rehearsal)")
    scale = None
    if not args.no_scale and not args.strong_total:
        scale = scale_line(ctx, world, rank, barrier, dist, max(20, args.steps // 4), 5,
                           args.rotate_mib << 20)
        scale["distinct_gpus"] = distinct
    strong = None
    if strong_n:
        strong = strong_line(ctx, world, rank, barrier, dist, max(5, args.steps // 8), 3,
                             args.strong_pieces, args.strong_piece)
    total_pkts = rx.n * args.steps * world
    mpkt_s = total_pkts / wall / 1e6
    ms_step = 1e3 * wall / args.steps
    cls_us = kt.get("rx_classify", 1e3 * gpu_step1)    # timing off: the whole step, an upper bound
    achieved = cls_bytes / (cls_us / 1e6) / 1e9

    traffic = None
    tf = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tf):
        try:
            with open(tf) as f:
                traffic = json.load(f)["workloads"].get(w.name, {}).get("rx_classify_hbm_bytes_per_launch")
        except Exception:
            traffic = None

    rocprof = None
    rf = os.path.join(ROOT, "profiles", "rocprof_classify.json")
    if os.path.exists(rf):
        try:
            with open(rf) as f:
                r = json.load(f)["workloads"].get(w.name)
            if r:
                rocprof = {"kernel_us": r["mean_us"], "source": r["source"],
                           "achieved": round(cls_bytes / r["mean_us"] / 1e3, 1),
                           "frac": round(cls_bytes / r["mean_us"] / 1e3 / HBM_PEAK_GBS, 4)}
        except Exception:
            rocprof = None

    line = {
        "metric": "device-resident Mpkt/s + GB/s, RX parse+cksum+port-demux, 64B & 1500B frames",
        "value": round(mpkt_s, 2),
        "unit": "Mpkt/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 5),
        "higher_is_better": True,
        "scaling": "strong" if args.strong_total else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (SURVEY.md §8(d) recipe, seeded per rank)",
        "config": {"workload": w.name, "baseline_config": args.config, "frames_per_gpu": rx.n,
                   "frame_bytes_per_gpu": rx.sum_len, "bound_ports": w.n_sockets,
                   "parallelism": f"shard{world}", "device_copies_rotated": rx.copies},
        "gbps_pipeline": round(rx.pipeline_bytes() * args.steps * world / wall / 1e9, 1),
        "gpu_us_per_step": round(1e3 * gpu_step, 3),
        "single_call_us": round(single_us, 3),
        "pipeline_depth": args.pipeline,
        "depth1": {"mpkt_s": round(rx.n * k_steps / wall1 / 1e6, 2), "gpu_us_per_step": round(1e3 * gpu_step1, 3),
                   "note": "the same calls one at a time on one stream (kernel timing loop)"},
        "kernel_us": {k: round(v, 3) for k, v in kt.items()},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel": "rx_classify",
                     "traffic_source": "profiles/traffic.json: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                                       "passes of this workload (tools/pmc_traffic.sh)",
                     "algorithmic_bytes_per_launch": cls_bytes,
                     "kernel_us_events": round(cls_us, 3),
                     "rocprof": rocprof},
        "cpu_baseline": None,
    }
    line["per_rank"] = per_rank
    line["distinct_gpus"] = distinct
    if scale is not None:
        line["scale"] = scale
    if strong is not None:
        line["strong"] = strong
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        gdig = gpu_digest(ctx, rx.args[0][5], rx.n, w.n_sockets) if rx.n <= (1 << 22) else None
        res, cores = cpu_baseline(w, args.cpu_seconds, gdig)
        best = res["best"]
        v, reps, secs = res["sweep"][best]
        eff = effective_cpus()
        line["cpu_baseline"] = {
            "value": round(v, 2), "unit": "Mpkt/s", "cores": min(best, eff), "kind": "port",
            "sample": f"{best} pinned threads (the best of the sweep) on {min(best, eff)} effective "
                      f"CPUs (affinity {cores}, cgroup quota {cpu_quota()}), each thread running the "
                      f"poller restatement over its own NUMA-local copy of the {rx.n}-frame {w.name} "
                      f"batch x {reps} passes ({secs:.1f} s), RX checksum verification on",
            "threads": best, "effective_cpus": eff,
            "threads_sweep_mpkt_s": {str(t): round(x[0], 2) for t, x in res["sweep"].items()},
            "all_cores": {"threads": cores, "mpkt_s": round(res["sweep"][cores][0], 2)},
            "affinity_cores": cores, "cgroup_cpu_quota": cpu_quota(),
            "one_thread": round(res["sweep"][1][0], 2),
            "one_thread_no_csum": round(res[(1, False)][0], 2),
            f"{cores}_threads_no_csum": round(res[(cores, False)][0], 2),
            "parity": res["parity"],
        }
        try:
            line["config1_cpu"] = config1_line(args.cpu_seconds / 2)
        except Exception as e:
            line["config1_cpu"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_extra:
        extra = []
        for cfg in (1, 3, 4, 5):
            if cfg != args.config:
                try:
                    extra.append(side_config(ctx, cfg, max(10, args.steps // 4), args.rotate_mib << 20))
                except Exception as e:   # a side line never hides the main measurement
                    extra.append({"config": cfg, "error": repr(e)})
        line["other_configs"] = extra
        e2e = []
        for cfg in (2, 3, 4):
            try:
                e2e.append(end_to_end(ctx, cfg, 10))
            except Exception as e:
                e2e.append({"config": cfg, "error": repr(e)})
        for cfg in (2, 3):
            try:
                e2e.append(end_to_end_async(ctx, cfg, 20))
            except Exception as e:
                e2e.append({"config": cfg, "async": True, "error": repr(e)})
        line["end_to_end"] = e2e
        try:
            line["sporadic_drop"] = sporadic_line(ctx, max(90, args.steps), args.rotate_mib << 20)
        except Exception as e:
            line["sporadic_drop"] = {"error": repr(e)}
        try:
            line["socket_path"] = socket_path_lines()
        except Exception as e:
            line["socket_path"] = [{"error": repr(e)}]
        tx = []
        for plen in (22, 1458):                  # 64 B and 1500 B frames
            try:
                tx.append(tx_line(ctx, plen, 1 << 20, 50))
            except Exception as e:
                tx.append({"payload": plen, "error": repr(e)})
        try:
            tx.append(tx_line(ctx, 2952, 1 << 18, 50, mtu=1500))     # 2 x 1514 B fragments each
        except Exception as e:
            tx.append({"payload": 2952, "mtu": 1500, "error": repr(e)})
        line["tx"] = tx
        try:
            line["reassembly"] = [reasm_line(ctx, 1 << 18, 2952, 10)]
            try:
                line["reassembly"].append(reasm_inplace_line(ctx, 1 << 18, 2952, 10))
            except Exception as e:
                line["reassembly"].append({"in_place": True, "error": repr(e)})
        except Exception as e:
            line["reassembly"] = [{"error": repr(e)}]
        rs = []
        for cfg, nq in ((2, 8), (5, 8)):
            try:
                rs.append(rss_line(ctx, cfg, nq, 50))
            except Exception as e:
                rs.append({"config": cfg, "error": repr(e)})
        line["rss"] = rs
        ga = []
        for cfg in (2, 3):
            try:
                ga.append(gather_line(ctx, cfg, 50))
                if cfg == 2:
                    ga.append(gather_line(ctx, cfg, 50, slot=0))
            except Exception as e:
                ga.append({"config": cfg, "error": repr(e)})
        line["gather"] = ga
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def dry_run(args, world, rank, dist):
    """The multi-rank plumbing without a GPU: each rank builds its shard of the workload (small
    --frames keeps it quick), the ranks rendezvous, and rank 0 prints what every rank would
    measure (workload, frames, seeds) plus the barrier/max-over-ranks reduction of a dummy
    wall time."""
    frames = args.frames
    if args.strong_total:
        frames = -(-args.strong_total // world)
    w = F.config_batch(args.config, n=frames, shard=rank)
    mine = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "workload": w.name,
            "frames": w.batch.n, "digest": _digest(w.batch.frames[:w.batch.frames_bytes], w.batch.length)}
    if not args.no_scale and not args.strong_total:
        w5 = F.config_batch(5, n=frames, shard=rank)
        mine["scale_workload"] = w5.name
        mine["scale_frames"] = w5.batch.n
        mine["scale_digest"] = _digest(w5.batch.frames[:w5.batch.frames_bytes], w5.batch.length)
        mine["scale_digest_rebased"] = _digest(w5.batch.frames[:w5.batch.frames_bytes], w5.batch.length,
                                               w5.batch.offset)
    if not args.no_strong and not args.strong_total:
        ws = strong_workload(world, rank, args.strong_pieces, args.strong_piece)
        mine["strong_workload"] = ws.name
        mine["strong_pieces"] = list(strong_pieces(world, rank, args.strong_pieces))
        mine["strong_frames"] = ws.batch.n
        # each piece's bytes, lengths and rebased offsets, cut back out of the rank's batch
        pd, k = [], args.strong_piece
        for j in range(len(mine["strong_pieces"])):
            o = ws.batch.offset[j * k:(j + 1) * k].astype(np.int64)
            a, b = int(o[0]), int(o[-1]) + int(ws.batch.length[(j + 1) * k - 1])
            pd.append(_digest(ws.batch.frames[a:b], ws.batch.length[j * k:(j + 1) * k], (o - a).astype(np.uint32)))
        mine["strong_piece_digests"] = pd
    per_rank = [mine]
    wall = 1.0 + rank
    if dist is not None:
        import torch
        dist.barrier()
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "baseline_config": args.config,
                          "scaling": "strong" if args.strong_total else "weak",
                          "max_wall": wall, "per_rank": per_rank}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
