"""Per-phase cycle stamps of rx_classify (diagnostic build, make stamps). Prints the mean cycles
per workgroup (wave 0) spent in each phase, for a tiny batch (latency) and a full batch."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["UDPDK_LIB_OVERRIDE"] = os.path.join(ROOT, "tools", "diag", os.environ.get("STAMPS_LIB", "libudpdk_amd.so"))
sys.path.insert(0, ROOT)
import numpy as np
from udpdk_amd import abi, frames as F

PH = ["prologue", "window wait+fields", "header sums", "demux pass", "fused completion", "descriptor staging+barrier",
      "state+stash+tail+next window", "counters+tile end"]
L = abi.lib()
L.udpdk_gpu_debug_buffer.argtypes = [C.c_void_p, C.c_void_p]
ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
dbg = ctx.alloc((2 * 8192 + 8192) * 16 * 8)   # classify rows, then rx_scatterw rows from 16384
L.udpdk_gpu_debug_buffer(ctx.handle, C.c_void_p(dbg.ptr))
CASES = [(2, 4096), (2, None), (4, 65536), (3, 65536)]
if os.environ.get("STAMPS_CASES"):      # e.g. "4:0,3:0" (0 = the config's full size)
    CASES = [(int(c), int(m) or None) for c, m in (x.split(":") for x in os.environ["STAMPS_CASES"].split(","))]
for cfg, n in CASES:
    w = F.config_batch(cfg, n=n)
    ctx.upload_snapshot(abi.snapshot_from_lists(w.port_lists(), w.n_sockets))
    # enough device copies that the 256 MiB Infinity Cache cannot hold them (as bench.py), so
    # the stamps show HBM-cold behaviour
    copies = max(1, -(-640 * 2**20 // (w.batch.frames.nbytes + 10 * w.batch.n)))
    dbs = []
    for _ in range(copies):
        db = abi.rx_upload(ctx, w.batch.frames, w.batch.offset, w.batch.length)
        db.frames_bytes = w.batch.frames_bytes
        dbs.append(db)
    L.udpdk_gpu_memset(ctx.handle, C.c_void_p(dbg.ptr), 0, 16 * 8 * 8192 + 64)
    out = abi.rx_alloc_out(ctx, w.batch.n, w.n_sockets, w.batch.n)
    abi.rx_run(ctx, dbs[0], out)
    for i in range(31):                 # back-to-back (warm GPU), the last launch's stamps stay
        abi._check(abi.rx_enqueue(ctx, dbs[i % copies], out), "udpdk_gpu_rx")
    abi.rx_stats(ctx)
    _, tiles = abi.geometry(w.batch.n, w.n_sockets)
    d = ctx.download(dbg, np.uint64, 16 * tiles).reshape(tiles, 16).astype(np.float64)
    print(f"{w.name} n={w.batch.n} tiles={tiles}")
    for k, name in enumerate(PH):
        print(f"   {name:20s} mean {d[:, k].mean():12.0f}  max {d[:, k].max():12.0f}")
    # timeline from the chip-synchronous 100 MHz realtime stamps (slots 12-13)
    raw = ctx.download(dbg, np.uint64, 16 * tiles).reshape(tiles, 16)
    st0 = raw[:, 12].astype(np.int64) - int(raw[:, 12].min())
    en0 = raw[:, 13].astype(np.int64) - int(raw[:, 12].min())
    dur = en0 - st0
    pct = lambda x: " ".join(f"{np.percentile(x, q) / 100:.2f}" for q in (0, 10, 50, 90, 100))
    print(f"   span {en0.max() / 100:.2f} us; start us p0/10/50/90/100: {pct(st0)}; "
          f"duration us: {pct(dur)}")
    xcc = (raw[:, 14] >> 32).astype(np.int64) & 0xF
    for x in np.unique(xcc)[:8]:
        m = xcc == x
        print(f"     xcc {x}: wgs {m.sum():5d} start p50 {np.median(st0[m]) / 100:.2f} "
              f"end max {en0[m].max() / 100:.2f}")
    hw = raw[:, 14].astype(np.int64)
    cu = ((hw >> 32) & 0xF) << 16 | ((hw >> 8) & 0xF) | ((hw >> 12) & 1) << 4 | ((hw >> 13) & 7) << 5
    ucu, inv, per = np.unique(cu, return_inverse=True, return_counts=True)
    simd = (hw >> 4) & 3
    print(f"   CUs used {len(ucu)}; WGs per CU min/median/max {per.min()}/{int(np.median(per))}/"
          f"{per.max()}; wave0 SIMD histogram {np.bincount(simd, minlength=4).tolist()}")
    # is a slow workgroup slow because of its CU (all its CU's workgroups slow) or on its own?
    cu_mean = np.bincount(inv, weights=dur) / per
    within = dur - cu_mean[inv]
    print(f"   duration std us: all {dur.std() / 100:.2f}, between CUs {cu_mean.std() / 100:.2f}, "
          f"within a CU {within.std() / 100:.2f}; CU mean p10/50/90 "
          f"{' '.join(f'{np.percentile(cu_mean, q) / 100:.2f}' for q in (10, 50, 90))}")
    se = (hw >> 13) & 7
    for x in np.unique(xcc)[:2]:
        m = xcc == x
        print(f"     xcc {x}: per-SE mean duration us "
              f"{[round(float(dur[m & (se == e)].mean()) / 100, 1) for e in np.unique(se[m])]}")
    late = st0 > 500                                   # started > 5 us after the first
    if late.any():
        print(f"   late WGs {late.sum()}: on CUs holding {np.bincount(per[inv[late]]).nonzero()[0].tolist()} WGs")
    tl = raw[:, 15].astype(np.int64)
    order = np.argsort(tl)
    print(f"   tile order: start of tile k vs k: corr {np.corrcoef(tl, st0)[0, 1]:.3f}; "
          f"end(last tile) {en0[order[-1]] / 100:.2f} us")
    for db in dbs:
        for b in (db.frames, db.offset, db.length):
            b.free()
    for b in (out.meta, out.lane_off, out.lane_pkt):
        b.free()
ctx.close()
