"""Host cost of the timed region's closing synchronisation: ctx.sync (every pipe's stream),
hipDeviceSynchronize, and the context stream alone after a join; on an idle GPU and right after
a batch (config 2, pipelined)."""
import ctypes as C, json, sys, time
sys.path.insert(0, '.')
import bench
from udpdk_amd import abi, frames as F

ctx = abi.GpuContext(0, max_frames=1 << 20, max_lanes=16)
hip = C.CDLL("libamdhip64.so")
stream = C.c_void_p(abi.lib().udpdk_gpu_stream(ctx.handle))
rx = bench.Rx(ctx, F.config_batch(2), 640 << 20)
ctx.pipeline(3)
for i in range(10):
    rx.step(i)
ctx.sync()
ev = C.c_void_p()
hip.hipEventCreateWithFlags(C.byref(ev), 2)          # hipEventDisableTiming


def event_spin():
    ctx.join()
    hip.hipEventRecord(ev, stream)
    while hip.hipEventQuery(ev) != 0:
        pass


def stream_spin():
    ctx.join()
    while hip.hipStreamQuery(stream) != 0:
        pass


def event_sync():
    ctx.join()
    hip.hipEventRecord(ev, stream)
    hip.hipEventSynchronize(ev)


ways = {"ctx.sync": ctx.sync, "hipDeviceSynchronize": lambda: hip.hipDeviceSynchronize(),
        "join+stream": lambda: (ctx.join(), hip.hipStreamSynchronize(stream)),
        "event_spin": event_spin, "stream_spin": stream_spin, "event_sync": event_sync}
res = {}
for name, f in ways.items():
    idle, busy = [], []
    for rep in range(50):
        t0 = time.perf_counter(); f(); idle.append(time.perf_counter() - t0)
        for i in range(20):
            rx.step(i)
        ctx.join()
        time.sleep(0.002)                      # the batches are done; only the wait's cost remains
        t0 = time.perf_counter(); f(); busy.append(time.perf_counter() - t0)
    idle.sort(); busy.sort()
    res[name] = {"idle_us_median": round(idle[25] * 1e6, 1), "after_batches_us_median": round(busy[25] * 1e6, 1)}
# a 20-step timed region end to end with each closing sync
for name, f in ways.items():
    w = []
    for rep in range(30):
        ctx.sync()
        t0 = time.perf_counter()
        for i in range(20):
            rx.step(i)
        ctx.join()
        f()
        w.append(time.perf_counter() - t0)
    w.sort()
    res[name]["steps20_us_per_step_median"] = round(w[15] / 20 * 1e6, 2)
print(json.dumps(res, indent=1))
