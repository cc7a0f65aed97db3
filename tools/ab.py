"""Same-box A/B of library builds (replaces the round-2 tools/ab/*.sh + one-off line scripts).

Variants are built on the CPU side first: `make variant VAR=t4096 VFLAGS="-DUDPDK_RX_HIST_CAP=(1u<<22)"`
→ tools/var/t4096.so. The name `base` is the in-tree udpdk_amd/libudpdk_amd.so. On the GPU box:

  python tools/ab.py --libs base,t4096 --bench "--config 5" --reps 2
  python tools/ab.py --libs base,new --line rss --reps 2 --tests tests/test_gpu_rss.py

--bench runs bench.py (default extra args: --steps 200 --warmup 20 --no-cpu-baseline --no-extra)
and prints value / pipelined step / depth-1 step / kernel times per variant and repetition.
--line runs one of bench.py's side lines in a child process per variant (LINES below).
--tests first runs those GPU tests once against every non-base variant (parity before timing).
Every child runs under its own timeout; the first failure ends the script (no retries).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

LINES = {
    "tx": "for plen in (22, 1458): out(bench.tx_line(ctx, plen, 1 << 20, 50))",
    "txfrag": "out(bench.tx_line(ctx, 2952, 1 << 18, 50, mtu=1500))",
    "txsize": "for n in (1 << 17, 1 << 18, 1 << 19, 1 << 20): out(bench.tx_line(ctx, 1458, n, 50))",
    "rss": "for cfg in (2, 5): out(bench.rss_line(ctx, cfg, 8, 50))",
    "reasm": "out(bench.reasm_line(ctx, 1 << 18, 2952, 10))",
    "reasmip": "out(bench.reasm_inplace_line(ctx, 1 << 18, 2952, 10))",
    "reasmx": "import reasm_probe_x\nreasm_probe_x.run(ctx, out)",
    "gather": "for cfg in (2, 3): out(bench.gather_line(ctx, cfg, 50))\n"
              "out(bench.gather_line(ctx, 2, 50, slot=0))",
    "sporadic": "out(bench.sporadic_line(ctx, 180, 640 << 20))",
    "cfg": "import os\nfor c in os.environ.get('CFGS', '4 5').split(): out(bench.side_config(ctx, int(c), 50, 640 << 20))",
}


def split_env(name: str):
    """'base@UDPDK_RX_SPAN=0' -> ('base', {'UDPDK_RX_SPAN': '0'}): a library variant run with extra
    environment (the library reads its form switches at context creation)."""
    lib, *kv = name.split("@")
    return lib, dict(x.split("=", 1) for x in kv)


def lib_path(name: str) -> str:
    name = split_env(name)[0]
    if name == "base":
        return os.path.join(ROOT, "udpdk_amd", "libudpdk_amd.so")
    return os.path.join(ROOT, "tools", "var", name + ".so")


def run(cmd, env, timeout, log):
    with open(log, "w") as f:
        r = subprocess.run(["timeout", "-k", "10", str(timeout)] + cmd, env=env, cwd=ROOT,
                           stdout=f, stderr=subprocess.STDOUT)
    if r.returncode:
        sys.stdout.write(open(log).read()[-3000:])
        raise SystemExit(f"{' '.join(cmd[:3])} failed rc={r.returncode} (log {log})")
    return [json.loads(l) for l in open(log) if l.startswith("{")]


def child_line(name: str):
    sys.path.insert(0, ROOT)
    import bench
    from udpdk_amd import abi
    ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)

    def out(d):
        print(json.dumps(d), flush=True)
    exec(LINES[name], {"bench": bench, "ctx": ctx, "out": out})


def summary(d: dict) -> str:
    if "value" in d:
        return (f"value {d['value']:.0f}  step {d.get('gpu_us_per_step')}  d1 {d['depth1']['gpu_us_per_step']}  "
                f"k {d.get('kernel_us')}")
    keys = [k for k in ("us_per_launch", "us_per_call", "gpu_us_per_step", "kernel_us", "frac_hbm",
                        "frac_hbm_pipeline", "mpkt_s", "clean_us_per_call", "sporadic_us_per_call",
                        "sporadic_over_clean", "depth1_clean_us", "depth1_stray_call_us") if k in d]
    return f"{d.get('workload', '')[:40]:40s} " + "  ".join(f"{k} {d[k]}" for k in keys)


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--_line":
        return child_line(sys.argv[2])
    p = argparse.ArgumentParser()
    p.add_argument("--libs", required=True)
    p.add_argument("--bench", default=None, help="extra bench.py arguments")
    p.add_argument("--line", default=None, choices=sorted(LINES))
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--tests", default=None)
    p.add_argument("--timeout", type=int, default=200)
    a = p.parse_args()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    libs = a.libs.split(",")
    for n in libs:
        if not os.path.exists(lib_path(n)):
            raise SystemExit(f"missing {lib_path(n)}")
    if a.tests:
        for n in libs:
            if split_env(n)[0] == "base":
                continue
            env = dict(os.environ, UDPDK_LIB_OVERRIDE=lib_path(n), TMPDIR="/tmp", **split_env(n)[1])
            log = os.path.join(ROOT, "gpurun_out", f"ab_test_{n}.log")
            run([sys.executable, "-u", "-m", "pytest", *a.tests.split(), "-m", "gpu", "-x", "-q",
                 "--timeout", "120", "--timeout-method", "thread"], env, 600, log)
            print(f"tests {n}: {open(log).read().strip().splitlines()[-1]}", flush=True)
    for rep in range(a.reps):
        for n in libs:
            env = dict(os.environ, UDPDK_LIB_OVERRIDE=lib_path(n), **split_env(n)[1])
            log = os.path.join(ROOT, "gpurun_out", f"ab_{n.replace('@', '_').replace('=', '')}_r{rep}.log")
            if a.line:
                res = run([sys.executable, os.path.abspath(__file__), "--_line", a.line], env, a.timeout, log)
            else:
                extra = (a.bench or "").split()
                dflt = ["--steps", "200", "--warmup", "20", "--no-cpu-baseline", "--no-extra", "--no-strong"]
                res = run([sys.executable, "bench.py", *dflt, *extra], env, a.timeout, log)
            for d in res:
                print(f"r{rep} {n:10s} {summary(d)}", flush=True)


if __name__ == "__main__":
    main()
