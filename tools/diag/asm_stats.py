"""Instruction mix per loop depth of a kernel in build/asm/rx_kernels.s (make asm), using the
compiler's own "Loop: Header=... Depth=N" block annotations."""
import collections
import re
import sys

kern = sys.argv[1] if len(sys.argv) > 1 else "_ZN5udpdk11rx_classifyILb1EEEvNS_6RxArgsE"
s = open("build/asm/rx_kernels.s").read()
start = s.index(kern + ":")
end = s.index(".Lfunc_end", start)
depth, header = 0, None
stats = collections.defaultdict(collections.Counter)
for l in s[start:end].split("\n"):
    m = re.search(r"(Loop|Inner Loop Header|Loop Header): .*?Depth=(\d+)", l)
    if re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", l):
        m2 = re.search(r"Header=(BB\d+_\d+) Depth=(\d+)", l) or re.search(r"Loop Header: Depth=(\d+)", l)
        if "Depth=" in l:
            d = int(re.search(r"Depth=(\d+)", l).group(1))
            h = re.search(r"Header=(BB\d+_\d+)", l)
            depth, header = d, (h.group(1) if h else l.split(":")[0].lstrip("."))
        else:
            depth, header = 0, None
        continue
    t = l.strip()
    if not l.startswith("\t") or not t or t.startswith((".", ";")):
        continue
    op = t.split()[0]
    k = ("branch" if op.startswith(("s_cbranch", "s_branch")) else "wait" if op.startswith("s_waitcnt")
         else "valu" if op.startswith("v_") else "salu" if op.startswith("s_")
         else "vmem" if op.startswith(("global_", "buffer_")) else "lds" if op.startswith("ds_") else "other")
    stats[(depth, header)][k] += 1
for key in sorted(stats, key=lambda x: (x[0], str(x[1]))):
    c = stats[key]
    print(f"depth {key[0]} header {key[1]}: total {sum(c.values())} {dict(c)}")
