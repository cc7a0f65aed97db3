"""Device-to-device copy rate on this box (diagnostic): what a plain read+write stream of the
in-place reassembly's size achieves, as the ceiling for reasm_emit_inplace's moved bytes."""
import torch

for mb in (128, 256, 386, 512, 768, 1024, 1500):
    n = mb << 20
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    y = torch.empty_like(x)
    x.random_(0, 255)
    for _ in range(3):
        y.copy_(x)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        y.copy_(x)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1000 / 20
    print(f"copy {mb} MiB: {us:.1f} us per copy, {2 * n / us / 1e6:.2f} TB/s read+write")
