"""Device-to-device copy rate (the practical ceiling of a read+write pass)."""
import time

import torch

dev = torch.device("cuda:0")
for mib in (64, 272, 1024):
    n = mib << 20
    a = torch.empty(n, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        b.copy_(a)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    print(f"{mib} MiB copy: {ms * 1e3:.1f} us, {2 * n / ms / 1e9:.0f} GB/s (read+write)", flush=True)
