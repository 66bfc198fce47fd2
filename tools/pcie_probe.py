"""PCIe copy rates on the box: pinned H2D, D2H, both at once (the host pipeline's ceiling)."""
import time

import torch

n = 256 << 20
dev = torch.device("cuda:0")
h1 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
d1 = torch.empty(n, dtype=torch.uint8, device=dev)
d2 = torch.empty(n, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def h2d():
    with torch.cuda.stream(s1):
        d1.copy_(h1, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h2.copy_(d2, non_blocking=True)


def both():
    h2d()
    d2h()


def chunks(sz):
    def f():
        for i in range(0, n, sz):
            with torch.cuda.stream(s1):
                d1[i:i + sz].copy_(h1[i:i + sz], non_blocking=True)
            with torch.cuda.stream(s2):
                h2[i:i + sz].copy_(d2[i:i + sz], non_blocking=True)
    return f


for name, fn in [("h2d", h2d), ("d2h", d2h), ("both", both), ("both_8M", chunks(8 << 20)),
                 ("both_32M", chunks(32 << 20))]:
    dt = t(fn)
    print(f"{name}: {n / dt / 1e9:.1f} GB/s per direction ({dt * 1e3:.2f} ms)", flush=True)


def dep(sz, host_sync, d2h_first=False):
    def f():
        evs = []
        outs = []
        for k, i in enumerate(range(0, n, sz)):
            if host_sync and k >= 2:
                outs[k - 2].synchronize()
            with torch.cuda.stream(s1):
                d1[i:i + sz].copy_(h1[i:i + sz], non_blocking=True)
                e = torch.cuda.Event()
                e.record(s1)
            s2.wait_event(e)
            with torch.cuda.stream(s2):
                h2[i:i + sz].copy_(d2[i:i + sz], non_blocking=True)
                o = torch.cuda.Event()
                o.record(s2)
            outs.append(o)
    return f


for name, fn in [("dep_32M", dep(32 << 20, False)), ("dep_sync_32M", dep(32 << 20, True)),
                 ("dep_sync_16M", dep(16 << 20, True)), ("dep_sync_64M", dep(64 << 20, True))]:
    dt = t(fn)
    print(f"{name}: {n / dt / 1e9:.1f} GB/s per direction ({dt * 1e3:.2f} ms)", flush=True)
