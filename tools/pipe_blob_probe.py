"""Host pipeline on the record batch (1 M x 1 KiB, x1): packed encode + decode, timed per call."""
import sys
import time

import torch

sys.path.insert(0, ".")
import zipora_amd as zr  # noqa: E402
from zipora_amd.device import RansHostPipe  # noqa: E402

R = 1 << 20
host = zr.synth("t", R * 1024, seed=3)
lens = [1024] * R
tab = zr.Rans64Encoder(zr.histogram(host[: 1 << 24]), 1).table
for gmib in [int(x) for x in (sys.argv[1:] or ["32"])]:
    pipe = RansHostPipe(tab, 1, gmib << 20)
    t0 = time.perf_counter()
    raw_off, _, rb, eb = pipe.layout(lens)
    t1 = time.perf_counter()
    pin = torch.empty(rb, dtype=torch.uint8, pin_memory=True)
    pin.copy_(torch.frombuffer(bytearray(host), dtype=torch.uint8))
    penc = torch.empty(eb, dtype=torch.uint8, pin_memory=True)
    pout = torch.empty(rb, dtype=torch.uint8, pin_memory=True)
    eo, el, st, tot = pipe.encode_packed(lens, pin, raw_off, penc)
    pipe.decode(lens, penc, eo, el, pout, raw_off)
    for _ in range(2):
        a = time.perf_counter()
        eo, el, st, tot = pipe.encode_packed(lens, pin, raw_off, penc)
        b = time.perf_counter()
        pipe.decode(lens, penc, eo, el, pout, raw_off)
        c = time.perf_counter()
        print(f"group {gmib} MiB: layout {t1 - t0:.2f} s, encode {(b - a) * 1e3:.1f} ms "
              f"({R * 1024 / (b - a) / 2**30:.1f} GiB/s, {tot / 2**20:.0f} MiB out), decode {(c - b) * 1e3:.1f} ms "
              f"({R * 1024 / (c - b) / 2**30:.1f} GiB/s)", flush=True)
    assert torch.equal(pin, pout)
    pipe.close()
