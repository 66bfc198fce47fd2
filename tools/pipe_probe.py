"""Host pipeline rate vs group size (64 x 4 MiB, x4096, uniform bytes)."""
import sys
import time

import torch

sys.path.insert(0, ".")
import zipora_amd as zr  # noqa: E402
from zipora_amd.device import RansHostPipe  # noqa: E402

B, n, N = 64, 4 << 20, 4096
host = zr.synth("u", B * n)
lens = [n] * B
hist = zr.histogram(host)
tab = zr.Rans64Encoder(hist, N).table
import os
ALIGN = int(os.environ.get("ALIGN", "16"))
for gmib in [int(x) for x in (sys.argv[1:] or ["4", "8", "16", "32", "64"])]:
    pipe = RansHostPipe(tab, N, gmib << 20)
    raw_off, enc_off, rb, eb = pipe.layout(lens, ALIGN)
    pin = torch.empty(rb, dtype=torch.uint8, pin_memory=True)
    pin.copy_(torch.frombuffer(bytearray(host), dtype=torch.uint8))
    penc = torch.empty(eb, dtype=torch.uint8, pin_memory=True)
    pout = torch.empty(rb, dtype=torch.uint8, pin_memory=True)
    el, st = pipe.encode(lens, pin, raw_off, penc, enc_off)
    pipe.decode(lens, penc, enc_off, el, pout, raw_off)
    te = td = 0
    for _ in range(3):
        t0 = time.perf_counter()
        el, st = pipe.encode(lens, pin, raw_off, penc, enc_off)
        t1 = time.perf_counter()
        pipe.decode(lens, penc, enc_off, el, pout, raw_off)
        t2 = time.perf_counter()
        te += t1 - t0
        td += t2 - t1
    assert torch.equal(pin, pout)
    print(f"align {ALIGN} group {gmib} MiB: encode {B * n * 3 / te / 2**30:.1f} GiB/s ({te / 3 * 1e3:.2f} ms), "
          f"decode {B * n * 3 / td / 2**30:.1f} GiB/s ({td / 3 * 1e3:.2f} ms)", flush=True)
    pipe.close()
