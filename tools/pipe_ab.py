"""Host pipeline (zr_rans_pipe_*) encode / decode rates of the library named by
ZR_LIB_PATH (groups of $GROUP_MIB MiB, default 32), pinned host areas, two shapes: 64 x 4 MiB x4096 (the headline's)
and 1 M x 1 KiB records x1 (configs[4]). Prints one line per shape."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import zipora_amd as zr  # noqa: E402
from zipora_amd.device import RansHostPipe  # noqa: E402


def rates(lens, N, kind, reps=3):
    lens = np.asarray(lens, dtype=np.uint64)
    total = int(lens.sum())
    host = zr.synth(kind, total, seed=7)
    hist = [int(v) for v in np.bincount(np.frombuffer(host, dtype=np.uint8), minlength=256)]
    pipe = RansHostPipe(zr.Rans64Encoder(hist, N).table, N, int(os.environ.get("GROUP_MIB", "32")) << 20)
    raw_off, _, rb, eb = pipe.layout(lens)
    pin = torch.empty(rb, dtype=torch.uint8, pin_memory=True)
    pin.copy_(torch.frombuffer(bytearray(host), dtype=torch.uint8))
    penc = torch.empty(eb, dtype=torch.uint8, pin_memory=True)
    pout = torch.empty(rb, dtype=torch.uint8, pin_memory=True)
    enc_off, enc_len, st, _ = pipe.encode_packed(lens, pin, raw_off, penc)
    pipe.decode(lens, penc, enc_off, enc_len, pout, raw_off)
    te = td = 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        enc_off, enc_len, st, _ = pipe.encode_packed(lens, pin, raw_off, penc)
        t1 = time.perf_counter()
        st2 = pipe.decode(lens, penc, enc_off, enc_len, pout, raw_off)
        td += time.perf_counter() - t1
        te += t1 - t0
    ok = not (st != 0).any() and not (st2 != 0).any() and torch.equal(pout, pin)
    pipe.close()
    g = total * reps / 2**30
    return ok, g / te, g / td, g / (te + td)


for name, lens, N, kind in [("rans 64x4MiB x4096", [4 << 20] * 64, 4096, "u"),
                            ("blob 1Mx1KiB x1", [1024] * (1 << 20), 1, "z")]:
    ok, e, d, rt = rates(lens, N, kind)
    print(f"{name}: ok={ok} encode {e:.2f} GiB/s decode {d:.2f} GiB/s encode+decode {rt:.2f} GiB/s", flush=True)
