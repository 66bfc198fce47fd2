#!/usr/bin/env python3
"""Per-workgroup timeline of the fast rANS decode (diagnostic build ZR_DEC_ABL=8).
Records (start/end s_memrealtime at 100 MHz, s_memtime cycles, HW_ID, XCC_ID) are
written by each workgroup into the workspace scratch area."""
import os, sys, collections
os.environ["ZR_DEC_ABL"] = "8"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import zipora_amd as zr
from zipora_amd.device import RansDeviceBatch

B, n, N = 64, 4 << 20, 4096
bt = RansDeviceBatch([n] * B, N, shared_table=True)
raw = torch.frombuffer(bytearray(zr.synth("u", B * n)), dtype=torch.uint8).cuda()
enc = bt.new_enc(); out = bt.new_raw()
bt.full_encode(raw, enc)
mode = sys.argv[1] if len(sys.argv) > 1 else "warm"
for _ in range(3):
    if mode == "bench":  # as in bench.py: the decode follows a full encode
        bt.full_encode(raw, enc)
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(); bt.decode(enc, out); e1.record()
    torch.cuda.synchronize()
    print(f"{mode}: decode call (hdr+scan+fast+redo) {e0.elapsed_time(e1)*1e3:.1f} us")
assert torch.equal(out, raw)
r = lambda x: (x + 255) // 256 * 256
nblk = (N + 255) // 256
off = r(B * N * 4) * 2 + r(B * nblk * 8) * 2 + r(B * nblk * 4)
base = (bt.ws.data_ptr() + 255) // 256 * 256 - bt.ws.data_ptr()
nwg = B * ((N + 1023) // 1024)
rec = bt.ws[base + off: base + off + nwg * 32].cpu().view(torch.int64).view(nwg, 4).tolist()
t0 = min(x[0] for x in rec)
starts = sorted((x[0] - t0) / 100.0 for x in rec)   # microseconds
ends = sorted((x[1] - t0) / 100.0 for x in rec)
cyc = [x[2] for x in rec]
dur = [(x[1] - x[0]) / 100.0 for x in rec]
cu = collections.Counter((x[3] >> 32, (x[3] >> 8) & 0xF, (x[3] >> 13) & 0x3, (x[3] >> 12) & 1) for x in rec)
print(f"wgs={nwg} distinct (xcc,cu,se,sh)={len(cu)} max wgs on one CU={max(cu.values())}")
print(f"start us: min {starts[0]:.1f} p50 {starts[len(starts)//2]:.1f} max {starts[-1]:.1f}")
print(f"end   us: min {ends[0]:.1f} p50 {ends[len(ends)//2]:.1f} max {ends[-1]:.1f}")
print(f"dur   us: min {min(dur):.1f} avg {sum(dur)/len(dur):.1f} max {max(dur):.1f}")
print(f"cycles: min {min(cyc)} avg {sum(cyc)/len(cyc):.0f} max {max(cyc)}  -> clock {sum(cyc)/len(cyc)/ (sum(dur)/len(dur)) / 1e3:.2f} GHz")
