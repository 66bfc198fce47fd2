#!/usr/bin/env python3
"""Diagnostic: fraction of 256-stream blocks the fast rANS decoder hands to the
generic re-decode, on the bench workload (64 x 4 MiB, 4096 streams)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import zipora_amd as zr
from zipora_amd.device import RansDeviceBatch
kind = sys.argv[1] if len(sys.argv) > 1 else "u"
B, n, N = 64, 4 << 20, 4096
bt = RansDeviceBatch([n] * B, N, shared_table=True)
raw = torch.frombuffer(bytearray(zr.synth(kind, B * n)), dtype=torch.uint8).cuda()
enc = bt.new_enc(); out = bt.new_raw()
bt.full_encode(raw, enc); bt.decode(enc, out); torch.cuda.synchronize()
r = lambda x: (x + 255) // 256 * 256
nblk = (N + 255) // 256
base = (bt.ws.data_ptr() + 255) // 256 * 256 - bt.ws.data_ptr()
ro = base + r(B * N * 4) * 2 + r(B * nblk * 8) * 2
redo = bt.ws[ro: ro + 4 * B * nblk].cpu().view(torch.int32)
print(f"kind={kind} redo blocks {int(redo.sum())}/{B * nblk}  roundtrip={'ok' if torch.equal(out, raw) else 'MISMATCH'}")
