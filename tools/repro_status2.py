#!/usr/bin/env python3
"""The any-slow (generic) path's status in the xN decoders: one buffer's state
set outside [2^16, 2^24), decode over a garbage-filled status array."""
import os, random, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import zipora_amd as zr
from zipora_amd.device import RansDeviceBatch

rng = random.Random(1)
for N, B, n, xs in [(2, 32785, 10, [0xBE000000006202BF, 5, 1 << 30]), (2, 30000, 10, [0xBE000000006202BF]),
                    (1024, 70, 4096, [0xBE000000006202BF, 5]), (4096, 20, 1 << 16, [1 << 40])]:
    for X in xs:
        lens = [n] * B
        bt = RansDeviceBatch(lens, N, shared_table=False)
        raw = bt.new_raw()
        raw.copy_(torch.randint(0, 256, (raw.numel(),), dtype=torch.uint8, device=raw.device))
        enc = bt.new_enc()
        bt.full_encode(raw, enc)
        torch.cuda.synchronize()
        tgt = B // 2 + 3
        o = bt.enc_off_host[tgt]
        s = 1 if N > 1 else 0
        host = enc.cpu()
        host[o + 8 * s:o + 8 * s + 8] = torch.tensor(list(X.to_bytes(8, "little")), dtype=torch.uint8)
        enc.copy_(host.to(enc.device))
        bt.status.fill_(-3)
        out = bt.new_raw()
        bt.decode(enc, out)
        torch.cuda.synchronize()
        st = bt.statuses()
        uw = [b for b in range(B) if st[b] == -3]
        print(f"N={N} B={B} X={X:#x}: target status {st[tgt]}, unwritten {len(uw)} {uw[:4]}", flush=True)
