#!/usr/bin/env python3
"""Diagnostic: run the rANS host-API parity cases through the device batch with a
chosen decoder build (env ZR_DEC / ZR_DEC_ABL) and report statuses / mismatches."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
import zipora_amd as zr
import oracle_ffi as O
from zipora_amd.device import RansDeviceBatch

u = O.gen_uniform(200000)
cases = [b"hello world, this is a test of enhanced 64-bit rANS encoding",
         bytes(((i * 123 + 45) % 256) for i in range(10000)), u[:4097], u[:100000]]
for data in cases:
    for N in [2, 3, 64, 257, 1000, 4096]:
        if N > len(data):
            continue
        bt = RansDeviceBatch([len(data)], N)
        raw = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        enc = bt.new_enc()
        bt.full_encode(raw, enc)
        out = bt.new_raw()
        bt.decode(enc, out)
        torch.cuda.synchronize()
        st = bt.statuses()
        r = lambda x: (x + 255) // 256 * 256
        nblk = (N + 255) // 256
        base = (bt.ws.data_ptr() + 255) // 256 * 256 - bt.ws.data_ptr()
        ro = base + r(N * 4) * 2 + r(nblk * 8) * 2
        redo = int(bt.ws[ro: ro + 4 * nblk].cpu().view(torch.int32).sum().item())
        ok = bt.raw_of(out, 0) == data
        print(f"n={len(data)} N={N} status={st} redo_blocks={redo}/{nblk} roundtrip={'ok' if ok else 'MISMATCH'}", flush=True)
