#!/usr/bin/env python3
"""Decode statuses of clean batches over a garbage-filled status array (every
buffer's status must be written by the decode): geometries from the
corrupted-input sweep. Usage: python3 tools/repro_status.py"""
import os, random, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch
import zipora_amd as zr
from zipora_amd.device import RansDeviceBatch
from fuzz_rans import data_of

rng = random.Random(5)
for N, B, lo, hi in [(2, 32785, 2, 40), (2, 32785, 2, 4), (2, 20000, 2, 40), (7, 9400, 7, 140),
                     (64, 1030, 64, 1280), (2, 33000, 0, 40), (1, 2000, 0, 3000)]:
    lens = [rng.randrange(lo, hi) for _ in range(B)]
    datas = [data_of("u", n, rng, zr) for n in lens]
    bt = RansDeviceBatch(lens, N, shared_table=False)
    raw = bt.new_raw()
    host = bytearray(bt.raw_bytes)
    for b, d in enumerate(datas):
        o = bt.raw_off_host[b]
        host[o:o + len(d)] = d
    raw.copy_(torch.frombuffer(bytes(host) if host else b"\0", dtype=torch.uint8).to(raw.device)[:raw.numel()])
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    est = bt.statuses()
    bt.status.fill_(-3)
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    st = bt.statuses()
    unwritten = [b for b in range(B) if st[b] == -3]
    badenc = [b for b in range(B) if est[b] != 0]
    outh = out.cpu().numpy().tobytes()
    wrong = [b for b in range(B) if st[b] == 0 and outh[bt.raw_off_host[b]:bt.raw_off_host[b] + lens[b]] != datas[b]]
    print(f"N={N} B={B} lens {lo}..{hi}: enc errors {len(badenc)}, unwritten decode statuses {len(unwritten)} "
          f"{unwritten[:5]} lens {[lens[b] for b in unwritten[:5]]}, wrong bytes {len(wrong)}", flush=True)
