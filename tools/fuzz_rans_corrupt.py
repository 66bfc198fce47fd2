#!/usr/bin/env python3
"""Randomised corrupted-input sweep of the rANS device decoders against the CPU
oracle (test infrastructure, run on the GPU box). Each case encodes a random
batch (tools/fuzz_rans.py geometries, narrow / wide / record batches), then
corrupts about half of its buffers (a state set to a random 64-bit value, a
stream length moved or raised, random bytes overwritten anywhere in the
buffer, enc_len cut short or raised) and decodes on the device over a
garbage-filled status array and a workspace filled with one of four patterns
(random bytes, all ones, zeros, or round 5's epoch-tagged arrival words: tag
<< 24 | error << 23 | count with the tags round 5's call counter gave a fresh
process and counts below the arrivals a buffer needs; ws_fill). Every buffer
must match the oracle (rans.rs:449-651 restated) error for error and byte for
byte.
Usage: python3 tools/fuzz_rans_corrupt.py [seconds] [seed]
"""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def ws_fill(ws, rng, kind, n_arrivals=8):
    """Fills a workspace tensor (uint8, device) with pattern `kind`: 0 random
    bytes, 1 0xFF, 2 zeros, 3 round 5's arrival words (the decoder no longer
    reads any of it; the patterns check that no status depends on it)."""
    import numpy as np
    import torch
    n = ws.numel()
    if kind == 0:
        h = np.random.default_rng(rng.randrange(1 << 30)).integers(0, 256, n, dtype=np.uint8)
    elif kind == 1:
        h = np.full(n, 0xFF, dtype=np.uint8)
    elif kind == 2:
        h = np.zeros(n, dtype=np.uint8)
    else:
        nw = n // 8
        k = np.arange(nw, dtype=np.uint64)
        # the tags of a fresh process's first 64 calls under round 5's counter
        tag = (np.uint64(0x9E3779B97F4A7C15) + np.uint64(1) + (k % np.uint64(64))) & np.uint64((1 << 40) - 1)
        cnt = k % np.uint64(max(1, n_arrivals))
        err = (k // np.uint64(3)) & np.uint64(1)
        words = (tag << np.uint64(24)) | (err << np.uint64(23)) | cnt
        h = np.zeros(n, dtype=np.uint8)
        h[:nw * 8] = words.view(np.uint8)
    ws.copy_(torch.from_numpy(h).to(ws.device))


def run(secs=None, max_cases=None, seed=12345, log=print):
    import torch
    import oracle_ffi as orc
    import zipora_amd as zr
    from zipora_amd.device import RansDeviceBatch
    from fuzz_rans import data_of

    rng = random.Random(seed)
    t_end = time.time() + secs if secs else None
    cases = bad_bufs = 0
    while (t_end is None or time.time() < t_end) and (max_cases is None or cases < max_cases):
        if rng.random() < 0.3:
            N, B = 1, rng.randrange(20, 2000)
            lens = [rng.randrange(0, 3000) for _ in range(B)]
        else:
            N = rng.choice([2, 7, 64, 256, 1000, 1024, 4096])
            B = rng.choice([1, 3]) if rng.random() < 0.3 else max(1, (1 << 16) // N + rng.randrange(1, 20))
            B = min(B, max(1, (8 << 20) // (20 * N)))
            lens = [rng.randrange(N, N * rng.choice([2, 8, 20])) if rng.random() < 0.9 else rng.randrange(0, N)
                    for _ in range(B)]
        kinds = [rng.choice(["u", "z", "t", "two"]) for _ in range(B)]
        datas = [data_of(k, n, rng, zr) for k, n in zip(kinds, lens)]
        bt = RansDeviceBatch(lens, N, shared_table=False)
        raw = bt.new_raw()
        for b, d in enumerate(datas):
            if d:
                o = bt.raw_off_host[b]
                raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).to(raw.device)
        enc = bt.new_enc()
        bt.full_encode(raw, enc)
        torch.cuda.synchronize()
        bt.raise_on_error()
        tabs = [orc.rans_table(orc.histogram(d)) for d in datas]
        host = bytearray(enc.cpu().numpy().tobytes())
        orig = bytes(host)
        enc_len = bt.enc_len.cpu().tolist()
        enc_len0 = list(enc_len)
        what = [""] * B
        for b in range(B):
            if rng.random() < 0.5:
                continue
            o, L = bt.enc_off_host[b], enc_len[b]
            cap = (bt.enc_off_host[b + 1] if b + 1 < B else bt.enc_bytes) - o  # the buffer's area
            single = N <= 1 or lens[b] < N
            kind = rng.randrange(5)
            what[b] = f"kind {kind} (L={L}, cap={cap}, single={single})"
            if kind == 0 and L >= 8:  # a state: any 64-bit value
                s = (L - 8) if single else 8 * rng.randrange(N)
                host[o + s:o + s + 8] = rng.getrandbits(64).to_bytes(8, "little")
            elif kind == 1 and not single:  # a stream length moved to the next or raised
                s = rng.randrange(N)
                ls = o + 8 * N + 4 * s
                v = int.from_bytes(host[ls:ls + 4], "little")
                d = rng.choice([1, 9, 100, 100000, 1 << 31])
                host[ls:ls + 4] = ((v + d) & 0xFFFFFFFF).to_bytes(4, "little")
                if rng.random() < 0.5 and s + 1 < N:
                    ls1 = ls + 4
                    v1 = int.from_bytes(host[ls1:ls1 + 4], "little")
                    host[ls1:ls1 + 4] = ((v1 - d) & 0xFFFFFFFF).to_bytes(4, "little")
            elif kind == 2 and L > 0:  # random bytes anywhere in the encoded buffer
                for _ in range(rng.randrange(1, 6)):
                    host[o + rng.randrange(L)] = rng.randrange(256)
            elif kind == 3 and L > 0:  # cut short
                enc_len[b] = rng.randrange(0, L)
            else:  # enc_len raised within the buffer's area (trailing zeros)
                enc_len[b] = min(cap, L + rng.randrange(1, 64))
            bad_bufs += 1
        enc.copy_(torch.frombuffer(host, dtype=torch.uint8).to(enc.device))
        bt.enc_len.copy_(torch.tensor(enc_len, dtype=torch.int64))
        bt.status.fill_(-3)
        fill = rng.randrange(4)
        ws_fill(bt.ws, rng, fill)
        out = bt.new_raw()
        bt.decode(enc, out)
        torch.cuda.synchronize()
        st = bt.statuses()
        for b in range(B):
            o = bt.enc_off_host[b]
            try:
                ref = orc.rans_decode(tabs[b], N, bytes(host[o:o + enc_len[b]]), lens[b])
            except orc.OracleError:
                ref = None
            ok = (st[b] != 0) if ref is None else (st[b] == 0 and bt.raw_of(out, b) == ref)
            if not ok:
                dump = os.path.join(ROOT, "gpurun_out", f"corrupt_case_{seed}_{cases}_{b}.json")
                import json
                os.makedirs(os.path.dirname(dump), exist_ok=True)
                json.dump({"N": N, "len": lens[b], "enc_len": enc_len[b], "enc_len0": enc_len0[b],
                           "orig": orig[o:o + max(enc_len0[b], enc_len[b])].hex(),
                           "corrupted": bytes(host[o:o + max(enc_len0[b], enc_len[b])]).hex(),
                           "data": datas[b].hex(), "status": st[b],
                           "decoded": bt.raw_of(out, b).hex(), "ws_fill": fill},
                          open(dump, "w"))
                raise AssertionError(f"MISMATCH case {cases} seed {seed}: N={N} B={B} buffer {b} "
                                     f"len={lens[b]} status={st[b]} oracle={'err' if ref is None else 'ok'} "
                                     f"corruption: {what[b] or 'none'}; enc_len {enc_len[b]}; workspace fill {fill}; "
                                     f"neighbours {what[max(0, b - 2):b + 3]}")
        cases += 1
        log(f"case {cases}: N={N} B={B} corrupted so far {bad_bufs} ok")
    return cases, bad_bufs


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 12345
    cases, bad = run(secs=secs, seed=seed, log=lambda m: print(m, flush=True))
    print(f"fuzz ok: {cases} cases, {bad} corrupted buffers, seed {seed}")


if __name__ == "__main__":
    main()
