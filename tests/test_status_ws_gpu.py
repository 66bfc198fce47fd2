"""Round 6: decode statuses do not depend on
what the workspace held before the call.

Round 5's wide decoder counted its workgroups' arrivals on epoch-tagged words
in the workspace (tag << 24 | error << 23 | count), and the corrupted-input
sweep met a stale word that already carried the current call's tag: a buffer's
status was left unwritten. The cause was the tag's source (a call counter that
started at the same constant in every process, so a fresh process's k-th call
repeated an earlier process's k-th tag) plus workspace memory that is never
cleared. The decoder now reads no workspace word as protocol state: the call
clears its statuses to ZR_OK on the stream and the kernels store
ZR_INVALID_INPUT where they find an error (zr_rans_decode_batch_dev,
dec_xn_body).

Every case here pre-fills the workspace with round 5's arrival words built
from the tags a fresh process's first 64 calls would have used (so the next
call's tag is among them), counts 0 .. n-1 and the error bit on and off, or
with all ones / random bytes, over a garbage-filled status array, for the
one-level and two-level arrival shapes of round 5 (narrow 64-lane workgroups
with N <= 512 and 513..1024; 1024-lane workgroups with N <= 8192 and
8193..16384), plus the k_dec_hdr path (more than 64 blocks per buffer), clean
and corrupted. Each status and each decoded buffer must equal the oracle's
(rans.rs:449-651; errors rans.rs:480-482, :563-568, :601-610)."""
import os
import random
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _corrupt(host, enc_len, bt, N, b, rng, kind):
    o, L = bt.enc_off_host[b], enc_len[b]
    if kind == 0:  # a stream length raised: "Invalid stream data length" or a short read
        s = rng.randrange(N)
        ls = o + 8 * N + 4 * s
        v = int.from_bytes(host[ls:ls + 4], "little")
        host[ls:ls + 4] = ((v + 100000) & 0xFFFFFFFF).to_bytes(4, "little")
    elif kind == 1:  # a state out of range
        s = 8 * rng.randrange(N)
        host[o + s:o + s + 8] = (rng.getrandbits(64) | (1 << 63)).to_bytes(8, "little")
    elif kind == 2:  # truncated below the header
        enc_len[b] = rng.randrange(0, 12 * N)
    else:  # truncated inside the streams
        enc_len[b] = max(12 * N, L - rng.randrange(1, 200))


@pytest.mark.parametrize("N,B,per", [
    (300, 40, 40),      # narrow (B N <= 2^16), 5 one-wave workgroups per buffer: one level
    (1000, 30, 30),     # narrow, 16 workgroups per buffer: two levels (sets of 8)
    (4096, 20, 16),     # 1024-lane workgroups, 4 per buffer: one level
    (12000, 6, 12),     # 1024-lane workgroups, 12 per buffer: two levels
    (20000, 4, 6),      # > 64 blocks of 256 streams per buffer: k_dec_hdr + k_scan first
])
@pytest.mark.parametrize("fill", [3, 1, 0])
def test_decode_status_independent_of_workspace(zr, oracle, N, B, per, fill):
    import torch
    from fuzz_rans_corrupt import ws_fill
    from zipora_amd.device import RansDeviceBatch
    rng = random.Random(N * 7 + fill)
    lens = [N * per + rng.randrange(0, N) for _ in range(B)]
    datas = [zr.synth("ut"[b % 2], n, seed=1000 + b) for b, n in enumerate(lens)]
    bt = RansDeviceBatch(lens, N, shared_table=False)
    raw = bt.new_raw()
    for b, d in enumerate(datas):
        o = bt.raw_off_host[b]
        raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    tabs = [oracle.rans_table(oracle.histogram(d)) for d in datas]
    # round 5's arrival shape of this geometry: arrivals per buffer word
    nwg = (N + 63) // 64 if B * N <= 1 << 16 else (N + 1023) // 1024
    n_arr = min(nwg, 8)
    for corrupt in (False, True):
        host = bytearray(enc.cpu().numpy().tobytes())
        enc_len = bt.enc_len.cpu().tolist()
        bad = set()
        if corrupt:
            # the last buffers and a few in between, so that errors come from
            # workgroups other than a buffer's first
            for b in sorted({B - 1, B - 2, B // 2, 1}):
                _corrupt(host, enc_len, bt, N, b, rng, len(bad) % 4)
                bad.add(b)
        e2 = torch.frombuffer(host, dtype=torch.uint8).cuda()
        bt.enc_len.copy_(torch.tensor(enc_len, dtype=torch.int64))
        for rep in range(2):  # the same workspace twice: stale content of a real call too
            if rep == 0:
                ws_fill(bt.ws, rng, fill, n_arrivals=n_arr)
            bt.status.fill_(-3)
            out = bt.new_raw()
            bt.decode(e2, out)
            torch.cuda.synchronize()
            st = bt.statuses()
            for b in range(B):
                o = bt.enc_off_host[b]
                try:
                    ref = oracle.rans_decode(tabs[b], N, bytes(host[o:o + enc_len[b]]), lens[b])
                except oracle.OracleError:
                    ref = None
                if ref is None:
                    assert st[b] == zr._lib.ZR_INVALID_INPUT, f"buffer {b}: status {st[b]}, oracle error"
                else:
                    assert st[b] == 0, f"buffer {b}: status {st[b]}, oracle ok (corrupted {b in bad})"
                    assert bt.raw_of(out, b) == ref, f"buffer {b}"
            if not corrupt:
                assert all(s == 0 for s in st)


@pytest.mark.parametrize("fill", [3, 1, 0])
def test_x1_and_mixed_status_independent_of_workspace(zr, oracle, fill):
    """The x1 decoders over an adversarial workspace: k_dec_x1_fast leaves a
    taken flag per record in the workspace for k_dec_x1_ring, written for every
    record in the same call. A record batch (N = 1: 3000 records of 0-2000 B,
    some corrupted: a raised state, a cut record) and a mixed batch (N = 4096,
    buffers shorter than N take the x1 layout beside xN ones), each decoded
    twice on one workspace: statuses and bytes equal the oracle's
    (rans.rs:510-552 decode_single, :555-651)."""
    import torch
    from fuzz_rans_corrupt import ws_fill
    from zipora_amd.device import RansDeviceBatch
    rng = random.Random(77 + fill)
    for N, lens in ((1, [rng.choice([0, 1, 15, 16, 17, 1024, rng.randrange(0, 2000)]) for _ in range(3000)]),
                    (4096, [4096 * 20 + 3, 100, 0, 4095, 4096 * 33, 1, 5000, 4096 * 7 + 11] * 3)):
        datas = [zr.synth("tu"[b % 2], n, seed=500 + b) if n else b"" for b, n in enumerate(lens)]
        B = len(lens)
        bt = RansDeviceBatch(lens, N, shared_table=True)
        raw = bt.new_raw()
        for b, d in enumerate(datas):
            if d:
                o = bt.raw_off_host[b]
                raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
        enc = bt.new_enc()
        bt.full_encode(raw, enc)
        torch.cuda.synchronize()
        bt.raise_on_error()
        tab = oracle.rans_table(oracle.histogram(b"".join(datas)))
        host = bytearray(enc.cpu().numpy().tobytes())
        enc_len = bt.enc_len.cpu().tolist()
        for b in range(0, B, 7):  # corrupt every 7th non-empty buffer
            o, L = bt.enc_off_host[b], enc_len[b]
            if L < 9:
                continue
            if (b // 7) % 2:
                s = (L - 8) if (N <= 1 or lens[b] < N) else 8 * rng.randrange(N)
                host[o + s + 7] |= 0x80  # a state far out of range
            else:
                enc_len[b] = L - 1 - rng.randrange(min(L - 1, 6))  # cut short
        e2 = torch.frombuffer(host, dtype=torch.uint8).cuda()
        bt.enc_len.copy_(torch.tensor(enc_len, dtype=torch.int64))
        for rep in range(2):
            if rep == 0:
                ws_fill(bt.ws, rng, fill, n_arrivals=8)
            bt.status.fill_(-3)
            out = bt.new_raw()
            bt.decode(e2, out)
            torch.cuda.synchronize()
            st = bt.statuses()
            for b in range(B):
                o = bt.enc_off_host[b]
                try:
                    ref = oracle.rans_decode(tab, N, bytes(host[o:o + enc_len[b]]), lens[b])
                except oracle.OracleError:
                    ref = None
                if ref is None:
                    assert st[b] == zr._lib.ZR_INVALID_INPUT, f"N={N} buffer {b}: status {st[b]}, oracle error"
                else:
                    assert st[b] == 0, f"N={N} buffer {b}: status {st[b]}, oracle ok"
                    assert bt.raw_of(out, b) == ref, f"N={N} buffer {b}"
