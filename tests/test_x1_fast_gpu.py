"""x1 record batches through k_dec_x1_fast (1024 records per workgroup, the
xN decoder's step with per-record output runs) and its hand-off to
k_dec_x1_ring (records the fast kernel does not take): bit-exact against the
oracle's decode_single (rans.rs:523-545).

Cases: whole groups only (every record of a wave live), records that end inside
a group (the per-lane store path), records whose reads outrun the ring (generic
re-decode), corrupted and truncated records (status and bytes equal to the
oracle's Ok/Err), unaligned outputs (the ring kernel's records) mixed in."""
import random

import pytest

pytestmark = pytest.mark.gpu


def _batch(zr, lens, datas, N=1, align=16):
    import torch
    from zipora_amd.device import RansDeviceBatch
    bt = RansDeviceBatch(lens, N, shared_table=True, align=align)
    raw = bt.new_raw()
    for b, d in enumerate(datas):
        if d:
            o = bt.raw_off_host[b]
            raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    return bt, enc


def _check(zr, oracle, lens, datas, N=1, align=16):
    import torch
    bt, enc = _batch(zr, lens, datas, N, align)
    t = oracle.rans_table(oracle.histogram(b"".join(datas)))
    for b, d in enumerate(datas):
        assert bt.encoded(enc, b) == oracle.rans_encode(t, N, d), f"encode, record {b}"
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    for b, d in enumerate(datas):
        assert bt.raw_of(out, b) == d, f"decode, record {b} (len {len(d)})"
    return bt, enc, t


@pytest.mark.parametrize("kind", ["u", "t"])
def test_x1_whole_groups_many_workgroups(zr, oracle, kind):
    # 3000 records of 1 KiB: three workgroups, every group regular
    lens = [1024] * 3000
    datas = [zr.synth(kind, n, seed=7 + b) for b, n in enumerate(lens)]
    _check(zr, oracle, lens, datas)


@pytest.mark.parametrize("N", [1, 4096])
def test_x1_ragged_records(zr, oracle, N):
    # lengths around every tile (16 and, since round 4, 32 steps), group (64),
    # line and output group (128) boundary, random ones, empty records; with
    # N = 4096 the records >= 4096 take the xN layout
    rnd = random.Random(11 + N)
    edge = [0, 1, 2, 7, 8, 15, 16, 17, 31, 32, 33, 63, 64, 65, 95, 96, 97, 127, 128, 129, 159, 160, 161,
            191, 192, 193, 255, 256, 257, 1000, 1023, 1024, 1025, 4095, 4096, 5000, 20000]
    lens = edge * 8 + [rnd.randrange(0, 3000) for _ in range(1800)]
    rnd.shuffle(lens)
    datas = [zr.synth("t", n, seed=100 + b) for b, n in enumerate(lens)]
    _check(zr, oracle, lens, datas, N)


def test_x1_aligned_and_unaligned_outputs(zr, oracle):
    # align=1: most records' outputs are not 16-B aligned (k_dec_x1_ring), the rest are
    # (k_dec_x1_fast); both kernels in one call
    rnd = random.Random(5)
    lens = [rnd.choice([1024, 1000, 16, 17, 333, 2048]) for _ in range(1500)]
    datas = [zr.synth("z", n, seed=b) for b, n in enumerate(lens)]
    _check(zr, oracle, lens, datas, align=1)


def test_x1_ring_outrun_falls_back(zr, oracle):
    # a shared table trained almost only on 'a': records of rare bytes cost ~12 bits
    # per symbol, more than the ring sustains, so those lanes decode again
    # with x1_dec_generic; their neighbours stay on the fast path
    rnd = random.Random(3)
    lens, datas = [], []
    for b in range(2048):
        if b % 97 == 5:
            d = bytes(rnd.randrange(256) for _ in range(1500))
        else:
            d = b"a" * 1400 + bytes(rnd.randrange(256) for _ in range(2))
        lens.append(len(d))
        datas.append(d)
    _check(zr, oracle, lens, datas)


def test_x1_corrupted_records_match_oracle(zr, oracle):
    """Flipped bits, damaged states and truncated records: each record's status
    (Ok / "Insufficient data" / "too short") and, when Ok, its bytes equal the
    oracle's decode of the same corrupted bytes."""
    import torch
    rnd = random.Random(9)
    lens = [1024] * 1100 + [rnd.randrange(1, 2000) for _ in range(900)]
    datas = [zr.synth("t", n, seed=300 + b) for b, n in enumerate(lens)]
    bt, enc = _batch(zr, lens, datas)
    t = oracle.rans_table(oracle.histogram(b"".join(datas)))
    enc_len = bt.enc_len.cpu().tolist()
    host = bytearray(enc.cpu().numpy().tobytes())
    recs = []
    for b in range(len(lens)):
        o, L = bt.enc_off_host[b], enc_len[b]
        r = bytearray(host[o:o + L])
        kind = b % 5
        if kind == 1 and L > 8:  # a flipped bit in the stream
            i = rnd.randrange(L - 8)
            r[i] ^= 1 << rnd.randrange(8)
        elif kind == 2 and L > 12:  # truncated stream, the state moved down
            cut = rnd.randrange(1, min(L - 8, 40))
            r = r[:L - 8 - cut] + r[L - 8:]
        elif kind == 3:  # a damaged state (some stay in [2^16, 2^24))
            v = int.from_bytes(r[-8:], "little") ^ (1 << rnd.randrange(24))
            r[-8:] = v.to_bytes(8, "little")
        elif kind == 4 and b % 3 == 0:  # too short
            r = r[:rnd.randrange(0, 8)]
        recs.append(bytes(r))
        host[o:o + len(r)] = r
        enc_len[b] = len(r)
    enc.copy_(torch.frombuffer(host, dtype=torch.uint8).cuda())
    bt.enc_len.copy_(torch.tensor(enc_len, dtype=torch.int64))
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    st = bt.statuses()
    for b, r in enumerate(recs):
        try:
            ref = oracle.rans_decode(t, 1, r, lens[b])
        except oracle.OracleError:
            ref = None
        if ref is None:
            assert st[b] != 0, f"record {b}: oracle errs, GPU ok"
        else:
            assert st[b] == 0, f"record {b}: oracle ok, GPU status {st[b]}"
            assert bt.raw_of(out, b) == ref, f"record {b}"
