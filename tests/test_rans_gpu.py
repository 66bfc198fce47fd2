"""rANS parity on the MI355X: HIP path through the C ABI vs the oracle (bit-exact)."""
import random

import pytest

pytestmark = pytest.mark.gpu

NS = [1, 2, 3, 4, 8, 64, 255, 256, 257, 1000, 4096]


def _cases(oracle):
    u = oracle.gen_uniform(200000)
    rep = b"This is a test message for parallel rANS processing with multiple streams to verify correctness across all variants." * 10
    skew = bytearray(100000)
    skew[50000] = 255
    return [
        b"hello world, this is a test of enhanced 64-bit rANS encoding",
        b"quad-stream parallel encoding test with four independent streams for better performance",
        bytes(((i * 123 + 45) % 256) for i in range(10000)),
        rep, b"a" * 10000, bytes(i % 256 for i in range(4096)), bytes(skew),
        u[:1], u[:7], u[:255], u[:256], u[:257], u[:4095], u[:4096], u[:4097], u[:100000],
        bytes([7]) * 3 + bytes([9]),
    ]


def test_rans_host_api_bit_exact(zr, oracle):
    for data in _cases(oracle):
        freqs = oracle.histogram(data)
        t = oracle.rans_table(freqs)
        for N in NS:
            if N > 8 and len(data) > 20000 and N not in (256, 4096):
                continue
            ref = oracle.rans_encode(t, N, data)
            enc = zr.Rans64Encoder(freqs, N)
            got = enc.encode(data)
            assert got == ref, f"encode mismatch n={len(data)} N={N}"
            dec = zr.Rans64Decoder(enc)
            assert dec.decode(ref, len(data)) == data


def test_rans_empty_and_zero(zr, oracle):
    freqs = [0] * 256
    enc = zr.Rans64Encoder(freqs, 4)
    assert enc.encode(b"") == bytes.fromhex("0000010000000000")
    assert zr.Rans64Decoder(enc).decode(b"", 0) == b""
    with pytest.raises(zr.ZiporaError):
        enc.encode(b"x")  # empty table: symbol not in frequency table


def test_rans_symbol_missing_errors(zr):
    f = zr.histogram(b"aaaa")
    for N in (1, 4, 300):
        with pytest.raises(zr.ZiporaError):
            zr.Rans64Encoder(f, N).encode(b"a" * 1000 + b"b")


def test_rans_truncation_errors(zr, oracle):  # rans.rs:971-1008
    data = b"hello world 1234567890 parallel test data string for testing truncated stream lengths"
    f = oracle.histogram(data)
    enc = zr.Rans64Encoder(f, 4)
    e = enc.encode(data)
    d = zr.Rans64Decoder(enc)
    with pytest.raises(zr.ZiporaError):
        d.decode(e[:-10], len(data))
    with pytest.raises(zr.ZiporaError):
        d.decode(e[:40], len(data))
    with pytest.raises(zr.ZiporaError):
        zr.Rans64Decoder(zr.Rans64Encoder(f, 1)).decode(b"\x01\x02", 5)


def _oracle_decode_or_error(oracle, t, N, data, n):
    try:
        return oracle.rans_decode(t, N, data, n)
    except oracle.OracleError:
        return None


def test_rans_decode_crafted_streams_match_oracle(zr, oracle):
    """Fuzz-style: corrupted states/lengths/bytes -> same Ok/Err and same bytes as the oracle."""
    rnd = random.Random(7)
    data = oracle.gen_uniform(3000)
    f = oracle.histogram(data)
    t = oracle.rans_table(f)
    for N in (1, 4, 300):
        good = bytearray(oracle.rans_encode(t, N, data))
        for trial in range(40):
            bad = bytearray(good)
            kind = trial % 4
            if kind == 0 and N > 1:  # state outside [2^16, 2^24): generic path
                s = rnd.randrange(N)
                val = rnd.choice([0, 1, 255, 65535, 1 << 24, (1 << 32) + 5, (1 << 63) + 12345])
                bad[8 * s: 8 * s + 8] = val.to_bytes(8, "little")
            elif kind == 1:
                i = rnd.randrange(len(bad))
                bad[i] ^= 1 << rnd.randrange(8)
            elif kind == 2 and N > 1:
                s = rnd.randrange(N)
                o = 8 * N + 4 * s
                v = int.from_bytes(bad[o: o + 4], "little")
                bad[o: o + 4] = max(0, v + rnd.choice([-3, -1, 1, 2])).to_bytes(4, "little")
            else:
                bad = bad[: rnd.randrange(1, len(bad))]
            ref = _oracle_decode_or_error(oracle, t, N, bytes(bad), len(data))
            dec = zr.Rans64Decoder(zr.Rans64Encoder(f, N))
            try:
                got = dec.decode(bytes(bad), len(data))
            except zr.ZiporaError:
                got = None
            assert got == ref, f"N={N} trial={trial}"


def _batch_roundtrip(zr, oracle, lens, N, kind, shared, align=16):
    import torch
    from zipora_amd.device import RansDeviceBatch
    bt = RansDeviceBatch(lens, N, shared_table=shared, align=align)
    raw = bt.new_raw()
    datas = []
    for b, n in enumerate(lens):
        d = zr.synth(kind, n, seed=1000 + b)
        datas.append(d)
        o = bt.raw_off_host[b]
        raw[o:o + n] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda() if n else raw[o:o]
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    if shared:
        allb = b"".join(datas)
        tables = [oracle.rans_table(oracle.histogram(allb))] * len(lens)
    else:
        tables = [oracle.rans_table(oracle.histogram(d)) for d in datas]
    for b, d in enumerate(datas):
        assert bt.encoded(enc, b) == oracle.rans_encode(tables[b], N, d), f"buffer {b}"
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    for b, d in enumerate(datas):
        assert bt.raw_of(out, b) == d


@pytest.mark.parametrize("N,shared", [(4096, False), (4096, True), (1, False), (256, False),
                                      (100, True)])
def test_rans_device_batch(zr, oracle, N, shared):
    lens = [0, 1, 4095, 4096, 4097, 50000, 123457, 1 << 18]
    _batch_roundtrip(zr, oracle, lens, N, "u", shared)


def test_rans_device_batch_text_zipf(zr, oracle):
    _batch_roundtrip(zr, oracle, [300000, 70000], 4096, "t", False)
    _batch_roundtrip(zr, oracle, [300000, 70000], 1024, "z", True)


def test_rans_blob_batch_x1(zr, oracle):
    """config-5 shape in miniature: many 1 KiB records, x1 each, shared trained table."""
    _batch_roundtrip(zr, oracle, [1024] * 300 + [17, 0, 2000], 1, "t", True)
    # unaligned record offsets (byte-granular layouts) take the byte-store paths
    _batch_roundtrip(zr, oracle, [1000, 3, 1021, 16, 15, 777], 1, "z", True, align=1)
    _batch_roundtrip(zr, oracle, [1000, 3, 1021, 16, 15, 777], 1, "z", False, align=1)


def test_rans_full_size_property(zr, oracle):
    """BASELINE config 2 at full size: 256 MiB as 64 x 4 MiB buffers, 4096 streams each.
    Round trip must be exact; 4 buffers are also byte-compared with the oracle."""
    import torch
    from zipora_amd.device import RansDeviceBatch
    B, n, N = 64, 4 << 20, 4096
    bt = RansDeviceBatch([n] * B, N)
    data = zr.synth("u", B * n)
    raw = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    assert torch.equal(out, raw)
    for b in (0, 17, 42, 63):
        d = data[b * n:(b + 1) * n]
        t = oracle.rans_table(oracle.histogram(d))
        assert bt.encoded(enc, b) == oracle.rans_encode(t, N, d)


def _pipe_roundtrip(zr, oracle, lens, N, kind, group_bytes, pinned=True):
    """Host-resident batch through zr_rans_pipe_*: every buffer's bytes equal the
    oracle's Rans64Encoder::encode under the shared table; decode restores the input."""
    import numpy as np
    import torch
    from zipora_amd.device import RansHostPipe
    datas = [zr.synth(kind, n, seed=3000 + b) for b, n in enumerate(lens)]
    freqs = oracle.histogram(b"".join(datas))
    table = zr.Rans64Encoder(freqs, N).table
    pipe = RansHostPipe(table, N, group_bytes)
    raw_off, enc_off, rb, eb = pipe.layout(lens)
    raw = torch.zeros(max(rb, 1), dtype=torch.uint8, pin_memory=pinned)
    for b, d in enumerate(datas):
        o = int(raw_off[b])
        raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8) if d else raw[o:o]
    enc = torch.zeros(max(eb, 1), dtype=torch.uint8, pin_memory=pinned)
    enc_len, st = pipe.encode(lens, raw, raw_off, enc, enc_off)
    assert (st == 0).all()
    t = oracle.rans_table(freqs)
    encb = enc.numpy()
    for b, d in enumerate(datas):
        o = int(enc_off[b])
        assert encb[o:o + int(enc_len[b])].tobytes() == oracle.rans_encode(t, N, d), f"buffer {b}"
    out = torch.zeros_like(raw)
    st = pipe.decode(lens, enc, enc_off, enc_len, out, raw_off)
    assert (st == 0).all()
    outb = out.numpy()
    for b, d in enumerate(datas):
        o = int(raw_off[b])
        assert outb[o:o + len(d)].tobytes() == d, f"buffer {b}"
    pipe.close()


def test_rans_host_pipe_packed(zr, oracle):
    """Packed encode: records back to back (offsets = exclusive scan of lengths),
    bytes equal the oracle's; decode from the packed layout restores the input."""
    import numpy as np
    import torch
    from zipora_amd.device import RansHostPipe
    for lens, N, kind, group in (([1024] * 3000 + [0, 17, 5], 1, "t", 256 << 10),
                                 ([300000, 0, 5, 70000, 1 << 20, 4096], 4096, "u", 512 << 10)):
        datas = [zr.synth(kind, n, seed=500 + b) for b, n in enumerate(lens)]
        freqs = oracle.histogram(b"".join(datas))
        pipe = RansHostPipe(zr.Rans64Encoder(freqs, N).table, N, group)
        raw_off, _, rb, eb = pipe.layout(lens)
        raw = torch.zeros(max(rb, 1), dtype=torch.uint8, pin_memory=True)
        for b, d in enumerate(datas):
            o = int(raw_off[b])
            if d:
                raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8)
        enc = torch.zeros(max(eb, 1), dtype=torch.uint8, pin_memory=True)
        enc_off, enc_len, st, total = pipe.encode_packed(lens, raw, raw_off, enc)
        assert (st == 0).all()
        assert total == int(enc_len.sum())
        assert enc_off.tolist() == (np.concatenate([[0], np.cumsum(enc_len)[:-1]]).tolist() if len(lens) else [])
        t = oracle.rans_table(freqs)
        encb = enc.numpy()
        for b, d in enumerate(datas):
            o = int(enc_off[b])
            assert encb[o:o + int(enc_len[b])].tobytes() == oracle.rans_encode(t, N, d), f"buffer {b}"
        out = torch.zeros_like(raw)
        st = pipe.decode(lens, enc, enc_off, enc_len, out, raw_off)
        assert (st == 0).all()
        outb = out.numpy()
        for b, d in enumerate(datas):
            o = int(raw_off[b])
            assert outb[o:o + len(d)].tobytes() == d
        pipe.close()


def test_rans_host_pipe(zr, oracle):
    # several groups per call (every device slot reused), a buffer larger than a group,
    # empty and tiny buffers, pageable memory
    lens = [300000, 0, 5, 70000, 1 << 20, 4096, 200000, 123457, 1, 90000]
    _pipe_roundtrip(zr, oracle, lens, 4096, "u", 256 << 10)
    _pipe_roundtrip(zr, oracle, lens, 64, "t", 64 << 10, pinned=False)
    _pipe_roundtrip(zr, oracle, [1024] * 200 + [17, 3], 1, "t", 32 << 10)
    _pipe_roundtrip(zr, oracle, [], 4, "u", 1 << 20)


def test_rans_host_pipe_errors(zr, oracle):
    import numpy as np
    import torch
    from zipora_amd.device import RansHostPipe
    freqs = oracle.histogram(b"aaaa")
    pipe = RansHostPipe(zr.Rans64Encoder(freqs, 4).table, 4, 1 << 16)
    lens = [100, 100]
    raw_off, enc_off, rb, eb = pipe.layout(lens)
    raw = torch.full((rb,), ord("a"), dtype=torch.uint8)
    raw[150] = ord("b")  # symbol missing from the table: buffer 1 fails, buffer 0 codes
    enc = torch.zeros(eb, dtype=torch.uint8)
    enc_len, st = pipe.encode(lens, raw, raw_off, enc, enc_off)
    assert st[0] == 0 and st[1] != 0
    # truncated input: decode reports the buffer, the other one is restored
    enc_len2 = enc_len.copy()
    enc_len2[1] = 10
    out = torch.zeros_like(raw)
    enc_len2[0] = enc_len[0]
    st = pipe.decode([100, 100], enc, enc_off, enc_len2, out, raw_off)
    assert st[0] == 0 and st[1] != 0
    assert bytes(out[:100].numpy()) == b"a" * 100


@pytest.mark.parametrize("align", [16, 1])
def test_shared_histogram_small_records(zr, align):
    """Shared histogram of many <= 1 KiB records (the blob-store path): equals the
    byte counts of the records' concatenation (rans.rs:708-714 caller semantics)."""
    import numpy as np
    import torch
    from zipora_amd.device import RansDeviceBatch
    rnd = random.Random(align)
    lens = [rnd.choice([0, 1, 15, 16, 17, 255, 1000, 1023, 1024]) for _ in range(1000)] + [1024] * 200
    bt = RansDeviceBatch(lens, 1, shared_table=True, align=align)
    raw = bt.new_raw()
    datas = []
    for b, n in enumerate(lens):
        d = zr.synth("z" if b % 2 else "u", n, seed=b)
        datas.append(d)
        o = bt.raw_off_host[b]
        if n:
            raw[o:o + n] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    # bytes outside the records must not be counted
    gaps = torch.ones_like(raw, dtype=torch.bool)
    for b, n in enumerate(lens):
        gaps[bt.raw_off_host[b]:bt.raw_off_host[b] + n] = False
    raw[gaps] = 0xAB
    bt.histogram(raw)
    torch.cuda.synchronize()
    want = np.bincount(np.frombuffer(b"".join(datas), dtype=np.uint8), minlength=256)
    assert bt.hist[:256].cpu().numpy().astype(np.int64).tolist() == want.tolist()
