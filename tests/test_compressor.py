"""RansCompressor record format (compression/mod.rs:416-512).

CPU tests pin the oracle composition and the re-normalisation quirk (finding
0.9); GPU tests compare the HIP path (host records and device batches) with
the oracle byte for byte and error for error."""
import struct

import pytest


def _train_cases(zr):
    text = zr.synth("t", 20000, seed=11)
    return [
        (text, text[:5000]),                       # typical: trained on the data itself
        (b"aaaaaaaaab", b"ab" * 50),               # skewed table
        (bytes(range(256)) * 4, bytes(range(256))),  # flat table: idempotent normalisation
        (zr.synth("z", 50000, seed=3), zr.synth("z", 3000, seed=4)),
        (b"hello world", b"hello"),
    ]


def _try(fn, *a):
    """fn(*a), or None when it raises (errors compare equal to errors)."""
    try:
        return fn(*a)
    except Exception:  # noqa: BLE001
        return None


def test_oracle_quirk_and_flat_roundtrip(zr, oracle):
    """Flat tables survive the second normalisation; skewed ones do not (finding 0.9)."""
    flat = oracle.rans_compressor_table(bytes(range(256)) * 4)
    data = bytes(range(256))
    rec = oracle.rans_compressor_compress(flat, data)
    assert len(rec) == 1028 + len(oracle.rans_encode(flat, 1, data))
    assert struct.unpack("<I", rec[1024:1028])[0] == 256
    assert oracle.rans_compressor_decompress(rec) == data
    skew = oracle.rans_compressor_table(b"aaaaaaaaab")
    again = oracle.rans_table([skew.freq[i] for i in range(256)])
    assert [again.freq[i] for i in range(256)] != [skew.freq[i] for i in range(256)]
    assert oracle.rans_compressor_compress(skew, b"") == b""
    assert oracle.rans_compressor_decompress(b"") == b""
    with pytest.raises(oracle.OracleError):
        oracle.rans_compressor_decompress(b"\x00" * 1027)
    with pytest.raises(oracle.OracleError):
        oracle.rans_compressor_table(b"")


@pytest.mark.gpu
def test_compressor_host_records(zr, oracle):
    for train, data in _train_cases(zr):
        c = zr.RansCompressor(train)
        t = oracle.rans_compressor_table(train)
        assert [c.table.freq[i] for i in range(256)] == [t.freq[i] for i in range(256)]
        rec = c.compress(data)
        assert rec == oracle.rans_compressor_compress(t, data)
        assert _try(c.decompress, rec) == _try(oracle.rans_compressor_decompress, rec)
    c = zr.RansCompressor(b"abc")
    assert c.compress(b"") == b"" and c.decompress(b"") == b""
    with pytest.raises(zr.ZiporaError):
        c.decompress(b"\x01" * 100)
    with pytest.raises(zr.ZiporaError):
        zr.RansCompressor(b"")
    with pytest.raises(zr.ZiporaError):
        c.compress(b"abd")  # 'd' not in the table


@pytest.mark.gpu
def test_compressor_device_batch(zr, oracle):
    """Blob-store style batch: one compressor, many records, empty and odd sizes."""
    import torch
    from zipora_amd.device import RansCompressorDeviceBatch
    for train in (bytes(range(256)) * 16, zr.synth("t", 1 << 16, seed=5)):
        lens = [1024] * 40 + [0, 1, 17, 3000, 0, 255]
        # records drawn from the training bytes: every symbol is in the table
        datas = [train[(97 * i) % (len(train) - n):][:n] if n else b"" for i, n in enumerate(lens)]
        c = zr.RansCompressor(train)
        t = oracle.rans_compressor_table(train)
        bt = RansCompressorDeviceBatch(lens)
        bt.upload_tables([c.table])
        raw = bt.new_raw()
        for b, d in enumerate(datas):
            o = bt.raw_off_host[b]
            if d:
                raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
        enc = bt.new_enc()
        bt.compress(raw, enc)
        torch.cuda.synchronize()
        st = bt.statuses()
        recs = []
        for b, d in enumerate(datas):
            ref = oracle.rans_compressor_compress(t, d)
            assert st[b] == 0, f"record {b}"
            got = bt.encoded(enc, b)
            assert got == ref, f"record {b}"
            recs.append(got)
        out = bt.new_raw()
        bt.decompress(enc, out)
        torch.cuda.synchronize()
        st = bt.statuses()
        for b, rec in enumerate(recs):
            want = _try(oracle.rans_compressor_decompress, rec)
            if want is None:
                assert st[b] != 0, f"record {b}"
            else:
                assert st[b] == 0, f"record {b}"
                assert bt.raw_of(out, b) == want, f"record {b}"
