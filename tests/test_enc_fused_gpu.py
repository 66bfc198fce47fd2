"""Round 5: encode and stream compaction in one launch (k_enc_lb,
zr_rans_set_encode_fused(1)). Each 256-stream encoder
workgroup compacts its own streams after a look-back on the byte sums of its
buffer's lower blocks; the output is the reference layout of encode_parallel
(rans.rs:369-420, header and streams at rans.rs:402-419), byte for byte."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def fused(zr):
    L = zr.load()
    was, was_w = L.zr_rans_get_encode_fused(), L.zr_rans_get_encoder_width()
    assert L.zr_rans_set_encoder_width(256) == 0  # (a form of the 256-lane encoder)
    assert L.zr_rans_set_encode_fused(1) == 0
    yield
    L.zr_rans_set_encode_fused(was)
    L.zr_rans_set_encoder_width(was_w)


def _roundtrip(zr, oracle, datas, N, shared=True):
    import concurrent.futures as cf
    import torch
    from zipora_amd.device import RansDeviceBatch
    lens = [len(d) for d in datas]
    bt = RansDeviceBatch(lens, N, shared_table=shared)
    raw = bt.new_raw()
    for b, d in enumerate(datas):
        o = bt.raw_off_host[b]
        if d:
            raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    bt.status.fill_(-9)  # every status written by the call
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    if shared:
        t = oracle.rans_table(oracle.histogram(b"".join(datas)))
        tabs = [t] * len(datas)
    else:
        tabs = [oracle.rans_table(oracle.histogram(d)) for d in datas]
    with cf.ThreadPoolExecutor(max_workers=16) as ex:
        refs = list(ex.map(lambda b: oracle.rans_encode(tabs[b], N, datas[b]), range(len(datas))))
    for b in range(len(datas)):
        assert bt.encoded(enc, b) == refs[b], f"buffer {b}"
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    assert torch.equal(out, raw)
    return bt


@pytest.mark.parametrize("kind", ["u", "t", "z"])
def test_fused_headline_batch(zr, oracle, fused, kind):
    """The bench's shape (64 x 4 MiB x 4096 streams), every buffer compared."""
    datas = [zr.synth(kind, 4 << 20, seed=0xF0 + b) for b in range(64)]
    _roundtrip(zr, oracle, datas, 4096)


def test_fused_ragged_and_mixed(zr, oracle, fused):
    """Ragged buffers (blocks with fewer than 256 streams, rows not a multiple of
    the tile), N not a multiple of 256, an x1 buffer and an empty one in the
    same batch, per-buffer tables; the batch over 2^16 streams (wide shape)."""
    N = 1000
    lens = [N * 300 + 7, N * 1024, 123, 0, N * 64 + N - 1] * 20
    datas = [zr.synth("tuz"[i % 3], n, seed=0x5A + i) for i, n in enumerate(lens)]
    _roundtrip(zr, oracle, datas, N, shared=False)


def test_fused_many_calls_reuse_slots(zr, oracle, fused):
    """More calls than ticket slots (64) in a row on one stream: every call's
    tickets start at 0 again (the last workgroup resets its slot)."""
    datas = [zr.synth("u", 1 << 20, seed=0x77 + b) for b in range(16)]
    import torch
    from zipora_amd.device import RansDeviceBatch
    bt = RansDeviceBatch([len(d) for d in datas], 4096, shared_table=True)
    raw = bt.new_raw()
    for b, d in enumerate(datas):
        o = bt.raw_off_host[b]
        raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    first = enc.clone()
    for _ in range(70):
        bt.encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    assert torch.equal(first, enc)
    t = oracle.rans_table(oracle.histogram(b"".join(datas)))
    assert bt.encoded(enc, 15) == oracle.rans_encode(t, 4096, datas[15])


def test_fused_symbol_missing_from_table(zr, oracle, fused):
    """A byte with f = 0 in one block of the last buffer: that buffer's status
    (written by its LAST block's workgroup, which looks back over all of them)
    is ZR_INVALID_INPUT, every other buffer's OK and byte-exact."""
    import torch
    from zipora_amd import _lib
    from zipora_amd.device import RansDeviceBatch
    N, B = 4096, 20
    lens = [N * 64] * B
    bt = RansDeviceBatch(lens, N, shared_table=True)
    raw = bt.new_raw()
    d0 = bytes(np.random.default_rng(1).integers(0, 128, lens[0], dtype=np.uint8))
    for b in range(B):
        o = bt.raw_off_host[b]
        raw[o:o + lens[b]] = torch.frombuffer(bytearray(d0), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    bt.full_encode(raw, enc)  # table from bytes < 128
    torch.cuda.synchronize()
    bt.raise_on_error()
    for pos in (12345, 7):  # a block in the middle, then block 7 of 16 (stream 7)
        raw[bt.raw_off_host[B - 1] + pos] = 200  # not in the table
        bt.status.fill_(-9)
        bt.encode(raw, enc)
        torch.cuda.synchronize()
        st = bt.statuses()
        assert st[B - 1] == _lib.ZR_INVALID_INPUT
        assert all(s == 0 for s in st[:B - 1])
    t = oracle.rans_table(oracle.histogram(d0))
    assert bt.encoded(enc, 0) == oracle.rans_encode(t, N, d0)
