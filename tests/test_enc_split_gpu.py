"""Round 4: the split xN encode (zr_rans_set_encode_split(q)). A batch of at
least 2^18 streams is encoded as encoder(the first q/4 of the buffers) -> one
dispatch of encoder(the rest) + compaction(the first part) (k_enc_cmp_fused) ->
compaction(the rest). Every buffer's bytes must equal the
oracle's Rans64Encoder::encode (rans.rs:369-420 encode_parallel, :354-366
encode_single for buffers shorter than N) and the unsplit schedule's, byte for
byte, statuses included; then decode back."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def split(zr):
    L = zr.load()
    was, was_w = L.zr_rans_get_encode_split(), L.zr_rans_get_encoder_width()
    assert L.zr_rans_set_encoder_width(256) == 0  # (a form of the 256-lane encoder)

    def set_s(q):
        assert L.zr_rans_set_encode_split(q) == 0

    yield set_s
    L.zr_rans_set_encode_split(was)
    L.zr_rans_set_encoder_width(was_w)


def _fill(bt, datas):
    import torch
    raw = bt.new_raw()
    for b, d in enumerate(datas):
        if d:
            o = bt.raw_off_host[b]
            raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    return raw


def _encode(bt, raw, on, set_split):
    import torch
    set_split(on)
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    return enc


@pytest.mark.parametrize("N,B,shared,q", [(4096, 64, True, 2), (4096, 64, False, 3), (2048, 131, True, 3),
                                         (4096, 66, False, 1), (2048, 131, True, 2)])
def test_split_encode_matches_oracle(zr, oracle, split, N, B, shared, q):
    """Ragged lengths, buffers shorter than N (x1 layout), empty ones and an odd
    buffer count (halves of B // 2 and B - B // 2), per-buffer or shared table."""
    import torch
    from zipora_amd.device import RansDeviceBatch
    rnd = random.Random(N * 1000 + B)
    base = [0, 1, N - 1, N, N + 1, 3 * N + 7, 16 * N]
    lens = [base[i] if i < len(base) else rnd.randrange(N, 24 * N) for i in range(B)]
    rnd.shuffle(lens)
    assert B * N >= 1 << 18
    kinds = "uzt"
    datas = [zr.synth(kinds[b % 3], n, seed=301 + b) for b, n in enumerate(lens)]
    bt = RansDeviceBatch(lens, N, shared_table=shared)
    raw = _fill(bt, datas)
    enc1 = _encode(bt, raw, q, split)
    bt.raise_on_error()
    if shared:
        allb = b"".join(datas)
        t = oracle.rans_table(oracle.histogram(allb))
    for b, d in enumerate(datas):
        if not shared:
            t = oracle.rans_table(oracle.histogram(d))
        assert bt.encoded(enc1, b) == oracle.rans_encode(t, N, d), f"buffer {b} (n={len(d)})"
    lens1 = bt.enc_len.clone()
    enc0 = _encode(bt, raw, 0, split)
    bt.raise_on_error()
    assert torch.equal(bt.enc_len, lens1)
    for b in range(B):
        assert bt.encoded(enc0, b) == bt.encoded(enc1, b), f"buffer {b}: split and unsplit differ"
    out = bt.new_raw()
    bt.decode(enc1, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    for b, d in enumerate(datas):
        assert bt.raw_of(out, b) == d


@pytest.mark.parametrize("bad,q", [(3, 2), (40, 2), (45, 3), (50, 3)])
def test_split_encode_missing_symbol(zr, split, bad, q):
    """A byte the shared table lacks ("Symbol {} not in frequency table",
    rans.rs:311-316) in a buffer of the first part (its compaction runs in the
    fused dispatch) or of the second: that buffer alone reports
    ZR_INVALID_INPUT, under either schedule."""
    import torch
    from zipora_amd import _lib
    from zipora_amd.device import RansDeviceBatch
    N, B = 4096, 64
    lens = [N * 16] * B
    bt = RansDeviceBatch(lens, N, shared_table=True)
    raw = bt.new_raw()
    d0 = bytes(np.random.default_rng(2).integers(0, 128, lens[0], dtype=np.uint8))
    for b in range(B):
        o = bt.raw_off_host[b]
        raw[o:o + lens[b]] = torch.frombuffer(bytearray(d0), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    bt.full_encode(raw, enc)  # the table of bytes < 128
    torch.cuda.synchronize()
    bt.raise_on_error()
    raw[bt.raw_off_host[bad] + 777] = 200
    for on in (q, 0):
        split(on)
        bt.encode(raw, enc)
        torch.cuda.synchronize()
        st = bt.statuses()
        assert st[bad] == _lib.ZR_INVALID_INPUT
        assert all(s == 0 for i, s in enumerate(st) if i != bad)
