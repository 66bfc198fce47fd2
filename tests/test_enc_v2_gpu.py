"""Round 4: the V2 encoder step (zr_rans.hip enc_entry_v2 / enc_step_v2: the state
kept as x, q = umulhi(y, R) >> sh, f = 1 through the start offset, output bits
OR-ed in place into the lane ring) at the symbol frequencies where it differs
from a plain division: f = 1, f < 16 (two renorm bytes per step), f = 4096
(a one-symbol table) and a symbol missing from the table, in the 256-lane xN
encoder and the record-batch ring encoder (k_enc_x1_ring). Every
encoded byte is compared with the oracle's encode (rans.rs:303-335 encode_symbol,
:354-366 encode_single, :369-420 encode_parallel), then decoded back."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rare_symbols(n, seed):
    """Mostly one byte; 200 bytes that occur once (normalised to f = 1), 12 that
    occur ~0.1 % each (f < 16: two renorm bytes when the state is high)."""
    rng = np.random.default_rng(seed)
    d = np.full(n, 200, dtype=np.uint8)
    pos = rng.choice(n, 200 + 12 * (n // 1000), replace=False)
    d[pos[:200]] = np.arange(200, dtype=np.uint8)
    rest = pos[200:]
    d[rest] = (201 + (np.arange(len(rest)) % 12)).astype(np.uint8)
    return d.tobytes()


def _kinds(n, b):
    k = b % 4
    if k == 0:
        return _rare_symbols(n, 31 + b)
    if k == 1:
        return bytes([7]) * n  # one symbol: f = 4096
    if k == 2:
        return bytes(np.random.default_rng(b).integers(0, 2, n, dtype=np.uint8) * 255)  # two symbols
    return bytes(np.random.default_rng(b).integers(0, 256, n, dtype=np.uint8))


@pytest.mark.parametrize("N", [4096, 1000, 1536])
def test_v2_edge_frequencies_xn(zr, oracle, N):
    import torch
    from zipora_amd.device import RansDeviceBatch
    B = 24 if N >= 4096 else 70
    lens = [N * (40 + 3 * b) + (b * 7) % N for b in range(B)]
    assert B * N > (1 << 16)  # the wide (>= 256-lane) encoder
    datas = [_kinds(n, b) for b, n in enumerate(lens)]
    bt = RansDeviceBatch(lens, N)
    raw = bt.new_raw()
    for b, d in enumerate(datas):
        o = bt.raw_off_host[b]
        raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    for b, d in enumerate(datas):
        t = oracle.rans_table(oracle.histogram(d))
        assert bt.encoded(enc, b) == oracle.rans_encode(t, N, d), f"buffer {b} (kind {b % 4})"
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    for b, d in enumerate(datas):
        assert bt.raw_of(out, b) == d, f"buffer {b}"


def test_v2_edge_frequencies_records(zr, oracle):
    """Records through the ring encoder with one shared table that has f = 1 and
    f < 16 symbols (trained on all records, blob_store/entropy.rs:212-238)."""
    import torch
    from zipora_amd.device import RansDeviceBatch
    R, n = 4096, 1024
    data = _rare_symbols(R * n, 5)
    bt = RansDeviceBatch([n] * R, 1, shared_table=True)
    raw = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    t = oracle.rans_table(oracle.histogram(data))
    for b in range(R):
        d = data[b * n:(b + 1) * n]
        assert bt.encoded(enc, b) == oracle.rans_encode(t, 1, d), f"record {b}"
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    assert torch.equal(out, raw)


def test_v2_symbol_missing_from_table(zr, oracle):
    """A buffer coded with another buffer's table (a byte with f = 0) reports
    "Symbol {} not in frequency table" (rans.rs:311-316) as ZR_INVALID_INPUT."""
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
    raw[bt.raw_off_host[B - 1] + 12345] = 200  # not in the table
    bt.encode(raw, enc)
    torch.cuda.synchronize()
    st = bt.statuses()
    assert st[B - 1] == _lib.ZR_INVALID_INPUT
    assert all(s == 0 for s in st[:B - 1])
