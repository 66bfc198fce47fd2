"""Round 5: the pipelined compaction (k_enc_compact_pipe, opt-in through
zr_rans_set_compact_pipe; measured slower than k_enc_compact_lds). Every
workgroup walks groups of 16 streams with three under way; a group whose image
is wider than the window, or whose longest stream has more 16-B rows than the
lane loads cover, runs the one-group body after the loop. Both kinds are compared with the oracle byte for
byte (the reference layout of encode_parallel, rans.rs:369-420, streams at
rans.rs:402-419), in the same batch."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def pipe(zr):
    L = zr.load()
    assert L.zr_rans_set_compact_pipe(8) == 0
    yield
    L.zr_rans_set_compact_pipe(0)


def _roundtrip(zr, oracle, datas, N, shared=True):
    import concurrent.futures as cf
    import torch
    from zipora_amd.device import RansDeviceBatch
    bt = RansDeviceBatch([len(d) for d in datas], N, shared_table=shared)
    raw = bt.new_raw()
    for b, d in enumerate(datas):
        o = bt.raw_off_host[b]
        if d:
            raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    enc.fill_(0xA5)  # every byte of the layout written by the call
    bt.status.fill_(-9)
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


def _wide_groups(n, N, groups, seed):
    """Low-entropy bytes, except the columns of the given stream groups (byte i
    goes to stream i % N, rans.rs:388-391), which get bytes the table makes
    rare: those groups' streams grow ~1.5x and their images pass the window."""
    rng = np.random.default_rng(seed)
    d = rng.integers(0, 4, n, dtype=np.uint8)
    cols = np.zeros(N, dtype=bool)
    for g in groups:
        cols[16 * g:16 * g + 16] = True
    m = cols[np.arange(n) % N]
    d[m] = rng.integers(0, 256, int(m.sum()), dtype=np.uint8)
    return bytes(d)


def test_pipe_headline_with_wide_groups(zr, oracle):
    """The bench's buffer shape (4 MiB x 4096 streams): 32 buffers, half of them
    with 1-3 groups that take the in-place body (first, middle, last group of
    the buffer and of a 256-stream block), the rest all pipelined."""
    N = 4096
    datas = []
    for b in range(32):
        if b % 2:
            datas.append(_wide_groups(4 << 20, N, [(0, 17, 255), (100,), (16, 15)][b % 3], 0x1000 + b))
        else:
            datas.append(zr.synth("uzt"[b % 3], 4 << 20, seed=0x2000 + b))
    _roundtrip(zr, oracle, datas, N)


def test_pipe_every_group_wide(zr, oracle):
    """Every group of every buffer wider than the window: the loop only marks,
    the one-group body does all the work."""
    N = 4096
    datas = [_wide_groups(4 << 20, N, range(N // 16), 0x3000 + b) for b in range(2)]
    # low-entropy bytes dominate the shared table: a random byte costs ~10 bits
    datas.append(bytes(np.random.default_rng(0x3100).integers(0, 4, 32 << 20, dtype=np.uint8)))
    _roundtrip(zr, oracle, datas, N)


def test_pipe_ragged_batch(zr, oracle):
    """Ragged lengths and an N that is no multiple of 16 or 256 (a short last
    group and block), x1 buffers and an empty one interleaved, per-buffer tables,
    more groups than the grid (each workgroup several loop steps)."""
    N = 1000
    lens = [N * 300 + 7, N * 1024, 123, 0, N * 64 + N - 1, N * 1100 + 999] * 24
    datas = [zr.synth("tuz"[i % 3], n, seed=0x4000 + i) for i, n in enumerate(lens)]
    _roundtrip(zr, oracle, datas, N, shared=False)


def test_pipe_flagged_buffer(zr, oracle):
    """A byte missing from the table in one buffer: that buffer's status is
    ZR_INVALID_INPUT (written by its group 0's setup), the others OK and exact."""
    import torch
    from zipora_amd import _lib
    from zipora_amd.device import RansDeviceBatch
    N, B = 4096, 12
    lens = [N * 256] * B
    bt = RansDeviceBatch(lens, N, shared_table=True)
    raw = bt.new_raw()
    d0 = bytes(np.random.default_rng(5).integers(0, 100, lens[0], dtype=np.uint8))
    for b in range(B):
        o = bt.raw_off_host[b]
        raw[o:o + lens[b]] = torch.frombuffer(bytearray(d0), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    raw[bt.raw_off_host[5] + 777777] = 200
    bt.status.fill_(-9)
    bt.encode(raw, enc)
    torch.cuda.synchronize()
    st = bt.statuses()
    assert st[5] == _lib.ZR_INVALID_INPUT
    assert all(s == 0 for i, s in enumerate(st) if i != 5)
    t = oracle.rans_table(oracle.histogram(d0))
    ref = oracle.rans_encode(t, N, d0)
    for b in (0, 4, 6, 11):
        assert bt.encoded(enc, b) == ref
