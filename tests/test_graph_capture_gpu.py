"""HIP graph capture of the device pipeline: the histogram, table
build, encode and decode captured once and replayed; each replay must produce
the oracle's bytes, and a replay over a corrupted stream must report it (the
decoder's capture-safe path keeps no host-side per-call state). The _dev calls
that stage host data refuse a capturing stream."""
import os
import sys

import pytest
import torch

import zipora_amd as zr
from zipora_amd.device import RansDeviceBatch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle_ffi as O  # noqa: E402

pytestmark = pytest.mark.gpu


def test_captured_step_replays_bit_exact():
    lens = [300_000, 4096 * 40 + 17, 100]
    N = 4096
    ds = [zr.synth("u", n, seed=40 + i) for i, n in enumerate(lens)]
    bt = RansDeviceBatch(lens, N, shared_table=True)
    raw = bt.new_raw()
    for b, d in enumerate(ds):
        o = bt.raw_off_host[b]
        raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    enc, out = bt.new_enc(), bt.new_raw()
    side = torch.cuda.Stream()

    def step(s):
        bt.histogram(raw, s, zeroed=True)
        bt.tables_from_hist(s, consume=True)
        bt.encode(raw, enc, s)
        bt.decode(enc, out, s)

    with torch.cuda.stream(side):
        step(side)  # eager warm-up (allocations, first-call setup)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        step(torch.cuda.current_stream())
    torch.cuda.synchronize()
    alld = b"".join(ds)
    tab = O.rans_table(O.histogram(alld))
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        bt.raise_on_error()
        for b, d in enumerate(ds):
            assert bt.raw_of(out, b) == d
            assert bt.encoded(enc, b) == O.rans_encode(tab, N, d)
    # a decode-only graph over a corrupted buffer 0: the error must be reported
    # on every replay, and the clean buffers still decoded
    dg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(dg, stream=side):
        bt.decode(enc, out, torch.cuda.current_stream())
    torch.cuda.synchronize()
    e0 = bt.enc_off_host[0]
    enc[e0 + 8 * N: e0 + 8 * N + 4] = torch.tensor([0xFF, 0xFF, 0xFF, 0x7F], dtype=torch.uint8).cuda()
    for _ in range(2):
        dg.replay()
        torch.cuda.synchronize()
        st = bt.statuses()
        assert st[0] != 0 and st[1] == 0 and st[2] == 0
        assert bt.raw_of(out, 1) == ds[1] and bt.raw_of(out, 2) == ds[2]


def test_host_staging_calls_refuse_capture():
    from zipora_amd import _lib
    bt = RansDeviceBatch([1000], 4, shared_table=True)
    t = zr.Rans64Encoder([1] * 256, 4).table
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    st = None
    with torch.cuda.graph(g, stream=side):
        arr = (_lib.RansTable * 1)(t)
        st = zr.load().zr_rans_dtab_upload(arr, 1, bt.tables.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert st == _lib.ZR_UNSUPPORTED


def test_capture_refusal_list():
    """The header's list of the _dev calls that refuse a capturing stream
    (include/zipora_amd.h: zr_rans_dtab_upload, zr_huff_decode_dev,
    zr_huff_encode_dev, zr_fse_compress_dev,
    zr_fse_decompress_dev, zr_ctx_huff_encode_dev, zr_ctx_huff_decode_dev, the
    RansCompressor batch calls), each called under an active capture: every one
    returns ZR_UNSUPPORTED and enqueues nothing (the captured graph is empty)."""
    import ctypes
    from zipora_amd import _lib
    from zipora_amd.device import RansCompressorDeviceBatch
    L = zr.load()
    bt = RansDeviceBatch([5000], 4096, shared_table=True)
    raw = bt.new_raw()
    data = zr.synth("t", 4000, seed=3)
    tree = zr.HuffmanEncoder(data).tree().raw
    ctx = zr.ContextualHuffmanEncoder(data, zr.HuffmanOrder.Order1)
    cb = RansCompressorDeviceBatch([4000])
    buf = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    out = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    meta = torch.zeros(4, dtype=torch.int64, device="cuda")
    ws = torch.empty(1 << 22, dtype=torch.uint8, device="cuda")
    cfg = _lib.FseConfig()
    L.zr_fse_config_default(ctypes.byref(cfg))
    side = torch.cuda.Stream()
    got = {}
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        s = torch.cuda.current_stream().cuda_stream
        m, st = meta.data_ptr(), meta.data_ptr() + 8
        got["huff_decode"] = L.zr_huff_decode_dev(tree, buf.data_ptr(), 8192, out.data_ptr(), 4000, st,
                                                  ws.data_ptr(), ws.numel(), s)
        got["huff_encode"] = L.zr_huff_encode_dev(tree, buf.data_ptr(), 4000, out.data_ptr(), out.numel(), m, st,
                                                  ws.data_ptr(), ws.numel(), s)
        got["fse_compress"] = L.zr_fse_compress_dev(ctypes.byref(cfg), None, buf.data_ptr(), 4000, out.data_ptr(),
                                                    m, st, ws.data_ptr(), ws.numel(), s)
        got["fse_decompress"] = L.zr_fse_decompress_dev(buf.data_ptr(), 4000, out.data_ptr(), out.numel(), 1, m, st,
                                                        ws.data_ptr(), ws.numel(), s)
        got["ctx_encode"] = L.zr_ctx_huff_encode_dev(ctx.handle, 0, buf.data_ptr(), 4000, out.data_ptr(), s)
        got["ctx_decode"] = L.zr_ctx_huff_decode_dev(ctx.handle, 0, buf.data_ptr(), 4000, out.data_ptr(), 4000, s)
        got["compressor_compress"] = L.zr_rans_compressor_compress_batch_dev(
            cb.cbatch, buf.data_ptr(), out.data_ptr(), cb.ws.data_ptr(), cb.ws_bytes, s)
        got["compressor_decompress"] = L.zr_rans_compressor_decompress_batch_dev(
            cb.cbatch, buf.data_ptr(), out.data_ptr(), cb.ws.data_ptr(), cb.ws_bytes, s)
    assert got == {k: _lib.ZR_UNSUPPORTED for k in got}, got


def test_captured_fused_table_step_replays():
    """The bench's graph mode (bench.py --graph 1): the one-launch histogram +
    table (zr_rans_dtab_from_data_dev, ticket slot fixed at capture), encode and
    decode captured once and replayed on one stream; every replay equals the
    oracle and the table's tickets reset between replays (a replay over other
    data builds that data's table)."""
    lens = [4096 * 50, 4096 * 50 + 9]
    N = 4096
    bt = RansDeviceBatch(lens, N, shared_table=True)
    raw = bt.new_raw()
    enc, out = bt.new_enc(), bt.new_raw()
    side = torch.cuda.Stream()

    def load(seed, kind):
        ds = [zr.synth(kind, n, seed=seed + i) for i, n in enumerate(lens)]
        for b, d in enumerate(ds):
            o = bt.raw_off_host[b]
            raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
        return ds

    def step(s):
        bt.table_from_data(raw, s)
        bt.encode(raw, enc, s)
        bt.decode(enc, out, s)

    ds = load(70, "u")
    with torch.cuda.stream(side):
        step(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        step(torch.cuda.current_stream())
    torch.cuda.synchronize()
    for rep, (seed, kind) in enumerate([(70, "u"), (80, "t"), (90, "z"), (70, "u")]):
        ds = load(seed, kind)
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        bt.raise_on_error()
        tab = O.rans_table(O.histogram(b"".join(ds)))
        for b, d in enumerate(ds):
            assert bt.raw_of(out, b) == d, (rep, b)
            assert bt.encoded(enc, b) == O.rans_encode(tab, N, d), (rep, b)


@pytest.mark.parametrize("nbytes", [4, 12, 64, 256, 4096, 100003])
def test_captured_memset_replays(nbytes):
    """zr_memset_dev captured into a graph and replayed four times clears every
    byte each time. (hipMemsetAsync itself, captured, wrote address-like words
    on the second and later replays for 64 B and more on this ROCm, which is why
    the library fills by its own kernel: tools/graph_memset_probe.py.)"""
    L = zr.load()
    t = torch.full((nbytes + 3,), 7, dtype=torch.uint8, device="cuda")
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        assert L.zr_memset_dev(t.data_ptr() + 1, 0, nbytes, torch.cuda.current_stream().cuda_stream) == 0
    for _ in range(4):
        t.fill_(7)
        g.replay()
        torch.cuda.synchronize()
        assert int(t[1:nbytes + 1].max()) == 0 and int(t[1:nbytes + 1].min()) == 0
        assert int(t[0]) == 7 and int(t[nbytes + 1]) == 7


def test_captured_wide_decode_statuses_on_replay():
    """The headline geometry (64 buffers x 4096 streams: the wide decoder, its
    statuses cleared at every call) captured and replayed four times: every
    replay's statuses are clean and a corrupted buffer is flagged on each."""
    B, n, N = 64, 4096 * 8 + 5, 4096
    ds = [zr.synth("u", n, seed=500 + b) for b in range(B)]
    bt = RansDeviceBatch([n] * B, N, shared_table=True)
    raw = bt.new_raw()
    for b, d in enumerate(ds):
        o = bt.raw_off_host[b]
        raw[o:o + n] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    enc, out = bt.new_enc(), bt.new_raw()
    bt.table_from_data(raw)
    bt.encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        bt.decode(enc, out, torch.cuda.current_stream())
    for rep in range(4):
        bt.status.fill_(-3)
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert bt.statuses() == [0] * B, rep
        assert torch.equal(out, raw)
    e0 = bt.enc_off_host[5]
    enc[e0 + 8 * N: e0 + 8 * N + 4] = torch.tensor([0xFF, 0xFF, 0xFF, 0x7F], dtype=torch.uint8).cuda()
    for rep in range(2):
        g.replay()
        torch.cuda.synchronize()
        st = bt.statuses()
        assert st[5] != 0 and all(s == 0 for i, s in enumerate(st) if i != 5), rep
