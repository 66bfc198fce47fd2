"""Round-2 rANS parity on the MI355X through the C ABI, against the oracle:
the literal BASELINE configs[1] at full size, both launch shapes of the coders,
wrapped-sum tables built on the device, the encoder's reciprocal division
checked exhaustively, allocation-free host calls from two threads, the
adaptive encoder, the pipe's error drain, the Huffman decoder's in-order
fallback, and the bench's N > 1 table exchange."""
import os
import random
import socket
import sys
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fill(bt, datas):
    import torch
    raw = bt.new_raw()
    for b, d in enumerate(datas):
        o = bt.raw_off_host[b]
        if d:
            raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    return raw


def test_rans_literal_config_full_size(zr, oracle):
    """BASELINE configs[1] as written: ONE 256 MiB uniform buffer, 4096-way
    interleaved streams (rans.rs:369-420), 65,536 symbols per stream. Encoded on
    the device (histogram -> Rans64Encoder::new -> encode), byte-compared with the
    oracle's Rans64Encoder::encode, decoded back."""
    import torch
    from zipora_amd.device import RansDeviceBatch
    n, N = 256 << 20, 4096
    data = zr.synth("u", n, seed=0x9E3779B97F4A7C15)
    bt = RansDeviceBatch([n], N, shared_table=True)
    raw = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    t = oracle.rans_table(oracle.histogram(data))
    ref = oracle.rans_encode(t, N, data)
    got = bt.encoded(enc, 0)
    assert len(got) == len(ref)
    assert got == ref
    del ref, got
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    assert torch.equal(out[:n], raw)


@pytest.mark.parametrize("N,B", [(4096, 24), (1000, 70), (1024, 70), (2048, 40), (8192, 10), (512, 140),
                                 (1536, 50)])
def test_rans_wide_shape_ragged(zr, oracle, N, B):
    """More than 2^16 streams in the batch: 256-lane encoder workgroups and
    1024-lane decoder workgroups, with ragged, tiny (x1 layout) and empty
    buffers mixed in."""
    import torch
    from zipora_amd.device import RansDeviceBatch
    rnd = random.Random(N)
    base = [0, 1, N - 1, N, N + 1, 50000, 123457, 1 << 18, 3 * N + 7]
    lens = [base[i % len(base)] if i < len(base) else rnd.randrange(N, 40 * N) for i in range(B)]
    assert B * N > (1 << 16)
    datas = [zr.synth("u" if b % 3 else "z", n, seed=77 + b) for b, n in enumerate(lens)]
    bt = RansDeviceBatch(lens, N)
    raw = _fill(bt, datas)
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    for b, d in enumerate(datas):
        t = oracle.rans_table(oracle.histogram(d))
        assert bt.encoded(enc, b) == oracle.rans_encode(t, N, d), f"buffer {b} (n={len(d)})"
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    for b, d in enumerate(datas):
        assert bt.raw_of(out, b) == d


@pytest.mark.parametrize("N", [64, 100, 1000, 4095, 4097])
def test_rans_narrow_shape_ragged(zr, oracle, N):
    """Few streams (one-wave workgroups): stream counts that are not multiples of
    the 64-lane workgroup, long streams, a shared table."""
    import torch
    from zipora_amd.device import RansDeviceBatch
    lens = [300000 + 13 * N, 5 * N + 3, N]
    datas = [zr.synth("t", n, seed=5 + b) for b, n in enumerate(lens)]
    bt = RansDeviceBatch(lens, N, shared_table=True)
    raw = _fill(bt, datas)
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    t = oracle.rans_table(oracle.histogram(b"".join(datas)))
    for b, d in enumerate(datas):
        assert bt.encoded(enc, b) == oracle.rans_encode(t, N, d), f"buffer {b}"
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    for b, d in enumerate(datas):
        assert bt.raw_of(out, b) == d


@pytest.mark.parametrize("N,per,B,skew", [(100, 1208, 3, False), (100, 1209, 3, False), (100, 1208, 2, True),
                                           (4096, 1208, 17, False), (4096, 1208, 17, True), (1000, 300, 70, True),
                                           (4096, 1209, 17, True)])
def test_rans_scratch_layouts(zr, oracle, N, per, B, skew):
    """Both scratch layouts of the xN encoder (RansWork::il): per-stream capacity
    2 * per + 16 = 2432 B is the largest lane-interleaved one, 2434 B the
    smallest stream-contiguous one. Groups of 16 streams whose destination spans
    two compaction windows, and (skew) streams of very different lengths in one
    group: every third stream of the period-N interleave sees one constant byte."""
    import torch
    from zipora_amd.device import RansDeviceBatch
    lens = [N * per - (b % 3) for b in range(B)]
    datas = []
    for b, n in enumerate(lens):
        d = np.frombuffer(zr.synth("u", n, seed=900 + b), dtype=np.uint8).copy()
        if skew:
            d[(np.arange(n) % N) % 3 == 0] = 65
        datas.append(d.tobytes())
    bt = RansDeviceBatch(lens, N)
    raw = _fill(bt, datas)
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    for b, d in enumerate(datas):
        t = oracle.rans_table(oracle.histogram(d))
        assert bt.encoded(enc, b) == oracle.rans_encode(t, N, d), f"buffer {b} (n={len(d)})"
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    for b, d in enumerate(datas):
        assert bt.raw_of(out, b) == d


def test_status_written_without_zeroing(zr, oracle):
    """encode/decode write every buffer's status themselves (no memset in the
    call): xN and x1 buffers, an empty one, a symbol missing from its table
    (rans.rs:311-316) and a header shorter than min_header_size
    (rans.rs:563-568), over a status array pre-filled with garbage."""
    import torch
    from zipora_amd._lib import ZR_INVALID_INPUT
    from zipora_amd.device import RansDeviceBatch
    N = 64
    lens = [0, 10, 5000, 5000, 70000]
    datas = [b"", bytes(range(10)), zr.synth("t", 5000, seed=3), b"ab" * 2500, zr.synth("u", 70000, seed=4)]
    bt = RansDeviceBatch(lens, N, shared_table=False)
    raw = _fill(bt, datas)
    enc = bt.new_enc()
    bt.histogram(raw)
    bt.tables_from_hist(consume=True)
    assert int(bt.hist.abs().sum().item()) == 0  # consumed
    raw[bt.raw_off_host[3] + 7] = 0xFF  # not in buffer 3's table
    bt.status.fill_(12345)
    bt.encode(raw, enc)
    torch.cuda.synchronize()
    assert bt.statuses() == [0, 0, 0, ZR_INVALID_INPUT, 0]
    for b in (0, 1, 2, 4):
        t = oracle.rans_table(oracle.histogram(datas[b]))
        assert bt.encoded(enc, b) == oracle.rans_encode(t, N, datas[b]), f"buffer {b}"
    bt.enc_len[2] = 5      # shorter than the N * 12 header
    bt.enc_len[3] = 0
    bt.status.fill_(-7)
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    assert bt.statuses() == [0, 0, ZR_INVALID_INPUT, ZR_INVALID_INPUT, 0]
    for b in (0, 1, 4):
        assert bt.raw_of(out, b) == datas[b]


@pytest.mark.parametrize("nzero", [1, 16])
def test_rans_generic_fallback_lanes(zr, oracle, nzero):
    """Streams the fast decoder cannot hold: a shared table in which almost every
    byte but 0 has frequency 1 (rans.rs:238-299 on a batch dominated by zeros), so a
    buffer of bytes 1..255 costs ~1.5 bytes per symbol and its lanes outrun their
    LDS rings; they fall back to the generic per-lane decoder inside the same
    kernel. One-wave (nzero=1) and 1024-lane (nzero=16) workgroups."""
    import numpy as np
    import torch
    from zipora_amd.device import RansDeviceBatch
    N, n = 4096, 256 << 10
    rnd = np.random.default_rng(7)
    hard = bytes(rnd.integers(1, 256, n, dtype=np.uint8))
    datas = [bytes(4 << 20)] * nzero + [hard]
    bt = RansDeviceBatch([len(d) for d in datas], N, shared_table=True)
    raw = _fill(bt, datas)
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    t = oracle.rans_table(oracle.histogram(b"".join(datas)))
    assert sum(f == 1 for f in t.freq[1:]) >= 250  # (pass 3 gives the remainder to one of them)
    assert bt.encoded(enc, nzero) == oracle.rans_encode(t, N, hard)
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    for b, d in enumerate(datas):
        assert bt.raw_of(out, b) == d, f"buffer {b}"


def test_rans_narrow_many_workgroups(zr, oracle):
    """One-wave workgroups beyond three per CU (N = 64, 900 buffers: 900
    workgroups): the decoder keeps its 4-byte slot entries there."""
    import torch
    from zipora_amd.device import RansDeviceBatch
    N, B = 64, 900
    rnd = random.Random(17)
    lens = [rnd.randrange(N, 3000) for _ in range(B)]
    datas = [zr.synth("t", n, seed=400 + b) for b, n in enumerate(lens)]
    bt = RansDeviceBatch(lens, N, shared_table=True)
    raw = _fill(bt, datas)
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    t = oracle.rans_table(oracle.histogram(b"".join(datas)))
    for b in range(0, B, 97):
        assert bt.encoded(enc, b) == oracle.rans_encode(t, N, datas[b]), f"buffer {b}"
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    assert torch.equal(out, raw)


@pytest.mark.parametrize("B", [3, 4])
def test_rans_many_blocks_separate_scan(zr, oracle, B):
    """More than SCAN_FUSE (64) 256-stream blocks per buffer (N = 20000): the
    block-sum scan runs as its own kernel before the compaction and the decoder
    (k_scan), in one-wave (B = 3) and 1024-lane (B = 4) workgroup shapes."""
    import torch
    from zipora_amd.device import RansDeviceBatch
    N = 20000
    lens = [5 * N + 7, 3 * N, N + 1, 7 * N + 11][:B]
    datas = [zr.synth("u" if b % 2 else "t", n, seed=31 + b) for b, n in enumerate(lens)]
    bt = RansDeviceBatch(lens, N)
    raw = _fill(bt, datas)
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    for b, d in enumerate(datas):
        t = oracle.rans_table(oracle.histogram(d))
        assert bt.encoded(enc, b) == oracle.rans_encode(t, N, d), f"buffer {b}"
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    for b, d in enumerate(datas):
        assert bt.raw_of(out, b) == d


def _dtab_words(bt, k=0):
    w = bt.tables.cpu().numpy().view(np.uint32)
    per = bt.tables.numel() // 4 // bt.n_tables
    return w[k * per:(k + 1) * per]


def test_device_table_wrapped_total(zr, oracle):
    """k_tab on histograms whose u32 sum wraps (rans.rs:209): the min(remaining)
    clamp of rans.rs:264-271 binds. Device table == oracle == host table."""
    import torch
    from zipora_amd.device import RansDeviceBatch
    rnd = random.Random(11)
    hists = []
    h = [0] * 256
    h[97], h[98], h[99] = 0xFFFFFFF0, 20, 5  # total wraps to 9
    hists.append(h)
    h = [0] * 256
    h[0], h[255] = 0x80000000, 0x80000001  # total wraps to 1
    hists.append(h)
    while len(hists) < 32:
        h = [rnd.choice([0, 0, 1, rnd.randrange(1, 1000)]) for _ in range(256)]
        for _ in range(rnd.randrange(1, 4)):
            h[rnd.randrange(256)] = rnd.randrange(1 << 30, 1 << 32)
        if sum(h) >= (1 << 32) and sum(h) & 0xFFFFFFFF:
            hists.append(h)
    assert all(sum(h) >= (1 << 32) for h in hists)
    bt = RansDeviceBatch([1] * len(hists), 1, shared_table=False)
    bt.hist.copy_(torch.tensor(np.array(hists, dtype=np.uint32).view(np.int32).reshape(-1)).cuda())
    bt.tables_from_hist()
    torch.cuda.synchronize()
    for k, h in enumerate(hists):
        t = oracle.rans_table(h)
        w = _dtab_words(bt, k)
        freq, start, slot = w[4:260], w[260:516], w[1028:1028 + 4096]
        assert list(freq) == list(t.freq), f"hist {k}"
        assert list(start) == list(t.start), f"hist {k}"
        host = zr.Rans64Encoder(h, 1).table
        assert list(host.freq) == list(t.freq)
        owner = np.zeros(4096, dtype=np.int64)
        for s in range(256):
            owner[t.start[s]:t.start[s] + t.freq[s]] = s
        assert (slot & 0xFF).tolist() == owner.tolist(), f"hist {k}"


def test_encoder_reciprocal_exhaustive(zr):
    """umulhi(x << 8, rcp) >> rsh == x / f for every f in 1..4096, x < 2^24 (the
    analogue of the reference's fast_div test, rans.rs:786-809), on the device."""
    assert zr.selftest_reciprocal() == 0


def test_host_calls_allocation_free_two_threads(zr, oracle):
    """10k x 1 KiB records through the synchronous zr_rans_encode/decode from two
    host threads: after warm-up the library allocates nothing (zr_device_alloc_count)."""
    recs = [zr.synth("t", 1024, seed=100 + i) for i in range(10000)]
    freqs = oracle.histogram(b"".join(recs))
    enc = zr.Rans64Encoder(freqs, 1)
    dec = zr.Rans64Decoder(enc)
    out = [None] * len(recs)
    errors = []

    def run(idx, barrier):
        try:
            barrier.wait()
            for i in idx:
                e = enc.encode(recs[i])
                out[i] = e
                assert dec.decode(e, 1024) == recs[i]
        except Exception as ex:  # noqa: BLE001
            errors.append(ex)

    def two_threads(lo, hi):
        b = threading.Barrier(2)
        ts = [threading.Thread(target=run, args=(range(lo + k, hi, 2), b)) for k in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errors, errors[:2]

    two_threads(0, 400)  # warm-up: both threads' call contexts grow to 1 KiB records
    before = zr.device_alloc_count()
    two_threads(400, len(recs))
    after = zr.device_alloc_count()
    assert after == before, f"{after - before} device allocations after warm-up"
    t = oracle.rans_table(freqs)
    for i in range(0, len(recs), 97):
        assert out[i] == oracle.rans_encode(t, 1, recs[i])


def test_adaptive_encoder(zr, oracle):
    """AdaptiveRans64Encoder (rans.rs:655-721) incl. the reference's own test
    (rans.rs:864-878): thresholds 73, 73^2, 73^4 and encode_adaptive."""
    a = zr.AdaptiveRans64Encoder()
    assert a.select_variant(50) == "x1"
    assert a.select_variant(100) == "x2"
    assert a.select_variant(10000) == "x4"
    assert a.select_variant(30000000) == "x8"
    for data in (b"test data for adaptive encoding", zr.synth("t", 73), zr.synth("z", 6000),
                 zr.synth("u", 100000), b""):
        N = {"x1": 1, "x2": 2, "x4": 4, "x8": 8}[a.select_variant(len(data))]
        got = a.encode_adaptive(data)
        assert got
        t = oracle.rans_table(oracle.histogram(data))
        assert got == oracle.rans_encode(t, N, data)


def test_pipe_error_then_reuse(zr, oracle):
    """an error return of the host pipe drains its streams and
    frees its slots, so the same pipe then codes a smaller batch correctly."""
    import torch
    from zipora_amd.device import RansHostPipe
    datas = [zr.synth("t", 1024, seed=i) for i in range(50)]
    freqs = oracle.histogram(b"".join(datas))
    pipe = RansHostPipe(zr.Rans64Encoder(freqs, 1).table, 1, 16 << 10)
    lens = [1024] * 50
    raw_off, _, rb, _ = pipe.layout(lens)
    raw = torch.zeros(rb, dtype=torch.uint8, pin_memory=True)
    for b, d in enumerate(datas):
        raw[int(raw_off[b]):int(raw_off[b]) + 1024] = torch.frombuffer(bytearray(d), dtype=torch.uint8)
    small = torch.zeros(3000, dtype=torch.uint8, pin_memory=True)  # far below 50 encoded records
    with pytest.raises(zr.ZiporaError):
        pipe.encode_packed(lens, raw, raw_off, small)
    lens2 = [1024] * 3
    raw_off2, _, rb2, eb2 = pipe.layout(lens2)
    raw2 = raw[:rb2].clone().pin_memory()
    enc2 = torch.zeros(eb2, dtype=torch.uint8, pin_memory=True)
    enc_off, enc_len, st, total = pipe.encode_packed(lens2, raw2, raw_off2, enc2)
    assert (st == 0).all()
    t = oracle.rans_table(freqs)
    e = enc2.numpy()
    for b in range(3):
        o = int(enc_off[b])
        assert e[o:o + int(enc_len[b])].tobytes() == oracle.rans_encode(t, 1, datas[b])
    pipe.close()


def test_huffman_decode_inorder_fallback(zr, oracle):
    """A stream whose guessed segment starts never resynchronise by themselves
    (a 3-bit all-zero code repeated over 70+ segments): the decoder's device
    rounds run out and its in-order pass finishes the job, without a host round
    trip. Output == oracle (decoder.rs:90-165)."""
    data = b"a" * 100000 + b"bcd"
    e = zr.HuffmanEncoder(data)
    bits = e.encode(data)
    t = oracle.huff_tree(oracle.histogram(data))
    assert bits == oracle.huff_encode(t, data)
    assert max(len(c) for c in oracle.huff_codes(t).values()) == 3
    assert zr.HuffmanDecoder(e.tree()).decode(bits, len(data)) == data
    with pytest.raises(zr.ZiporaError):  # "Decoded length mismatch"
        zr.HuffmanDecoder(e.tree()).decode(bits[:1000], 2700)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        import zipora_amd as zr
        from zipora_amd import dist as zd
        from zipora_amd.device import RansDeviceBatch
        import oracle_ffi as O
        lens = [200000 + 31 * rank, 70000]
        datas = [zr.synth("z", n, seed=zd.shard_seed(9, rank) + b) for b, n in enumerate(lens)]
        bt = RansDeviceBatch(lens, 4096, shared_table=True)
        raw = _fill(bt, datas)
        enc = bt.new_enc()
        # bench.py's N > 1 step: device histogram -> all-reduce -> k_tab -> encode
        bt.histogram(raw)
        zd.allreduce_histogram(bt.hist)
        bt.tables_from_hist()
        bt.encode(raw, enc)
        torch.cuda.synchronize()
        bt.raise_on_error()
        shards = [None] * world
        dist.all_gather_object(shards, b"".join(datas))
        t = O.rans_table(O.histogram(b"".join(shards)))
        ok = all(bt.encoded(enc, b) == O.rans_encode(t, 4096, d) for b, d in enumerate(datas))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_shared_table_exchange_two_ranks_on_device():
    """the int32 device histogram -> all_reduce -> k_tab
    sequence of bench.py with two ranks (gloo, both on cuda:0): every rank's
    streams equal the oracle's encoding under the union's table."""
    import torch.multiprocessing as mp
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert all(ok for _, ok in res)


def test_wide_decode_errors_in_later_workgroups(zr, oracle):
    """The 1024-lane decoder with its fused header (no k_dec_hdr): the last
    workgroup of a buffer to finish stores its status from the errors every
    workgroup added to the buffer's arrival word, so errors anywhere in a
    buffer survive. Corrupted buffers (lengths moved between two streams of the
    third workgroup, a changed state, a flipped stream bit, a truncated buffer,
    a total over enc_len) decode error-for-error and byte-for-byte like the
    oracle (rans.rs:555-651), over a status array pre-filled with garbage."""
    import random
    import torch
    from zipora_amd.device import RansDeviceBatch
    N, n, B = 4096, 1 << 18, 33  # 33 x 4096 streams > 2^16: the 1024-lane shape
    datas = [zr.synth("t" if b % 2 else "u", n, seed=900 + b) for b in range(B)]
    bt = RansDeviceBatch([n] * B, N, shared_table=False)
    raw = _fill(bt, datas)
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    tabs = [oracle.rans_table(oracle.histogram(d)) for d in datas]
    host = bytearray(enc.cpu().numpy().tobytes())
    enc_len = bt.enc_len.cpu().tolist()
    rnd = random.Random(17)

    def u32(buf, o):
        return int.from_bytes(buf[o:o + 4], "little")

    for b in range(1, B, 2):
        o, L = bt.enc_off_host[b], enc_len[b]
        kind = (b // 2) % 5
        if kind == 0:  # 9 bytes of stream s moved to stream s+1 (same total)
            s = rnd.randrange(2048, 3072)
            ls, ls1 = o + 8 * N + 4 * s, o + 8 * N + 4 * (s + 1)
            host[ls:ls + 4] = (u32(host, ls) - 9).to_bytes(4, "little")
            host[ls1:ls1 + 4] = (u32(host, ls1) + 9).to_bytes(4, "little")
        elif kind == 1:  # a state in [2^16, 2^24) changed
            s = rnd.randrange(1024, N)
            host[o + 8 * s:o + 8 * s + 8] = (0x10000 + rnd.randrange(1 << 20)).to_bytes(8, "little")
        elif kind == 2:  # a flipped bit in the stream area
            i = o + 12 * N + rnd.randrange(L - 12 * N)
            host[i] ^= 1 << rnd.randrange(8)
        elif kind == 3:  # truncated: the last stream is short
            enc_len[b] = L - rnd.randrange(1, 40)
        else:  # a length past enc_len ("Invalid stream data length")
            s = rnd.randrange(N)
            ls = o + 8 * N + 4 * s
            host[ls:ls + 4] = (u32(host, ls) + 100000).to_bytes(4, "little")
    enc.copy_(torch.frombuffer(host, dtype=torch.uint8).cuda())
    bt.enc_len.copy_(torch.tensor(enc_len, dtype=torch.int64))
    bt.status.fill_(-3)
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    st = bt.statuses()
    for b in range(B):
        o = bt.enc_off_host[b]
        try:
            ref = oracle.rans_decode(tabs[b], N, bytes(host[o:o + enc_len[b]]), n)
        except oracle.OracleError:
            ref = None
        if ref is None:
            assert st[b] != 0, f"buffer {b}: the oracle errs, the GPU reports ok"
        else:
            assert st[b] == 0, f"buffer {b}: the oracle decodes, GPU status {st[b]}"
            assert bt.raw_of(out, b) == ref, f"buffer {b}"


def test_wide_decode_errors_grid_beyond_residency(zr, oracle):
    """The decoder's status protocol without waits: every
    workgroup of a buffer adds itself to the buffer's arrival word when its
    lanes are done and the last one stores the status, so a grid of more
    workgroups than the GPU holds at once (300 buffers x 4 workgroups of 1024
    lanes, one per CU) reports errors found by the LAST workgroups of the last
    buffers; a clean call with the same workspace then reports OK everywhere (a
    stale arrival word of the earlier call restarts), and a corrupted call again
    reports the errors (rans.rs:480-482, :601-610: the oracle decides)."""
    import random
    import torch
    from zipora_amd.device import RansDeviceBatch
    N, n, B = 4096, 8 * 4096, 300
    datas = [zr.synth("u" if b % 3 else "t", n, seed=4000 + b) for b in range(B)]
    bt = RansDeviceBatch([n] * B, N, shared_table=False)
    raw = _fill(bt, datas)
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    tabs = [oracle.rans_table(oracle.histogram(d)) for d in datas]
    clean = bytearray(enc.cpu().numpy().tobytes())
    clean_len = bt.enc_len.cpu().tolist()
    host, enc_len = bytearray(clean), list(clean_len)
    rnd = random.Random(23)

    def u32(buf, o):
        return int.from_bytes(buf[o:o + 4], "little")

    bad_bufs = list(range(B - 24, B))  # the last buffers: their workgroups start last
    for b in bad_bufs:
        o, L = bt.enc_off_host[b], enc_len[b]
        if b % 3 == 0:  # truncated: the last stream (workgroup 3) runs out of bytes
            enc_len[b] = L - rnd.randrange(1, 8)
        elif b % 3 == 1:  # 5 bytes of a stream of workgroup 3 moved to its neighbour
            s = rnd.randrange(3072, N - 1)
            ls, ls1 = o + 8 * N + 4 * s, o + 8 * N + 4 * (s + 1)
            host[ls:ls + 4] = (u32(host, ls) - 5).to_bytes(4, "little")
            host[ls1:ls1 + 4] = (u32(host, ls1) + 5).to_bytes(4, "little")
        else:  # a state of workgroup 3 below 2^16: the generic decoder, then an error or not
            s = rnd.randrange(3072, N)
            host[o + 8 * s:o + 8 * s + 8] = rnd.randrange(1, 1 << 16).to_bytes(8, "little")

    def run(buf, lens):
        enc.copy_(torch.frombuffer(bytes(buf), dtype=torch.uint8).cuda())
        bt.enc_len.copy_(torch.tensor(lens, dtype=torch.int64))
        bt.status.fill_(-3)
        out = bt.new_raw()
        bt.decode(enc, out)
        torch.cuda.synchronize()
        return bt.statuses(), out

    def check(st, out, buf, lens):
        n_err = 0
        for b in range(B):
            o = bt.enc_off_host[b]
            try:
                ref = oracle.rans_decode(tabs[b], N, bytes(buf[o:o + lens[b]]), n)
            except oracle.OracleError:
                ref = None
            if ref is None:
                n_err += 1
                assert st[b] != 0, f"buffer {b}: the oracle errs, the GPU reports ok"
            else:
                assert st[b] == 0, f"buffer {b}: the oracle decodes, GPU status {st[b]}"
                assert bt.raw_of(out, b) == ref, f"buffer {b}"
        return n_err

    assert check(*run(host, enc_len), host, enc_len) >= 16
    st, out = run(clean, clean_len)
    assert all(v == 0 for v in st)
    assert check(st, out, clean, clean_len) == 0
    assert check(*run(host, enc_len), host, enc_len) >= 16


@pytest.mark.parametrize("kind,B,n", [("u", 64, 4 << 20), ("t", 3, 100_000), ("z", 1, 5000), ("u", 1, 0),
                                      ("t", 3000, 1000)])  # (the last: records, k_hist_small's fused form)
def test_table_from_data_fused(zr, oracle, kind, B, n):
    """zr_rans_dtab_from_data_dev (histogram + table build in the last k_hist
    workgroup): the table equals the oracle's
    Rans64Encoder::new of the batch's byte counts (rans.rs:208-299) and the
    two-launch path's byte for byte, hist is left zero, the table memory may
    hold garbage on entry, and repeated calls agree (the ticket counters are
    left zero by each call). The batch then encodes exactly as the oracle does."""
    import torch
    from zipora_amd.device import RansDeviceBatch
    datas = [zr.synth(kind, n, seed=77 + b) for b in range(B)]
    bt = RansDeviceBatch([n] * B, 4096, shared_table=True)
    raw = _fill(bt, datas)
    ref = RansDeviceBatch([n] * B, 4096, shared_table=True)
    ref.histogram(raw)
    ref.tables_from_hist()
    g = torch.Generator(device="cpu").manual_seed(5)
    bt.tables.copy_(torch.randint(0, 256, (bt.tables.numel(),), dtype=torch.uint8, generator=g).cuda())
    for _ in range(3):
        bt.table_from_data(raw)
        torch.cuda.synchronize()
        assert int(bt.hist.abs().sum().item()) == 0
        w, wr = _dtab_words(bt), _dtab_words(ref)
        assert (w[:2] == wr[:2]).all() and (w[4:] == wr[4:]).all()  # (words 2-3: padding, never written)
    all_bytes = b"".join(datas)
    t = oracle.rans_table(oracle.histogram(all_bytes))
    assert list(w[4:260]) == list(t.freq) and list(w[260:516]) == list(t.start)
    if n >= 4096:
        enc = bt.new_enc()
        bt.encode(raw, enc)
        torch.cuda.synchronize()
        bt.raise_on_error()
        for b in range(min(B, 3)):
            assert bt.encoded(enc, b) == oracle.rans_encode(t, 4096, datas[b])


@pytest.mark.parametrize("N,B,n,first_bad", [
    (4096, 8, 8 * 4096, 3584),     # one-wave shape: 64 workgroups per buffer, last set = workgroups 56..63
    (12288, 8, 6 * 12288, 8192),   # 1024-lane shape: 12 workgroups per buffer, last set = workgroups 8..11
])
def test_decode_errors_two_level_arrival(zr, oracle, N, B, n, first_bad):
    """a buffer of more than DA_SET = 8 decoder workgroups
    reports in two levels (sets of 8 on their own arrival words, the last of
    each set on the buffer's word), so an error bit must pass through a set
    word. Corruptions the oracle decides (truncation, moved lengths, a state
    below 2^16) placed only in streams of the LAST set's workgroups; the status
    must equal the oracle's, then a clean call on the same workspace reports OK
    and decodes, then the corrupted call errs again (rans.rs:480-482, :601-610)."""
    import torch
    from zipora_amd.device import RansDeviceBatch
    datas = [zr.synth("u" if b % 2 else "t", n, seed=5100 + b) for b in range(B)]
    bt = RansDeviceBatch([n] * B, N, shared_table=False)
    raw = _fill(bt, datas)
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    tabs = [oracle.rans_table(oracle.histogram(d)) for d in datas]
    clean = bytearray(enc.cpu().numpy().tobytes())
    clean_len = bt.enc_len.cpu().tolist()
    host, enc_len = bytearray(clean), list(clean_len)
    rnd = random.Random(N)

    def u32(buf, o):
        return int.from_bytes(buf[o:o + 4], "little")

    for b in range(1, B):  # buffer 0 stays clean: both statuses in one call
        o, L = bt.enc_off_host[b], enc_len[b]
        k = b % 3
        if k == 0:  # truncated: the last streams run out of bytes
            enc_len[b] = L - rnd.randrange(1, 8)
        elif k == 1:  # bytes moved between two streams of the last set
            s = rnd.randrange(first_bad, N - 1)
            ls, ls1 = o + 8 * N + 4 * s, o + 8 * N + 4 * (s + 1)
            mv = min(5, u32(host, ls))  # (short streams: N = 12288 codes 6 symbols each)
            host[ls:ls + 4] = (u32(host, ls) - mv).to_bytes(4, "little")
            host[ls1:ls1 + 4] = (u32(host, ls1) + mv).to_bytes(4, "little")
        else:  # a state of the last set below 2^16
            s = rnd.randrange(first_bad, N)
            host[o + 8 * s:o + 8 * s + 8] = rnd.randrange(1, 1 << 16).to_bytes(8, "little")

    def run(buf, lens):
        enc.copy_(torch.frombuffer(bytes(buf), dtype=torch.uint8).cuda())
        bt.enc_len.copy_(torch.tensor(lens, dtype=torch.int64))
        bt.status.fill_(-3)
        out = bt.new_raw()
        bt.decode(enc, out)
        torch.cuda.synchronize()
        return bt.statuses(), out

    def check(st, out, buf, lens):
        n_err = 0
        for b in range(B):
            o = bt.enc_off_host[b]
            try:
                ref = oracle.rans_decode(tabs[b], N, bytes(buf[o:o + lens[b]]), n)
            except oracle.OracleError:
                ref = None
            if ref is None:
                n_err += 1
                assert st[b] != 0, f"buffer {b}: the oracle errs, the GPU reports ok"
            else:
                assert st[b] == 0, f"buffer {b}: the oracle decodes, GPU status {st[b]}"
                assert bt.raw_of(out, b) == ref, f"buffer {b}"
        return n_err

    assert check(*run(host, enc_len), host, enc_len) >= 3
    st, out = run(clean, clean_len)
    assert all(v == 0 for v in st)
    assert check(st, out, clean, clean_len) == 0
    assert check(*run(host, enc_len), host, enc_len) >= 3
