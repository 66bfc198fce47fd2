"""FSE parity on the MI355X: HIP path (zr_fse.hip) through the C ABI vs the oracle, bit-exact.

Cases follow the reference's tests/fse_tests.rs (strict round trips, edge sizes,
skew, all-256, deterministic random, presets, decoder-config independence,
static-table unseen symbol) and the stream-format rules of fse.rs:1105-1312.
"""
import random

import pytest

pytestmark = pytest.mark.gpu


def _cases(oracle):
    u = oracle.gen_uniform(70000)
    adv = bytes(4000) + bytes(range(1, 151))
    adv2 = b"\xff" * 4000 + bytes(range(1, 151))
    mod = b"a" * 700 + b"b" * 150 + b"c" * 150 + bytes(range(100))
    all256 = bytes((i % 256) for i in range(2048))
    tri = b"".join(bytes([b]) * (b + 1) for b in range(256))
    fox = (b"The quick brown fox jumps over the lazy dog. " * 120)[:5000]
    return [
        b"", b"a", b"\xff", b"x" * 99, b"x" * 100, b"x" * 101, bytes(4096), b"\xff" * 500,
        (b"abc" * 333), adv, adv2, mod, all256, tri, u[:128], u[:1000], u[:4096], u, fox,
        b"The quick brown fox jumps over the lazy dog. The quick brown fox jumps over the lazy dog.",
        bytes([0, 1, 2, 3]) * 50, b"A" * 200, bytes(range(256)),
    ]


def test_fse_default_bit_exact(zr, oracle):
    for data in _cases(oracle):
        ref = oracle.fse_compress(data)
        got = zr.fse_compress(data)
        assert got == ref, f"compress mismatch n={len(data)}"
        assert zr.fse_decompress(ref) == data


def test_fse_kat_b6_b7(zr):
    assert zr.fse_compress(b"\x78" * 100).hex() == "f5640000000c010078001000000100000000000000"
    assert zr.fse_compress(b"\x78" * 99) == bytes.fromhex("f563000000ff") + b"\x78" * 99


def test_fse_parallel_blocks_bit_exact(zr, oracle):
    z = zr.synth("z", 3 * 1024 * 1024 + 777, seed=3)
    t = zr.synth("t", 1 << 20, seed=1)
    u = oracle.gen_uniform(600000)
    for data in (z, t, u):
        for pb, bs in ((8, 64 * 1024), (8, 16 * 1024), (4, 128 * 1024), (2, 4096), (1, 4096),
                       (8, 1000), (8, 150), (8, 99), (3, 100)):
            if len(data) > 1_100_000 and bs < 4096:
                continue
            cfg = zr.FseConfig(parallel_blocks=pb, block_size=bs)
            oc = oracle.fse_config(parallel_blocks=pb, block_size=bs)
            ref = oracle.fse_compress(data, oc)
            got = zr.fse_compress_with_config(data, cfg)
            assert got == ref, f"parallel mismatch n={len(data)} pb={pb} bs={bs}"
            if pb > 1:
                assert zr.fse_decompress(ref) == data
                assert oracle.fse_decompress(got) == data


def test_fse_presets_and_decoder_independence(zr, oracle):
    data = (b"mismatch test data with skewed frequencies! " * 70)[:3000] + b"z" * 2000
    fox = (b"The quick brown fox jumps over the lazy dog. " * 120)[:5000]
    for mk in (zr.FseConfig.fast_compression, zr.FseConfig.balanced, zr.FseConfig.high_compression,
               zr.FseConfig.realtime):
        cfg = mk()
        for d in (data, fox):
            enc = zr.FseEncoder(cfg).compress(d)
            oc = oracle.fse_config(table_log=cfg.table_log, compression_level=cfg.compression_level,
                                   max_table_size=cfg.max_table_size,
                                   parallel_blocks=cfg.parallel_blocks or 0, block_size=cfg.block_size)
            assert enc == oracle.fse_compress(d, oc)
            assert zr.fse_decompress(enc) == d
            assert zr.fse_decompress_with_config(enc, cfg) == d


def test_fse_config_validation(zr):
    with pytest.raises(zr.ZiporaError):
        zr.FseEncoder(zr.FseConfig(table_log=4))
    with pytest.raises(zr.ZiporaError):
        zr.FseEncoder(zr.FseConfig(table_log=16))
    with pytest.raises(zr.ZiporaError):
        zr.FseEncoder(zr.FseConfig(compression_level=0))
    with pytest.raises(zr.ZiporaError):
        zr.FseEncoder(zr.FseConfig(table_log=15, max_table_size=1024))
    with pytest.raises(zr.ZiporaError):
        zr.FseEncoder(zr.FseConfig(max_symbol=70000))


def test_fse_static_table_and_dictionary(zr, oracle):
    # tests/fse_tests.rs test_fse_unseen_symbol_with_static_table_errors
    e = zr.FseEncoder(zr.FseConfig(adaptive=False))
    train = b"a" * 200
    assert e.compress(train) == oracle.fse_compress(train)
    with pytest.raises(zr.ZiporaError):
        e.compress(b"Z" * 200)
    # a static table reused on data it covers: bit-exact with the oracle given the same table
    e2 = zr.FseEncoder(zr.FseConfig(adaptive=False))
    first = b"abcdefgh" * 100
    e2.compress(first)
    second = b"hgfedcba" * 37 + b"aaaa" * 20
    ref = oracle.fse_compress_freqs(second, oracle.histogram(first))
    assert e2.compress(second) == ref
    assert zr.fse_decompress(ref) == second
    # FseEncoder::with_dictionary: dictionary counts added (fse.rs:807-812)
    dic = b"The quick brown fox jumps over the lazy dog"
    d = b"The lazy dog sleeps while the quick brown fox jumps around. " * 20
    ed = zr.FseEncoder.with_dictionary(zr.FseConfig.high_compression(), dic)
    h = [a + b for a, b in zip(oracle.histogram(d), oracle.histogram(dic))]
    oc = oracle.fse_config(table_log=15, compression_level=19, max_table_size=256 * 1024,
                           parallel_blocks=4, block_size=128 * 1024)
    enc = ed.compress(d)
    assert enc == oracle.fse_compress_freqs(d, h, oc)
    assert zr.fse_decompress(enc) == d


def test_fse_decoder_errors_match_oracle(zr, oracle):
    data = zr.synth("z", 300000, seed=5)
    cfg = oracle.fse_config(parallel_blocks=4, block_size=16384)
    par = oracle.fse_compress(data, cfg)
    single = oracle.fse_compress(data)
    bad = [b"\x00", b"\xf7abc", b"\xf6", b"\xf6\x00\x00\x00\x00", b"\xf6\xff\xff\xff\x7f\x00",
           b"\xf5\x01", b"\xf5\x05\x00\x00\x00\x03", b"\xf5\x05\x00\x00\x00\x0c\x01",
           b"\xf5\x05\x00\x00\x00\xff\x01\x02", b"\xf5\x00\x00\x00\x00",
           b"\xf5\x05\x00\x00\x00\x0c\x00\x00" + bytes(8),
           par[:3], par[:100], single[:50], single[:-1], par[:-7]]
    for s in bad:
        try:
            want = oracle.fse_decompress(s)
        except oracle.OracleError:
            want = None
        try:
            got = zr.fse_decompress(s)
        except zr.ZiporaError:
            got = None
        assert got == want, f"stream {s[:16].hex()} (len {len(s)})"


def test_fse_crafted_fuzz_vs_oracle(zr, oracle):
    rng = random.Random(1234)
    base = [oracle.fse_compress(zr.synth("t", 5000, seed=9)),
            oracle.fse_compress(zr.synth("z", 40000, seed=2), oracle.fse_config(parallel_blocks=4, block_size=8192))]
    for it in range(120):
        s = bytearray(rng.choice(base))
        for _ in range(rng.randint(1, 4)):
            k = rng.randrange(len(s))
            s[k] = rng.randrange(256)
        if rng.random() < 0.3:
            s = s[:rng.randrange(1, len(s))]
        s = bytes(s)
        try:
            size = oracle.fse_decompress(s)
        except oracle.OracleError:
            size = None
        try:
            got = zr.fse_decompress(s)
        except zr.ZiporaError:
            got = None
        assert got == size, f"fuzz case {it}"


def test_fse_device_full_size(zr, oracle):
    """Config 3: 2^28 B Zipf, 0xF6 Some(8), 64 KiB and 16 KiB blocks (bit-exact vs oracle)."""
    import torch
    n = 1 << 28
    data = torch.empty(n, dtype=torch.uint8, device="cuda")
    host = zr.synth("z", n, seed=11)
    data.copy_(torch.frombuffer(bytearray(host), dtype=torch.uint8))
    for bs in (64 * 1024, 16 * 1024):
        cfg = zr.FseConfig(parallel_blocks=8, block_size=bs)
        dev = zr.FseDevice(cfg)
        enc = dev.compress(data)
        ref = oracle.fse_compress(host, oracle.fse_config(parallel_blocks=8, block_size=bs))
        assert enc.numel() == len(ref)
        assert bytes(enc.cpu().numpy().tobytes()) == ref
        dec = dev.decompress(enc, n)
        assert torch.equal(dec, data)


def test_fse_block_states_out_of_range_vs_oracle(zr, oracle):
    """0xF6 streams whose block states were replaced by values outside the
    decoder's bulk range [2^16, 2^48) (0, small, huge) or by random ones: the
    device decode (status and bytes) equals the oracle's. Body layout
    (fse.rs:1026-1044): F6 | nblocks u32 | size u32 x nblocks | bodies, each
    body ending with its u64 state."""
    import struct
    data = zr.synth("z", 40 * 16384 + 777, seed=21)
    par = bytearray(oracle.fse_compress(data, oracle.fse_config(parallel_blocks=4, block_size=16384)))
    assert par[0] == 0xF6
    nb = struct.unpack_from("<I", par, 1)[0]
    sizes = struct.unpack_from(f"<{nb}I", par, 5)
    ends, o = [], 5 + 4 * nb
    for sz in sizes:
        o += sz
        ends.append(o)
    rng = random.Random(77)
    values = [0, 1, 5, 4095, 65535, 65536, (1 << 48) - 1, 1 << 48, (1 << 50) + 123, (1 << 64) - 1]
    for it in range(12):
        s = bytearray(par)
        for b in rng.sample(range(nb), 6):
            v = rng.choice(values) if it % 3 else rng.getrandbits(rng.choice([16, 32, 48, 64]))
            struct.pack_into("<Q", s, ends[b] - 8, v)
        s = bytes(s)
        try:
            want = oracle.fse_decompress(s)
        except oracle.OracleError:
            want = None
        try:
            got = zr.fse_decompress(s)
        except zr.ZiporaError:
            got = None
        assert got == want, f"case {it}"
