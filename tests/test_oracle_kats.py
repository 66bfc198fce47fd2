"""Pins the CPU oracle: SURVEY.md Appendix B known-answer vectors and the
reference's own exact asserts. (No GPU.)"""
import pytest


def h(s):
    return bytes.fromhex(s.replace(" ", ""))


def raw(pairs):
    r = [0] * 256
    for k, v in pairs.items():
        r[k] = v
    return r


# ---------------------------------------------------------------- Appendix B
def test_b1_b2_rans_x1(oracle):
    t = oracle.rans_table(raw({0x61: 1, 0x62: 4095}))
    assert (t.freq[0x61], t.start[0x61], t.freq[0x62], t.start[0x62]) == (2, 0, 4094, 2)
    assert oracle.rans_encode(t, 1, b"ab") == h("22 00 00 08 00 00 00 00 00")
    assert oracle.rans_encode(t, 1, b"ba") == h("00 02 01 08 00 00 00 00 00")
    assert oracle.rans_decode(t, 1, h("22 00 00 08 00 00 00 00 00"), 2) == b"ab"


def test_b3_rans_x1(oracle):
    t = oracle.rans_table(raw({0x61: 1, 0x62: 1}))
    assert oracle.rans_encode(t, 1, b"ab") == h("00 10 04 00 00 00 00 00")


def test_b4_rans_x2(oracle):
    t = oracle.rans_table(raw({0x61: 2, 0x62: 2}))
    assert oracle.rans_encode(t, 2, b"abab") == h(
        "00 00 04 00 00 00 00 00 00 18 04 00 00 00 00 00 00 00 00 00 00 00 00 00")


@pytest.mark.parametrize("n", [1, 2, 4, 8, 4096])
def test_b5_empty(oracle, n):
    t = oracle.rans_table(raw({0x61: 2}))
    assert oracle.rans_encode(t, n, b"") == h("00 00 01 00 00 00 00 00")


def test_b6_b7_fse(oracle):
    assert oracle.fse_compress(b"\x78" * 100) == h(
        "F5 64 00 00 00 0C 01 00 78 00 10 00 00 01 00 00 00 00 00 00 00")
    assert oracle.fse_compress(b"\x78" * 99) == h("F5 63 00 00 00 FF") + b"\x78" * 99


@pytest.mark.parametrize("data,expect", [
    (b"aab", "04"), (b"aaabbc", "80 06"), (b"abc", "18"), (b"abcd", "48 01"),
    (b"aaaaaaaaa", "00 00")])
def test_b8_b12_huffman(oracle, data, expect):
    t = oracle.huff_tree(oracle.histogram(data))
    assert oracle.huff_encode(t, data) == h(expect)
    assert oracle.huff_decode(t, h(expect), len(data)) == data


def test_b9_b11_codes(oracle):
    c = oracle.huff_codes(oracle.huff_tree(oracle.histogram(b"aaabbc")))
    assert c == {0x61: "00", 0x62: "01", 0x63: "1"}
    c = oracle.huff_codes(oracle.huff_tree(oracle.histogram(b"abcd")))
    assert c == {0x61: "000", 0x63: "001", 0x64: "01", 0x62: "1"}


def test_b13_fixed_rank_codes(oracle):
    d = bytes(range(256))
    t = oracle.huff_tree(oracle.histogram(d))
    assert t.max_code_length == 8
    assert oracle.huff_encode(t, d) == d


def test_b14_o1_identity(oracle):
    d = oracle.gen_uniform(5000)
    c = oracle.Ctx(b"training bytes for order one", 1)
    assert c.order == 1
    assert c.encode(d) == d
    assert c.decode(d, len(d)) == d
    for nway in (1, 2, 4, 8):
        e = c.encode_xn(nway, d)
        assert len(e) == len(d)
        assert c.decode_xn(nway, e, len(d)) == d


# ---------------------------------------------------------------- reference asserts
def test_rans_normalize_uniform(oracle):  # rans.rs:734-752
    t = oracle.rans_table(raw({i: 100 for i in range(16)}))
    used = [t.freq[i] for i in range(16)]
    assert sum(t.freq) == 4096 and max(used) - min(used) <= 1


def test_rans_frequency_normalization(oracle):  # rans.rs:882-896
    r = [1] * 256
    r[65], r[66] = 100, 50
    t = oracle.rans_table(r)
    assert t.total_freq == 4096 and all(t.freq[i] > 0 for i in range(256))


def test_rans_roundtrips_reference_cases(oracle):  # rans.rs:811-1039
    cases = [
        (b"hello world, this is a test of enhanced 64-bit rANS encoding", 1),
        (b"parallel encoding test with dual streams", 2),
        (b"quad-stream parallel encoding test with four independent streams for better performance", 4),
        (bytes(((i * 123 + 45) % 256) for i in range(10000)), 8),
    ]
    rep = b"This is a test message for parallel rANS processing with multiple streams to verify correctness across all variants." * 10
    cases += [(rep, n) for n in (1, 2, 4, 8)]
    cases += [(b"a" * 10000, 1), (bytes(i % 256 for i in range(4096)), 1)]
    skew = bytearray(100000)
    skew[50000] = 255
    cases.append((bytes(skew), 1))
    for data, n in cases:
        t = oracle.rans_table(oracle.histogram(data))
        enc = oracle.rans_encode(t, n, data)
        assert oracle.rans_decode(t, n, enc, len(data)) == data


def test_rans_truncation_errors(oracle):  # rans.rs:971-1008
    data = b"hello world 1234567890 parallel test data string for testing truncated stream lengths"
    t = oracle.rans_table(oracle.histogram(data))
    enc = oracle.rans_encode(t, 4, data)
    with pytest.raises(oracle.OracleError):
        oracle.rans_decode(t, 4, enc[:-10], len(data))
    with pytest.raises(oracle.OracleError):
        oracle.rans_decode(t, 4, enc[:40], len(data))


def test_fse_mul_hi_wraps(oracle):  # fse.rs:618-628, wrapping middle sum
    x = (3 << 32) | 0xFFFFFFFE
    true_hi = (x * 0xFFFFFFFFFFFFFFFF) >> 64
    assert oracle.lib().or_fse_mul_hi(x, 0xFFFFFFFFFFFFFFFF) != true_hi
    assert oracle.lib().or_fse_mul_hi(12345, 0xFFFFFFFFFFFFFFFF) == (12345 * 0xFFFFFFFFFFFFFFFF) >> 64


def test_fse_mode_byte_rejects_unknown(oracle):  # tests/fse_tests.rs:822-830
    crafted = bytes([0x02, 0, 0, 0, 5, 0, 0, 0, 5, 0, 0, 0, 1, 2, 3, 4, 5, 1, 2, 3, 4, 5])
    with pytest.raises(oracle.OracleError):
        oracle.fse_decompress(crafted, cap=64)


def test_fse_roundtrips_reference_cases(oracle):  # tests/fse_tests.rs:632-845
    cases = [b"", b"a", b"\xff", b"x" * 99, b"x" * 100, b"x" * 101, bytes(4096), b"\xff" * 500,
             (b"abc" * 333)]
    d = bytearray(4000)
    d += bytes(range(1, 151))
    cases.append(bytes(d))
    d = bytearray(b"\xff" * 4000) + bytes(range(1, 151))
    cases.append(bytes(d))
    cases.append(b"a" * 700 + b"b" * 150 + b"c" * 150 + bytes(range(100)))
    cases.append(bytes(i % 256 for i in range(2048)))
    cases.append(b"".join(bytes([b]) * (b + 1) for b in range(256)))
    u = oracle.gen_uniform(128 + 1000 + 4096 + 70000)
    off = 0
    for sz in (128, 1000, 4096, 70000):
        cases.append(u[off: off + sz])
        off += sz
    for data in cases:
        assert oracle.fse_decompress(oracle.fse_compress(data)) == data
    par = oracle.fse_config(parallel_blocks=4, block_size=1024)
    data = bytes(i % 251 for i in range(16384))
    enc = oracle.fse_compress(data, par)
    assert enc[0] == 0xF6
    assert oracle.fse_decompress(enc) == data


def test_huffman_reference_asserts(oracle):  # huffman/tests.rs:8-29, decoder.rs:175-185
    t = oracle.huff_tree(raw({65: 100}))
    assert t.max_code_length == 1 and oracle.huff_codes(t)[65] == "0"
    t = oracle.huff_tree(raw({65: 100, 66: 50}))
    assert t.max_code_length == 1
    t = oracle.huff_tree(oracle.histogram(b"hello world"))
    enc = oracle.huff_encode(t, b"hello world")
    with pytest.raises(oracle.OracleError):
        oracle.huff_decode(t, enc, 1_000_000)
    data = b"hello world! this is a test message for huffman coding."
    t = oracle.huff_tree(oracle.histogram(data))
    assert oracle.huff_decode(t, oracle.huff_encode(t, data), len(data)) == data


def test_huffman_decode_quirks(oracle):
    t = oracle.huff_tree(oracle.histogram(b"abc"))
    assert oracle.huff_decode(t, b"", 5) == b""  # decoder.rs:91-93: empty input -> Ok(empty)
    with pytest.raises(oracle.OracleError):
        oracle.huff_decode(t, b"\x18", 9)  # length mismatch (decoder.rs:157-163)
