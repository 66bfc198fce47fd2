"""The reference's own exact asserts for this path, ported as tests of the HIP
path through the C ABI (the reference holds no codec byte vectors; these
asserts are the byte-level facts it does hold).

  huffman/tests.rs:630-705   BitStreamWriter/Reader LSB-first bytes
  fse.rs:1369-1394           histogram == naive count on its exact input/lengths
  rans.rs:755-764            Rans64State::new() == RANS64_L (65536)
  rans.rs:767-779            Rans64Symbol::new(10, 5).fast_div(1000) == (200, 0)
  rans.rs:786-809            fast_div == hardware division, every freq
  fse.rs:1464-1474           FastDivision::new(7) (CPU only, see its test)

The Huffman writer/reader is not a separate object in this backend: the
encoder packs the concatenated codes LSB-first (encoder.rs:108-129) and the
decoder reads them back the same way (decoder.rs:112-148). Each bit pattern the
reference writes is therefore produced by a symbol sequence whose codes
concatenate to exactly those bits, and the encoded bytes must equal the bytes
the reference's assert names.
"""
import pytest

import zipora_amd as zr

gpu = pytest.mark.gpu


# --------------------------------------------------------------------------
# helpers (test-side restatements, not product code)
# --------------------------------------------------------------------------
def pack_lsb_first(writes):
    """BitStreamWriter::write(value, bits) ... finish() (encoder.rs:27-66):
    bit i of each value goes out i-th, bytes fill from bit 0, the last byte is
    zero-padded."""
    acc, n, out = 0, 0, bytearray()
    for value, bits in writes:
        for i in range(bits):
            acc |= ((value >> i) & 1) << n
            n += 1
            if n == 8:
                out.append(acc)
                acc, n = 0, 0
    if n:
        out.append(acc)
    return bytes(out)


def bits_of(writes):
    return [(v >> i) & 1 for v, b in writes for i in range(b)]


def parse_codes(tree, bits):
    """The symbol sequence whose codes (tree.get_code) concatenate to `bits`."""
    codes = {}
    for s in range(256):
        c = tree.get_code(s)
        if c is not None:
            codes[tuple(int(b) for b in c)] = s
    out, cur = [], []
    for b in bits:
        cur.append(b)
        if tuple(cur) in codes:
            out.append(codes[tuple(cur)])
            cur = []
    assert not cur, "bit pattern does not end on a code boundary"
    return bytes(out)


def chain_tree(n):
    """n equal-frequency symbols 0..n-1: the max-heap chain shape (tree.rs:52-133)."""
    f = [0] * 256
    for i in range(n):
        f[i] = 1
    return zr.HuffmanTree.from_frequencies(f)


def fixed_tree():
    """all 256 symbols: the fixed 8-bit rank code (tree.rs:122-126, :136-175)."""
    return zr.HuffmanTree.from_frequencies([1] * 256)


# --------------------------------------------------------------------------
# huffman/tests.rs:630-705
# --------------------------------------------------------------------------
@gpu
def test_bitstream_writer_basic():
    # writer.write(0b10101010, 8) -> [0b10101010]
    t = fixed_tree()
    assert t.get_code(0xAA) == [bool((0xAA >> i) & 1) for i in range(8)]
    enc = zr.HuffmanEncoder(tree=t).encode(bytes([0xAA]))
    assert enc == bytes([0b10101010])
    assert zr.HuffmanDecoder(t).decode(enc, 1) == bytes([0xAA])


@gpu
def test_bitstream_writer_partial_byte():
    # writer.write(0b1010, 4) -> [0b1010]
    t = chain_tree(3)
    syms = parse_codes(t, bits_of([(0b1010, 4)]))
    enc = zr.HuffmanEncoder(tree=t).encode(syms)
    assert enc == bytes([0b1010]) == pack_lsb_first([(0b1010, 4)])
    assert zr.HuffmanDecoder(t).decode(enc, len(syms)) == syms


@gpu
def test_bitstream_writer_multiple_writes():
    # write(0b1010, 4); write(0b0101, 4) -> [0b01011010] (LSB first). The last
    # bit is a 0 that no code of the tree ends on: the sequence stops one bit
    # short and the encoder's zero padding supplies it (encoder.rs:123-129).
    t = chain_tree(3)
    bits = bits_of([(0b1010, 4), (0b0101, 4)])
    assert bits[-1] == 0
    syms = parse_codes(t, bits[:-1])
    enc = zr.HuffmanEncoder(tree=t).encode(syms)
    assert enc == bytes([0b01011010]) == pack_lsb_first([(0b1010, 4), (0b0101, 4)])
    assert zr.HuffmanDecoder(t).decode(enc, len(syms)) == syms


@gpu
def test_bitstream_reader_basic_and_partial():
    # reader over [0b10101010]: read(8) == 0b10101010; read(4), read(4) == 0b1010, 0b1010
    data = bytes([0b10101010])
    assert zr.HuffmanDecoder(fixed_tree()).decode(data, 1) == data
    t = chain_tree(3)
    nib = parse_codes(t, bits_of([(0b1010, 4)]))
    assert zr.HuffmanDecoder(t).decode(data, 2 * len(nib)) == nib + nib


@gpu
def test_bitstream_roundtrip():
    # write (0b101,3) (0b11110000,8) (0b1,1) (0b111111,6); read them back
    writes = [(0b101, 3), (0b11110000, 8), (0b1, 1), (0b111111, 6)]
    t = chain_tree(4)
    syms = parse_codes(t, bits_of(writes))
    enc = zr.HuffmanEncoder(tree=t).encode(syms)
    assert enc == pack_lsb_first(writes)
    dec = zr.HuffmanDecoder(t).decode(enc, len(syms))
    assert dec == syms
    # and the read-back values: the bits of the decoded codes, in order
    got = [int(b) for s in dec for b in t.get_code(s)]
    pos = 0
    for value, nb in writes:
        v = sum(got[pos + i] << i for i in range(nb))
        assert v == value
        pos += nb


# --------------------------------------------------------------------------
# fse.rs:1369-1394: counts == naive count, exact input and lengths
# --------------------------------------------------------------------------
def _fse_hist_input():
    data = bytearray([0xAB] * 100)            # long equal-byte run
    data += bytes(range(256))                 # every symbol once
    data += bytes((i * 31 % 251) for i in range(1000))  # pseudo-random
    return bytes(data)


HIST_LENS = [0, 1, 3, 63, 64, 65, 67, None]


@gpu
@pytest.mark.parametrize("ln", HIST_LENS)
def test_fse_histogram_matches_naive_count(ln):
    """k_fse_hist (FseEncoder::analyze_frequencies' counting) on the device."""
    import ctypes
    data = _fse_hist_input()
    sl = data[:len(data) if ln is None else ln]
    expected = [0] * 256
    for b in sl:
        expected[b] += 1
    freqs = (ctypes.c_uint32 * 256)()
    buf = (ctypes.c_uint8 * max(1, len(sl))).from_buffer_copy(sl or b"\0")
    assert zr.load().zr_byte_histogram(buf, len(sl), freqs) == 0
    assert list(freqs) == expected


@gpu
@pytest.mark.parametrize("ln", [x for x in HIST_LENS if x != 0])
def test_rans_device_histogram_matches_naive_count(ln):
    """k_hist / k_hist_small (the rANS pipeline's histogram) on the same input."""
    import torch
    from zipora_amd.device import RansDeviceBatch
    data = _fse_hist_input()
    sl = data[:len(data) if ln is None else ln]
    expected = [0] * 256
    for b in sl:
        expected[b] += 1
    for N in (1, 4096):
        bt = RansDeviceBatch([len(sl)], N, shared_table=True)
        raw = bt.new_raw()
        raw[:len(sl)] = torch.frombuffer(bytearray(sl), dtype=torch.uint8).cuda()
        bt.histogram(raw)
        torch.cuda.synchronize()
        assert [int(v) for v in bt.hist.cpu().tolist()] == expected


# --------------------------------------------------------------------------
# rans.rs:755-809
# --------------------------------------------------------------------------
@gpu
@pytest.mark.parametrize("N", [1, 2, 4, 8, 4096])
def test_rans_initial_state_is_rans64_l(N):
    """Rans64State::new().state() == RANS64_L (rans.rs:755-764): the encoder's
    empty-input output is that state, u64 LE (rans.rs:339-344)."""
    enc = zr.Rans64Encoder([1] * 256, N)
    assert enc.encode(b"") == (65536).to_bytes(8, "little")


@gpu
def test_rans_symbol_fast_div_1000_by_5():
    """Rans64Symbol::new(10, 5): start 10, freq 5, fast_div(1000) == (200, 0) (rans.rs:767-779)."""
    sym = zr.Rans64Symbol(10, 5)
    assert (sym.start, sym.freq) == (10, 5)
    assert sym.fast_div(1000) == (200, 0)


@gpu
def test_rans_fast_div_matches_hardware_division():
    """rans.rs:786-809: every freq 1..=TOTFREQ, the reference's x list. The
    values below 2^24 go through the encoder's 24-bit reciprocal division."""
    M = (1 << 64) - 1
    bad = []
    for f in range(1, 4097):
        xs = [0, 1, f - 1, f, f + 1, 1000, 65536, 65536 * f, (1 << 32) - 1, M // f, M - 1, M]
        got = zr.Rans64Symbol(0, f).fast_div(xs)
        for x, (q, r) in zip(xs, got):
            if (q, r) != divmod(x, f):
                bad.append((f, x, q, r))
    assert not bad, bad[:5]


@gpu
def test_rans_fast_div_zero_and_large_freq():
    """fast_div's other inputs (rans.rs:137-152): freq 0 returns (0, 0) for every
    x (the early return at :138-140); a freq above TOTFREQ (Rans64Symbol::new
    takes any u32) divides exactly, as the 64-bit reciprocal does."""
    M = (1 << 64) - 1
    xs = [0, 1, 4095, 65536, (1 << 24) - 1, 1 << 24, M // 3, M]
    assert zr.Rans64Symbol(0, 0).fast_div(xs) == [(0, 0)] * len(xs)
    for f in (4097, 65537, (1 << 31) + 1, (1 << 32) - 1):
        assert zr.Rans64Symbol(0, f).fast_div(xs) == [divmod(x, f) for x in xs], f


# --------------------------------------------------------------------------
# fse.rs:1464-1474 -- CPU restatement only: FseTable builds a FastDivision of
# the frequency total (fse.rs:480) but no coding step ever calls it, so the
# device path has no counterpart; the restatement pins the helper's semantics.
# --------------------------------------------------------------------------
def _fast_division(divisor):
    """FastDivision::new (fse.rs:55-78)."""
    if divisor == 0:
        return 1, 0, 0
    shift = 32 - (32 - divisor.bit_length())  # 32 - leading_zeros
    mult = -(-(1 << (32 + shift)) // divisor)  # div_ceil
    return divisor, mult, shift


def test_fast_division_7():
    d, m, sh = _fast_division(7)
    for i in range(100):
        q = i if d <= 1 else (i * m) >> (32 + sh)  # divide (fse.rs:81-87)
        assert q == i // 7
        assert i - q * d == i % 7  # modulo (fse.rs:90-93)


# --------------------------------------------------------------------------
# fse.rs:1612-1618 and fse.rs:1621-1635: the FSE decoder's tail
# --------------------------------------------------------------------------
def test_fse_truncated_input_decoding_oracle(oracle):
    """fse.rs:1612-1618: FseDecoder::new().decompress(&[0u8; 3]) is an error
    (mode byte 0x00 is neither 0xF5 nor 0xF6)."""
    with pytest.raises(oracle.OracleError):
        oracle.fse_decompress(bytes(3))


@gpu
def test_fse_truncated_input_decoding():
    """fse.rs:1612-1618 through the C ABI."""
    with pytest.raises(zr.ZiporaError):
        zr.fse_decompress(bytes(3))


def test_fse_renormalize_decode_single_byte_steps(oracle):
    """fse.rs:1621-1635: with 2 bytes left (< BLOCK_SIZE = 4) renormalize_decode
    of state 100 reads one byte: Some(_), pos 2 -> 1. The state is then
    (100 << 8) | input[1] (fse.rs:726-729)."""
    x, pos = oracle.fse_renormalize_decode(100, bytes([0x12, 0x34]), 2)
    assert pos == 1
    assert x == (100 << 8) | 0x34
    # and the other branches of fse.rs:712-733: a word read, no read at pos 0,
    # no read at x >= 2^16, the max(x, 1) floor
    x, pos = oracle.fse_renormalize_decode(100, bytes([1, 2, 3, 4, 5]), 5)
    assert (x, pos) == ((100 << 32) | 0x05040302, 1)
    assert oracle.fse_renormalize_decode(100, bytes([7]), 0) == (100, 0)
    assert oracle.fse_renormalize_decode(1 << 16, bytes([7, 8]), 2) == (1 << 16, 2)
    assert oracle.fse_renormalize_decode(0, b"", 0) == (1, 0)
    # pos past the input: a word position beyond len shifts the state
    # and reads nothing (fse.rs:722-726's `*pos + BLOCK_SIZE <= input.len()`);
    # a one-byte read past it indexes out of bounds, which panics in the reference
    assert oracle.fse_renormalize_decode(100, bytes([1, 2, 3]), 9) == (100 << 32, 5)
    x, pos = oracle.fse_renormalize_decode(100, bytes([1, 2, 3, 4, 5, 6]), 7)
    assert (x, pos) == ((100 << 32), 3)
    with pytest.raises(oracle.OracleError):
        oracle.fse_renormalize_decode(100, bytes([1]), 3)


def _f5_with_word_area(words, state, orig_len, nsym=256):
    """A crafted 0xF5 stream (fse.rs:887-966 layout): F5 | len u32 | 12 |
    nsym u16 | (sym u8, freq u32) x nsym | word area | state u64, with the
    uniform normalised table (4096 / nsym per symbol) and the given word area."""
    import struct
    f = 4096 // nsym
    hdr = bytes([0xF5]) + struct.pack("<IBH", orig_len, 12, nsym)
    tab = b"".join(struct.pack("<BI", s, f) for s in range(nsym))
    return hdr + tab + bytes(words) + struct.pack("<Q", state)


@gpu
def test_fse_decode_last_bytes_path_vs_oracle(oracle):
    """k_fse_dec through renormalize_decode's single-byte branch (fse.rs:726-729):
    word areas of 1, 2, 3, 5, 6 and 7 bytes, so that the last renormalisations
    of the stream read single bytes with 3, 2 and 1 bytes left (the fse.rs:1621-1635
    case is the 2-byte area). Status and bytes equal the oracle's."""
    import random
    rng = random.Random(1635)
    cases = 0
    for area in (1, 2, 3, 5, 6, 7):
        for nsym in (256, 16, 2):
            for _ in range(4):
                words = bytes(rng.randrange(256) for _ in range(area))
                # small states renormalise at once; 2^16.. states after a few symbols
                state = rng.choice([100, 1, 0, 4095, 65535, rng.randrange(1 << 16, 1 << 24),
                                    rng.randrange(1 << 24, 1 << 48)])
                n = rng.choice([1, 2, 3, 8, 40])
                s = _f5_with_word_area(words, state, n, nsym)
                try:
                    want = oracle.fse_decompress(s)
                except oracle.OracleError:
                    want = None
                try:
                    got = zr.fse_decompress(s)
                except zr.ZiporaError:
                    got = None
                assert got == want, f"area {area} nsym {nsym} state {state} n {n}"
                cases += want is not None
    assert cases > 0
