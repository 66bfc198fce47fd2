"""Huffman parity on the MI355X: zr_huff.hip through the C ABI vs the oracle, bit-exact.

Covers huffman/tests.rs-style inputs, chain codes (most frequent symbol
longest), the fixed 8-bit fallback (>= 66 symbols), the single-symbol tree,
decoder length/plausibility errors, fuzzed streams, and the contextual
order-1/2 coder with 1/2/4/8-way interleaving.
"""
import random

import pytest

pytestmark = pytest.mark.gpu


def _inputs(zr, oracle):
    rng = random.Random(3)
    chain = b"".join(bytes([65 + i]) * (1 << i) for i in range(20))  # codes up to 19 bits
    skew = b"".join(bytes([i]) * max(1, int(1.9 ** i)) for i in range(22))  # long chain codes
    return [
        b"a", b"ab", b"aab", b"aaabbc", b"abc", b"abcd", b"aaaaaaaaa", b"hello world",
        b"The quick brown fox jumps over the lazy dog",
        bytes(range(256)), bytes(range(65)) * 3, bytes(range(66)) * 3, chain, skew,
        zr.synth("t", 100000, seed=1), zr.synth("z", 200000, seed=2), oracle.gen_uniform(50000),
        bytes(rng.randrange(256) for _ in range(3000)), b"x" * 70000,
    ]


def test_huff_o0_encode_decode_bit_exact(zr, oracle):
    for d in _inputs(zr, oracle):
        f = oracle.histogram(d)
        t = oracle.huff_tree(f)
        ref = oracle.huff_encode(t, d)
        enc = zr.HuffmanEncoder(d)
        got = enc.encode(d)
        assert got == ref, f"encode mismatch n={len(d)}"
        assert zr.HuffmanDecoder(enc.tree()).decode(ref, len(d)) == d


def test_huff_o0_1mib_text(zr, oracle):
    d = zr.synth("t", 1 << 20, seed=7)
    t = oracle.huff_tree(oracle.histogram(d))
    ref = oracle.huff_encode(t, d)
    enc = zr.HuffmanEncoder(d)
    assert enc.encode(d) == ref
    assert zr.HuffmanDecoder(enc.tree()).decode(ref, len(d)) == d


def test_huff_o0_missing_symbol_errors(zr):
    f = [0] * 256
    f[ord("a")] = 3
    f[ord("b")] = 1
    enc = zr.HuffmanEncoder.from_frequencies(f)
    with pytest.raises(zr.ZiporaError):
        enc.encode(b"abc")
    assert enc.encode(b"") == b""


def _dec(zr, oracle, tree_freq, stream, n):
    t = oracle.huff_tree(tree_freq)
    try:
        want = oracle.huff_decode(t, stream, n)
    except oracle.OracleError:
        want = None
    try:
        got = zr.HuffmanDecoder(zr.HuffmanTree.from_frequencies(tree_freq)).decode(stream, n)
    except zr.ZiporaError:
        got = None
    return got, want


def test_huff_o0_decoder_edges(zr, oracle):
    d = b"aaabbc" * 50
    f = oracle.histogram(d)
    enc = oracle.huff_encode(oracle.huff_tree(f), d)
    cases = [(enc, len(d)), (enc, len(d) + 1), (enc, len(d) + 50), (enc[:-1], len(d)), (enc, 1), (enc, 0),
             (b"", 5), (enc + b"\xff\xff", len(d)), (enc, 64 * len(enc) + 1), (enc[:1], 64)]
    for s, n in cases:
        got, want = _dec(zr, oracle, f, s, n)
        assert got == want, (len(s), n)
    # single-symbol tree: one symbol per bit plus the final fix-up
    f1 = oracle.histogram(b"zzzz")
    for n in (1, 8, 9, 10, 16, 17, 18):
        got, want = _dec(zr, oracle, f1, b"\x00\x00", n)
        assert got == want, n
    # fixed 8-bit tree (>= 66 symbols) incl. placeholder codes
    ff = oracle.histogram(bytes(range(70)))
    for s in (bytes(range(256)), bytes([255, 200, 69, 70, 0])):
        got, want = _dec(zr, oracle, ff, s, len(s))
        assert got == want


def test_huff_o0_decode_fuzz(zr, oracle):
    rng = random.Random(11)
    for it in range(60):
        d = zr.synth("t", rng.randrange(1, 5000), seed=it)
        f = oracle.histogram(d)
        s = bytearray(oracle.huff_encode(oracle.huff_tree(f), d))
        for _ in range(rng.randrange(0, 4)):
            if s:
                s[rng.randrange(len(s))] = rng.randrange(256)
        n = len(d) + rng.choice([0, 0, 0, -1, 1, 5])
        got, want = _dec(zr, oracle, f, bytes(s), max(0, n))
        assert got == want, it


@pytest.mark.parametrize("order", [1, 2])
def test_contextual_bit_exact(zr, oracle, order):
    for d in (zr.synth("t", 200000, seed=4), b"ab", b"abc", bytes(range(256)) * 3, b"q" * 1000):
        oc = oracle.Ctx(d, order)
        ec = zr.ContextualHuffmanEncoder(d, order)
        assert int(ec.order()) == oc.order
        ref = oc.encode(d)
        assert ec.encode(d) == ref
        assert zr.ContextualHuffmanDecoder(ec).decode(ref, len(d)) == d
        if oc.order == 1:
            for nw in (1, 2, 4, 8):
                r = oc.encode_xn(nw, d)
                assert ec.encode_with_interleaving(d, nw) == r, nw
                assert ec.decode_with_interleaving(r, len(d), nw) == d


def test_contextual_order0_fallback_and_errors(zr, oracle):
    ec = zr.ContextualHuffmanEncoder(b"a", zr.HuffmanOrder.Order1)  # order 0 over b"a"
    oc = oracle.Ctx(b"a", 1)
    assert oc.order == 0 and int(ec.order()) == 0
    assert ec.encode(b"aaaa") == oc.encode(b"aaaa")
    with pytest.raises(zr.ZiporaError):
        ec.encode_x2(b"aaaa")
    e2 = zr.ContextualHuffmanEncoder(b"abcd", zr.HuffmanOrder.Order2)
    with pytest.raises(zr.ZiporaError):
        e2.encode_x4(b"abcd")
    e1 = zr.ContextualHuffmanEncoder(b"abcd", zr.HuffmanOrder.Order1)
    with pytest.raises(zr.ZiporaError):
        zr.ContextualHuffmanDecoder(e1).decode(b"abc", 4)
    assert zr.ContextualHuffmanDecoder(e1).decode(b"", 4) == b""
    assert e1.decode_x4(b"", 10) == b""
    with pytest.raises(zr.ZiporaError):
        e1.decode_x4(b"abc", 10)


def test_contextual_device_full_size(zr):
    """Config 4 shard: 128 MiB text-like, order 1 identity coding + 8-way transpose (property)."""
    import torch
    n = 128 << 20
    d = torch.frombuffer(bytearray(zr.synth("t", n, seed=5)), dtype=torch.uint8).cuda()
    ec = zr.ContextualHuffmanEncoder(b"train", zr.HuffmanOrder.Order1)
    dev = zr.HuffmanO1Device(ec)
    enc = torch.empty_like(d)
    out = torch.empty_like(d)
    dev.encode_async(d, enc)
    dev.decode_async(enc, out, n)
    torch.cuda.synchronize()
    assert torch.equal(enc, d) and torch.equal(out, d)
    dev.encode_async(d, enc, 8)
    dev.decode_async(enc, out, n, 8)
    torch.cuda.synchronize()
    assert torch.equal(out, d)
    q = n // 8
    assert torch.equal(enc.view(q, 8)[:, 3], d[3 * q:4 * q])
