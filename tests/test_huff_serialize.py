"""Serialized Huffman trees and the HuffmanCompressor record (tree.rs:226-356,
compression/mod.rs:320-408).

The reference serializes by walking a HashMap, so its bytes vary between runs.
Here serialize writes ascending symbols (canonical); tests compare bytes in the
canonical order and, for other orders, the decoded trees' behaviour."""
import random
import struct

import pytest


def _freq_cases(zr):
    text = zr.synth("t", 4000, seed=2)
    z = zr.synth("z", 8000, seed=3)
    f_chain = [0] * 256
    for i, s in enumerate(b"abcdefgh"):
        f_chain[s] = 1 << i  # a long chain code
    f_fixed = [1] * 256  # > 64-deep chain -> fixed 8-bit rank codes with placeholders
    f_fixed[7] = 0
    f_one = [0] * 256
    f_one[65] = 9
    return [list(__import__("numpy").bincount(__import__("numpy").frombuffer(d, dtype="uint8"), minlength=256))
            for d in (text, z, b"aab", b"hello world")] + [f_chain, f_fixed, f_one, [0] * 256]


def test_oracle_serialize_known_answer(oracle):
    # freq a=2, b=1: the max-heap pops a first -> a = "0", b = "1" (tree.rs:93-111)
    f = [0] * 256
    f[ord("a")], f[ord("b")] = 2, 1
    t = oracle.huff_tree(f)
    assert oracle.huff_tree_serialize(t) == bytes([2, 0, 0x61, 1, 0x00, 0x62, 1, 0x01])
    back = oracle.huff_tree_deserialize(oracle.huff_tree_serialize(t))
    assert oracle.huff_codes(back) == oracle.huff_codes(t)
    assert oracle.huff_tree_serialize(oracle.huff_tree([0] * 256)) == b"\x00\x00"
    with pytest.raises(oracle.OracleError):
        oracle.huff_tree_deserialize(b"\x01")
    with pytest.raises(oracle.OracleError):
        oracle.huff_tree_deserialize(bytes([1, 0, 0x61, 9, 0xFF]))  # 9-bit code needs 2 bytes


def test_oracle_roundtrip_any_order(zr, oracle):
    rnd = random.Random(5)
    for f in _freq_cases(zr):
        t = oracle.huff_tree([int(x) for x in f])
        ser = oracle.huff_tree_serialize(t)
        data = bytes(s for s in range(256) if f[s]) * 3
        enc = oracle.huff_encode(t, data) if data else b""
        for _ in range(3):
            order = list(range(256))
            rnd.shuffle(order)
            back = oracle.huff_tree_deserialize(ser, order)
            if data:
                assert oracle.huff_decode(back, enc, len(data)) == data


@pytest.mark.gpu
def test_tree_serialize_parity(zr, oracle):
    rnd = random.Random(9)
    for f in _freq_cases(zr):
        f = [int(x) for x in f]
        t = zr.HuffmanTree.from_frequencies(f)
        ot = oracle.huff_tree(f)
        ser = t.serialize()
        assert ser == oracle.huff_tree_serialize(ot)
        back = zr.HuffmanTree.deserialize(ser)
        assert [back.raw.code_len[s] for s in range(256)] == [ot.code_len[s] for s in range(256)]
        data = bytes(s for s in range(256) if f[s]) * 5
        if not data:
            continue
        enc = oracle.huff_encode(ot, data)
        dec = zr.HuffmanDecoder(back).decode(enc, len(data))
        assert dec == data
        # the same codes listed in another (HashMap-like) order deserialize alike
        entries, o = [], 2
        for _ in range(struct.unpack("<H", ser[:2])[0]):
            L = ser[o + 1]
            nb = (L + 7) // 8
            entries.append(ser[o:o + 2 + nb])
            o += 2 + nb
        rnd.shuffle(entries)
        shuffled = ser[:2] + b"".join(entries)
        assert zr.HuffmanDecoder(zr.HuffmanTree.deserialize(shuffled)).decode(enc, len(data)) == data


@pytest.mark.gpu
def test_tree_deserialize_errors(zr, oracle):
    for bad in (b"", b"\x01", bytes([1, 0, 0x61]), bytes([1, 0, 0x61, 9, 0xFF]),
                bytes([2, 0, 0x61, 1, 0x00, 0x62, 2, 0x00])):  # the last: a = "0" blocks b = "00"
        with pytest.raises(oracle.OracleError):
            oracle.huff_tree_deserialize(bad)
        with pytest.raises(zr.ZiporaError):
            zr.HuffmanTree.deserialize(bad)


@pytest.mark.gpu
def test_tree_deserialize_overwrite(zr, oracle):
    """An empty remaining code replaces the node it reaches (tree.rs:360-366): b = "0"
    after a = "0" overwrites a without an error, as in the reference."""
    ser = bytes([2, 0, 0x61, 1, 0x00, 0x62, 1, 0x00])
    ot = oracle.huff_tree_deserialize(ser)
    t = zr.HuffmanTree.deserialize(ser)
    enc = bytes([0b0110])
    assert zr.HuffmanDecoder(t).decode(enc, 3) == oracle.huff_decode(ot, enc, 3)


@pytest.mark.gpu
def test_huffman_compressor_records(zr, oracle):
    for train, data in ((zr.synth("t", 20000, seed=1), None), (b"aab", b"abba"), (b"x", b"xxxx"),
                        (bytes(range(256)) * 2 + b"\x00" * 50, bytes(range(200)))):
        data = data if data is not None else train[:3000]
        c = zr.HuffmanCompressor(train)
        ot = oracle.huff_tree(oracle.histogram(train))
        rec = c.compress(data)
        assert rec == oracle.huff_compressor_compress(ot, data)
        assert c.decompress(rec) == oracle.huff_compressor_decompress(rec) == data
        assert c.tree_data() == oracle.huff_tree_serialize(ot)
    c = zr.HuffmanCompressor(b"abc")
    assert c.compress(b"") == b"" and c.decompress(b"") == b""
    for bad in (b"\x01\x02\x03", struct.pack("<I", 100) + b"\x00" * 10):
        with pytest.raises(zr.ZiporaError):
            c.decompress(bad)
        with pytest.raises(oracle.OracleError):
            oracle.huff_compressor_decompress(bad)
    with pytest.raises(zr.ZiporaError):
        c.compress(b"abd")  # 'd' is not in the tree


def _ctx_cases(zr):
    text = zr.synth("t", 30000, seed=8)
    return [(text, 0), (text, 1), (text, 2), (b"ab", 2), (b"a", 1), (b"", 0), (bytes(range(256)) * 3, 2),
            (zr.synth("u", 300000, seed=9), 2)]  # > 1024 order-2 contexts: the top-1024 cut


def test_oracle_ctx_serialize_layout(zr, oracle):
    c = oracle.Ctx(b"abcab", 1)
    ser = c.serialize()
    order, ntrees, nctx = ser[0], *struct.unpack("<II", ser[1:9])
    assert (order, ntrees, nctx) == (1, 4, 3)  # contexts a, b, c precede a symbol
    pairs = [struct.unpack("<II", ser[9 + 8 * k:17 + 8 * k]) for k in range(nctx)]
    assert pairs == [(0x61, 1), (0x62, 2), (0x63, 3)]


@pytest.mark.gpu
def test_ctx_serialize_parity(zr, oracle):
    for train, order in _ctx_cases(zr):
        enc = zr.ContextualHuffmanEncoder(train, order)
        ser = enc.serialize()
        assert ser == oracle.Ctx(train, order).serialize(), (len(train), order)
        back = zr.ContextualHuffmanEncoder.deserialize(ser)
        assert back.order() == enc.order()
        assert back.serialize() == ser
        data = train[:5000]
        if data:  # (drawn from the training bytes: every symbol has a code)
            e = enc.encode(data)
            assert back.encode(data) == e
            assert zr.ContextualHuffmanDecoder(back).decode(e, len(data)) == data


@pytest.mark.gpu
def test_ctx_deserialize_errors(zr):
    good = zr.ContextualHuffmanEncoder(b"hello world", 1).serialize()
    for bad in (b"", b"\x03" + good[1:], good[:3], good[:8], good[:12], good[:-1]):
        with pytest.raises(zr.ZiporaError):
            zr.ContextualHuffmanEncoder.deserialize(bad)
