"""Huffman O0 decode on streams whose guessed segment starts do not
resynchronise: the device decoder seeds equal-length code sets on
their boundaries and resolves any other non-synchronising code set with the
parallel segment-map composition (k_huff_map + k_huff_compose) instead of an
in-order walk. Byte-compared with the oracle's decoder (decoder.rs:90-165)."""
import os
import random
import sys
import time

import pytest

import zipora_amd as zr

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle_ffi as O  # noqa: E402

pytestmark = pytest.mark.gpu


def serialize(codes):
    """HuffmanTree::serialize layout (tree.rs:226-262) of {symbol: bit list}."""
    out = bytearray(len(codes).to_bytes(2, "little"))
    for sym, bits in sorted(codes.items()):
        out += bytes([sym, len(bits)])
        for i in range(0, len(bits), 8):
            out.append(sum(b << j for j, b in enumerate(bits[i:i + 8])))
    return bytes(out)


def bits_le(v, n):
    return [(v >> i) & 1 for i in range(n)]


def roundtrip(tree_bytes, data):
    t = zr.HuffmanTree.deserialize(tree_bytes)
    enc = zr.HuffmanEncoder(tree=t).encode(data)
    ot = O.huff_tree_deserialize(tree_bytes)
    assert enc == O.huff_encode(ot, data)
    t0 = time.time()
    dec = zr.HuffmanDecoder(t).decode(enc, len(data))
    dt = time.time() - t0
    assert dec == data
    assert dec == O.huff_decode(ot, enc, len(data))
    return dt


def test_uniform_8_symbols_1mib():
    """8 equiprobable symbols, 1 MiB: the reference's tree for them (max-heap,
    tree.rs:52-133) is a chain, which resynchronises at every 1 bit."""
    rnd = random.Random(8)
    data = bytes(rnd.randrange(8) for _ in range(1 << 20))
    e = zr.HuffmanEncoder(data)
    enc = e.encode(data)
    assert enc == O.huff_encode(O.huff_tree(O.histogram(data)), data)
    assert zr.HuffmanDecoder(e.tree()).decode(enc, len(data)) == data


@pytest.mark.parametrize("k", [3, 5, 6, 7])
def test_fixed_length_codes_seeded(k):
    """A deserialized tree of 2^k codes of k bits (k does not divide the 4096-bit
    segment): every wrong guess stays wrong forever; the starts are seeded on
    multiples of k."""
    codes = {s: bits_le(s, k) for s in range(1 << k)}
    rnd = random.Random(k)
    data = bytes(rnd.randrange(1 << k) for _ in range(1 << 20))
    assert roundtrip(serialize(codes), data) < 20


def test_block_code_resolve():
    """7-bit codes plus 14-bit escape codes ("1111111" + 7 bits): every code
    length is a multiple of 7, so a parse that starts off a boundary never
    finds one, and the lengths differ, so no equal-length seeding: the guessed
    starts t*4096 (t mod 7 of them misaligned in a row) stay wrong past the
    four synchronisation rounds and the parallel resolve must place them."""
    codes = {s: bits_le(s, 7) for s in range(127)}
    for j, s in enumerate(range(127, 255)):
        codes[s] = [1] * 7 + bits_le(j, 7)
    rnd = random.Random(77)
    data = bytes(rnd.choice(range(255)) for _ in range(1 << 20))
    assert roundtrip(serialize(codes), data) < 20
