"""Huffman tree construction (H1) is host code in libzipora_amd.so: parity with
the oracle's BinaryHeap restatement, no GPU needed."""
import random


def walk(children, syms, is_leaf, bits):
    """Decode one code (bits: list of 0/1) from the root; returns (symbol, used)."""
    cur, used = 0, 0
    while not is_leaf(cur):
        cur = children(cur)[bits[used]]
        used += 1
    return syms(cur), used


def _mine(t):
    return (lambda i: (t.child[i][0], t.child[i][1])), (lambda i: t.sym[i]), (lambda i: t.child[i][0] < 0)


def _oracle(t):
    return (lambda i: (t.node_child[i][0], t.node_child[i][1])), (lambda i: t.node_sym[i]), \
        (lambda i: bool(t.node_leaf[i]))


def _freq_cases():
    rng = random.Random(5)
    cases = [[0] * 256, [0] * 97 + [5] + [0] * 158, [1] * 256, list(range(256)), [1 << 20] * 66 + [0] * 190]
    for _ in range(300):
        k = rng.choice([1, 2, 3, 5, 10, 40, 65, 66, 70, 128, 200, 256])
        f = [0] * 256
        for s in rng.sample(range(256), k):
            f[s] = rng.choice([1, 2, 3, rng.randrange(1, 1000), rng.randrange(1, 1 << 31)])
        cases.append(f)
    return cases


def test_tree_codes_match_oracle(zr, oracle):
    for f in _freq_cases():
        t = zr.HuffmanTree.from_frequencies(f).raw
        o = oracle.huff_tree(f)
        assert (t.kind, t.n_symbols, t.max_code_length) == (o.kind, o.n_symbols, o.max_code_length)
        for s in range(256):
            assert (t.code_len[s], t.code[s]) == (o.code_len[s], o.code[s])


def test_decode_tree_matches_oracle(zr, oracle):
    rng = random.Random(9)
    for f in _freq_cases():
        t = zr.HuffmanTree.from_frequencies(f).raw
        o = oracle.huff_tree(f)
        if t.kind != 2:
            continue
        for _ in range(64):  # random bit strings decode to the same symbol / length
            bits = [rng.randrange(2) for _ in range(70)]
            assert walk(*_mine(t), bits) == walk(*_oracle(o), bits)
        for s in range(256):
            if t.code_len[s]:
                bits = [(t.code[s] >> j) & 1 for j in range(t.code_len[s])] + [0]
                assert walk(*_mine(t), bits) == (s, t.code_len[s])


def test_reference_tree_asserts(zr):
    # huffman/tests.rs:8-29: single symbol -> code [false]; two symbols -> max length 1
    t = zr.HuffmanTree.from_data(b"aaaa")
    assert t.get_code(ord("a")) == [False] and t.max_code_length() == 1
    t = zr.HuffmanTree.from_data(b"aabb")
    assert t.max_code_length() == 1
    assert zr.HuffmanTree.from_data(b"").max_code_length() == 0
    # Appendix B9-B11: aaabbc -> a=00 b=01 c=1 (most frequent longest)
    t = zr.HuffmanTree.from_data(b"aaabbc")
    assert t.get_code(ord("a")) == [False, False]
    assert t.get_code(ord("b")) == [False, True]
    assert t.get_code(ord("c")) == [True]


def test_contextual_orders(zr):
    assert zr.ContextualHuffmanEncoder(b"ab", zr.HuffmanOrder.Order1).order() == zr.HuffmanOrder.Order1
    assert zr.ContextualHuffmanEncoder(b"a", zr.HuffmanOrder.Order1).order() == zr.HuffmanOrder.Order0
    assert zr.ContextualHuffmanEncoder(b"ab", zr.HuffmanOrder.Order2).order() == zr.HuffmanOrder.Order1
    assert zr.ContextualHuffmanEncoder(b"abc", zr.HuffmanOrder.Order2).order() == zr.HuffmanOrder.Order2
