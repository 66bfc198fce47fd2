"""The entropy facade (src/entropy/mod.rs:56-330): EntropyAlgorithm,
EntropyConfig presets, EntropyStats. The CPU tests are the reference's own
tests (mod.rs:322-372) and the decision table on given counts; the GPU tests
count bytes with the device histogram and compare select_for_data with a
restatement of mod.rs:124-153 over numpy counts."""
import math
import random

import numpy as np
import pytest

from zipora_amd.entropy import EntropyAlgorithm as A
from zipora_amd.entropy import EntropyConfig, EntropyStats, entropy_from_counts


def test_entropy_stats_calculation():  # mod.rs:327-336
    s = EntropyStats.new(1000, 600, 4.5)
    assert s.input_size == 1000 and s.output_size == 600
    assert abs(s.compression_ratio - 0.6) < 0.001
    assert abs(s.bits_per_symbol - 4.8) < 0.001
    assert abs(s.efficiency - 0.9375) < 0.001
    assert abs(s.space_savings() - 40.0) < 0.001


def test_entropy_stats_edge_cases():  # mod.rs:355-367
    s = EntropyStats.new(0, 0, 0.0)
    assert s.compression_ratio == 0.0 and s.bits_per_symbol == 0.0 and s.efficiency == 0.0
    s = EntropyStats.new(100, 0, 4.0)
    assert s.compression_ratio == 0.0 and s.space_savings() == 100.0


def test_entropy_from_counts():  # mod.rs:338-353 on counts
    assert abs(entropy_from_counts([1] * 256) - 8.0) < 0.001
    assert entropy_from_counts([0] * 42 + [100] + [0] * 213) < 0.001
    assert entropy_from_counts([0] * 256) == 0.0


def test_names_availability_presets():
    assert A.default() is A.Auto
    assert [a.name_str() for a in A] == ["Huffman", "rANS", "FSE", "kFSE", "Dictionary", "Auto"]
    assert all(a.is_available() for a in A)
    assert A.available_algorithms() == [A.Huffman, A.Rans, A.Dictionary, A.Auto, A.Fse, A.KFse]
    d = EntropyConfig.default()
    assert (d.algorithm, d.compression_level, d.adaptive, d.dict_size, d.fast_decode) == (A.Auto, 3, True, 0, False)
    f = EntropyConfig.fast()
    assert (f.algorithm, f.compression_level, f.fast_decode) == (A.Huffman, 1, True)
    h = EntropyConfig.high_compression()
    assert (h.algorithm, h.compression_level, h.dict_size) == (A.Fse, 19, 32 * 1024)
    assert EntropyConfig.balanced() == EntropyConfig.default()


def _select_ref(data):
    """mod.rs:124-153 restated over numpy counts (test oracle)."""
    if not data:
        return A.Huffman
    c = np.bincount(np.frombuffer(data, dtype=np.uint8), minlength=256)
    total = float(len(data))
    e = 0.0
    for f in c:
        if f > 0:
            p = int(f) / total
            e -= p * math.log2(p)
    r = 1.0 - int((c > 0).sum()) / 256.0
    if r > 0.8:
        return A.Dictionary
    if e < 4.0 and len(data) > 1024:
        return A.Fse
    if 4.0 <= e <= 6.0 and len(data) > 256:
        return A.Rans
    return A.Huffman


def test_decision_table_on_counts():
    assert A.select_from_counts([5] * 40 + [0] * 216, 200) is A.Dictionary   # 40 symbols: r = 0.84
    c = [0] * 256
    for i in range(60):
        c[i] = 1000 if i < 4 else 1                                         # low entropy, 60 symbols
    assert A.select_from_counts(c, sum(c)) is A.Fse
    assert A.select_from_counts(c, 1000) is A.Huffman                        # not > 1024 bytes
    assert A.select_from_counts([1] * 256, 256) is A.Huffman                # 8 bits
    c = [40] * 32 + [10] * 32 + [0] * 192                                    # 64 symbols, ~5.7 bits
    assert 4.0 <= entropy_from_counts(c) <= 6.0
    assert A.select_from_counts(c, sum(c)) is A.Rans


@pytest.mark.gpu
def test_select_for_data_gpu(zr):
    rnd = random.Random(3)
    cases = [b"", b"a", bytes(range(256)), b"x" * 5000, bytes(rnd.randrange(4) for _ in range(3000)),
             bytes(rnd.randrange(40) for _ in range(3000)), bytes(rnd.randrange(52) for _ in range(300)),
             zr.synth("t", 4096, seed=9), zr.synth("z", 100000, seed=2), zr.synth("u", 70000, seed=5),
             bytes(rnd.randrange(60) for _ in range(257)), bytes(rnd.randrange(60) for _ in range(256))]
    for d in cases:
        assert A.select_for_data(d) is _select_ref(d), len(d)
    assert abs(EntropyStats.calculate_entropy(bytes(range(256))) - 8.0) < 0.001  # mod.rs:341-343
    assert EntropyStats.calculate_entropy(b"*" * 100) < 0.001                     # mod.rs:346-348
    assert EntropyStats.calculate_entropy(b"") == 0.0                              # mod.rs:351-352
