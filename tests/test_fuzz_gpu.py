"""Fixed-seed slices of the randomised parity sweeps (tools/fuzz_rans.py, fuzz_fse.py, fuzz_huff.py, fuzz_rans_corrupt.py):
random batch geometries (narrow and wide shapes, ragged and edge lengths), data
kinds, shared or per-buffer tables and encoder widths, every buffer's encoded
bytes equal to the oracle's (rans.rs:338-420) and decoded back on the device."""
import importlib.util
import os

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fuzz():
    spec = importlib.util.spec_from_file_location("fuzz_rans", os.path.join(ROOT, "tools", "fuzz_rans.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("seed", [2024, 31337])
def test_rans_random_batches_match_oracle(zr, oracle, seed):
    cases, bufs = _fuzz().run(max_cases=40, seed=seed, log=lambda m: None)
    assert cases == 40 and bufs > 40


def _fuzz_fse():
    spec = importlib.util.spec_from_file_location("fuzz_fse", os.path.join(ROOT, "tools", "fuzz_fse.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_fse_random_configs_match_oracle(zr, oracle):
    """Random FSE data and configs (tools/fuzz_fse.py): bytes equal to the
    oracle's, decompression error for error with it."""
    assert _fuzz_fse().run(max_cases=200, seed=99, log=lambda m: None) == 200


def test_huffman_random_inputs_match_oracle(zr, oracle):
    """Random data through the order-0 and contextual order-1/2 coders
    (tools/fuzz_huff.py): bytes equal to the oracle's, decoded back."""
    spec = importlib.util.spec_from_file_location("fuzz_huff", os.path.join(ROOT, "tools", "fuzz_huff.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    assert m.run(max_cases=150, seed=7, log=lambda m_: None) == 150


def test_rans_corrupted_batches_match_oracle(zr, oracle):
    """Corrupted encodings (tools/fuzz_rans_corrupt.py: states, lengths, random
    bytes, enc_len) decoded over a garbage-filled status array: error for error
    and byte for byte with the oracle."""
    spec = importlib.util.spec_from_file_location("fuzz_rans_corrupt",
                                                  os.path.join(ROOT, "tools", "fuzz_rans_corrupt.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    cases, bad = m.run(max_cases=40, seed=707, log=lambda m_: None)
    assert cases == 40 and bad > 0
