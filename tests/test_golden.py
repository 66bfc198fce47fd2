"""Golden fixtures (tests/golden/*.json, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces every committed vector (regression pin).
GPU: the HIP path produces the same bytes through the C ABI.
"""
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from make_golden import make_input  # noqa: E402


def load(name):
    with open(os.path.join(HERE, "golden", f"{name}.json")) as f:
        return json.load(f)["cases"]


def test_golden_oracle_rans(oracle):
    for c in load("rans"):
        d = make_input(c["input"])
        t = oracle.rans_table(oracle.histogram(d))
        enc = oracle.rans_encode(t, c["streams"], d)
        assert enc.hex() == c["encoded"]
        assert oracle.rans_decode(t, c["streams"], enc, len(d)) == d


def test_golden_oracle_fse(oracle):
    for c in load("fse"):
        d = make_input(c["input"])
        enc = oracle.fse_compress(d, oracle.fse_config(**c["config"]))
        assert enc.hex() == c["compressed"]
        if not (c["config"].get("parallel_blocks") == 1 and len(d) > 2 * c["config"]["block_size"]):
            assert oracle.fse_decompress(enc) == d


def test_golden_oracle_huffman(oracle):
    for c in load("huffman_o0"):
        d = make_input(c["input"])
        t = oracle.huff_tree(oracle.histogram(d))
        assert {str(s): v for s, v in oracle.huff_codes(t).items()} == c["codes"]
        enc = oracle.huff_encode(t, d)
        assert enc.hex() == c["encoded"]
        assert oracle.huff_decode(t, enc, len(d)) == d


@pytest.mark.gpu
def test_golden_gpu_rans(zr):
    for c in load("rans"):
        d = make_input(c["input"])
        e = zr.Rans64Encoder(zr.histogram(d), c["streams"])
        assert e.encode(d).hex() == c["encoded"]
        assert zr.Rans64Decoder(e).decode(bytes.fromhex(c["encoded"]), len(d)) == d


@pytest.mark.gpu
def test_golden_gpu_fse(zr):
    for c in load("fse"):
        d = make_input(c["input"])
        cfg = zr.FseConfig(**c["config"])
        assert zr.fse_compress_with_config(d, cfg).hex() == c["compressed"]
        if not (c["config"].get("parallel_blocks") == 1 and len(d) > 2 * c["config"]["block_size"]):
            assert zr.fse_decompress(bytes.fromhex(c["compressed"])) == d


@pytest.mark.gpu
def test_golden_gpu_huffman(zr):
    for c in load("huffman_o0"):
        d = make_input(c["input"])
        e = zr.HuffmanEncoder(d)
        assert e.encode(d).hex() == c["encoded"]
        assert zr.HuffmanDecoder(e.tree()).decode(bytes.fromhex(c["encoded"]), len(d)) == d
