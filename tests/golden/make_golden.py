#!/usr/bin/env python3
"""Generate tests/golden/*.json from the CPU oracle (oracle/liboracle.so).

The reference is Rust and cannot be built or run here, so
these fixtures are oracle outputs on the reference's own test inputs
(rans.rs:811-1039, tests/fse_tests.rs:632-845, huffman/tests.rs:7-620). Before
writing anything the script re-checks the oracle against SURVEY.md Appendix B
(B1-B14); tests/test_golden.py then pins the oracle to the files and the GPU
path to the same bytes.

    python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_ffi as O  # noqa: E402


def xorshift_bytes(n, seed=0x9E3779B97F4A7C15):
    """tests/fse_tests.rs:711-717 (byte = state >> 32)."""
    out = bytearray()
    s = seed
    M = (1 << 64) - 1
    for _ in range(n):
        s ^= (s << 13) & M
        s ^= s >> 7
        s ^= (s << 17) & M
        out.append((s >> 32) & 0xFF)
    return bytes(out)


def make_input(spec):
    """Inputs are stored as small recipes: ["hex", h] | ["xorshift", n, seed] |
    ["repeat", hex, count, limit] | ["seq", n, mul, add] | ["ramp"] (b repeated b+1 times)."""
    kind = spec[0]
    if kind == "hex":
        return bytes.fromhex(spec[1])
    if kind == "xorshift":
        return xorshift_bytes(spec[1], spec[2])
    if kind == "repeat":
        d = bytes.fromhex(spec[1]) * spec[2]
        return d[:spec[3]] if len(spec) > 3 and spec[3] else d
    if kind == "seq":
        return bytes(((i * spec[2] + spec[3]) % 256) for i in range(spec[1]))
    if kind == "ramp":  # byte b repeated b+1 times, b < limit (fse_tests.rs all-256 skew case)
        return b"".join(bytes([b]) * (b + 1) for b in range(spec[1] if len(spec) > 1 else 256))
    if kind == "concat":
        return b"".join(make_input(x) for x in spec[1:])
    raise ValueError(spec)


def H(b):
    return ["hex", b.hex()]


def R(b, count, limit=0):
    return ["repeat", b.hex(), count, limit]


XS = 0x9E3779B97F4A7C15


def check_appendix_b():
    t = O.rans_table([0] * 0x61 + [1, 4095] + [0] * (256 - 0x63))
    assert O.rans_encode(t, 1, b"ab").hex() == "220000080000000000"
    assert O.fse_compress(b"\x78" * 100).hex() == "f5640000000c010078001000000100000000000000"
    t = O.huff_tree(O.histogram(b"aaabbc"))
    assert O.huff_encode(t, b"aaabbc").hex() == "8006"


def rans_cases():
    specs = [
        H(b"hello world, this is a test of enhanced 64-bit rANS encoding"),
        H(b"quad-stream parallel encoding test with four independent streams for better performance"),
        R(b"This is a test message for parallel rANS processing with multiple streams to verify "
          b"correctness across all variants.", 4),
        ["seq", 1500, 123, 45], R(b"a", 1000), ["seq", 512, 1, 0], ["xorshift", 1500, 0x1234567], H(b"x"),
    ]
    out = []
    for sp in specs:
        d = make_input(sp)
        t = O.rans_table(O.histogram(d))
        for n in (1, 2, 4, 8, 64):
            out.append({"streams": n, "input": sp, "encoded": O.rans_encode(t, n, d).hex()})
    return out


def fse_cases():
    fox = R(b"The quick brown fox jumps over the lazy dog. ", 50, 2000)
    cases = [
        (H(b""), {}), (H(b"a"), {}), (H(b"\xff"), {}), (R(b"x", 99), {}), (R(b"x", 100), {}),
        (R(b"x", 101), {}), (R(b"\0", 4096), {}), (R(b"\xff", 500), {}), (R(b"abc", 333), {}),
        (["concat", R(b"\0", 4000), ["seq", 150, 1, 1]], {}),
        (["concat", R(b"\xff", 4000), ["seq", 150, 1, 1]], {}),
        (["concat", R(b"a", 700), R(b"b", 150), R(b"c", 150), ["seq", 100, 1, 0]], {}),
        (["seq", 2048, 1, 0], {}), (["ramp", 100], {}),
        (["xorshift", 128, XS], {}), (["xorshift", 1000, XS], {}), (["xorshift", 4096, XS], {}),
        (fox, {}), (fox, {"parallel_blocks": 4, "block_size": 400}),
        (["xorshift", 2500, 99], {"parallel_blocks": 8, "block_size": 512}),
        (fox, {"parallel_blocks": 1, "block_size": 400}),
        (fox, {"parallel_blocks": 4, "block_size": 120}),
    ]
    out = []
    for sp, cfg in cases:
        d = make_input(sp)
        out.append({"config": cfg, "input": sp, "compressed": O.fse_compress(d, O.fse_config(**cfg)).hex()})
    return out


def huff_cases():
    specs = [H(b"aab"), H(b"aaabbc"), H(b"abc"), H(b"abcd"), R(b"a", 9), H(b"hello world"),
             H(b"The quick brown fox jumps over the lazy dog"), ["seq", 256, 1, 0], ["seq", 210, 1, 0],
             ["ramp", 60], ["xorshift", 1000, 7],
             ["concat"] + [R(bytes([i]), 1 << min(i, 10)) for i in range(12)]]
    out = []
    for sp in specs:
        d = make_input(sp)
        t = O.huff_tree(O.histogram(d))
        codes = {str(s): c for s, c in O.huff_codes(t).items()}
        out.append({"input": sp, "codes": codes, "encoded": O.huff_encode(t, d).hex()})
    return out


def main():
    check_appendix_b()
    fx = {"rans": rans_cases(), "fse": fse_cases(), "huffman_o0": huff_cases()}
    for k, v in fx.items():
        p = os.path.join(HERE, f"{k}.json")
        with open(p, "w") as f:
            json.dump({"generator": "tests/golden/make_golden.py (oracle/zr_oracle.c)", "cases": v}, f)
        print(p, os.path.getsize(p))


if __name__ == "__main__":
    main()
