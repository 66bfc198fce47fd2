#!/usr/bin/env python3
"""Randomised parity sweep of the Huffman device paths against the CPU oracle
(test infrastructure, run on the GPU box): order-0 encode/decode
(huffman/encoder.rs, decoder.rs restated) and the contextual order-1/2 coder
with 1/2/4/8-way interleaving (huffman/interleaved.rs), on random data
(uniform, Zipf, text, one symbol, two symbols, chains whose codes run long,
sizes 1 B-2 MiB). Encoded bytes equal the oracle's; decode returns the input.
Usage: python3 tools/fuzz_huff.py [seconds] [seed]
"""
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def data_of(kind, n, rng, zr):
    if kind == "one":
        return bytes([rng.randrange(256)]) * n
    if kind == "two":
        a, b = rng.randrange(256), rng.randrange(256)
        return bytes(np.where(np.random.default_rng(rng.randrange(1 << 30)).integers(0, 2, n) == 0, a, b)
                     .astype(np.uint8))
    if kind == "chain":  # symbol i about 1.9^i times: codes of up to ~20 bits
        k = rng.randrange(3, 22)
        base = b"".join(bytes([(s * 7) % 256]) * max(1, int(1.9 ** s)) for s in range(k))
        reps = max(1, n // max(1, len(base)))
        d = bytearray(base * reps)
        random.Random(rng.randrange(1 << 30)).shuffle(d)
        return bytes(d[:max(1, n)])
    return zr.synth(kind, n, seed=rng.randrange(1 << 62))


def run(secs=None, max_cases=None, seed=12345, log=print):
    import oracle_ffi as orc
    import zipora_amd as zr

    rng = random.Random(seed)
    t_end = time.time() + secs if secs else None
    cases = 0
    while (t_end is None or time.time() < t_end) and (max_cases is None or cases < max_cases):
        n = rng.choice([1, 2, 3, 17, 255, 4096, rng.randrange(1, 5000), rng.randrange(5000, 200000),
                        rng.randrange(200000, 2 << 20)])
        kind = rng.choice(["u", "z", "t", "one", "two", "chain"])
        d = data_of(kind, n, rng, zr)
        mode = rng.choice(["o0", "o1", "o2"])
        desc = f"n={len(d)} kind={kind} mode={mode}"
        if mode == "o0":
            t = orc.huff_tree(orc.histogram(d))
            ref = orc.huff_encode(t, d)
            enc = zr.HuffmanEncoder(d)
            got = enc.encode(d)
            if got != ref:
                raise AssertionError(f"MISMATCH case {cases} seed {seed}: {desc}")
            if zr.HuffmanDecoder(enc.tree()).decode(ref, len(d)) != d:
                raise AssertionError(f"DECODE case {cases} seed {seed}: {desc}")
        else:
            order = 1 if mode == "o1" else 2
            oc = orc.Ctx(d, order)
            ec = zr.ContextualHuffmanEncoder(d, order)
            if int(ec.order()) != oc.order:
                raise AssertionError(f"ORDER case {cases} seed {seed}: {desc}")
            ref = oc.encode(d)
            if ec.encode(d) != ref:
                raise AssertionError(f"MISMATCH case {cases} seed {seed}: {desc}")
            if zr.ContextualHuffmanDecoder(ec).decode(ref, len(d)) != d:
                raise AssertionError(f"DECODE case {cases} seed {seed}: {desc}")
            if oc.order == 1:
                nw = rng.choice([1, 2, 4, 8])
                r = oc.encode_xn(nw, d)
                if ec.encode_with_interleaving(d, nw) != r or ec.decode_with_interleaving(r, len(d), nw) != d:
                    raise AssertionError(f"INTERLEAVED x{nw} case {cases} seed {seed}: {desc}")
                desc += f" x{nw}"
        cases += 1
        log(f"case {cases}: {desc} ok")
    return cases


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 150.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 12345
    cases = run(secs=secs, seed=seed, log=lambda m: print(m, flush=True))
    print(f"fuzz ok: {cases} cases, seed {seed}")


if __name__ == "__main__":
    main()
