#!/usr/bin/env python3
"""Randomised parity sweep of the FSE device path against the CPU oracle (test
infrastructure, run on the GPU box): random data (uniform, Zipf, text, one
symbol, two symbols, short runs around the 100-byte literal threshold), random
table_log / compression_level / parallel_blocks / block_size; the compressed
bytes must equal the oracle's (fse.rs:1105-1312 restated) and both sides must
decompress each other's stream. Usage: python3 tools/fuzz_fse.py [seconds] [seed]
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
    if n == 0:
        return b""
    if kind == "one":
        return bytes([rng.randrange(256)]) * n
    if kind == "two":
        a, b = rng.randrange(256), rng.randrange(256)
        return bytes(np.where(np.random.default_rng(rng.randrange(1 << 30)).integers(0, 2, n) == 0, a, b)
                     .astype(np.uint8))
    return zr.synth(kind, n, seed=rng.randrange(1 << 62))


def run(secs=None, max_cases=None, seed=12345, log=print):
    import oracle_ffi as orc
    import zipora_amd as zr

    rng = random.Random(seed)
    t_end = time.time() + secs if secs else None
    cases = 0
    while (t_end is None or time.time() < t_end) and (max_cases is None or cases < max_cases):
        n = rng.choice([0, 1, 2, 99, 100, 101, 255, 4096, rng.randrange(1, 5000), rng.randrange(5000, 300000),
                        rng.randrange(300000, 3 << 20)])
        kind = rng.choice(["u", "z", "t", "one", "two"])
        d = data_of(kind, n, rng, zr)
        tl = rng.randrange(5, 16)
        lvl = rng.choice([1, 3, 6, 9, 19])
        pb = rng.choice([None, None, 1, 2, 3, 4, 8])
        bs = rng.choice([64 * 1024, 16 * 1024, 128 * 1024, 4096, 1000, 150])
        if pb and n > 1_100_000 and bs < 4096:
            bs = 4096
        cfg = zr.FseConfig(table_log=tl, compression_level=lvl, max_table_size=max(64 * 1024, 1 << tl),
                           parallel_blocks=pb, block_size=bs)
        oc = orc.fse_config(table_log=tl, compression_level=lvl, max_table_size=max(64 * 1024, 1 << tl),
                            parallel_blocks=pb or 0, block_size=bs)
        desc = f"n={n} kind={kind} table_log={tl} level={lvl} pb={pb} bs={bs}"
        try:
            want = orc.fse_compress(d, oc)
        except orc.OracleError:
            want = None
        try:
            got = zr.fse_compress_with_config(d, cfg)
        except zr.ZiporaError:
            got = None
        if got != want:
            raise AssertionError(f"MISMATCH case {cases} seed {seed}: {desc}: "
                                 f"got {None if got is None else len(got)} want {None if want is None else len(want)}")
        if want is not None:
            # decompression, error for error with the oracle (parallel_blocks =
            # Some(1) with more than two blocks of data emits the body without
            # its mode byte, fse.rs:975-977, which neither side can read back)
            try:
                ref = orc.fse_decompress(want)
            except orc.OracleError:
                ref = None
            try:
                back = zr.fse_decompress(got)
            except zr.ZiporaError:
                back = None
            if back != ref or (pb != 1 and ref != d):
                raise AssertionError(f"ROUND TRIP case {cases} seed {seed}: {desc}")
        cases += 1
        log(f"case {cases}: {desc} {'ok' if want is not None else 'both refused'}")
    return cases


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 150.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 12345
    cases = run(secs=secs, seed=seed, log=lambda m: print(m, flush=True))
    print(f"fuzz ok: {cases} cases, seed {seed}")


if __name__ == "__main__":
    main()
