"""C ABI boundary checks that need no GPU: the library loads, exports every symbol
include/*.h declares, and the host-side table construction (Rans64Encoder::new,
rans.rs:208-299) matches the oracle bit for bit."""
import ctypes
import glob
import os
import random
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"\b(zr_[a-z0-9_]+)\s*\(", txt):
            syms.add(m.group(1))
    syms.discard("zr_error_cb")
    return sorted(syms)


def test_library_exports_every_header_symbol(zr):
    lib = zr.load()
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, f"not exported: {missing}"
    assert len(header_symbols()) >= 20


def test_python_signatures_cover_header(zr):
    from zipora_amd import _lib
    bound = {n for n, _, _ in _lib.SIGNATURES}
    missing = [s for s in header_symbols() if s not in bound]
    assert not missing, f"no ctypes signature for: {missing}"


def test_version_and_errors(zr):
    lib = zr.load()
    assert b"gfx950" in lib.zr_version()
    # invalid input reports through the thread-local last error
    st = lib.zr_synth_fill(7, 0, None, 0)
    assert st == -1 and "synth" in zr.last_error()


def _freq_cases():
    rnd = random.Random(1234)
    cases = [[0] * 256 for _ in range(1)]
    cases[0][97] = 5
    for _ in range(60):
        f = [0] * 256
        k = rnd.choice([1, 2, 3, 5, 16, 64, 200, 256])
        for s in rnd.sample(range(256), k):
            f[s] = rnd.choice([1, 2, 3, rnd.randint(1, 10), rnd.randint(1, 100000), rnd.randint(1, 1 << 28)])
        cases.append(f)
    f = [1] * 256
    f[65], f[66] = 100, 50
    cases.append(f)
    cases.append([0] * 255 + [7])
    big = [0] * 256
    big[0], big[255] = 99999, 1
    cases.append(big)
    cases.append([1 << 24] * 256)  # u32 wrapping sum
    return cases


def test_host_table_build_matches_oracle(zr, oracle):
    lib = zr.load()
    from zipora_amd import _lib
    for f in _freq_cases() + [[0] * 256]:
        t = _lib.RansTable()
        st = lib.zr_rans_table_build((ctypes.c_uint32 * 256)(*f), ctypes.byref(t))
        o = oracle.RansTable()
        ost = oracle.lib().or_rans_table_build((ctypes.c_uint32 * 256)(*f), ctypes.byref(o))
        assert st == ost
        assert list(t.freq) == list(o.freq)
        assert list(t.start) == list(o.start)
        assert t.total_freq == o.total_freq


def test_encode_bound_covers_worst_case(zr):
    lib = zr.load()
    for n, N in [(0, 1), (1, 1), (100, 4), (1 << 20, 4096)]:
        assert lib.zr_rans_encode_bound(n, N) >= 2 * n + 12 * N + 8


def test_synth_is_deterministic(zr, oracle):
    a = zr.synth("u", 4096)
    assert a == oracle.gen_uniform(4096)  # same xorshift as tests/fse_tests.rs:711-717
    z = zr.synth("z", 1 << 16)
    hist = oracle.histogram(z)
    assert hist[0] > hist[1] > hist[10] > hist[100]
    t = zr.synth("t", 1 << 16)
    assert len(set(t)) <= 64


def test_adaptive_select_variant_thresholds(zr):
    """AdaptiveRans64Encoder::select_variant (rans.rs:669-681) and the reference's
    test (rans.rs:864-878); host code, no GPU."""
    a = zr.AdaptiveRans64Encoder()
    assert [a.select_variant(n) for n in (50, 100, 10000, 30000000)] == ["x1", "x2", "x4", "x8"]
    edges = {0: "x1", 72: "x1", 73: "x2", 73 ** 2 - 1: "x2", 73 ** 2: "x4", 73 ** 4 - 1: "x4", 73 ** 4: "x8"}
    assert {n: a.select_variant(n) for n in edges} == edges


def test_stream_count_limit_checked_before_any_launch(zr):
    """the stream-count limit (2^26: a 32-row decoder tile spans < 2^31 B)
    is refused up front (no kernel, no timer)."""
    from zipora_amd import _lib
    lib = zr.load()
    bt = _lib.RansBatch()
    bt.n_buffers, bt.n_streams, bt.max_len = 1, 1 << 26, 1 << 28
    for fn in (lib.zr_rans_encode_batch_dev, lib.zr_rans_decode_batch_dev):
        assert fn(ctypes.byref(bt), None, None, None, 0, None) == _lib.ZR_UNSUPPORTED
        assert "2^26" in zr.last_error()


def test_diagnostic_switches_are_tools_only():
    """the product library reads no diagnostic environment
    switches (they exist only in the -DZR_DIAG tools build) and bench.py refuses
    to print a metric line while one is set."""
    import subprocess
    import sys
    src = open(os.path.join(ROOT, "zipora_amd", "csrc", "zr_rans.hip")).read()

    def open_conditions(text):  # the preprocessor conditions open at the end of text
        stack = []
        for line in text.splitlines():
            t = line.strip()
            if t.startswith("#if"):
                stack.append(t)
            elif t.startswith("#endif"):
                stack.pop()
        return stack

    for m in re.finditer(r'getenv\("(ZR_[A-Z_]+)"\)', src):
        assert "#ifdef ZR_DIAG" in open_conditions(src[:m.start()]), m.group(1)
    env = dict(os.environ, ZR_ABLATE="1")
    r = subprocess.run([sys.executable, "-c", "import zipora_amd._lib as l; print(l.diag_env())"],
                       cwd=ROOT, env=env, capture_output=True, text=True)
    assert "ZR_ABLATE" in r.stdout
