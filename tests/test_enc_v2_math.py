"""The V2 encoder's quotient (zr_rans.hip: enc_entry_v2, k_enc_xn / k_enc_x1_ring):
q = umulhi(y, R) >> sh must equal y / f for every symbol frequency f and every
y < 2^24 the step can see (y = x >> nb, x in [2^16, 2^24)); f = 1 uses
R = 2^32 - 1 (q = y - 1) with 4095 added to the entry's start. The division is
rans.rs:303-335's `x / freq` (encode_symbol). CPU only: the parity tests run the
kernels themselves against the oracle."""
import numpy as np


def entry_v2(f):
    """(R, sh) as enc_entry_v2 computes them."""
    if f == 1:
        return 0xFFFFFFFF, 0
    sh = (f - 1).bit_length() - 1  # ceil(log2 f) - 1
    R = ((1 << (32 + sh)) + f - 1) // f
    return R, sh


def _ys(f, rng):
    top = 1 << 24
    k = np.arange(1, top // f + 1, dtype=np.int64)
    step = max(1, len(k) // 2000)
    ys = np.concatenate([np.arange(1, 4096), rng.integers(1, top, 4000), k[::step] * f - 1, k[::step] * f,
                         [top - 1, top - 2]])
    ys = ys[(ys >= 1) & (ys < top)]
    return np.unique(ys).astype(np.uint64)


def test_reciprocal_exact_for_every_freq():
    rng = np.random.default_rng(7)
    for f in range(1, 4097):
        R, sh = entry_v2(f)
        assert 0 < R < (1 << 32)
        ys = _ys(f, rng)
        q = ((ys * np.uint64(R)) >> np.uint64(32)) >> np.uint64(sh)
        want = ys - np.uint64(1) if f == 1 else ys // np.uint64(f)
        assert np.array_equal(q, want), f


def test_update_matches_reference_step():
    """x' = q * (4096 - f) + y + start' equals (y / f) * 4096 + y % f + start
    (rans.rs:330-334), f = 1 included through the start offset."""
    rng = np.random.default_rng(11)
    for f in [1, 2, 3, 7, 16, 255, 1000, 2047, 4095, 4096]:
        R, sh = entry_v2(f)
        start = int(rng.integers(0, 4096 - f + 1))
        st = start + (4095 if f == 1 else 0)
        cmpl = (4096 - f) & 0xFFF
        for x in rng.integers(1 << 16, 1 << 24, 2000):
            x = int(x)
            nb = 16 if x >= (f << 20) else (8 if x >= (f << 12) else 0)
            y = x >> nb
            q = ((y * R) >> 32) >> sh
            got = (q * cmpl + y + st) & 0xFFFFFFFF
            assert got == (y // f) * 4096 + y % f + start, (f, x)
