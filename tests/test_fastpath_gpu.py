"""Round-3: the fast device decoders must take their fast path on the data the
bench and the BASELINE configs use. The generic per-lane loop behind them
(dec_lane_generic / x1_dec_generic) is bit-exact too, so parity tests alone
cannot see a refill schedule that sends lanes to it; zr_rans_fallback_lanes
counts them. (Round 3 found a one-tile-lag schedule that sent most lanes of the
headline there: parity stayed green, the decoder ran 6x slower.)"""
import pytest

pytestmark = pytest.mark.gpu


def _batch_roundtrip(zr, oracle, lens, N, kind, seed, check_bufs=2, skew=False):
    import numpy as np
    import torch
    from zipora_amd.device import RansDeviceBatch
    bt = RansDeviceBatch(lens, N, shared_table=True)
    raw = bt.new_raw()
    datas = []
    for b, n in enumerate(lens):
        d = zr.synth(kind, n, seed=seed + b)
        if skew:  # every third stream of the interleave sees one constant byte
            a = np.frombuffer(d, dtype=np.uint8).copy()
            a[(np.arange(n) % N) % 3 == 0] = 65
            d = a.tobytes()
        datas.append(d)
        o = bt.raw_off_host[b]
        raw[o:o + n] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    zr.fallback_lanes(reset=True)
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    fb = zr.fallback_lanes(reset=True)
    assert torch.equal(out, raw)
    if check_bufs:
        import concurrent.futures as cf
        t = oracle.rans_table(oracle.histogram(b"".join(datas)))
        nb = min(check_bufs, len(lens))
        # (the oracle releases the GIL: the buffers are encoded on 16 threads)
        with cf.ThreadPoolExecutor(max_workers=16) as ex:
            refs = list(ex.map(lambda b: oracle.rans_encode(t, N, datas[b]), range(nb)))
        for b in range(nb):
            assert bt.encoded(enc, b) == refs[b], f"buffer {b}"
    return fb


@pytest.mark.parametrize("kind", ["u", "z", "t"])
def test_headline_shape_takes_fast_path(zr, oracle, kind):
    """64 x 4 MiB x 4096 streams (the bench's workload, 1024-lane decoder):
    uniform, Zipf(1.1) and text-like bytes decode with no generic lanes."""
    # every buffer of the uniform batch (the bench's input kind) byte-compared
    fb = _batch_roundtrip(zr, oracle, [4 << 20] * 64, 4096, kind, 0x51 + ord(kind),
                          check_bufs=64 if kind == "u" else 2)
    assert fb == 0, f"{fb} of {64 * 4096} streams fell back to the generic decoder ({kind})"


def test_skewed_streams_fast_path(zr, oracle):
    """Streams that consume their bytes at very different rates in one wave
    (a constant byte in every third stream: ~0.4 bits per symbol there, ~9.5
    in the others): the refill schedule keeps every lane on the fast path."""
    fb = _batch_roundtrip(zr, oracle, [4 << 20] * 16, 4096, "u", 0x3A, skew=True)
    assert fb == 0, f"{fb} streams fell back"


def test_literal_shape_takes_fast_path(zr, oracle):
    """One 256 MiB buffer x 4096 streams (configs[1] as written, one-wave shape)."""
    fb = _batch_roundtrip(zr, oracle, [256 << 20], 4096, "u", 0x77, check_bufs=0)
    assert fb == 0, f"{fb} of 4096 streams fell back"


def test_ragged_wide_shape_fast_path(zr, oracle):
    """Streams whose lengths are not a multiple of the 32-step tile (tail loop
    with a segment still in flight), wide shape."""
    lens = [(4 << 20) + 4096 * 17 + 5] * 20
    fb = _batch_roundtrip(zr, oracle, lens, 4096, "u", 0x99)
    assert fb == 0


def test_record_batch_full_size(zr, oracle):
    """configs[4] at full size: 2^20 x 1 KiB uniform records through the x1
    coders with one shared table (RansBlobStore over one trained table,
    blob_store/entropy.rs:212-238; Rans64Encoder::<ParallelX1>, rans.rs:354-366,
    :523-552). Round trip of the whole batch, no generic records, and 256
    sampled records byte-compared with the oracle's encode."""
    import numpy as np
    import torch
    from zipora_amd.device import RansDeviceBatch
    R, n = 1 << 20, 1024
    data = zr.synth("u", R * n, seed=0xB10B)
    bt = RansDeviceBatch([n] * R, 1, shared_table=True)
    assert bt.raw_bytes == R * n
    raw = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    enc = bt.new_enc()
    bt.full_encode(raw, enc)
    torch.cuda.synchronize()
    bt.raise_on_error()
    hist = np.bincount(np.frombuffer(data, dtype=np.uint8), minlength=256)
    t = oracle.rans_table([int(v) for v in hist])
    rnd = np.random.default_rng(4)
    for b in sorted(set(int(v) for v in rnd.integers(0, R, 256)) | {0, R - 1}):
        d = data[b * n:(b + 1) * n]
        assert bt.encoded(enc, b) == oracle.rans_encode(t, 1, d), f"record {b}"
    zr.fallback_lanes(reset=True)
    out = bt.new_raw()
    bt.decode(enc, out)
    torch.cuda.synchronize()
    bt.raise_on_error()
    fb = zr.fallback_lanes(reset=True)
    assert torch.equal(out, raw)
    assert fb == 0, f"{fb} of {R} records fell back to the generic decoder"


@pytest.mark.parametrize("N", [1 << 18])
def test_single_buffer_many_streams(zr, oracle, N):
    """BASELINE.md C2 / SURVEY.md section 7 minimum slice: ONE 256 MiB uniform
    buffer at N = 2^18 interleaved streams (1024 symbols per stream; the
    reference takes any N, rans.rs:165-168): the whole encoded buffer
    byte-compared with the oracle's encode_parallel (rans.rs:369-420), decoded
    back with no generic lanes."""
    fb = _batch_roundtrip(zr, oracle, [256 << 20], N, "u", 0x2E18, check_bufs=1)
    assert fb == 0, f"{fb} of {N} streams fell back"


@pytest.mark.parametrize("lens,N,kind,check", [
    ([4 << 20] * 16, 4096, "z", 2),
    ([(4 << 20) + 4096 * 17 + 5] * 20, 4096, "u", 2),   # ragged rows (tail with refills in flight)
    ([256 << 20], 1 << 19, "u", 1),          # one buffer, N = 2^19 (two rounds of workgroups)
    ([3_000_001, 1_000_003, 77_777], 1 << 16, "t", 3),  # ragged buffers (the last one x1), 3 x 2^16 lanes
])
def test_wide_decoder_shapes(zr, oracle, lens, N, kind, check):
    """k_dec_xn_fast on the shapes round 5 ran through its LDS-DMA variant (now
    removed): the same bytes as the oracle's encode and the input back, no
    generic lanes."""
    fb = _batch_roundtrip(zr, oracle, lens, N, kind, 0xD3A + N, check_bufs=check)
    assert fb == 0, f"{fb} streams fell back"
