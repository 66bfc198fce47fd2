"""rANS order-0 -- host mirror of src/entropy/rans.rs over the HIP C ABI.

Same names and argument meaning as the reference:
  Rans64Encoder(frequencies, P).encode(data)           rans.rs:208, :338
  Rans64Decoder(encoder).decode(encoded, output_length) rans.rs:449, :510
P is the stream count of rans::ParallelVariant (rans.rs:165-196): the
reference's ParallelX1/X2/X4/X8 plus any other N (the trait is public).
Errors raise ZiporaError (InvalidData), like Result<_, ZiporaError>.
"""
import ctypes

from . import _lib
from .errors import ZiporaError, check


class ParallelVariant:
    def __init__(self, n, name=None):
        self.N = int(n)
        self.NAME = name or f"x{n}"


ParallelX1 = ParallelVariant(1, "x1")
ParallelX2 = ParallelVariant(2, "x2")
ParallelX4 = ParallelVariant(4, "x4")
ParallelX8 = ParallelVariant(8, "x8")


def _variant(p):
    return p if isinstance(p, ParallelVariant) else ParallelVariant(int(p))


def _u8(data):
    data = bytes(data)
    return (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0"), len(data)


class Rans64Symbol:
    """Rans64Symbol::new(start, freq) (rans.rs:89-104)."""

    def __init__(self, start, freq):
        self.start = start
        self.freq = freq

    def fast_div(self, x):
        """Rans64Symbol::fast_div (rans.rs:137-152): (x / freq, x % freq), on the
        device (the encoder's reciprocal division below 2^24). x: int or list."""
        xs = [int(x)] if isinstance(x, int) else [int(v) for v in x]
        n = len(xs)
        xa = (ctypes.c_uint64 * max(1, n))(*xs)
        qa = (ctypes.c_uint64 * max(1, n))()
        ra = (ctypes.c_uint64 * max(1, n))()
        check(_lib.load().zr_rans_symbol_fast_div(self.start, self.freq, xa, n, qa, ra))
        res = [(qa[i], ra[i]) for i in range(n)]
        return res[0] if isinstance(x, int) else res


class Rans64Encoder:
    """Rans64Encoder::<P>::new(&[u32; 256]) (rans.rs:208-235)."""

    def __init__(self, frequencies, parallel=ParallelX1):
        self.P = _variant(parallel)
        freqs = [int(f) & 0xFFFFFFFF for f in frequencies]
        if len(freqs) != 256:
            raise ValueError("frequencies must have 256 entries")
        self.table = _lib.RansTable()
        arr = (ctypes.c_uint32 * 256)(*freqs)
        check(_lib.load().zr_rans_table_build(arr, ctypes.byref(self.table)))

    def encode(self, data):
        """Rans64Encoder::encode (rans.rs:338-420)."""
        L = _lib.load()
        buf, n = _u8(data)
        cap = L.zr_rans_encode_bound(n, self.P.N)
        out = (ctypes.c_uint8 * cap)()
        ol = ctypes.c_size_t(0)
        check(L.zr_rans_encode(ctypes.byref(self.table), self.P.N, buf, n, out, cap, ctypes.byref(ol)))
        return ctypes.string_at(out, ol.value)

    def get_symbol(self, symbol):
        return Rans64Symbol(self.table.start[symbol], self.table.freq[symbol])

    def total_freq(self):
        return self.table.total_freq

    def variant_name(self):
        return self.P.NAME


class Rans64Decoder:
    """Rans64Decoder::<P>::new(&encoder) (rans.rs:449-468)."""

    def __init__(self, encoder):
        self.P = encoder.P
        self.table = encoder.table

    def decode(self, encoded_data, output_length):
        """Rans64Decoder::decode (rans.rs:510-651)."""
        L = _lib.load()
        buf, n = _u8(encoded_data)
        out = (ctypes.c_uint8 * max(1, output_length))()
        check(L.zr_rans_decode(ctypes.byref(self.table), self.P.N, buf, n, out, output_length))
        return ctypes.string_at(out, output_length)


class AdaptiveRans64Encoder:
    """AdaptiveRans64Encoder (rans.rs:655-721): picks P by the data size."""

    _NAMES = {1: "x1", 2: "x2", 4: "x4", 8: "x8"}
    _VARIANTS = {1: ParallelX1, 2: ParallelX2, 4: ParallelX4, 8: ParallelX8}

    def __init__(self):
        pass

    @classmethod
    def new(cls):
        return cls()

    def select_variant(self, data_size):
        """select_variant (rans.rs:669-681): "x1" < 73 <= "x2" < 73^2 <= "x4" < 73^4 <= "x8"."""
        return self._NAMES[_lib.load().zr_rans_adaptive_streams(int(data_size))]

    def variant_for(self, data_size):
        return self._VARIANTS[_lib.load().zr_rans_adaptive_streams(int(data_size))]

    def encode_adaptive(self, data):
        """encode_adaptive (rans.rs:684-706): histogram + Rans64Encoder::<P>::new + encode."""
        L = _lib.load()
        buf, n = _u8(data)
        cap = L.zr_rans_encode_bound(n, 8)
        out = (ctypes.c_uint8 * cap)()
        ol = ctypes.c_size_t(0)
        used = ctypes.c_uint32(0)
        check(L.zr_rans_encode_adaptive(buf, n, out, cap, ctypes.byref(ol), ctypes.byref(used)))
        return ctypes.string_at(out, ol.value)


def selftest_reciprocal():
    """Mismatches of the device encoder division over every freq 1..4096 and x < 2^24."""
    v = ctypes.c_uint64(0)
    check(_lib.load().zr_rans_selftest_reciprocal(ctypes.byref(v)))
    return v.value


def fallback_lanes(reset=True):
    """Streams/records the fast device decoders sent to their generic per-lane
    loop since the last reset (diagnostic; waits for the device)."""
    v = ctypes.c_uint64(0)
    check(_lib.load().zr_rans_fallback_lanes(ctypes.byref(v), 1 if reset else 0))
    return v.value


def device_alloc_count():
    v = ctypes.c_uint64(0)
    check(_lib.load().zr_device_alloc_count(ctypes.byref(v)))
    return v.value


def histogram(data):
    import numpy as np
    d = np.frombuffer(bytes(data), dtype=np.uint8)
    return [int(x) for x in np.bincount(d, minlength=256)]


__all__ = ["ParallelVariant", "ParallelX1", "ParallelX2", "ParallelX4", "ParallelX8",
           "Rans64Encoder", "Rans64Decoder", "Rans64Symbol", "AdaptiveRans64Encoder", "ZiporaError", "histogram",
           "selftest_reciprocal", "device_alloc_count", "fallback_lanes"]
