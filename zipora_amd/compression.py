"""RansCompressor (src/compression/mod.rs:416-512) over the C ABI.

A record is 256 x u32 LE normalised frequencies | u32 LE original size | x1 rANS
stream; empty data <-> empty record. `decompress` rebuilds the coder from the
stored (already normalised) frequencies with Rans64Encoder::new, exactly as the
reference does (mod.rs:514), including its non-idempotent re-normalisation of
skewed tables (SURVEY.md finding 0.9).
"""
import ctypes

from . import _lib
from .errors import check
from .rans import _u8


class RansCompressor:
    """RansCompressor::new(training_data) (mod.rs:425-452)."""

    def __init__(self, training_data):
        L = _lib.load()
        self.table = _lib.RansTable()
        buf, n = _u8(training_data)
        check(L.zr_rans_compressor_train(buf, n, ctypes.byref(self.table)))

    def compress(self, data):
        """Compressor::compress (mod.rs:457-477)."""
        L = _lib.load()
        buf, n = _u8(data)
        cap = L.zr_rans_compressor_bound(n)
        out = (ctypes.c_uint8 * cap)()
        ol = ctypes.c_size_t(0)
        check(L.zr_rans_compressor_compress(ctypes.byref(self.table), buf, n, out, cap, ctypes.byref(ol)))
        return ctypes.string_at(out, ol.value)

    def decompress(self, data):
        """Compressor::decompress (mod.rs:479-516): uses the record's stored table, not self's."""
        L = _lib.load()
        buf, n = _u8(data)
        size = ctypes.c_size_t(0)
        check(L.zr_rans_compressor_decompressed_size(buf, n, ctypes.byref(size)))
        out = (ctypes.c_uint8 * max(1, size.value))()
        ol = ctypes.c_size_t(0)
        check(L.zr_rans_compressor_decompress(buf, n, out, size.value, ctypes.byref(ol)))
        return ctypes.string_at(out, ol.value)

    def estimate_ratio(self, _data):
        return 0.6  # mod.rs:519-521

    def algorithm(self):
        return "Rans"  # Algorithm::Rans (mod.rs:523-525)
