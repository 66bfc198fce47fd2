"""Entropy stages of the PA-Zip / DictZip blob store over the C ABI.

  apply_fse_compression / remove_fse_compression   dict_zip/compression_types.rs:2272-2340
  PaZipFseConfig (dict_zip's FseConfig + presets)  dict_zip/compression_types.rs:2080-2146
  DictZipEntropyStage (encode/decode per record)   dict_zip/blob_store.rs:1075-1224
"""
import ctypes
import enum
from dataclasses import dataclass

from . import _lib
from .errors import check
from .huffman import ContextualHuffmanEncoder, HuffmanOrder


def _u8(data):
    data = bytes(data)
    return (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0"), len(data)


@dataclass
class PaZipFseConfig:
    """dict_zip's FseConfig (compression_types.rs:2080-2103); to_entropy_config
    fixes parallel_blocks None and 64 KiB blocks and tables (:2107-2123)."""
    max_symbol: int = 255
    table_log: int = 12
    adaptive: bool = True
    compression_level: int = 3
    fast_decode: bool = False

    @classmethod
    def for_pa_zip(cls):  # :2126-2133
        return cls(table_log=11, adaptive=True, compression_level=6, fast_decode=False)

    @classmethod
    def fast_pa_zip(cls):  # :2136-2145
        return cls(table_log=9, adaptive=False, compression_level=1, fast_decode=True)

    def to_c(self):
        c = _lib.FseConfig()
        c.table_log = self.table_log
        c.compression_level = self.compression_level
        c.max_table_size = 64 * 1024
        c.parallel_blocks = 0
        c.block_size = 64 * 1024
        c.adaptive = int(bool(self.adaptive))
        return c


def apply_fse_compression(encoded_data, config=None):
    """"UN" | raw (below 32 bytes or when FSE does not shrink), else "FS" | FSE stream."""
    L = _lib.load()
    c = (config or PaZipFseConfig()).to_c()
    buf, n = _u8(encoded_data)
    cap = L.zr_pazip_fse_bound(n, ctypes.byref(c))
    out = (ctypes.c_uint8 * cap)()
    ol = ctypes.c_size_t(0)
    check(L.zr_pazip_fse_apply(ctypes.byref(c), buf, n, out, cap, ctypes.byref(ol)))
    return ctypes.string_at(out, ol.value)


def remove_fse_compression(fse_data, config=None):
    L = _lib.load()
    c = (config or PaZipFseConfig()).to_c()
    buf, n = _u8(fse_data)
    size = ctypes.c_size_t(0)
    check(L.zr_pazip_fse_removed_size(buf, n, ctypes.byref(size)))
    out = (ctypes.c_uint8 * max(1, size.value))()
    ol = ctypes.c_size_t(0)
    check(L.zr_pazip_fse_remove(ctypes.byref(c), buf, n, out, size.value, ctypes.byref(ol)))
    return ctypes.string_at(out, ol.value)


class EntropyAlgorithm(enum.IntEnum):  # blob_store.rs:112-120
    None_ = 0
    HuffmanO1 = 1
    Fse = 2


class DictZipEntropyStage:
    """The DictZipBlobStore's per-record entropy stage: encode after PA-Zip,
    decode before it. HuffmanO1 uses an order-1 model of the dictionary."""

    def __init__(self, algorithm, interleaved=0, dictionary=b"", ratio_require=0.8):
        self.algorithm = EntropyAlgorithm(algorithm)
        self.interleaved = int(interleaved)
        self.ratio_require = float(ratio_require)
        self.model = (ContextualHuffmanEncoder(dictionary, HuffmanOrder.Order1)
                      if self.algorithm == EntropyAlgorithm.HuffmanO1 else None)

    def _h(self):
        return self.model.handle if self.model is not None else None

    def encode(self, data):
        """-> (bytes, EntropyAlgorithm used)."""
        L = _lib.load()
        buf, n = _u8(data)
        cap = 2 * n + 4096
        if self.model is not None:
            cap = max(cap, L.zr_ctx_huff_encode_bound(self._h(), n) + 16)
        out = (ctypes.c_uint8 * cap)()
        ol = ctypes.c_size_t(0)
        used = ctypes.c_int32(0)
        check(L.zr_dictzip_entropy_encode(int(self.algorithm), self.interleaved, self._h(), self.ratio_require,
                                          buf, n, out, cap, ctypes.byref(ol), ctypes.byref(used)))
        return ctypes.string_at(out, ol.value), EntropyAlgorithm(used.value)

    def decode(self, data, algorithm, original_size):
        L = _lib.load()
        buf, n = _u8(data)
        algorithm = EntropyAlgorithm(algorithm)
        if algorithm == EntropyAlgorithm.Fse:
            size = ctypes.c_size_t(0)
            check(L.zr_fse_decompressed_size(buf, n, ctypes.byref(size)))
            cap = size.value
        else:
            cap = max(n, original_size)
        out = (ctypes.c_uint8 * max(1, cap))()
        ol = ctypes.c_size_t(0)
        check(L.zr_dictzip_entropy_decode(int(algorithm), self._h(), buf, n, original_size, out, cap,
                                          ctypes.byref(ol)))
        return ctypes.string_at(out, ol.value)
