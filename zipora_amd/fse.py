"""FSE -- host mirror of src/entropy/fse.rs over the HIP C ABI.

Same names and argument meaning as the reference:
  FseConfig (+ fast_compression / high_compression / realtime / balanced)  fse.rs:204-316
  FseEncoder(config).compress(data)                                       fse.rs:773, :854
  FseDecoder() / FseDecoder.with_config(config), .decompress(data)         fse.rs:1084-1105
  fse_compress / fse_decompress / *_with_config / fse_zip / fse_unzip     fse.rs:1328-1355
Errors raise ZiporaError (like Result<_, ZiporaError>). All coding runs in
the HIP kernels of zr_fse.hip; the device-resident entry points take torch
CUDA tensors (FseDevice).
"""
import ctypes
from dataclasses import dataclass
from typing import Optional

from . import _lib
from .errors import ZiporaError, check


@dataclass
class FseConfig:
    max_symbol: int = 255
    table_log: int = 12
    adaptive: bool = True
    min_frequency: int = 1
    max_table_size: int = 64 * 1024
    fast_decode: bool = False
    dict_size: int = 0
    compression_level: int = 3
    parallel_blocks: Optional[int] = None
    entropy_optimization: bool = True
    block_size: int = 64 * 1024
    advanced_states: bool = False

    @classmethod
    def default(cls):
        return cls()

    @classmethod
    def fast_compression(cls):  # fse.rs:267-278
        return cls(table_log=10, compression_level=1, fast_decode=True, max_table_size=4 * 1024,
                   entropy_optimization=False, advanced_states=False)

    @classmethod
    def high_compression(cls):  # fse.rs:280-294
        return cls(table_log=15, compression_level=19, adaptive=True, max_table_size=256 * 1024,
                   dict_size=32 * 1024, entropy_optimization=True, advanced_states=True,
                   parallel_blocks=4, block_size=128 * 1024)

    @classmethod
    def realtime(cls):  # fse.rs:296-310
        return cls(table_log=8, compression_level=1, adaptive=False, fast_decode=True,
                   max_table_size=1024, entropy_optimization=False, advanced_states=False,
                   parallel_blocks=None, block_size=8 * 1024)

    @classmethod
    def balanced(cls):  # fse.rs:312-314
        return cls()

    def validate(self):
        """FseConfig::validate (fse.rs:317-348)."""
        if self.table_log < 5 or self.table_log > 15:
            raise ZiporaError(f"Table log must be 5-15, got {self.table_log}")
        if self.max_symbol > 65535:
            raise ZiporaError(f"Max symbol too large: {self.max_symbol}")
        if self.compression_level < 1 or self.compression_level > 22:
            raise ZiporaError(f"Compression level must be 1-22, got {self.compression_level}")
        if (1 << self.table_log) > self.max_table_size:
            raise ZiporaError(f"Table size {1 << self.table_log} exceeds max {self.max_table_size}")

    def to_c(self):
        c = _lib.FseConfig()
        c.table_log = self.table_log
        c.compression_level = self.compression_level
        c.max_table_size = self.max_table_size
        c.parallel_blocks = 0 if self.parallel_blocks is None else int(self.parallel_blocks)
        c.block_size = self.block_size
        c.adaptive = int(bool(self.adaptive))
        return c


# the facade's EntropyStats (mod.rs:241-330); the FSE coders record sizes only
# (entropy 0.0: a float diagnostic off the hot path)
from .entropy import EntropyStats  # noqa: E402


def _u8(data):
    data = bytes(data)
    return (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0"), len(data)


class FseEncoder:
    def __init__(self, config=None, dictionary=None):
        self._config = config if config is not None else FseConfig()
        self._config.validate()  # FseEncoder::new (fse.rs:773-786)
        self._dictionary = bytes(dictionary) if dictionary is not None else None
        self._freqs = None  # raw frequencies of the current table (FseEncoder::table)
        self._stats = EntropyStats()

    @classmethod
    def new(cls, config):
        return cls(config)

    @classmethod
    def with_dictionary(cls, config, dictionary):
        """FseEncoder::with_dictionary (fse.rs:789-794)."""
        return cls(config, dictionary)

    def analyze_frequencies(self, data):
        """analyze_frequencies (fse.rs:796-816): device histogram of data, plus
        the dictionary's byte counts; the table is built from it on the device."""
        L = _lib.load()
        freqs = (ctypes.c_uint32 * 256)()
        buf, n = _u8(data)
        check(L.zr_byte_histogram(buf, n, freqs))
        f = list(freqs)
        if self._dictionary:
            dbuf, dn = _u8(self._dictionary)
            dfreq = (ctypes.c_uint32 * 256)()
            check(L.zr_byte_histogram(dbuf, dn, dfreq))
            f = [(a + b) & 0xFFFFFFFF for a, b in zip(f, dfreq)]
        if not any(f):
            raise ZiporaError("No symbols found in frequency table")
        self._freqs = f

    def compress(self, data):
        """FseEncoder::compress (fse.rs:854-884)."""
        L = _lib.load()
        c = self._config.to_c()
        buf, n = _u8(data)
        if n == 0:
            return b""
        # fse.rs:859-862: a fresh table when adaptive (or on the first call)
        fresh = self._config.adaptive or self._freqs is None
        if fresh and (self._dictionary or not self._config.adaptive):
            self.analyze_frequencies(data)
        if self._config.adaptive and not self._dictionary:
            fp = None  # the histogram runs inside the compress launch
        else:
            fp = (ctypes.c_uint32 * 256)(*self._freqs)
        cap = L.zr_fse_compress_bound(n, ctypes.byref(c))
        out = (ctypes.c_uint8 * max(1, cap))()
        ol = ctypes.c_size_t(0)
        check(L.zr_fse_compress_freqs(ctypes.byref(c), fp, buf, n, out, cap, ctypes.byref(ol)))
        self._stats = EntropyStats(n, ol.value)
        return ctypes.string_at(out, ol.value)

    def stats(self):
        return self._stats

    def reset(self):
        """FseEncoder::reset (fse.rs:1052-1059): forgets the table."""
        self._freqs = None
        self._stats = EntropyStats()

    def config(self):
        return self._config


class FseDecoder:
    def __init__(self, config=None):
        self._config = config if config is not None else FseConfig()

    @classmethod
    def new(cls):
        return cls()

    @classmethod
    def with_config(cls, config):
        config.validate()
        return cls(config)

    def decompress(self, data):
        """FseDecoder::decompress (fse.rs:1105-1312)."""
        L = _lib.load()
        buf, n = _u8(data)
        size = ctypes.c_size_t(0)
        check(L.zr_fse_decompressed_size(buf, n, ctypes.byref(size)))
        cap = size.value
        out = (ctypes.c_uint8 * max(1, cap))()
        ol = ctypes.c_size_t(0)
        check(L.zr_fse_decompress(buf, n, out, cap, ctypes.byref(ol)))
        return ctypes.string_at(out, ol.value)

    def reset(self):
        pass


def fse_compress(data):
    return FseEncoder(FseConfig()).compress(data)


def fse_decompress(data):
    return FseDecoder().decompress(data)


def fse_compress_with_config(data, config):
    return FseEncoder(config).compress(data)


def fse_decompress_with_config(data, config):
    return FseDecoder.with_config(config).decompress(data)


fse_zip = fse_compress
fse_unzip = fse_decompress


class FseDevice:
    """Device-resident FSE over torch CUDA uint8 tensors (stream = torch's current)."""

    def __init__(self, config=None, max_len=0, device="cuda"):
        import torch
        self.torch = torch
        self.config = config if config is not None else FseConfig()
        self.config.validate()
        self.c = self.config.to_c()
        self.L = _lib.load()
        self.device = device
        self.meta = torch.zeros(4, dtype=torch.int64, device=device)  # out_len, status
        self._ws = None
        self._dws = None
        if max_len:
            self.reserve(max_len)

    def reserve(self, n):
        need = self.L.zr_fse_workspace_bytes(n, ctypes.byref(self.c))
        if self._ws is None or self._ws.numel() < need:
            self._ws = self.torch.empty(need + 256, dtype=self.torch.uint8, device=self.device)

    def bound(self, n):
        return self.L.zr_fse_compress_bound(n, ctypes.byref(self.c))

    def n_blocks(self, n):
        c = self.config
        if c.parallel_blocks and c.block_size and n > 2 * c.block_size and c.parallel_blocks > 1:
            return (n + c.block_size - 1) // c.block_size
        return 1

    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream().cuda_stream)

    def compress_async(self, src, out, n=None):
        n = src.numel() if n is None else n
        self.reserve(n)
        check(self.L.zr_fse_compress_dev(ctypes.byref(self.c), None, src.data_ptr(), n, out.data_ptr(),
                                         self.meta.data_ptr(), self.meta.data_ptr() + 8,
                                         self._ws.data_ptr(), self._ws.numel(), self._stream()))

    def decompress_async(self, enc, n_enc, out, max_blocks):
        need = self.L.zr_fse_decode_workspace_bytes(max_blocks)
        if self._dws is None or self._dws.numel() < need:
            self._dws = self.torch.empty(need + 256, dtype=self.torch.uint8, device=self.device)
        check(self.L.zr_fse_decompress_dev(enc.data_ptr(), n_enc, out.data_ptr(), out.numel(), max_blocks,
                                           self.meta.data_ptr(), self.meta.data_ptr() + 8,
                                           self._dws.data_ptr(), self._dws.numel(), self._stream()))

    def result(self):
        """(length, status) of the last async call (synchronises)."""
        m = self.meta.cpu()
        return int(m[0]), int(m[1] & 0xFFFFFFFF) - (1 << 32) * bool(m[1] & 0x80000000)

    def compress(self, src):
        out = self.torch.empty(self.bound(src.numel()), dtype=self.torch.uint8, device=self.device)
        self.compress_async(src, out)
        ln, st = self.result()
        if st:
            raise ZiporaError(f"FSE compression failed ({st})")
        return out[:ln]

    def decompress(self, enc, out_len, max_blocks=None):
        out = self.torch.empty(max(1, out_len), dtype=self.torch.uint8, device=self.device)
        mb = max_blocks if max_blocks is not None else max(1, self.n_blocks(out_len))
        self.decompress_async(enc, enc.numel(), out, mb)
        ln, st = self.result()
        if st:
            raise ZiporaError(f"FSE decompression failed ({st})")
        return out[:ln]


__all__ = ["FseConfig", "FseEncoder", "FseDecoder", "EntropyStats", "FseDevice", "fse_compress",
           "fse_decompress", "fse_compress_with_config", "fse_decompress_with_config", "fse_zip",
           "fse_unzip"]
