"""The entropy facade of src/entropy/mod.rs:56-330:
EntropyAlgorithm (name, is_available, available_algorithms, select_for_data),
EntropyConfig presets and EntropyStats.

select_for_data and EntropyStats.calculate_entropy count the bytes with the
device histogram kernel (zr_byte_histogram, the same k_fse_hist that FSE's
analyze_frequencies uses); what remains is host arithmetic on 256 counts, in
the reference's f64 order (mod.rs:301-319, :123-152). The reference is built
with its default features, so `zstd` is on and Fse / KFse exist
(Cargo.toml:27).
"""
import ctypes
import enum
import math
from dataclasses import dataclass

from . import _lib
from .errors import check


def byte_counts(data):
    """[u32; 256] byte frequencies of data, counted on the device."""
    data = bytes(data)
    freqs = (ctypes.c_uint32 * 256)()
    if data:
        buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data)
        check(_lib.load().zr_byte_histogram(buf, len(data), freqs))
    return list(freqs)


def entropy_from_counts(counts):
    """EntropyStats::calculate_entropy (mod.rs:301-319) on given counts: the
    Shannon entropy in bits, summed over the bins in index order."""
    total = float(sum(counts))
    if total == 0:
        return 0.0
    e = 0.0
    for f in counts:
        if f > 0:
            p = f / total
            e -= p * math.log2(p)
    return e


class EntropyAlgorithm(enum.Enum):
    """EntropyAlgorithm (mod.rs:56-72); Auto is the default."""
    Huffman = "Huffman"
    Rans = "rANS"
    Fse = "FSE"
    KFse = "kFSE"
    Dictionary = "Dictionary"
    Auto = "Auto"

    def name_str(self):
        """EntropyAlgorithm::name (mod.rs:76-87)."""
        return self.value

    def is_available(self):
        """EntropyAlgorithm::is_available (mod.rs:90-105): every variant of this build."""
        return True

    @staticmethod
    def available_algorithms():
        """EntropyAlgorithm::available_algorithms (mod.rs:108-121), in the reference's order."""
        A = EntropyAlgorithm
        return [A.Huffman, A.Rans, A.Dictionary, A.Auto, A.Fse, A.KFse]

    @staticmethod
    def default():
        return EntropyAlgorithm.Auto

    @staticmethod
    def select_from_counts(counts, size):
        """The decision of select_for_data (mod.rs:137-152) on a histogram."""
        A = EntropyAlgorithm
        e = entropy_from_counts(counts)
        unique = sum(1 for f in counts if f > 0)
        r = 1.0 - unique / 256.0
        if r > 0.8:
            return A.Dictionary  # high repetitiveness
        if e < 4.0 and size > 1024:
            return A.Fse  # low entropy, larger data
        if 4.0 <= e <= 6.0 and size > 256:
            return A.Rans  # medium entropy, medium size
        return A.Huffman

    @staticmethod
    def select_for_data(data):
        """EntropyAlgorithm::select_for_data (mod.rs:124-153)."""
        data = bytes(data)
        if not data:
            return EntropyAlgorithm.Huffman  # default for empty data
        return EntropyAlgorithm.select_from_counts(byte_counts(data), len(data))


@dataclass
class EntropyConfig:
    """EntropyConfig (mod.rs:158-196) and its presets (mod.rs:198-236)."""
    algorithm: EntropyAlgorithm = EntropyAlgorithm.Auto
    fse_config: object = None
    compression_level: int = 3
    adaptive: bool = True
    dict_size: int = 0
    fast_decode: bool = False

    def __post_init__(self):
        if self.fse_config is None:
            from .fse import FseConfig
            self.fse_config = FseConfig()

    @classmethod
    def default(cls):
        return cls()

    @classmethod
    def fast(cls):
        from .fse import FseConfig
        return cls(algorithm=EntropyAlgorithm.Huffman, compression_level=1, fast_decode=True,
                   fse_config=FseConfig.fast_compression())

    @classmethod
    def high_compression(cls):
        from .fse import FseConfig
        return cls(algorithm=EntropyAlgorithm.Fse, compression_level=19, adaptive=True, dict_size=32 * 1024,
                   fse_config=FseConfig.high_compression())

    @classmethod
    def balanced(cls):
        return cls()


@dataclass
class EntropyStats:
    """EntropyStats (mod.rs:241-300): sizes, ratio, bits per symbol, entropy, efficiency."""
    input_size: int = 0
    output_size: int = 0
    entropy: float = 0.0

    @classmethod
    def new(cls, input_size, output_size, entropy):
        return cls(input_size, output_size, entropy)

    @property
    def compression_ratio(self):
        return self.output_size / self.input_size if self.input_size > 0 else 0.0

    @property
    def bits_per_symbol(self):
        return (self.output_size * 8) / self.input_size if self.input_size > 0 else 0.0

    @property
    def efficiency(self):
        b = self.bits_per_symbol
        return self.entropy / b if b > 0.0 else 0.0

    def space_savings(self):
        """EntropyStats::space_savings (mod.rs:295-298), percent."""
        return (1.0 - self.compression_ratio) * 100.0

    @staticmethod
    def calculate_entropy(data):
        """EntropyStats::calculate_entropy (mod.rs:301-319); the counts on the device."""
        data = bytes(data)
        if not data:
            return 0.0
        return entropy_from_counts(byte_counts(data))


__all__ = ["EntropyAlgorithm", "EntropyConfig", "EntropyStats", "byte_counts", "entropy_from_counts"]
