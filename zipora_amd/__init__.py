"""zipora_amd -- MI355X-native (gfx950) entropy-coding backend for zipora's src/entropy.

Host mirror of the reference's Rust surface over the C ABI of libzipora_amd.so
(include/zipora_amd.h). Every codec call runs hand-written HIP kernels; there is
no CPU fallback.
"""
from ._lib import load, last_error, LIB_PATH  # noqa: F401
from .errors import ZiporaError  # noqa: F401
from .rans import (AdaptiveRans64Encoder, ParallelVariant, ParallelX1, ParallelX2, ParallelX4,  # noqa: F401
                   ParallelX8, Rans64Decoder, Rans64Encoder, Rans64Symbol, device_alloc_count, fallback_lanes,
                   histogram, selftest_reciprocal)

__version__ = "0.1.0"


def synth(kind, n, seed=0):
    """Deterministic synthetic bytes: 'u' uniform xorshift, 'z' Zipf(1.1), 't' text-like."""
    import ctypes
    k = {"u": 0, "z": 1, "t": 2}[kind]
    buf = (ctypes.c_uint8 * max(1, n))()
    from .errors import check
    check(load().zr_synth_fill(k, seed, buf, n))
    return ctypes.string_at(buf, n)
from .fse import (EntropyStats, FseConfig, FseDecoder, FseDevice, FseEncoder,  # noqa: F401,E402
                  fse_compress, fse_compress_with_config, fse_decompress, fse_decompress_with_config,
                  fse_unzip, fse_zip)
from .huffman import (ContextualHuffmanDecoder, ContextualHuffmanEncoder, HuffmanCompressor,  # noqa: F401,E402
                      HuffmanDecoder, HuffmanEncoder, HuffmanO1Device, HuffmanOrder, HuffmanTree, InterleavingFactor)
from .compression import RansCompressor  # noqa: F401,E402
# the src/entropy/mod.rs facade (EntropyAlgorithm there is zipora_amd.entropy.EntropyAlgorithm;
# the top-level name is dict_zip's, as in the reference's pa-zip stage)
from . import entropy  # noqa: F401,E402
from .entropy import EntropyConfig  # noqa: F401,E402
from .pazip import (DictZipEntropyStage, EntropyAlgorithm, PaZipFseConfig,  # noqa: F401,E402
                    apply_fse_compression, remove_fse_compression)
