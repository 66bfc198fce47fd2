"""ctypes binding of libzipora_amd.so (the C ABI declared in include/zipora_amd.h).

The product path fails loudly when the HIP library is missing: there is no CPU
fallback anywhere in this package.
"""
import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libzipora_amd.so")
# tools only: ZR_DIAG_LIB=1 loads the -DZR_DIAG build (profiling ablations that
# read ZR_ABLATE / ZR_DEC_ABL / ZR_COMPACT_OLD), ZR_LIB_PATH another build (A/B
# runs); bench.py refuses to print a metric line under either
DIAG_LIB_PATH = os.path.join(_PKG, "libzipora_amd_diag.so")
DIAG_ENV = ("ZR_CMP_ABL", "ZR_DIAG_LIB", "ZR_LIB_PATH", "ZR_ABLATE", "ZR_DEC_ABL", "ZR_COMPACT_OLD")


def diag_env():
    """The diagnostic switches set in this process's environment."""
    return [k for k in DIAG_ENV if os.environ.get(k)]

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_sz = ctypes.c_size_t
c_vp = ctypes.c_void_p

ZR_OK = 0
ZR_INVALID_INPUT = -1
ZR_MEMORY_ERROR = -2
ZR_UNSUPPORTED = -4
ZR_INTERNAL = -5


class RansTable(ctypes.Structure):
    _fields_ = [("freq", ctypes.c_uint32 * 256), ("start", ctypes.c_uint32 * 256),
                ("total_freq", ctypes.c_uint32)]


class RansBatch(ctypes.Structure):
    _fields_ = [("n_buffers", ctypes.c_uint32), ("n_streams", ctypes.c_uint32),
                ("max_len", ctypes.c_uint64), ("len", c_vp), ("raw_off", c_vp),
                ("enc_off", c_vp), ("enc_len", c_vp), ("status", c_vp), ("tables", c_vp),
                ("table_stride", ctypes.c_uint32), ("min_len", ctypes.c_uint64)]


class FseConfig(ctypes.Structure):
    _fields_ = [("table_log", ctypes.c_uint32), ("compression_level", ctypes.c_int32),
                ("max_table_size", ctypes.c_uint64), ("parallel_blocks", ctypes.c_uint64),
                ("block_size", ctypes.c_uint64), ("adaptive", ctypes.c_int32)]


class HuffTree(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("n_symbols", ctypes.c_int32),
                ("max_code_length", ctypes.c_uint32), ("code_len", ctypes.c_uint8 * 256),
                ("code", ctypes.c_uint64 * 256), ("n_nodes", ctypes.c_int32),
                ("child", (ctypes.c_int16 * 2) * 511), ("sym", ctypes.c_uint8 * 511)]


# (name, restype, argtypes) for every exported symbol; tests check this list
# against include/zipora_amd.h.
SIGNATURES = [
    ("zr_last_error", ctypes.c_char_p, []),
    ("zr_set_error_callback", None, [c_vp]),
    ("zr_version", ctypes.c_char_p, []),
    ("zr_device_count", ctypes.c_int32, [c_i32p]),
    ("zr_set_device", ctypes.c_int32, [ctypes.c_int32]),
    ("zr_rans_table_build", ctypes.c_int32, [c_u32p, ctypes.POINTER(RansTable)]),
    ("zr_rans_encode_bound", c_sz, [c_sz, ctypes.c_uint32]),
    ("zr_rans_encode", ctypes.c_int32, [ctypes.POINTER(RansTable), ctypes.c_uint32, c_u8p, c_sz,
                                        c_u8p, c_sz, ctypes.POINTER(c_sz)]),
    ("zr_rans_decode", ctypes.c_int32, [ctypes.POINTER(RansTable), ctypes.c_uint32, c_u8p, c_sz,
                                        c_u8p, c_sz]),
    ("zr_rans_adaptive_streams", ctypes.c_uint32, [c_sz]),
    ("zr_rans_encode_adaptive", ctypes.c_int32, [c_u8p, c_sz, c_u8p, c_sz, ctypes.POINTER(c_sz), c_u32p]),
    ("zr_rans_selftest_reciprocal", ctypes.c_int32, [c_u64p]),
    ("zr_comm_unique_id", ctypes.c_int32, [c_u8p]),
    ("zr_comm_init", ctypes.c_int32, [c_u8p, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(c_vp)]),
    ("zr_comm_count", ctypes.c_int32, [c_vp, c_i32p]),
    ("zr_histogram_allreduce_dev", ctypes.c_int32, [c_vp, c_vp, ctypes.c_uint32, c_vp]),
    ("zr_table_broadcast_dev", ctypes.c_int32, [c_vp, c_vp, ctypes.c_uint32, ctypes.c_int32, c_vp]),
    ("zr_comm_destroy", ctypes.c_int32, [c_vp]),
    ("zr_rans_fallback_lanes", ctypes.c_int32, [c_u64p, ctypes.c_int32]),
    ("zr_rans_symbol_fast_div", ctypes.c_int32, [ctypes.c_uint32, ctypes.c_uint32, c_u64p, c_sz, c_u64p, c_u64p]),
    ("zr_device_alloc_count", ctypes.c_int32, [c_u64p]),
    ("zr_rans_dtab_bytes", c_sz, []),
    ("zr_rans_dtab_upload", ctypes.c_int32, [ctypes.POINTER(RansTable), ctypes.c_uint32, c_vp, c_vp]),
    ("zr_histogram_dev", ctypes.c_int32, [c_vp, ctypes.POINTER(RansBatch), ctypes.c_int32, c_vp, c_vp]),
    ("zr_rans_dtab_from_hist_dev", ctypes.c_int32, [c_vp, ctypes.c_uint32, c_vp, c_vp]),
    ("zr_rans_dtab_from_hist_consume_dev", ctypes.c_int32, [c_vp, ctypes.c_uint32, c_vp, c_vp]),
    ("zr_rans_dtab_from_data_dev", ctypes.c_int32, [c_vp, ctypes.POINTER(RansBatch), c_vp, c_vp, c_vp]),
    ("zr_rans_decoder_kernel", ctypes.c_char_p, [ctypes.c_uint32, ctypes.c_uint32]),
    ("zr_rans_workspace_bytes", c_sz, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]),
    ("zr_rans_encode_batch_dev", ctypes.c_int32, [ctypes.POINTER(RansBatch), c_vp, c_vp, c_vp, c_sz,
                                                  c_vp]),
    ("zr_rans_decode_batch_dev", ctypes.c_int32, [ctypes.POINTER(RansBatch), c_vp, c_vp, c_vp, c_sz,
                                                  c_vp]),
    ("zr_rans_pipe_create", ctypes.c_int32, [ctypes.POINTER(RansTable), ctypes.c_uint32, ctypes.c_uint64,
                                             ctypes.POINTER(c_vp)]),
    ("zr_rans_pipe_destroy", ctypes.c_int32, [c_vp]),
    ("zr_rans_pipe_encode", ctypes.c_int32, [c_vp, ctypes.c_uint32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                             c_vp]),
    ("zr_rans_pipe_encode_packed", ctypes.c_int32, [c_vp, ctypes.c_uint32, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp,
                                                    c_vp, c_vp, c_vp]),
    ("zr_rans_pipe_decode", ctypes.c_int32, [c_vp, ctypes.c_uint32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                             c_vp]),
    ("zr_rans_compressor_train", ctypes.c_int32, [c_u8p, c_sz, ctypes.POINTER(RansTable)]),
    ("zr_rans_compressor_bound", c_sz, [c_sz]),
    ("zr_rans_compressor_compress", ctypes.c_int32, [ctypes.POINTER(RansTable), c_u8p, c_sz, c_u8p, c_sz,
                                                     ctypes.POINTER(c_sz)]),
    ("zr_rans_compressor_decompressed_size", ctypes.c_int32, [c_u8p, c_sz, ctypes.POINTER(c_sz)]),
    ("zr_rans_compressor_decompress", ctypes.c_int32, [c_u8p, c_sz, c_u8p, c_sz, ctypes.POINTER(c_sz)]),
    ("zr_rans_compressor_workspace_bytes", c_sz, [ctypes.c_uint32, ctypes.c_uint64]),
    ("zr_rans_compressor_compress_batch_dev", ctypes.c_int32, [ctypes.POINTER(RansBatch), c_vp, c_vp, c_vp,
                                                               c_sz, c_vp]),
    ("zr_rans_compressor_decompress_batch_dev", ctypes.c_int32, [ctypes.POINTER(RansBatch), c_vp, c_vp, c_vp,
                                                                 c_sz, c_vp]),
    ("zr_host_register", ctypes.c_int32, [c_vp, c_sz]),
    ("zr_host_unregister", ctypes.c_int32, [c_vp]),
    ("zr_fse_config_default", None, [ctypes.POINTER(FseConfig)]),
    ("zr_fse_compress_bound", c_sz, [c_sz, ctypes.POINTER(FseConfig)]),
    ("zr_fse_compress", ctypes.c_int32, [ctypes.POINTER(FseConfig), c_u8p, c_sz, c_u8p, c_sz,
                                         ctypes.POINTER(c_sz)]),
    ("zr_fse_decompress", ctypes.c_int32, [c_u8p, c_sz, c_u8p, c_sz, ctypes.POINTER(c_sz)]),
    ("zr_fse_decompressed_size", ctypes.c_int32, [c_u8p, c_sz, ctypes.POINTER(c_sz)]),
    ("zr_fse_workspace_bytes", c_sz, [c_sz, ctypes.POINTER(FseConfig)]),
    ("zr_fse_compress_dev", ctypes.c_int32, [ctypes.POINTER(FseConfig), c_vp, c_vp, c_sz, c_vp, c_vp,
                                             c_vp, c_vp, c_sz, c_vp]),
    ("zr_fse_compress_freqs", ctypes.c_int32, [ctypes.POINTER(FseConfig), c_u32p, c_u8p, c_sz, c_u8p,
                                               c_sz, ctypes.POINTER(c_sz)]),
    ("zr_byte_histogram", ctypes.c_int32, [c_u8p, c_sz, c_u32p]),
    ("zr_fse_decode_workspace_bytes", c_sz, [ctypes.c_uint64]),
    ("zr_fse_decompress_dev", ctypes.c_int32, [c_vp, c_sz, c_vp, c_sz, ctypes.c_uint64, c_vp, c_vp,
                                               c_vp, c_sz, c_vp]),
    ("zr_pazip_fse_bound", c_sz, [c_sz, ctypes.POINTER(FseConfig)]),
    ("zr_pazip_fse_apply", ctypes.c_int32, [ctypes.POINTER(FseConfig), c_u8p, c_sz, c_u8p, c_sz,
                                            ctypes.POINTER(c_sz)]),
    ("zr_pazip_fse_removed_size", ctypes.c_int32, [c_u8p, c_sz, ctypes.POINTER(c_sz)]),
    ("zr_pazip_fse_remove", ctypes.c_int32, [ctypes.POINTER(FseConfig), c_u8p, c_sz, c_u8p, c_sz,
                                             ctypes.POINTER(c_sz)]),
    ("zr_dictzip_entropy_encode", ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, c_vp, ctypes.c_float, c_u8p,
                                                   c_sz, c_u8p, c_sz, ctypes.POINTER(c_sz), c_i32p]),
    ("zr_dictzip_entropy_decode", ctypes.c_int32, [ctypes.c_int32, c_vp, c_u8p, c_sz, c_sz, c_u8p, c_sz,
                                                   ctypes.POINTER(c_sz)]),
    ("zr_huff_tree_build", ctypes.c_int32, [c_u32p, ctypes.POINTER(HuffTree)]),
    ("zr_huff_encode_bound", c_sz, [ctypes.POINTER(HuffTree), c_sz]),
    ("zr_huff_encode", ctypes.c_int32, [ctypes.POINTER(HuffTree), c_u8p, c_sz, c_u8p, c_sz,
                                        ctypes.POINTER(c_sz)]),
    ("zr_huff_decode", ctypes.c_int32, [ctypes.POINTER(HuffTree), c_u8p, c_sz, c_u8p, c_sz]),
    ("zr_huff_workspace_bytes", c_sz, [c_sz, c_sz]),
    ("zr_huff_encode_dev", ctypes.c_int32, [ctypes.POINTER(HuffTree), c_vp, c_sz, c_vp, c_sz, c_vp,
                                            c_vp, c_vp, c_sz, c_vp]),
    ("zr_huff_decode_dev", ctypes.c_int32, [ctypes.POINTER(HuffTree), c_vp, c_sz, c_vp, c_sz, c_vp,
                                            c_vp, c_sz, c_vp]),
    ("zr_huff_tree_serialized_bound", c_sz, []),
    ("zr_huff_tree_serialize", ctypes.c_int32, [ctypes.POINTER(HuffTree), c_u8p, c_sz, ctypes.POINTER(c_sz)]),
    ("zr_huff_tree_deserialize", ctypes.c_int32, [c_u8p, c_sz, ctypes.POINTER(HuffTree)]),
    ("zr_huff_compressor_train", ctypes.c_int32, [c_u8p, c_sz, ctypes.POINTER(HuffTree)]),
    ("zr_huff_compressor_bound", c_sz, [ctypes.POINTER(HuffTree), c_sz]),
    ("zr_huff_compressor_compress", ctypes.c_int32, [ctypes.POINTER(HuffTree), c_u8p, c_sz, c_u8p, c_sz,
                                                     ctypes.POINTER(c_sz)]),
    ("zr_huff_compressor_decompressed_size", ctypes.c_int32, [c_u8p, c_sz, ctypes.POINTER(c_sz)]),
    ("zr_huff_compressor_decompress", ctypes.c_int32, [c_u8p, c_sz, c_u8p, c_sz, ctypes.POINTER(c_sz)]),
    ("zr_ctx_huff_new", ctypes.c_int32, [c_u8p, c_sz, ctypes.c_int32, ctypes.POINTER(c_vp)]),
    ("zr_ctx_huff_free", None, [c_vp]),
    ("zr_ctx_huff_serialized_size", c_sz, [c_vp]),
    ("zr_ctx_huff_serialize", ctypes.c_int32, [c_vp, c_u8p, c_sz, ctypes.POINTER(c_sz)]),
    ("zr_ctx_huff_deserialize", ctypes.c_int32, [c_u8p, c_sz, ctypes.POINTER(c_vp)]),
    ("zr_ctx_huff_order", ctypes.c_int32, [c_vp]),
    ("zr_ctx_huff_encode_bound", c_sz, [c_vp, c_sz]),
    ("zr_ctx_huff_encode", ctypes.c_int32, [c_vp, ctypes.c_int32, c_u8p, c_sz, c_u8p, c_sz,
                                            ctypes.POINTER(c_sz)]),
    ("zr_ctx_huff_decode", ctypes.c_int32, [c_vp, ctypes.c_int32, c_u8p, c_sz, c_u8p, c_sz,
                                            ctypes.POINTER(c_sz)]),
    ("zr_ctx_huff_encode_dev", ctypes.c_int32, [c_vp, ctypes.c_int32, c_vp, c_sz, c_vp, c_vp]),
    ("zr_ctx_huff_decode_dev", ctypes.c_int32, [c_vp, ctypes.c_int32, c_vp, c_sz, c_vp, c_sz, c_vp]),
    ("zr_ctx_huff_tree0", ctypes.c_int32, [c_vp, ctypes.POINTER(HuffTree)]),
    ("zr_malloc_dev", ctypes.c_int32, [ctypes.POINTER(c_vp), c_sz]),
    ("zr_free_dev", ctypes.c_int32, [c_vp]),
    ("zr_memcpy_h2d", ctypes.c_int32, [c_vp, c_vp, c_sz, c_vp]),
    ("zr_memcpy_d2h", ctypes.c_int32, [c_vp, c_vp, c_sz, c_vp]),
    ("zr_memset_dev", ctypes.c_int32, [c_vp, ctypes.c_int, c_sz, c_vp]),
    ("zr_release_call_contexts", ctypes.c_int32, []),
    ("zr_memcpy_dev", ctypes.c_int32, [c_vp, c_vp, c_sz, ctypes.c_uint32, c_vp]),
    ("zr_stream_sync", ctypes.c_int32, [c_vp]),
    ("zr_timer_enable", ctypes.c_int32, [ctypes.c_int32]),
    ("zr_timer_select", ctypes.c_int32, [ctypes.c_char_p]),
    ("zr_timer_reset", ctypes.c_int32, []),
    ("zr_timer_read", ctypes.c_int32, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_uint64)]),
    ("zr_synth_fill", ctypes.c_int32, [ctypes.c_int32, ctypes.c_uint64, c_u8p, c_sz]),
]

_lib = None


def load(build_if_missing=True):
    """Load the HIP library (building it in-tree first if it is absent)."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        # torch bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's):
        # load it first so the process holds ONE HIP runtime and torch streams
        # and allocations are valid handles for this library too.
        import torch  # noqa: F401
    except Exception:
        pass
    diag = bool(os.environ.get("ZR_DIAG_LIB"))
    path = DIAG_LIB_PATH if diag else LIB_PATH
    if os.environ.get("ZR_LIB_PATH"):  # tools only (A/B of two builds on one box)
        path = os.environ["ZR_LIB_PATH"]
    if not os.path.exists(path):
        if not build_if_missing:
            raise RuntimeError(f"zipora_amd: HIP library missing at {path}; run "
                               "`python -m zipora_amd.build`")
        from . import build as _b
        _b.build(diag=diag)
    L = ctypes.CDLL(path)
    for name, res, args in SIGNATURES:
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def last_error():
    m = load().zr_last_error()
    return m.decode() if m else ""
