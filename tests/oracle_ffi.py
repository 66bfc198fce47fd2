"""ctypes binding of the CPU oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
The oracle restates infinilabs/zipora src/entropy (see oracle/zr_oracle.c).
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

u8p = ctypes.POINTER(ctypes.c_uint8)
sz = ctypes.c_size_t


class RansTable(ctypes.Structure):
    _fields_ = [("freq", ctypes.c_uint32 * 256), ("start", ctypes.c_uint32 * 256),
                ("total_freq", ctypes.c_uint32)]


class FseConfig(ctypes.Structure):
    _fields_ = [("table_log", ctypes.c_uint32), ("compression_level", ctypes.c_int32),
                ("max_table_size", ctypes.c_uint64), ("parallel_blocks", ctypes.c_uint64),
                ("block_size", ctypes.c_uint64), ("adaptive", ctypes.c_int32)]


class HuffTree(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("n_symbols", ctypes.c_int32),
                ("max_code_length", ctypes.c_uint32), ("code_len", ctypes.c_uint8 * 256),
                ("code", ctypes.c_uint64 * 256), ("n_nodes", ctypes.c_int32),
                ("node_leaf", ctypes.c_uint8 * 1024), ("node_sym", ctypes.c_uint8 * 1024),
                ("node_child", (ctypes.c_int16 * 2) * 1024)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
                os.path.join(ORACLE_DIR, "zr_oracle.c")):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.or_rans_table_build.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(RansTable)]
        L.or_rans_encode_bound.argtypes = [sz, ctypes.c_uint32]
        L.or_rans_encode_bound.restype = sz
        L.or_rans_encode.argtypes = [ctypes.POINTER(RansTable), ctypes.c_uint32, u8p, sz, u8p,
                                     ctypes.POINTER(sz)]
        L.or_rans_decode.argtypes = [ctypes.POINTER(RansTable), ctypes.c_uint32, u8p, sz, u8p, sz]
        L.or_rans_encode_mirror.argtypes = L.or_rans_encode.argtypes
        L.or_rans_decode_mirror.argtypes = L.or_rans_decode.argtypes
        L.or_fse_config_default.argtypes = [ctypes.POINTER(FseConfig)]
        L.or_fse_compress_bound.argtypes = [sz, ctypes.POINTER(FseConfig)]
        L.or_fse_compress_bound.restype = sz
        L.or_fse_compress.argtypes = [ctypes.POINTER(FseConfig), u8p, sz, u8p, ctypes.POINTER(sz)]
        L.or_fse_compress_freqs.argtypes = [ctypes.POINTER(FseConfig), ctypes.POINTER(ctypes.c_uint32), u8p,
                                            sz, u8p, ctypes.POINTER(sz)]
        L.or_fse_decompress.argtypes = [u8p, sz, u8p, sz, ctypes.POINTER(sz)]
        L.or_fse_decompressed_size.argtypes = [u8p, sz, ctypes.POINTER(sz)]
        L.or_fse_mul_hi.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.or_fse_mul_hi.restype = ctypes.c_uint64
        L.or_fse_renormalize_decode.argtypes = [ctypes.c_uint64, u8p, sz, ctypes.POINTER(sz)]
        L.or_fse_renormalize_decode.restype = ctypes.c_uint64
        L.or_fse_normalize_exact.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_uint32)]
        L.or_huff_tree_build.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(HuffTree)]
        L.or_huff_encode_bound.argtypes = [ctypes.POINTER(HuffTree), u8p, sz]
        L.or_huff_encode_bound.restype = sz
        L.or_huff_encode.argtypes = [ctypes.POINTER(HuffTree), u8p, sz, u8p, ctypes.POINTER(sz)]
        L.or_huff_decode.argtypes = [ctypes.POINTER(HuffTree), u8p, sz, u8p, sz, ctypes.POINTER(sz)]
        L.or_huff_tree_serialize.argtypes = [ctypes.POINTER(HuffTree), u8p]
        L.or_huff_tree_serialize.restype = sz
        L.or_huff_tree_deserialize.argtypes = [u8p, sz, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(HuffTree)]
        L.or_ctx_new.argtypes = [u8p, sz, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.or_ctx_new.restype = ctypes.c_void_p
        L.or_ctx_free.argtypes = [ctypes.c_void_p]
        L.or_ctx_serialize.argtypes = [ctypes.c_void_p, u8p]
        L.or_ctx_serialize.restype = sz
        L.or_ctx_order.argtypes = [ctypes.c_void_p]
        L.or_ctx_encode_bound.argtypes = [ctypes.c_void_p, u8p, sz]
        L.or_ctx_encode_bound.restype = sz
        L.or_ctx_encode.argtypes = [ctypes.c_void_p, u8p, sz, u8p, ctypes.POINTER(sz)]
        L.or_ctx_encode_xn.argtypes = [ctypes.c_void_p, ctypes.c_int, u8p, sz, u8p, ctypes.POINTER(sz)]
        L.or_ctx_decode.argtypes = [ctypes.c_void_p, u8p, sz, u8p, sz, ctypes.POINTER(sz)]
        L.or_ctx_decode_xn.argtypes = [ctypes.c_void_p, ctypes.c_int, u8p, sz, u8p, sz,
                                       ctypes.POINTER(sz)]
        L.or_gen_uniform.argtypes = [ctypes.c_uint64, u8p, sz]
        L.or_rans_x1_records.argtypes = [ctypes.POINTER(RansTable), ctypes.c_void_p, sz, sz, ctypes.POINTER(sz)]
        _lib = L
    return _lib


class OracleError(Exception):
    pass


def _buf(data):
    data = bytes(data)
    b = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data + b"\0" if not data else data)
    return b, len(data)


def _out(n):
    return (ctypes.c_uint8 * max(1, n))()


def _check(st, what):
    if st != 0:
        raise OracleError(f"{what} failed with status {st}")


def histogram(data):
    import numpy as np
    d = np.frombuffer(bytes(data), dtype=np.uint8)
    return [int(x) for x in np.bincount(d, minlength=256)]


# ---------------------------------------------------------------- rANS
def rans_table(raw):
    t = RansTable()
    arr = (ctypes.c_uint32 * 256)(*raw)
    _check(lib().or_rans_table_build(arr, ctypes.byref(t)), "rans_table")
    return t


def rans_encode(table, n_streams, data):
    b, n = _buf(data)
    cap = lib().or_rans_encode_bound(n, n_streams)
    out = _out(cap)
    ol = sz(0)
    _check(lib().or_rans_encode(ctypes.byref(table), n_streams, b, n, out, ctypes.byref(ol)),
           "rans_encode")
    return ctypes.string_at(out, ol.value)


def rans_decode(table, n_streams, enc, n):
    b, ln = _buf(enc)
    out = _out(n)
    _check(lib().or_rans_decode(ctypes.byref(table), n_streams, b, ln, out, n), "rans_decode")
    return ctypes.string_at(out, n)


def rans_encode_mirror(table, n_streams, data):
    """rans_encode with the reference's data structures (index vectors, Vec growth)."""
    b, n = _buf(data)
    out = _out(lib().or_rans_encode_bound(n, n_streams))
    ol = sz(0)
    _check(lib().or_rans_encode_mirror(ctypes.byref(table), n_streams, b, n, out, ctypes.byref(ol)),
           "rans_encode_mirror")
    return ctypes.string_at(out, ol.value)


def rans_decode_mirror(table, n_streams, enc, n):
    b, ln = _buf(enc)
    out = _out(n)
    _check(lib().or_rans_decode_mirror(ctypes.byref(table), n_streams, b, ln, out, n), "rans_decode_mirror")
    return ctypes.string_at(out, n)


# ------------------------------------------------------- RansCompressor
# compression/mod.rs:416-512 composed from the rANS restatement above.
def rans_compressor_table(train):
    """RansCompressor::new (mod.rs:425-452): byte counts (the min-1 fix-up at
    :438-448 never fires: present symbols already count >= 1) -> Rans64Encoder::new."""
    if not train:
        raise OracleError("rANS compressor requires training data")
    return rans_table(histogram(train))


def rans_compressor_compress(table, data):
    """Compressor::compress (mod.rs:457-477)."""
    import struct
    if not data:
        return b""
    hdr = b"".join(struct.pack("<I", table.freq[i]) for i in range(256))
    return hdr + struct.pack("<I", len(data) & 0xFFFFFFFF) + rans_encode(table, 1, data)


def rans_compressor_decompress(rec):
    """Compressor::decompress (mod.rs:479-516): Rans64Encoder::new on the STORED
    normalised frequencies (re-normalises them: finding 0.9)."""
    import struct
    if not rec:
        return b""
    if len(rec) < 1028:
        raise OracleError("Invalid rANS compressed data format")
    freqs = list(struct.unpack("<256I", rec[:1024]))
    size = struct.unpack("<I", rec[1024:1028])[0]
    return rans_decode(rans_table(freqs), 1, rec[1028:], size)


# ---------------------------------------------------------------- FSE
def fse_config(**kw):
    c = FseConfig()
    lib().or_fse_config_default(ctypes.byref(c))
    for k, v in kw.items():
        if k == "parallel_blocks" and v is None:
            v = 0
        setattr(c, k, v)
    return c


def fse_compress(data, config=None):
    c = config or fse_config()
    b, n = _buf(data)
    out = _out(lib().or_fse_compress_bound(n, ctypes.byref(c)))
    ol = sz(0)
    _check(lib().or_fse_compress(ctypes.byref(c), b, n, out, ctypes.byref(ol)), "fse_compress")
    return ctypes.string_at(out, ol.value)


def fse_compress_freqs(data, freqs, config=None):
    c = config or fse_config()
    b, n = _buf(data)
    out = _out(lib().or_fse_compress_bound(n, ctypes.byref(c)))
    ol = sz(0)
    _check(lib().or_fse_compress_freqs(ctypes.byref(c), (ctypes.c_uint32 * 256)(*freqs), b, n, out,
                                       ctypes.byref(ol)), "fse_compress_freqs")
    return ctypes.string_at(out, ol.value)


def fse_renormalize_decode(state, data, pos):
    """FseTable::renormalize_decode (fse.rs:704-735): returns (state, pos)."""
    p = sz(pos)
    b, n = _buf(data)
    x = lib().or_fse_renormalize_decode(state, b, n, ctypes.byref(p))
    if x == 0:  # input[*pos] past the input: a panic in the reference (fse.rs:729)
        raise OracleError("renormalize_decode: index out of bounds")
    return x, p.value


def fse_decompress(data, cap=None):
    b, n = _buf(data)
    if cap is None:
        s = sz(0)
        st = lib().or_fse_decompressed_size(b, n, ctypes.byref(s))
        _check(st, "fse_size")
        cap = s.value
    out = _out(cap)
    ol = sz(0)
    _check(lib().or_fse_decompress(b, n, out, cap, ctypes.byref(ol)), "fse_decompress")
    return ctypes.string_at(out, ol.value)


# ---------------------------------------------------------------- Huffman
def huff_tree(freq):
    t = HuffTree()
    _check(lib().or_huff_tree_build((ctypes.c_uint32 * 256)(*freq), ctypes.byref(t)), "huff_tree")
    return t


def huff_codes(t):
    """symbol -> code as a '0'/'1' string in emission order."""
    return {s: "".join("1" if (t.code[s] >> j) & 1 else "0" for j in range(t.code_len[s]))
            for s in range(256) if t.code_len[s]}


def huff_encode(t, data):
    b, n = _buf(data)
    out = _out(lib().or_huff_encode_bound(ctypes.byref(t), b, n))
    ol = sz(0)
    _check(lib().or_huff_encode(ctypes.byref(t), b, n, out, ctypes.byref(ol)), "huff_encode")
    return ctypes.string_at(out, ol.value)


def huff_decode(t, enc, n):
    b, ln = _buf(enc)
    out = _out(n)
    ol = sz(0)
    _check(lib().or_huff_decode(ctypes.byref(t), b, ln, out, n, ctypes.byref(ol)), "huff_decode")
    return ctypes.string_at(out, ol.value)


def huff_tree_serialize(t):
    """HuffmanTree::serialize (tree.rs:226-262), symbols ascending."""
    out = _out(2 + 256 * 10)
    n = lib().or_huff_tree_serialize(ctypes.byref(t), out)
    return ctypes.string_at(out, n)


def huff_tree_deserialize(data, order=None):
    """HuffmanTree::deserialize (tree.rs:265-356); `order` = HashMap insertion order."""
    b, n = _buf(data)
    t = HuffTree()
    o = (ctypes.c_int * 256)(*order) if order is not None else None
    _check(lib().or_huff_tree_deserialize(b, n, o, ctypes.byref(t)), "huff_tree_deserialize")
    return t


def huff_compressor_compress(t, data):
    """HuffmanCompressor::compress (compression/mod.rs:345-369)."""
    import struct
    if not data:
        return b""
    body = huff_encode(t, data)
    tree = huff_tree_serialize(t)
    return struct.pack("<I", len(tree)) + tree + struct.pack("<I", len(data) & 0xFFFFFFFF) + body


def huff_compressor_decompress(rec, order=None):
    """HuffmanCompressor::decompress (compression/mod.rs:371-407)."""
    import struct
    if not rec:
        return b""
    if len(rec) < 8:
        raise OracleError("Huffman compressed data too short")
    ts = struct.unpack("<I", rec[:4])[0]
    if len(rec) < 8 + ts:
        raise OracleError("Huffman compressed data truncated")
    t = huff_tree_deserialize(rec[4:4 + ts], order)
    size = struct.unpack("<I", rec[4 + ts:8 + ts])[0]
    return huff_decode(t, rec[8 + ts:], size)


# ------------------------------------------------- PA-Zip / DictZip stages
def pazip_fse_config(table_log=12, compression_level=3, adaptive=True):
    """dict_zip FseConfig::to_entropy_config (compression_types.rs:2107-2123)."""
    return fse_config(table_log=table_log, compression_level=compression_level, adaptive=int(adaptive),
                      parallel_blocks=0, block_size=64 * 1024, max_table_size=64 * 1024)


def pazip_apply(data, cfg):
    """apply_fse_compression (compression_types.rs:2272-2299)."""
    if not data:
        return b""
    if len(data) < 32:
        return b"UN" + data
    if not (5 <= cfg.table_log <= 15 and 1 <= cfg.compression_level <= 22):
        raise OracleError("invalid FSE config")
    comp = fse_compress(data, cfg)
    return b"\xfeS" + comp if len(comp) < len(data) else b"UN" + data


def pazip_remove(data, cfg):
    """remove_fse_compression (compression_types.rs:2310-2340)."""
    if not data:
        return b""
    if len(data) < 2:
        return data
    if data[:2] == b"UN":
        return data[2:]
    if not (5 <= cfg.table_log <= 15 and 1 <= cfg.compression_level <= 22):
        raise OracleError("invalid FSE config")
    body = data[2:] if data[:2] == b"\xfeS" else data
    return fse_decompress(body) if body else b""


def dictzip_encode(algo, interleave, ctx, ratio, data):
    """apply_entropy_encoding + check_compression_ratio (blob_store.rs:1075-1161, :1292-1304)."""
    import numpy as np
    if algo == 0:
        return data, 0
    if algo == 1:
        nway = {0: 1, 1: 1, 2: 2, 4: 4, 8: 8}.get(interleave)
        if nway is None:
            raise OracleError("Invalid interleaving factor")
        enc = ctx.encode(data) if nway == 1 else ctx.encode_xn(nway, data)
    else:
        enc = fse_compress(data, fse_config(parallel_blocks=interleave if interleave > 1 else 0))
    if data and np.float32(len(enc)) / np.float32(len(data)) <= np.float32(ratio):
        return enc, algo
    return data, 0


def dictzip_decode(algo, ctx, data, original_size):
    """decode_entropy (blob_store.rs:1164-1224): O1 with the plain decoder and original_size."""
    if algo == 0:
        return data
    if algo == 1:
        return ctx.decode(data, original_size)
    return fse_decompress(data)


# ---------------------------------------------------------------- contextual
class Ctx:
    def __init__(self, train, order):
        b, n = _buf(train)
        st = ctypes.c_int(0)
        self.h = lib().or_ctx_new(b, n, order, ctypes.byref(st))
        _check(st.value, "ctx_new")

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_ctx_free(self.h)

    @property
    def order(self):
        return lib().or_ctx_order(self.h)

    def encode(self, data):
        b, n = _buf(data)
        out = _out(lib().or_ctx_encode_bound(self.h, b, n))
        ol = sz(0)
        _check(lib().or_ctx_encode(self.h, b, n, out, ctypes.byref(ol)), "ctx_encode")
        return ctypes.string_at(out, ol.value)

    def encode_xn(self, nway, data):
        b, n = _buf(data)
        out = _out(lib().or_ctx_encode_bound(self.h, b, n))
        ol = sz(0)
        _check(lib().or_ctx_encode_xn(self.h, nway, b, n, out, ctypes.byref(ol)), "ctx_encode_xn")
        return ctypes.string_at(out, ol.value)

    def decode(self, enc, n):
        b, ln = _buf(enc)
        out = _out(n)
        ol = sz(0)
        _check(lib().or_ctx_decode(self.h, b, ln, out, n, ctypes.byref(ol)), "ctx_decode")
        return ctypes.string_at(out, ol.value)

    def serialize(self):
        """ContextualHuffmanEncoder::serialize (interleaved.rs:476-503), canonical order."""
        out = _out(9 + 8 * 1024 + 1025 * (4 + 2 + 256 * 10))  # order 2 keeps <= 1024 contexts
        n = lib().or_ctx_serialize(self.h, out)
        return ctypes.string_at(out, n)

    def decode_xn(self, nway, enc, n):
        b, ln = _buf(enc)
        out = _out(n)
        ol = sz(0)
        _check(lib().or_ctx_decode_xn(self.h, nway, b, ln, out, n, ctypes.byref(ol)), "ctx_decode_xn")
        return ctypes.string_at(out, ol.value)


def rans_x1_records(table, buf, offset, n_rec, rec_len):
    """x1 encode+decode of n_rec records of rec_len bytes of `buf` (a bytes-like
    object kept alive by the caller) starting at `offset`, one C call (the GIL is
    released for the whole group). Returns the encoded byte total."""
    base = ctypes.addressof(ctypes.c_char.from_buffer(buf)) if isinstance(buf, bytearray) else \
        ctypes.cast(ctypes.c_char_p(buf), ctypes.c_void_p).value
    tot = sz(0)
    _check(lib().or_rans_x1_records(ctypes.byref(table), base + offset, n_rec, rec_len, ctypes.byref(tot)),
           "rans_x1_records")
    return tot.value


def gen_uniform(n, seed=0x9E3779B97F4A7C15):
    out = _out(n)
    lib().or_gen_uniform(seed, out, n)
    return ctypes.string_at(out, n)
