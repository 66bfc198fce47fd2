"""Huffman -- host mirror of src/entropy/huffman over the HIP C ABI.

Same names and argument meaning as the reference:
  HuffmanTree.from_frequencies / from_data, get_code, max_code_length   tree.rs:52-216
  HuffmanEncoder(data) / HuffmanEncoder.from_frequencies, encode, tree   encoder.rs:76-134
  HuffmanDecoder(tree).decode(encoded, output_length)                    decoder.rs:85-165
  HuffmanOrder, InterleavingFactor                                       interleaved.rs:16-75
  ContextualHuffmanEncoder(data, order): encode, encode_with_interleaving,
    encode_x1..x8, decode_with_interleaving, decode_x1..x8, order, tree_count
  ContextualHuffmanDecoder(encoder).decode(encoded, output_length)       interleaved.rs:1039-1209
The tree is built by host C++ in libzipora_amd.so (<= 256 leaves); every
encode/decode runs in HIP kernels (zr_huff.hip). Errors raise ZiporaError.
"""
import ctypes
import struct
import enum

from . import _lib
from .errors import ZiporaError, check


def _u8(data):
    data = bytes(data)
    return (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0"), len(data)


class HuffmanTree:
    def __init__(self, t):
        self._t = t

    @classmethod
    def from_frequencies(cls, frequencies):
        f = [int(x) & 0xFFFFFFFF for x in frequencies]
        if len(f) != 256:
            raise ValueError("frequencies must have 256 entries")
        t = _lib.HuffTree()
        check(_lib.load().zr_huff_tree_build((ctypes.c_uint32 * 256)(*f), ctypes.byref(t)))
        return cls(t)

    @classmethod
    def from_data(cls, data):
        import numpy as np
        h = np.bincount(np.frombuffer(bytes(data), dtype=np.uint8), minlength=256)
        return cls.from_frequencies([int(x) for x in h])

    def get_code(self, symbol):
        """Vec<bool> of the symbol's code (emission order), or None."""
        L = self._t.code_len[symbol]
        if L == 0:
            return None
        c = self._t.code[symbol]
        return [bool((c >> j) & 1) for j in range(L)]

    def max_code_length(self):
        return self._t.max_code_length

    def symbol_count(self):
        return self._t.n_symbols

    @property
    def raw(self):
        return self._t

    def serialize(self):
        """HuffmanTree::serialize (tree.rs:226-262), symbols in ascending order."""
        L = _lib.load()
        cap = L.zr_huff_tree_serialized_bound()
        out = (ctypes.c_uint8 * cap)()
        ol = ctypes.c_size_t(0)
        check(L.zr_huff_tree_serialize(ctypes.byref(self._t), out, cap, ctypes.byref(ol)))
        return ctypes.string_at(out, ol.value)

    @classmethod
    def deserialize(cls, data):
        """HuffmanTree::deserialize (tree.rs:265-306)."""
        data = bytes(data)
        buf = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
        t = _lib.HuffTree()
        check(_lib.load().zr_huff_tree_deserialize(buf, len(data), ctypes.byref(t)))
        return cls(t)


class HuffmanEncoder:
    def __init__(self, data=None, tree=None):
        self._tree = tree if tree is not None else HuffmanTree.from_data(data if data is not None else b"")

    @classmethod
    def new(cls, data):
        return cls(data)

    @classmethod
    def from_frequencies(cls, frequencies):
        return cls(tree=HuffmanTree.from_frequencies(frequencies))

    def encode(self, data):
        """HuffmanEncoder::encode (encoder.rs:88-131)."""
        L = _lib.load()
        buf, n = _u8(data)
        t = self._tree.raw
        cap = L.zr_huff_encode_bound(ctypes.byref(t), n)
        out = (ctypes.c_uint8 * max(1, cap))()
        ol = ctypes.c_size_t(0)
        check(L.zr_huff_encode(ctypes.byref(t), buf, n, out, cap, ctypes.byref(ol)))
        return ctypes.string_at(out, ol.value)

    def tree(self):
        return self._tree

    def estimate_compression_ratio(self, data):
        data = bytes(data)
        if not data:
            return 0.0
        t = self._tree.raw
        bits = sum(t.code_len[b] for b in data)
        return bits / (len(data) * 8)


class HuffmanDecoder:
    def __init__(self, tree):
        self._tree = tree

    def decode(self, encoded_data, output_length):
        """HuffmanDecoder::decode (decoder.rs:90-165)."""
        L = _lib.load()
        buf, n = _u8(encoded_data)
        out = (ctypes.c_uint8 * max(1, output_length))()
        check(L.zr_huff_decode(ctypes.byref(self._tree.raw), buf, n, out, output_length))
        if n == 0 or output_length == 0:
            return b""
        return ctypes.string_at(out, output_length)


class HuffmanOrder(enum.IntEnum):
    Order0 = 0
    Order1 = 1
    Order2 = 2


class InterleavingFactor(enum.IntEnum):
    X1 = 1
    X2 = 2
    X4 = 4
    X8 = 8

    def streams(self):
        return int(self)


class ContextualHuffmanEncoder:
    """ContextualHuffmanEncoder::new(data, order) (interleaved.rs:94-266)."""

    def __init__(self, data, order=HuffmanOrder.Order1):
        L = _lib.load()
        buf, n = _u8(data)
        h = ctypes.c_void_p()
        check(L.zr_ctx_huff_new(buf, n, int(order), ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            _lib.load().zr_ctx_huff_free(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def order(self):
        return HuffmanOrder(_lib.load().zr_ctx_huff_order(self._h))

    def tree_count(self):
        """trees.len(): trees[0] plus one tree per context (interleaved.rs:94-266)."""
        return struct.unpack("<I", self.serialize()[1:5])[0]

    def serialize(self):
        """ContextualHuffmanEncoder::serialize (interleaved.rs:476-503), contexts ascending."""
        L = _lib.load()
        cap = L.zr_ctx_huff_serialized_size(self._h)
        out = (ctypes.c_uint8 * max(1, cap))()
        ol = ctypes.c_size_t(0)
        check(L.zr_ctx_huff_serialize(self._h, out, cap, ctypes.byref(ol)))
        return ctypes.string_at(out, ol.value)

    @classmethod
    def deserialize(cls, data):
        """ContextualHuffmanEncoder::deserialize (interleaved.rs:506-595)."""
        L = _lib.load()
        buf, n = _u8(data)
        h = ctypes.c_void_p()
        check(L.zr_ctx_huff_deserialize(buf, n, ctypes.byref(h)))
        self = cls.__new__(cls)
        self._h = h
        return self

    def _encode(self, nway, data):
        L = _lib.load()
        buf, n = _u8(data)
        cap = L.zr_ctx_huff_encode_bound(self._h, n)
        out = (ctypes.c_uint8 * max(1, cap))()
        ol = ctypes.c_size_t(0)
        check(L.zr_ctx_huff_encode(self._h, nway, buf, n, out, cap, ctypes.byref(ol)))
        return ctypes.string_at(out, ol.value)

    def _decode(self, nway, data, n):
        L = _lib.load()
        buf, ln = _u8(data)
        out = (ctypes.c_uint8 * max(1, n))()
        ol = ctypes.c_size_t(0)
        check(L.zr_ctx_huff_decode(self._h, nway, buf, ln, out, n, ctypes.byref(ol)))
        return ctypes.string_at(out, ol.value)

    def encode(self, data):
        """encode (interleaved.rs:269-392)."""
        return self._encode(0, data)

    def encode_with_interleaving(self, data, factor):
        """encode_with_interleaving (interleaved.rs:604-626); Order-1 only."""
        return self._encode(int(factor), data)

    def decode_with_interleaving(self, data, output_size, factor):
        return self._decode(int(factor), data, output_size)

    def encode_x1(self, data):
        return self.encode_with_interleaving(data, InterleavingFactor.X1)

    def encode_x2(self, data):
        return self.encode_with_interleaving(data, InterleavingFactor.X2)

    def encode_x4(self, data):
        return self.encode_with_interleaving(data, InterleavingFactor.X4)

    def encode_x8(self, data):
        return self.encode_with_interleaving(data, InterleavingFactor.X8)

    def decode_x1(self, data, n):
        return self.decode_with_interleaving(data, n, InterleavingFactor.X1)

    def decode_x2(self, data, n):
        return self.decode_with_interleaving(data, n, InterleavingFactor.X2)

    def decode_x4(self, data, n):
        return self.decode_with_interleaving(data, n, InterleavingFactor.X4)

    def decode_x8(self, data, n):
        return self.decode_with_interleaving(data, n, InterleavingFactor.X8)


class ContextualHuffmanDecoder:
    def __init__(self, encoder):
        self._enc = encoder

    def decode(self, encoded_data, output_length):
        """ContextualHuffmanDecoder::decode (interleaved.rs:1050-1209)."""
        return self._enc._decode(0, encoded_data, output_length)


class HuffmanO1Device:
    """Device-resident order-1/2 coding over torch CUDA uint8 tensors."""

    def __init__(self, encoder):
        import torch
        self.torch = torch
        self.enc = encoder
        self.L = _lib.load()

    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream().cuda_stream)

    def encode_async(self, src, out, nway=0):
        check(self.L.zr_ctx_huff_encode_dev(self.enc.handle, nway, src.data_ptr(), src.numel(),
                                            out.data_ptr(), self._stream()))

    def decode_async(self, enc, out, n, nway=0):
        check(self.L.zr_ctx_huff_decode_dev(self.enc.handle, nway, enc.data_ptr(), enc.numel(),
                                            out.data_ptr(), n, self._stream()))


__all__ = ["HuffmanTree", "HuffmanEncoder", "HuffmanDecoder", "HuffmanOrder", "InterleavingFactor",
           "ContextualHuffmanEncoder", "ContextualHuffmanDecoder", "HuffmanO1Device", "ZiporaError"]


class HuffmanCompressor:
    """HuffmanCompressor (compression/mod.rs:320-408): tree_size u32 | serialized
    tree | size u32 | bits; decompress uses the record's own tree."""

    def __init__(self, training_data):
        data = bytes(training_data)
        buf = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
        t = _lib.HuffTree()
        check(_lib.load().zr_huff_compressor_train(buf, len(data), ctypes.byref(t)))
        self.tree = HuffmanTree(t)

    def tree_data(self):
        return self.tree.serialize()

    def compress(self, data):
        L = _lib.load()
        data = bytes(data)
        buf = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
        cap = L.zr_huff_compressor_bound(ctypes.byref(self.tree.raw), len(data))
        out = (ctypes.c_uint8 * cap)()
        ol = ctypes.c_size_t(0)
        check(L.zr_huff_compressor_compress(ctypes.byref(self.tree.raw), buf, len(data), out, cap,
                                            ctypes.byref(ol)))
        return ctypes.string_at(out, ol.value)

    def decompress(self, data):
        L = _lib.load()
        data = bytes(data)
        buf = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
        size = ctypes.c_size_t(0)
        check(L.zr_huff_compressor_decompressed_size(buf, len(data), ctypes.byref(size)))
        out = (ctypes.c_uint8 * max(1, size.value))()
        ol = ctypes.c_size_t(0)
        check(L.zr_huff_compressor_decompress(buf, len(data), out, size.value, ctypes.byref(ol)))
        return ctypes.string_at(out, ol.value)

    def algorithm(self):
        return "Huffman"  # Algorithm::Huffman (mod.rs:404-406)
