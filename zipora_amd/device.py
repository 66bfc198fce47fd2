"""Device-resident batch pipeline over the C ABI (torch supplies device memory and streams).

A batch is B independent buffers, each one reference rANS stream set with
P::N = n_streams. Buffers live contiguously in one raw area and one encoded
area; offsets are device uint64 tensors. This is the hot path bench.py times.
"""
import ctypes

import torch

from . import _lib
from .errors import ZiporaError, check


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class RansDeviceBatch:
    """Geometry + workspace for batched rANS on one GPU.

    lens: list/tensor of decoded lengths; buffers are packed back to back in the
    raw area (raw_off) and at fixed bound-sized slots in the encoded area
    (enc_off), so encode needs no host round trip.
    """

    def __init__(self, lens, n_streams, device="cuda", shared_table=False, align=16):
        self.L = _lib.load()
        lens = [int(x) for x in lens]
        self.B = len(lens)
        self.N = int(n_streams)
        self.device = torch.device(device)
        self.max_len = max(lens) if lens else 0
        raw_off, enc_off = [], []
        r = e = 0
        for n in lens:
            raw_off.append(r)
            enc_off.append(e)
            r += (n + align - 1) // align * align
            e += (self.L.zr_rans_encode_bound(n, self.N) + align - 1) // align * align
        self.raw_bytes, self.enc_bytes = r, e
        self.lens_host = lens
        self.raw_off_host, self.enc_off_host = raw_off, enc_off
        dev = self.device
        u64 = torch.uint64 if hasattr(torch, "uint64") else torch.int64
        self.len = torch.tensor(lens, dtype=torch.int64, device=dev)
        self.raw_off = torch.tensor(raw_off, dtype=torch.int64, device=dev)
        self.enc_off = torch.tensor(enc_off, dtype=torch.int64, device=dev)
        self.enc_len = torch.zeros(self.B, dtype=torch.int64, device=dev)
        self.status = torch.zeros(self.B, dtype=torch.int32, device=dev)
        self.shared = bool(shared_table)
        self.n_tables = 1 if self.shared else self.B
        tb = self.L.zr_rans_dtab_bytes()
        self.tables = torch.zeros(self.n_tables * tb, dtype=torch.uint8, device=dev)
        self.hist = torch.zeros(self.n_tables * 256, dtype=torch.int32, device=dev)
        wsb = self.L.zr_rans_workspace_bytes(self.B, self.N, self.max_len)
        self.ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        self.ws_bytes = wsb
        self.cbatch = _lib.RansBatch()
        c = self.cbatch
        c.n_buffers, c.n_streams, c.max_len = self.B, self.N, self.max_len
        c.len, c.raw_off, c.enc_off = self.len.data_ptr(), self.raw_off.data_ptr(), self.enc_off.data_ptr()
        c.enc_len, c.status = self.enc_len.data_ptr(), self.status.data_ptr()
        c.tables = self.tables.data_ptr()
        c.table_stride = 0 if self.shared else 1
        c.min_len = min(lens) if lens else 0

    # ---- areas
    def new_raw(self):
        return torch.zeros(max(1, self.raw_bytes), dtype=torch.uint8, device=self.device)

    def new_enc(self):
        return torch.zeros(max(1, self.enc_bytes), dtype=torch.uint8, device=self.device)

    # ---- pipeline stages
    def histogram(self, raw, stream=None, zeroed=False):
        """Count raw's bytes into self.hist. zeroed=True: the caller knows hist is
        all zero (fresh, or after tables_from_hist(consume=True)), so no memset."""
        if not zeroed:
            check(self.L.zr_memset_dev(_ptr(self.hist), 0, self.hist.numel() * 4, _stream(stream)))
        check(self.L.zr_histogram_dev(_ptr(raw), ctypes.byref(self.cbatch), int(self.shared),
                                      _ptr(self.hist), _stream(stream)))

    def tables_from_hist(self, stream=None, consume=False):
        """Rans64Encoder::new per histogram, on device. consume=True also zeroes
        hist once read (the next histogram(zeroed=True) accumulates from zero)."""
        fn = self.L.zr_rans_dtab_from_hist_consume_dev if consume else self.L.zr_rans_dtab_from_hist_dev
        check(fn(_ptr(self.hist), self.n_tables, _ptr(self.tables), _stream(stream)))

    def table_from_data(self, raw, stream=None):
        """Shared table of the whole batch in one launch (histogram + the table
        build in its last workgroup). self.hist must be all zero (fresh, or left
        so by this call or tables_from_hist(consume=True)); it stays zero."""
        if not self.shared:
            raise ValueError("table_from_data builds the one shared table")
        check(self.L.zr_rans_dtab_from_data_dev(_ptr(raw), ctypes.byref(self.cbatch), _ptr(self.hist),
                                                _ptr(self.tables), _stream(stream)))

    def upload_tables(self, host_tables):
        arr = (_lib.RansTable * len(host_tables))(*host_tables)
        check(self.L.zr_rans_dtab_upload(arr, len(host_tables), _ptr(self.tables), _stream()))

    def encode(self, raw, enc, stream=None):
        check(self.L.zr_rans_encode_batch_dev(ctypes.byref(self.cbatch), _ptr(raw), _ptr(enc),
                                              _ptr(self.ws), self.ws_bytes, _stream(stream)))

    def decode(self, enc, raw, stream=None):
        check(self.L.zr_rans_decode_batch_dev(ctypes.byref(self.cbatch), _ptr(enc), _ptr(raw),
                                              _ptr(self.ws), self.ws_bytes, _stream(stream)))

    def full_encode(self, raw, enc, stream=None):
        """histogram -> Rans64Encoder::new on device -> encode (no host round trip)."""
        self.histogram(raw, stream)
        self.tables_from_hist(stream)
        self.encode(raw, enc, stream)

    # ---- results
    def statuses(self):
        return self.status.cpu().tolist()

    def raise_on_error(self):
        st = self.statuses()
        bad = [i for i, s in enumerate(st) if s != 0]
        if bad:
            raise ZiporaError(_lib.ZR_INVALID_INPUT, f"rANS batch: buffers {bad[:8]} failed")

    def encoded(self, enc, b):
        off = self.enc_off_host[b]
        n = int(self.enc_len[b].item())
        return bytes(enc[off: off + n].cpu().numpy().tobytes())

    def raw_of(self, raw, b):
        off = self.raw_off_host[b]
        return bytes(raw[off: off + self.lens_host[b]].cpu().numpy().tobytes())


class RansHostPipe:
    """Host-resident rANS batches through the overlapped copy/code pipeline
    (zr_rans_pipe_*): every array is host memory; one shared table.

    The areas are uint8 CPU tensors (pinned ones reach the full PCIe rate);
    offsets follow RansDeviceBatch's layout unless given.
    """

    def __init__(self, table, n_streams, group_bytes=32 << 20):
        import numpy as np
        self._np = np
        self.L = _lib.load()
        self.N = int(n_streams)
        self._table = table
        h = ctypes.c_void_p()
        check(self.L.zr_rans_pipe_create(ctypes.byref(table), self.N, int(group_bytes), ctypes.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            check(self.L.zr_rans_pipe_destroy(self.h))
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def layout(self, lens, align=16):
        """(raw_off, enc_off, raw_bytes, enc_bytes) packing buffers back to back."""
        np = self._np
        lens = np.asarray(lens, dtype=np.uint64)
        bound = np.array([self.L.zr_rans_encode_bound(int(n), self.N) for n in lens], dtype=np.uint64)
        ra = (lens + align - 1) // align * align
        ea = (bound + align - 1) // align * align
        raw_off = np.concatenate([[0], np.cumsum(ra)[:-1]]).astype(np.uint64) if len(lens) else ra
        enc_off = np.concatenate([[0], np.cumsum(ea)[:-1]]).astype(np.uint64) if len(lens) else ea
        return raw_off, enc_off, int(ra.sum()), int(ea.sum())

    @staticmethod
    def _p(a):
        if isinstance(a, torch.Tensor):
            assert a.device.type == "cpu" and a.is_contiguous()
            return ctypes.c_void_p(a.data_ptr())
        return ctypes.c_void_p(a.ctypes.data)

    def encode(self, lens, raw, raw_off, enc, enc_off):
        """-> (enc_len, status) numpy arrays; raises on a call-level error."""
        np = self._np
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        B = len(lens)
        enc_len = np.zeros(B, dtype=np.uint64)
        status = np.zeros(B, dtype=np.int32)
        check(self.L.zr_rans_pipe_encode(self.h, B, self._p(lens), self._p(raw),
                                         self._p(np.ascontiguousarray(raw_off, dtype=np.uint64)),
                                         self._p(enc), self._p(np.ascontiguousarray(enc_off, dtype=np.uint64)),
                                         self._p(enc_len), self._p(status)))
        return enc_len, status

    def encode_packed(self, lens, raw, raw_off, enc):
        """Records back to back in enc -> (enc_off, enc_len, status, total)."""
        np = self._np
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        B = len(lens)
        enc_off = np.zeros(B, dtype=np.uint64)
        enc_len = np.zeros(B, dtype=np.uint64)
        status = np.zeros(B, dtype=np.int32)
        total = ctypes.c_uint64(0)
        cap = enc.numel() if isinstance(enc, torch.Tensor) else enc.nbytes
        check(self.L.zr_rans_pipe_encode_packed(self.h, B, self._p(lens), self._p(raw),
                                                self._p(np.ascontiguousarray(raw_off, dtype=np.uint64)),
                                                self._p(enc), cap, self._p(enc_off), self._p(enc_len),
                                                self._p(status), ctypes.byref(total)))
        return enc_off, enc_len, status, total.value

    def decode(self, lens, enc, enc_off, enc_len, raw, raw_off):
        """-> status numpy array."""
        np = self._np
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        B = len(lens)
        status = np.zeros(B, dtype=np.int32)
        check(self.L.zr_rans_pipe_decode(self.h, B, self._p(lens), self._p(enc),
                                         self._p(np.ascontiguousarray(enc_off, dtype=np.uint64)),
                                         self._p(np.ascontiguousarray(enc_len, dtype=np.uint64)),
                                         self._p(raw), self._p(np.ascontiguousarray(raw_off, dtype=np.uint64)),
                                         self._p(status)))
        return status


class RansCompressorDeviceBatch(RansDeviceBatch):
    """Device batches of RansCompressor records (compression/mod.rs:416-512): x1
    streams behind a 1028-byte header, one compressor (shared table) per batch."""

    def __init__(self, lens, device="cuda", align=16):
        super().__init__(lens, 1, device=device, shared_table=True, align=align)
        L = self.L
        enc_off, e = [], 0
        for n in self.lens_host:
            enc_off.append(e)
            e += (L.zr_rans_compressor_bound(n) + align - 1) // align * align
        self.enc_bytes = e
        self.enc_off_host = enc_off
        self.enc_off = torch.tensor(enc_off, dtype=torch.int64, device=self.device)
        wsb = L.zr_rans_compressor_workspace_bytes(self.B, self.max_len)
        self.ws = torch.empty(wsb, dtype=torch.uint8, device=self.device)
        self.ws_bytes = wsb
        self.cbatch.enc_off = self.enc_off.data_ptr()

    def compress(self, raw, enc, stream=None):
        """Compressor::compress per record, on device (table: upload_tables / tables_from_hist)."""
        check(self.L.zr_rans_compressor_compress_batch_dev(ctypes.byref(self.cbatch), _ptr(raw), _ptr(enc),
                                                           _ptr(self.ws), self.ws_bytes, _stream(stream)))

    def decompress(self, enc, raw, stream=None):
        """Compressor::decompress per record, on device (table rebuilt from the stored header)."""
        check(self.L.zr_rans_compressor_decompress_batch_dev(ctypes.byref(self.cbatch), _ptr(enc), _ptr(raw),
                                                             _ptr(self.ws), self.ws_bytes, _stream(stream)))
