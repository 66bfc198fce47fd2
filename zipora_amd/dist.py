"""Multi-GPU plumbing for the entropy path.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on
ROCm). The path shards: every rank codes its own buffers as complete reference
streams, so the data path has no collective. The only exchange is the
shared-table mode's 256-bin histogram: one all-reduce(SUM) of 256 counters
(1 KiB as u32, 2 KiB as i64), after which every rank normalises locally
(rans.rs:238-299 is deterministic) and holds the identical table.
"""
import torch
import torch.distributed as dist


def world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def allreduce_histogram(hist):
    """Sum a 256-bin histogram (int32/uint32 or int64 tensor, any device) over ranks in place.

    int32 counts are the device histograms' u32 bit patterns: the sum wraps mod
    2^32 exactly as the reference's u32 counts do. RCCL reduces device tensors
    in place; gloo (CPU tests) reduces a host copy of a device tensor."""
    if world() == 1:
        return hist
    if hist.is_cuda and dist.get_backend() == "gloo":
        h = hist.cpu()
        allreduce_histogram(h)
        hist.copy_(h)
        return hist
    if hist.dtype == torch.int32 or hist.dtype == torch.int64:
        dist.all_reduce(hist, op=dist.ReduceOp.SUM)
        return hist
    # uint32 histograms: reduce as int64 (RCCL/gloo have no u32 SUM) and write back
    h64 = hist.to(torch.int64)
    dist.all_reduce(h64, op=dist.ReduceOp.SUM)
    hist.copy_(h64.to(hist.dtype))
    return hist


class RcclComm:
    """The library's own RCCL communicator (zr_comm_*, zr_comm.cpp): what a
    Rust host binding libzipora_amd.so uses for the shared table, with no
    PyTorch in the data path. The 128-byte unique id is moved between the
    processes by any host channel; `exchange_id` below uses torch.distributed's
    object broadcast when a process group exists (world size 1: none needed)."""

    def __init__(self, nranks=1, rank=0, unique_id=None):
        import ctypes
        from . import _lib
        from .errors import check
        self._L = _lib.load()
        self._check = check
        if unique_id is None:
            unique_id = RcclComm.unique_id() if nranks == 1 else exchange_id(rank)
        self.id = bytes(unique_id)
        self.nranks, self.rank = int(nranks), int(rank)
        idbuf = (ctypes.c_uint8 * 128).from_buffer_copy(self.id)
        h = ctypes.c_void_p()
        check(self._L.zr_comm_init(idbuf, self.nranks, self.rank, ctypes.byref(h)))
        self._h = h

    @staticmethod
    def unique_id():
        import ctypes
        from . import _lib
        from .errors import check
        buf = (ctypes.c_uint8 * 128)()
        check(_lib.load().zr_comm_unique_id(buf))
        return bytes(buf)

    def allreduce_histogram(self, hist, stream=None):
        """In-place u32 SUM over the ranks of a device histogram (int32/uint32 tensor:
        the RCCL call reduces numel() u32 counters, so any other dtype is refused)."""
        if hist.dtype not in (torch.int32, torch.uint32) or not hist.is_contiguous() or not hist.is_cuda:
            raise TypeError(f"RcclComm.allreduce_histogram needs a contiguous int32/uint32 device tensor, "
                            f"got {hist.dtype} on {hist.device}")
        if stream is None:
            stream = torch.cuda.current_stream(hist.device).cuda_stream
        self._check(self._L.zr_histogram_allreduce_dev(self._h, hist.data_ptr(), hist.numel(), stream))
        return hist

    def count(self):
        """RCCL's own rank count of the communicator (ncclCommCount)."""
        import ctypes
        n = ctypes.c_int32(0)
        self._check(self._L.zr_comm_count(self._h, ctypes.byref(n)))
        return int(n.value)

    def broadcast_tables(self, tables, n_tables, root=0, stream=None):
        if stream is None:
            stream = torch.cuda.current_stream(tables.device).cuda_stream
        self._check(self._L.zr_table_broadcast_dev(self._h, tables.data_ptr(), n_tables, root, stream))

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            self._check(self._L.zr_comm_destroy(h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def exchange_id(rank):
    """Rank 0's RCCL unique id, delivered to every rank over the existing
    torch.distributed process group (host objects only)."""
    obj = [RcclComm.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


class TorchComm:
    """The same exchange on torch.distributed's process group (RCCL for the
    "nccl" backend): the fallback of `shared_table_comm`."""

    def allreduce_histogram(self, hist, stream=None):
        return allreduce_histogram(hist)

    def close(self):
        pass


def shared_table_comm(nranks, rank):
    """The shared-table communicator of a multi-rank run: the library's own
    RCCL communicator (zr_comm_*), or, when it cannot be set up on every rank,
    the torch.distributed group's on every rank (reported on stderr; the run
    goes on). The ranks agree twice: before the collective init (a rank that
    has no id or no zr_comm keeps every rank out of it) and after it (a rank
    whose init failed on the Python side, e.g. the library call returned an
    error, makes every rank destroy its communicator and fall back together,
    so no two ranks run the exchange on different collectives). A failure
    INSIDE ncclCommInitRank is not covered: that init is collective, so the
    other ranks may stay blocked in their own init and never reach the second
    agreement (RCCL's own init timeout then ends them)."""
    import sys
    uid, err = None, None
    if rank == 0:
        try:
            uid = RcclComm.unique_id()
        except Exception as e:  # noqa: BLE001
            err = e
    obj = [uid]
    dist.broadcast_object_list(obj, src=0)
    uid = obj[0]
    ok = 1 if uid is not None and hasattr(_lib_load(), "zr_comm_init") else 0
    comm = None
    if _all_ranks(ok):
        try:
            comm = RcclComm(nranks, rank, unique_id=uid)
        except Exception as e:  # noqa: BLE001
            err = e
        if _all_ranks(1 if comm is not None else 0):
            return comm
        if comm is not None:
            try:
                comm.close()
            except Exception as e:  # noqa: BLE001  (the fallback below still applies)
                err = err or f"zr_comm_destroy failed: {e}"
            err = err or "another rank's zr_comm_init failed"
    print(f"zipora_amd: no zr_comm communicator ({err}); histogram all-reduce on torch.distributed",
          file=sys.stderr)
    return TorchComm()


def _all_ranks(flag):
    """True on every rank iff flag is true on every rank (all_reduce MIN on the group)."""
    t = torch.tensor([int(bool(flag))], dtype=torch.int32)
    if dist.get_backend() != "gloo":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item()) == 1


def _lib_load():
    from . import _lib
    return _lib.load()


def max_over_ranks(seconds, device=None):
    """The bench contract's timing: the slowest rank's wall time."""
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=device)
    if world() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard_seed(base, rank):
    """Weak scaling: every rank codes its own synthetic shard of the same size."""
    return (base + 0x9E3779B97F4A7C15 * rank) & ((1 << 64) - 1)
