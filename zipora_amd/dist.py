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


def max_over_ranks(seconds, device=None):
    """The bench contract's timing: the slowest rank's wall time."""
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=device)
    if world() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard_seed(base, rank):
    """Weak scaling: every rank codes its own synthetic shard of the same size."""
    return (base + 0x9E3779B97F4A7C15 * rank) & ((1 << 64) - 1)
