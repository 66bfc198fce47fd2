"""The shared-table exchange on the library's own RCCL communicator (zr_comm_*,
zr_comm.cpp): a world-size-1 communicator on the GPU, so the RCCL calls the
multi-GPU bench makes (ncclCommInitRank, in-place u32 all-reduce, broadcast)
really run. The 2-rank arithmetic of the exchange is covered on CPU with gloo
(test_dist_gloo.py); one GPU cannot host two RCCL ranks."""
import pytest
import torch

import zipora_amd as zr

pytestmark = pytest.mark.gpu


def test_rccl_world1_allreduce_and_broadcast():
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import oracle_ffi as O
    from zipora_amd import dist as zd
    from zipora_amd.device import RansDeviceBatch
    comm = zd.RcclComm(1, 0)
    try:
        data = zr.synth("t", 1 << 20, seed=11)
        bt = RansDeviceBatch([len(data)], 4096, shared_table=True)
        raw = bt.new_raw()
        raw[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        bt.histogram(raw)
        before = bt.hist.clone()
        comm.allreduce_histogram(bt.hist)  # one rank: the sum is the histogram itself
        torch.cuda.synchronize()
        assert torch.equal(before, bt.hist)
        assert [int(v) for v in bt.hist.cpu().tolist()] == O.histogram(data)
        bt.tables_from_hist()
        tab0 = bt.tables.clone()
        comm.broadcast_tables(bt.tables, 1, root=0)
        torch.cuda.synchronize()
        assert torch.equal(tab0, bt.tables)
        # the broadcast table codes the buffer exactly as the oracle does
        enc = bt.new_enc()
        bt.encode(raw, enc)
        torch.cuda.synchronize()
        bt.raise_on_error()
        assert bt.encoded(enc, 0) == O.rans_encode(O.rans_table(O.histogram(data)), 4096, data)
    finally:
        comm.close()


def test_rccl_u32_sum_wraps():
    """The all-reduce is a u32 SUM (wraps mod 2^32 per bin, like the reference's
    u32 counters); with one rank it must leave every bit pattern untouched."""
    from zipora_amd import dist as zd
    comm = zd.RcclComm(1, 0)
    try:
        h = torch.tensor([-1, 0x7FFFFFFF, -2147483648, 5] * 64, dtype=torch.int32, device="cuda")
        ref = h.clone()
        comm.allreduce_histogram(h)
        torch.cuda.synchronize()
        assert torch.equal(h, ref)
    finally:
        comm.close()


def test_comm_rejects_bad_rank():
    from zipora_amd import dist as zd
    with pytest.raises(zr.ZiporaError):
        zd.RcclComm(2, 5, unique_id=bytes(128))


def test_rccl_allreduce_captured_step_replays():
    """The header's claim that the RCCL calls may be captured: the shared-table
    step of the multi-GPU bench (histogram, in-place u32 all-reduce on a
    world-1 communicator, consuming table build, encode, decode) captured into
    a HIP graph and replayed three times, each replay equal to the oracle."""
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import oracle_ffi as O
    from zipora_amd import dist as zd
    from zipora_amd.device import RansDeviceBatch
    comm = zd.RcclComm(1, 0)
    try:
        lens = [4096 * 30 + 7, 4096 * 30]
        bt = RansDeviceBatch(lens, 4096, shared_table=True)
        raw = bt.new_raw()
        enc, out = bt.new_enc(), bt.new_raw()
        side = torch.cuda.Stream()

        def step(s):
            bt.histogram(raw, s, zeroed=True)
            comm.allreduce_histogram(bt.hist, s.cuda_stream)
            bt.tables_from_hist(s, consume=True)
            bt.encode(raw, enc, s)
            bt.decode(enc, out, s)

        def load(seed, kind):
            ds = [zr.synth(kind, n, seed=seed + i) for i, n in enumerate(lens)]
            for b, d in enumerate(ds):
                o = bt.raw_off_host[b]
                raw[o:o + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
            return ds

        load(1, "t")
        with torch.cuda.stream(side):
            step(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            step(torch.cuda.current_stream())
        for seed, kind in ((1, "t"), (2, "z"), (3, "u")):
            ds = load(seed, kind)
            out.zero_()
            g.replay()
            torch.cuda.synchronize()
            bt.raise_on_error()
            tab = O.rans_table(O.histogram(b"".join(ds)))
            for b, d in enumerate(ds):
                assert bt.raw_of(out, b) == d
                assert bt.encoded(enc, b) == O.rans_encode(tab, 4096, d)
    finally:
        comm.close()
