#!/usr/bin/env python3
"""bench.py -- rANS O0 encode+decode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 256 MiB of uniform-random bytes per GPU,
coded as 64 independent 4 MiB buffers, each a reference rANS stream set with
4096-way lane-interleaved streams (rans::ParallelVariant N = 4096). One step =
histogram -> [RCCL all-reduce of the 256-bin histogram when N > 1: the shared
frequency table] -> Rans64Encoder::new on device -> encode -> decode, all
device-resident. value = uncompressed bytes of all ranks / (t_enc + t_dec).

    python bench.py --gpus 1 --steps 10 --warmup 3
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks, one process per GPU. Without WORLD_SIZE in the environment and N > 1, "
                        "bench.py starts the N rank processes itself; under torchrun it must equal WORLD_SIZE")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--buffers", type=int, default=64)
    p.add_argument("--buffer-mib", type=int, default=4)
    p.add_argument("--streams", type=int, default=4096)
    p.add_argument("--kind", default="u")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-host-path", action="store_true")
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the configs[1]-literal / configs[2] / configs[4] sub-lines of the default run")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--workload", default="rans", choices=["rans", "fse", "o1", "blob"],
                   help="rans = BASELINE metric (configs[1]); fse = configs[2]; o1 = configs[3] "
                        "(per-GPU shard); blob = configs[4] (per-GPU batch) -- secondary lines")
    p.add_argument("--groups", type=int, default=1,
                   help="rans: code the buffers as G groups on G HIP streams after the shared table "
                        "(encode+compaction+decode of one group overlap the others')")
    p.add_argument("--graph", type=int, default=0,
                   help="rANS workload, one rank: untimed steps replay a HIP graph of the step "
                        "(the event-timed steps run eagerly)")
    p.add_argument("--pipeline", action="store_true",
                   help="rans: two distinct batches alternate; each step codes one (encode -> decode on the "
                        "main stream) while the histogram + table of the next one run on a second stream")
    p.add_argument("--records", type=int, default=1 << 20)
    p.add_argument("--fse-block-kib", type=int, default=64)
    p.add_argument("--dry-run", action="store_true",
                   help="launcher check without a GPU: the ranks join a gloo group, time an empty step and "
                        "rank 0 prints the rank count (no kernels, no metric)")
    return p.parse_args()


CPU_MIN_SECONDS = 3.0  # each CPU baseline repeats its sample for >= this wall time (~48 core-seconds on 16)


def _cpu_repeat(fn, items, threads, min_s=CPU_MIN_SECONDS):
    """Run fn over items on a thread pool (the oracle releases the GIL in C),
    repeating whole passes until min_s of wall time; returns (seconds, passes)."""
    import concurrent.futures as cf
    items = list(items)
    passes = 0
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(max_workers=threads) as ex:
        while True:
            list(ex.map(fn, items))
            passes += 1
            dt = time.perf_counter() - t0
            if dt >= min_s:
                return dt, passes


def host_info(threads):
    """The GPU box's host CPU, as the CPU baseline ran on it."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"model": model, "nproc": aff, "os_cpu_count": os.cpu_count(), "threads_used": threads,
            "note": "all-core leg = min(nproc, --cpu-threads); the GPU box allots 16 host cores per GPU"}


def cpu_threads(args):
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    return max(1, min(aff, args.cpu_threads))


def cpu_baseline(data, n, B, N, threads, sample_bytes=None):
    """The oracle (C restatement of src/entropy/rans.rs, 'port') on host cores, two legs:
    (i) one thread with the reference's data structures (per-stream index vectors of
    rans.rs:385-391 / :629-633, Vec growth; or_rans_*_mirror), (ii) every allotted core,
    buffers spread over threads. Each: histogram + Rans64Encoder::new + encode + decode.
    sample_bytes: code only the first sample_bytes of each buffer (bounded sample)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    O.lib()
    m = min(n, sample_bytes) if sample_bytes else n

    # pieces: whole buffers, or (sampled) consecutive m-byte slices of the buffers,
    # each coded as its own x N stream set; up to 4 per thread
    per = n // m
    pieces = [b * n + i * m for b in range(B) for i in range(per)][:4 * threads]

    def one(k, mirror=False):
        d = data[pieces[k]:pieces[k] + m]
        t = _table_fast(O, d)
        if mirror:
            enc = O.rans_encode_mirror(t, N, d)
            dec = O.rans_decode_mirror(t, N, enc, m)
        else:
            enc = O.rans_encode(t, N, d)
            dec = O.rans_decode(t, N, enc, m)
        assert dec == d
        return len(enc)

    nb1 = min(len(pieces), 4)
    dt1, p1 = _cpu_repeat(lambda k: one(k, True), range(nb1), 1)
    nb = len(pieces)
    dt, passes = _cpu_repeat(one, range(nb), threads)
    what = f"{m >> 20} MiB" + (f" slices of the {n >> 20} MiB buffer(s), each its own x{N} stream set"
                               if m < n else f" buffers, x{N} streams")
    return {"value": round(passes * nb * m / 2**30 / dt, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"all-core leg: {passes} passes over {nb} x {what} of the same uniform workload, "
                      f"histogram+Rans64Encoder::new+encode+decode, {threads} threads over buffers, {dt:.2f} s wall",
            "single_thread": {"value": round(p1 * nb1 * m / 2**30 / dt1, 4), "unit": "GiB/s", "cores": 1,
                              "kind": "port",
                              "sample": f"{p1} passes over {nb1} x {what}, reference data structures (per-stream "
                                        f"index vectors rans.rs:385-391/:629-633, Vec growth), {dt1:.2f} s wall"},
            "host": host_info(threads)}


def _table_fast(O, d):
    import numpy as np
    h = np.bincount(np.frombuffer(d, dtype=np.uint8), minlength=256).astype(np.uint32)
    return O.rans_table([int(x) for x in h])


TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")


def pmc_traffic(workload, kernel):
    """HBM bytes per dispatch of `kernel` in `workload` from profiles/traffic.json, the
    committed PMC summary of the current round (tools/profile_round.sh +
    tools/summarize_prof.py: FETCH_SIZE x2 + WRITE_SIZE, separate passes)."""
    if not os.path.exists(TRAFFIC_FILE):
        return None, None
    with open(TRAFFIC_FILE) as fh:
        doc = json.load(fh)
    wl = doc.get("workloads", {}).get(workload, {})
    t = wl.get(kernel)
    src = f"profiles/traffic.json ({doc.get('source', '?')})"
    return (round(t["hbm_bytes"]) if t else None), src


def kernel_ms(L, name):
    ms, cnt = ctypes.c_double(0), ctypes.c_uint64(0)
    L.zr_timer_read(name.encode(), ctypes.byref(ms), ctypes.byref(cnt))
    return ms.value / max(1, cnt.value), cnt.value


def cpu_baseline_fse(host, bs, threads):
    """The oracle (C restatement of src/entropy/fse.rs, 'port'): FSE 0xF6
    compress+decompress on bounded 8 MiB slices, two legs: every allotted core
    (slices spread over threads) and one thread."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    O.lib()
    sl = 8 << 20
    ns = min(len(host) // sl, 2 * threads)
    cfg = O.fse_config(parallel_blocks=8, block_size=bs)

    def one(i):
        d = host[i * sl:(i + 1) * sl]
        enc = O.fse_compress(d, cfg)
        assert O.fse_decompress(enc, len(d)) == d
        return len(enc)

    dt, passes = _cpu_repeat(one, range(ns), threads)
    dt1, p1 = _cpu_repeat(one, range(1), 1)
    what = f"0xF6 stream (Some(8), {bs >> 10} KiB blocks), compress+decompress"
    return {"value": round(passes * ns * sl / 2**30 / dt, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{passes} passes over {ns} x 8 MiB slices of the same Zipf workload, each an independent "
                      f"{what}, {threads} threads, {dt:.2f} s wall",
            "single_thread": {"value": round(p1 * sl / 2**30 / dt1, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
                              "sample": f"{p1} passes over 1 x 8 MiB slice, {what}, {dt1:.2f} s wall"}}


def fse_host_rates(L, torch, host, bs, reps=3):
    """configs[2] starting and ending in host memory (north_star: the rate with the
    H2D and D2H copies): zr_fse_compress / zr_fse_decompress on pinned host
    buffers (the C ABI's host entry points: copy in, code on the device, copy out)."""
    import ctypes
    from zipora_amd import _lib as zl
    n = len(host)
    cfg = zl.FseConfig()
    L.zr_fse_config_default(ctypes.byref(cfg))
    cfg.parallel_blocks, cfg.block_size = 8, bs
    pin = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    pin.copy_(torch.frombuffer(bytearray(host), dtype=torch.uint8))
    cap = L.zr_fse_compress_bound(n, ctypes.byref(cfg))
    penc = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
    pout = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    ol, dl = ctypes.c_size_t(0), ctypes.c_size_t(0)
    u8 = lambda t: ctypes.cast(t.data_ptr(), ctypes.POINTER(ctypes.c_uint8))  # noqa: E731
    te = td = 0.0
    for r in range(reps + 1):  # the first call grows the call context's buffers
        t0 = time.perf_counter()
        if L.zr_fse_compress(ctypes.byref(cfg), u8(pin), n, u8(penc), cap, ctypes.byref(ol)):
            raise SystemExit("FSE host compress failed")
        t1 = time.perf_counter()
        if L.zr_fse_decompress(u8(penc), ol.value, u8(pout), n, ctypes.byref(dl)):
            raise SystemExit("FSE host decompress failed")
        t2 = time.perf_counter()
        if r:
            te += t1 - t0
            td += t2 - t1
    if dl.value != n or not torch.equal(pout, pin):
        raise SystemExit("FSE host round trip mismatch")
    return {"host_resident_gibps": round(n * reps / (te + td) / 2**30, 3),
            "host_encode_gibps": round(n * reps / te / 2**30, 3),
            "host_decode_gibps": round(n * reps / td / 2**30, 3),
            "host_path": "zr_fse_compress/zr_fse_decompress, pinned host buffers, synchronous H2D + kernels + D2H"}


def run_fse(args, torch, dist, world, rank, dev, zr, L):
    from zipora_amd import dist as zd
    """configs[2]: FSE encode+decode, 256 MiB Zipf(1.1) per GPU, 0xF6 blocks (Some(8))."""
    total = 256 << 20
    bs = args.fse_block_kib << 10
    host = zr.synth("z", total, seed=0x9E3779B97F4A7C15 + rank)
    raw = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(dev)
    cfg = zr.FseConfig(parallel_blocks=8, block_size=bs)
    fd = zr.FseDevice(cfg, max_len=total, device=dev)
    enc = torch.empty(fd.bound(total), dtype=torch.uint8, device=dev)
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    nblk = fd.n_blocks(total)
    fd2 = zr.FseDevice(cfg, device=dev)  # separate meta for decode
    cap = enc.numel()

    def step():
        fd.compress_async(raw, enc)
        fd2.decompress_async(enc, cap, out, nblk)

    step()
    torch.cuda.synchronize(dev)
    clen, st = fd.result()
    dlen, st2 = fd2.result()
    if st or st2 or dlen != total or not torch.equal(out, raw):
        raise SystemExit(f"FSE warmup mismatch (status {st}/{st2}, len {dlen})")
    dt, dom, dom_ms, kms, _ = _measure(torch, dist, world, dev, L, step, args,
                                    ["fse_decode", "fse_encode", "fse_histogram"])
    if not torch.equal(out, raw):
        raise SystemExit("FSE decode mismatch in timed region")
    res = {
        "metric": "GiB/s encode+decode (device-resident), FSE, 256 MiB Zipf(1.1), MI355X",
        "value": round(world * total * args.steps / dt / 2**30, 3), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (Zipf alpha=1.1 bytes, inverse CDF over the xorshift64 generator)",
        "config": {"workload": f"FSE 0xF6 encode+decode, 256 MiB Zipf per GPU, parallel_blocks=Some(8), "
                               f"block_size={bs >> 10} KiB ({nblk} blocks, one coder lane each)",
                   "block_size": bs, "blocks": nblk, "parallelism": f"shard{world}"},
        "roofline": _roofline(dom, dom_ms, {"fse_decode": clen + total, "fse_encode": total + clen,
                                            "fse_histogram": total}, f"fse{bs >> 10}",
                              {"fse_decode": "k_fse_dec", "fse_encode": "k_fse_enc", "fse_histogram": "k_fse_hist"}),
        "kernels_ms": kms, "kernels_ms_source": KMS_SOURCE,
        "compressed_bytes": clen, "ratio": round(clen / total, 5),
    }
    del raw, enc, out
    if rank == 0 and world == 1 and not args.no_host_path:
        res.update(fse_host_rates(L, torch, host, bs))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_fse(host, bs, cpu_threads(args))
    return res


RANS_SYMS = {"rans_encode": "k_enc_xn", "rans_decode": "k_dec_xn_fast", "rans_compact": "k_enc_compact_lds",
             "histogram": "k_hist"}
KMS_SOURCE = ("instrumented passes before the timed region (8 steps per kernel, that kernel alone HIP-event "
              "timed on every 4th step); the roofline's avg_launch_ms is the dominant kernel's, timed alone on "
              "every 4th step of the timed region")


COPY_GBS = None  # the achievable-copy ceiling, measured once per run
COPY_NOTE = None


def copy_ceiling(torch, dev, L, nbytes=256 << 20, reps=20):
    """Device-to-device copy of 256 MiB by the library's 16-B-per-lane streaming
    kernel (zr_memcpy_dev: each wave its own contiguous chunk, eight 16-B loads
    per lane in flight, non-temporal), read + write bytes /
    time, the best of three grid sizes, timed with HIP events on the stream it
    runs on: the practical one-pass ceiling reported beside the 8 TB/s spec peak."""
    global COPY_GBS, COPY_NOTE
    if COPY_GBS is None:
        a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        b = torch.empty_like(a)
        st = torch.cuda.current_stream(dev)
        best, best_g = 0.0, 0
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        if not hasattr(L, "zr_memcpy_dev"):  # (an older library in an A/B run: no ceiling)
            COPY_GBS, COPY_NOTE = 0.0, "unmeasured"
            return COPY_GBS
        for g in (4 * cus, 8 * cus, 16 * cus):
            for _ in range(3):
                L.zr_memcpy_dev(b.data_ptr(), a.data_ptr(), nbytes, g, st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(reps):
                L.zr_memcpy_dev(b.data_ptr(), a.data_ptr(), nbytes, g, st.cuda_stream)
            e1.record(st)
            e1.synchronize()
            gbs = 2 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
            if gbs > best:
                best, best_g = gbs, g
        COPY_GBS = best
        COPY_NOTE = (f"zr_memcpy_dev 256 MiB, per-wave chunks, 8 x 16 B/lane in flight, grid {best_g} x 256, "
                     "read+write bytes / time")
        del a, b
    return COPY_GBS


def _roofline(dom, dom_ms, bytes_of, traffic_wl, sym, kms=None):
    """roofline object of the dominant kernel: algorithmic bytes per launch / its
    average launch time in the timed region; traffic = PMC HBM bytes per launch;
    frac_of_copy = achieved / the measured copy ceiling."""
    nbytes = bytes_of[dom]
    ach = nbytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    tr, src = pmc_traffic(traffic_wl, sym[dom])
    r = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": tr, "traffic_source": src,
         "kernel": f"{sym[dom]} ({dom})", "bytes_per_launch": nbytes, "avg_launch_ms": round(dom_ms, 4)}
    if kms and dom in kms:  # the same kernel in the instrumented pass (every kernel timed)
        r["avg_launch_ms_instrumented"] = kms[dom]
    if COPY_GBS:
        r["copy_ceiling"] = round(COPY_GBS, 1)
        r["copy_ceiling_source"] = COPY_NOTE
        r["frac_of_copy"] = round(ach / COPY_GBS, 4)
    return r


def _measure(torch, dist, world, dev, L, fn, args, names, also=()):
    """Warm up, then instrumented passes (one named kernel HIP-event timed per
    pass) that give kernels_ms and pick the dominant kernel, then the timed
    region proper: args.steps steps in which the dominant kernel (and the kernels
    in `also`, in turn) is event-timed on every TIME_EVERY-th step
    (hipExtLaunchKernelGGL's begin/end events).
    -> (seconds, dominant name, its ms per launch in the timed region, kernels_ms,
        {kernel: ms per launch in the timed region} for the dominant and `also`)"""
    for _ in range(args.warmup):
        fn()
    torch.cuda.synchronize(dev)
    select = getattr(L, "zr_timer_select", None)
    kms = {}
    if select is None:  # (an older library in an A/B run: every kernel timed at once)
        L.zr_timer_reset()
        _timer_enable(L, 1)
        for _ in range(max(1, min(args.steps, 10))):
            fn()
        torch.cuda.synchronize(dev)
        _timer_enable(L, 0)
        kms = {k: round(kernel_ms(L, k)[0], 4) for k in names}
        dominant = max(names, key=lambda k: kms[k])
        L.zr_timer_reset()
        _timer_enable(L, 1)
        dt = _timed(torch, dist, world, dev, fn, args.steps, 0)
        _timer_enable(L, 0)
        tms = {k: kernel_ms(L, k)[0] for k in [dominant, *also]}
        return dt, dominant, tms[dominant], kms, tms
    # one kernel timed per pass, on every TIME_EVERY-th step: timed all at once
    # the kernels ran 5-12 % longer, and timed on consecutive steps longer again
    # (rocprofv3 kernel trace of the same runs, prof_r03)
    for k in names:
        L.zr_timer_reset()
        select(k.encode())
        for i in range(2 * TIME_EVERY):
            _timer_enable(L, 1 if i % TIME_EVERY == 0 else 0)
            fn()
        torch.cuda.synchronize(dev)
        _timer_enable(L, 0)
        kms[k] = round(kernel_ms(L, k)[0], 4)
    dominant = max(names, key=lambda k: kms[k])
    timed = [dominant] + [k for k in also if k != dominant]
    L.zr_timer_reset()

    # every TIME_EVERY-th step of the timed region times one kernel of `timed`,
    # in turn: a timed launch costs the queue ~12 us (7 us before it, 5 after;
    # kernel trace, prof_r03), which every step would otherwise carry
    def timer(i):
        on = i % TIME_EVERY == 0
        if on:
            select(timed[(i // TIME_EVERY) % len(timed)].encode())
        _timer_enable(L, 1 if on else 0)

    dt = _timed(torch, dist, world, dev, fn, args.steps, 0, timer=timer)
    _timer_enable(L, 0)
    tms = {}
    for k in timed:  # (a kernel no timed step reached keeps its instrumented-pass time)
        ms, cnt = kernel_ms(L, k)
        tms[k] = ms if cnt else kms[k]
    L.zr_timer_reset()
    select(b"")
    # the roofline's launch time: the kernel's average in the timed region (HIP
    # events on its own stream); the committed rocprofv3 --stats summary of the
    # same command is the check on it
    return dt, dominant, tms[dominant], kms, tms


TIME_EVERY = 4
_TIMER_ON = False  # a step runs with the library's kernel timer on (graph mode: eagerly)


def _timer_enable(L, on):
    global _TIMER_ON
    _TIMER_ON = bool(on)
    L.zr_timer_enable(1 if on else 0)


def _timed(torch, dist, world, dev, fn, steps, warmup, timer=None):
    from zipora_amd import dist as zd
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        if timer is not None:
            timer(i)
        fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    return zd.max_over_ranks(time.perf_counter() - t0, dev)


def _exchange_info(zd, comm, world):
    """How the shared table's histogram crossed the ranks: RCCL's own rank count
    of the library communicator (ncclCommCount via zr_comm_count), or the
    torch.distributed fallback, or none (one rank)."""
    if comm is None:
        return {"rccl_ranks": None, "histogram_exchange": "none (one rank)"}
    if isinstance(comm, zd.RcclComm):
        return {"rccl_ranks": comm.count(), "histogram_exchange": "zr_comm (RCCL all-reduce, u32 SUM)"}
    return {"rccl_ranks": None, "histogram_exchange": "torch.distributed all_reduce (zr_comm unavailable)"}


def _line(metric, value, world, args, dt, data, config, roofline, extra):
    r = {"metric": metric, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
         "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
         "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": data, "config": config,
         "roofline": roofline}
    r.update(extra)
    return r


def cpu_baseline_o1(host, threads):
    """Oracle ContextualHuffman order-1 (interleaved.rs) encode+decode, 4 MiB slices."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    O.lib()
    sl = 4 << 20
    ns = min(len(host) // sl, 2 * threads)

    def one(i):
        d = host[i * sl:(i + 1) * sl]
        c = O.Ctx(d[:1 << 16], 1)
        assert c.decode(c.encode(d), len(d)) == d

    dt, passes = _cpu_repeat(one, range(ns), threads)
    dt1, p1 = _cpu_repeat(one, range(1), 1)
    return {"value": round(passes * ns * sl / 2**30 / dt, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{passes} passes over {ns} x 4 MiB slices of the same text, order-1 encode+decode, "
                      f"{threads} threads, {dt:.2f} s wall",
            "single_thread": {"value": round(p1 * sl / 2**30 / dt1, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
                              "sample": f"{p1} passes over one 4 MiB slice, order-1 encode+decode, {dt1:.2f} s wall"}}


def cpu_baseline_blob(host, threads):
    """Oracle rANS x1 per 1 KiB record with one shared table (RansCompressor-style):
    every allotted core over record groups, and one thread."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    O.lib()
    per = 4096
    nrec = min(len(host) // 1024, per * threads)
    t = _table_fast(O, host[:nrec * 1024])
    buf = bytes(host[:nrec * 1024])

    def one(k):  # a whole record group per oracle call: the C loop runs without the GIL
        lo = k * per
        O.rans_x1_records(t, buf, lo * 1024, min(nrec, lo + per) - lo, 1024)

    dt, passes = _cpu_repeat(one, range((nrec + per - 1) // per), threads)
    dt1, p1 = _cpu_repeat(one, range(1), 1)
    return {"value": round(passes * nrec * 1024 / 2**30 / dt, 4), "unit": "GiB/s", "cores": threads,
            "kind": "port",
            "sample": f"{passes} passes over {nrec} x 1 KiB records of the same batch, x1 encode+decode with "
                      f"one shared table, {threads} threads, {dt:.2f} s wall",
            "single_thread": {"value": round(p1 * per * 1024 / 2**30 / dt1, 4), "unit": "GiB/s", "cores": 1,
                              "kind": "port",
                              "sample": f"{p1} passes over {per} x 1 KiB records, x1 encode+decode, shared table, "
                                        f"{dt1:.2f} s wall"}}


PUBLISHED_O0 = {"value_mbps": {"entropy 0.5": 58.3, "entropy 2.0": 53.1, "entropy 6.0": 38.1},
                "what": "HuffmanEncoder::new + encode, 64 KiB, 1 thread, AMD EPYC 7B13 (Zen 3), rustc 1.91.1",
                "source": "docs/PERFORMANCE.md:77 (benches/entropy_bench.rs:48-59)"}


def huffman_o0_line(zr, L=None):
    """BASELINE configs[0]: HuffmanEncoder O0 encode+decode of 1 MiB synthetic bytes
    on the CPU reference path (examples/entropy_coding_demo.rs:36-65): the oracle's
    restatement of tree.rs/encoder.rs/decoder.rs (bit-serial pack, tree walk), one
    thread, on text-like (`t`) and uniform (`u`) bytes, printed beside the
    reference's published encode rate (docs/PERFORMANCE.md:77, 64 KiB). The same
    calls through the library's host API (tree on the host, kernels on the GPU,
    H2D/D2H included) are shown beside it, checked byte for byte."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    O.lib()
    out = {"metric": "MB/s Huffman O0 encode+decode, 1 MiB, CPU reference path (configs[0])", "unit": "MB/s",
           "published_reference": PUBLISHED_O0, "inputs": {}}

    def rate(fn, nbytes, min_s=1.0):
        k, t0 = 0, time.perf_counter()
        while True:
            fn()
            k += 1
            dt = time.perf_counter() - t0
            if dt >= min_s:
                return round(k * nbytes / dt / 1e6, 2)

    for kind in ("t", "u"):
        row = {}
        for n in (1 << 20, 1 << 16):
            d = zr.synth(kind, n, seed=0x9E3779B97F4A7C15)
            t = O.huff_tree(O.histogram(d))
            enc = O.huff_encode(t, d)
            assert O.huff_decode(t, enc, n) == d
            r = {"encode_incl_tree_mbps": rate(lambda: O.huff_encode(O.huff_tree(O.histogram(d)), d), n),
                 "decode_mbps": rate(lambda: O.huff_decode(t, enc, n), n),
                 "encode_decode_mbps": rate(lambda: O.huff_decode(t, O.huff_encode(O.huff_tree(O.histogram(d)),
                                                                                   d), n), n),
                 "bits_per_byte": round(8 * len(enc) / n, 4)}
            if n == 1 << 20:
                he = zr.HuffmanEncoder(d)
                g = he.encode(d)
                assert g == enc, "GPU Huffman O0 differs from the oracle"
                dec = zr.HuffmanDecoder(he.tree())
                assert dec.decode(g, n) == d
                r["gpu_host_api_encode_decode_mbps"] = rate(
                    lambda: zr.HuffmanDecoder(zr.HuffmanEncoder(d).tree()).decode(zr.HuffmanEncoder(d).encode(d),
                                                                                   n), n)
            row[f"{n >> 10}KiB"] = r
        out["inputs"][kind] = row
    out["value"] = out["inputs"]["t"]["1024KiB"]["encode_decode_mbps"]
    out["cpu_baseline"] = {"value": out["value"], "unit": "MB/s", "cores": 1, "kind": "port",
                           "sample": "1 MiB of text-like bytes, tree build + encode + decode, >= 1 s of repeats"}
    out["note"] = ("configs[0] is the CPU plumbing case (no GPU in the reference's path); "
                   "gpu_host_api_* is zr_huff_encode/zr_huff_decode from host memory, the tree built twice "
                   "per round trip as the Python mirror does")
    return out


def run_o1(args, torch, dist, world, rank, dev, zr, L):
    """configs[3] per GPU: 128 MiB text-like shard (1 GiB over 8 GPUs), order-1
    ContextualHuffman encode + decode (identity coding: two HBM copies)."""
    from zipora_amd import dist as zd
    n = 128 << 20
    host = zr.synth("t", n, seed=zd.shard_seed(1, rank))
    raw = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(dev)
    enc_model = zr.ContextualHuffmanEncoder(host[:1 << 16], zr.HuffmanOrder.Order1)
    d = zr.HuffmanO1Device(enc_model)
    enc = torch.empty_like(raw)
    out = torch.empty_like(raw)

    def step():
        d.encode_async(raw, enc)
        d.decode_async(enc, out, n)

    dt, dom, dom_ms, kms, _ = _measure(torch, dist, world, dev, L, step, args, ["huff_o1_decode", "huff_o1_encode"])
    if not torch.equal(out, raw):
        raise SystemExit("O1 round trip mismatch")
    extra = {"kernels_ms": kms, "kernels_ms_source": KMS_SOURCE}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        extra["cpu_baseline"] = cpu_baseline_o1(host, cpu_threads(args))
    return _line("GiB/s encode+decode (device-resident), Huffman O1, 1 GiB text over 8 GPUs", world * n * args.steps
                 / dt / 2**30, world, args, dt, "synthetic (order-1 Markov text, seed per rank)",
                 {"workload": "ContextualHuffman order-1 encode+decode, 128 MiB text per GPU (1/8 of 1 GiB)",
                  "parallelism": f"shard{world}"},
                 _roofline(dom, dom_ms, {"huff_o1_decode": 2 * n, "huff_o1_encode": 2 * n}, "o1",
                           {"huff_o1_decode": "k_copy16", "huff_o1_encode": "k_copy16"}), extra)


def run_blob(args, torch, dist, world, rank, dev, zr, L):
    """configs[4] per GPU: R x 1 KiB text records, rANS x1 per record with a
    shared trained table (RansBlobStore / RansCompressor record codec)."""
    from zipora_amd import dist as zd
    from zipora_amd.device import RansDeviceBatch
    R, rl = args.records, 1024
    total = R * rl
    host = zr.synth("t", total, seed=zd.shard_seed(5, rank))
    raw = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(dev)
    bt = RansDeviceBatch([rl] * R, 1, device=dev, shared_table=True)
    enc = bt.new_enc()
    out = bt.new_raw()

    comm = zd.shared_table_comm(world, rank) if world > 1 else None  # the shared trained table over ranks

    fused = comm is None and hasattr(L, "zr_rans_dtab_from_data_dev")  # histogram + table in one launch

    def step():
        if fused:
            bt.table_from_data(raw)
        else:
            bt.histogram(raw)
            if comm is not None:
                comm.allreduce_histogram(bt.hist)
            bt.tables_from_hist()
        bt.encode(raw, enc)
        bt.decode(enc, out)

    dt, dom, dom_ms, kms, _ = _measure(torch, dist, world, dev, L, step, args, ["rans_decode_x1", "rans_encode_x1"])
    exch = _exchange_info(zd, comm, world)
    if comm is not None:
        comm.close()
    bt.raise_on_error()
    if not torch.equal(out, raw):
        raise SystemExit("blob round trip mismatch")
    comp = int(bt.enc_len.sum().item())
    extra = {"kernels_ms": kms, "kernels_ms_source": KMS_SOURCE,
             "compressed_bytes": comp, "ratio": round(comp / total, 5), **exch}
    if world == 1 and not args.no_host_path:
        extra.update(host_pipe_rates(zr, bt, host, [1024] * R, 1, args.steps))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        extra["cpu_baseline"] = cpu_baseline_blob(host, cpu_threads(args))
    return _line("GiB/s encode+decode (device-resident), rANS x1 record batch, 1 M x 1 KiB", world * total *
                 args.steps / dt / 2**30, world, args, dt, "synthetic (order-1 Markov text records)",
                 {"workload": f"{R} x 1 KiB records per GPU, rANS x1 per record, shared trained table",
                  "records": R, "parallelism": f"shard{world}"},
                 _roofline(dom, dom_ms, {"rans_decode_x1": comp + total, "rans_encode_x1": total + comp}, "blob",
                           {"rans_decode_x1": "k_dec_x1_fast", "rans_encode_x1": "k_enc_x1_ring"}), extra)



def host_pipe_rates(zr, bt, host, lens, N, steps):
    """Host-resident batches through zr_rans_pipe_* (pinned host areas; H2D, coding and
    D2H of successive 32 MiB groups overlap). The shared table is the device batch's."""
    import numpy as np
    import torch
    from zipora_amd.device import RansHostPipe
    lens = np.asarray(lens, dtype=np.uint64)  # converted once, outside the timed calls
    # the shared table of the whole batch (the device step consumes bt.hist)
    hist = [int(v) for v in np.bincount(np.frombuffer(host, dtype=np.uint8), minlength=256)]
    pipe = RansHostPipe(zr.Rans64Encoder(hist, N).table, N)
    raw_off, _, rb, eb = pipe.layout(lens)
    pin = torch.empty(rb, dtype=torch.uint8, pin_memory=True)
    pin.copy_(torch.frombuffer(bytearray(host), dtype=torch.uint8))
    penc = torch.empty(eb, dtype=torch.uint8, pin_memory=True)
    pout = torch.empty(rb, dtype=torch.uint8, pin_memory=True)
    # packed output: records back to back, so only encoded bytes cross PCIe
    enc_off, enc_len, st, _ = pipe.encode_packed(lens, pin, raw_off, penc)  # warm: grows the slots
    pipe.decode(lens, penc, enc_off, enc_len, pout, raw_off)
    reps = max(1, min(3, steps))
    te = td = 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        enc_off, enc_len, st, _ = pipe.encode_packed(lens, pin, raw_off, penc)
        t1 = time.perf_counter()
        st2 = pipe.decode(lens, penc, enc_off, enc_len, pout, raw_off)
        td += time.perf_counter() - t1
        te += t1 - t0
    if (st != 0).any() or (st2 != 0).any() or not torch.equal(pout, pin):
        raise SystemExit("host pipeline mismatch")
    total = int(lens.sum())
    pipe.close()
    return {"host_resident_gibps": round(total * reps / (te + td) / 2**30, 3),
            "host_encode_gibps": round(total * reps / te / 2**30, 3),
            "host_decode_gibps": round(total * reps / td / 2**30, 3)}


def run_rans(args, torch, dist, world, rank, dev, zr, L, B, n, N, diag=(), host=None, host_path=True,
             cpu=True):
    """configs[1]: rANS O0 encode+decode of B x n bytes per GPU, N-way streams,
    one shared table (histogram -> [RCCL all-reduce] -> table -> encode -> decode)."""
    from zipora_amd import dist as zd
    from zipora_amd.device import RansDeviceBatch
    total = B * n
    if host is None:
        host = zr.synth(args.kind, total, seed=0x9E3779B97F4A7C15 + rank)
    raw = torch.frombuffer(bytearray(host[:total]), dtype=torch.uint8).to(dev)
    bt = RansDeviceBatch([n] * B, N, device=dev, shared_table=True)
    enc = bt.new_enc()
    out = bt.new_raw()
    stream = torch.cuda.current_stream(dev)

    # hist starts zeroed (allocation) and the consuming table build re-zeroes it,
    # so the step carries no memset (A/B runs against an older library, which
    # lacks the consuming entry point, memset instead)
    consume = hasattr(L, "zr_rans_dtab_from_hist_consume_dev")

    # the shared frequency table over ranks: the library's own RCCL communicator
    # (zr_comm_*; the unique id travels over the torch process group, host side)
    comm = zd.shared_table_comm(world, rank) if world > 1 else None

    # --groups G > 1: after the shared table, the B buffers are coded as G groups
    # of B / G on G streams (each group its own batch and workspace over the same
    # table), so one group's compaction and decode overlap the others' encoding
    G = max(1, getattr(args, "groups", 1)) if B % max(1, getattr(args, "groups", 1)) == 0 else 1
    groups = []
    if G > 1:
        bg = B // G
        for g in range(G):
            sub = RansDeviceBatch([n] * bg, N, device=dev, shared_table=True)
            sub.cbatch.tables = bt.tables.data_ptr()  # the whole batch's table
            lo, hi = g * bg * n, (g + 1) * bg * n
            eo = bt.enc_off_host[g * bg]
            groups.append((sub, raw[lo:hi], enc[eo:], out[lo:hi], torch.cuda.Stream(dev)))
        ev_tab = torch.cuda.Event()

    # one rank: histogram and table in one launch (the table built by the last
    # histogram workgroup); more ranks: the all-reduce sits between the two
    fused = comm is None and hasattr(L, "zr_rans_dtab_from_data_dev")

    # --pipeline: batches A and B (distinct data) alternate. Step k codes batch
    # k % 2 with the table made in step k - 1, and on a second stream makes the
    # table of batch (k + 1) % 2 once step k - 1 is done with it: the
    # histogram's HBM pass runs beside the latency-bound encoder
    pipe = bool(getattr(args, "pipeline", False)) and G == 1 and fused
    if pipe:
        host_b = zr.synth(args.kind, total, seed=0x2545F4914F6CDD1D + rank)
        raw_b = torch.frombuffer(bytearray(host_b), dtype=torch.uint8).to(dev)
        bt_b = RansDeviceBatch([n] * B, N, device=dev, shared_table=True)
        pp = {"k": 0, "batches": [(bt, raw), (bt_b, raw_b)], "side": torch.cuda.Stream(dev),
              "tab": [torch.cuda.Event(), torch.cuda.Event()], "done": [torch.cuda.Event(), torch.cuda.Event()]}
        bt.table_from_data(raw, stream)
        pp["tab"][0].record(stream)

    def step():
        if pipe:
            k = pp["k"]
            x, y = k & 1, (k & 1) ^ 1
            (bx, rx), (by, ry) = pp["batches"][x], pp["batches"][y]
            side = pp["side"]
            side.wait_event(pp["done"][y])  # step k - 1 has finished with batch y's table
            by.table_from_data(ry, side)
            pp["tab"][y].record(side)
            stream.wait_event(pp["tab"][x])
            bx.encode(rx, enc, stream)
            bx.decode(enc, out, stream)
            pp["done"][x].record(stream)
            pp["k"] = k + 1
            return
        if fused:
            bt.table_from_data(raw, stream)
        else:
            bt.histogram(raw, stream, zeroed=consume)
            if comm is not None:  # in-place u32 all-reduce of the 256 counts over xGMI
                comm.allreduce_histogram(bt.hist, stream.cuda_stream)
            bt.tables_from_hist(stream, consume=consume)
        if G == 1:
            bt.encode(raw, enc, stream)
            bt.decode(enc, out, stream)
            return
        ev_tab.record(stream)
        for sub, r, e, o, st in groups:
            st.wait_event(ev_tab)
            sub.encode(r, e, st)
            sub.decode(e, o, st)
        for *_, st in groups:
            stream.wait_stream(st)

    def last_raw():  # the batch the last step decoded (and its status array)
        if not pipe:
            return bt, raw
        return pp["batches"][(pp["k"] - 1) & 1]

    step()
    torch.cuda.synchronize(dev)
    fn = step
    graph = bool(getattr(args, "graph", 0)) and not pipe and G == 1 and comm is None
    if graph:
        # the whole step (histogram + table, encode with its compaction, the
        # decode's status clear and decode) captured once; untimed steps replay
        # it on the same stream, the event-timed ones run eagerly (a graph
        # bakes in the timer state it was captured with)
        cap = torch.cuda.Stream(dev)
        cap.wait_stream(stream)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap):
            cs = torch.cuda.current_stream(dev)
            if fused:
                bt.table_from_data(raw, cs)
            else:
                bt.histogram(raw, cs, zeroed=consume)
                bt.tables_from_hist(cs, consume=consume)
            bt.encode(raw, enc, cs)
            bt.decode(enc, out, cs)
        torch.cuda.synchronize(dev)
        out.zero_()
        g.replay()
        torch.cuda.synchronize(dev)
        if not diag:
            bt.raise_on_error()
            if not torch.equal(out, raw):
                raise SystemExit("decode mismatch after the first graph replay")

        def fn():
            if _TIMER_ON:
                step()
            else:
                g.replay()
    if not diag:
        b_, r_ = last_raw()
        b_.raise_on_error()
        if not torch.equal(out, r_):
            raise SystemExit("decode mismatch after the first step")

    dt, dom, dom_ms, kms, tms = _measure(torch, dist, world, dev, L, fn, args,
                                         ["rans_encode", "rans_decode", "rans_compact", "histogram"],
                                         also=["rans_decode"])
    if not diag:
        b_, r_ = last_raw()
        b_.raise_on_error()
        if not torch.equal(out, r_):
            raise SystemExit("decode mismatch in timed region")
        if pipe:  # the other batch, coded once more on its own
            b2, r2 = pp["batches"][pp["k"] & 1]
            torch.cuda.synchronize(dev)
            b2.encode(r2, enc, stream)
            b2.decode(enc, out, stream)
            torch.cuda.synchronize(dev)
            b2.raise_on_error()
            if not torch.equal(out, r2):
                raise SystemExit("decode mismatch (second pipelined batch)")
    if G > 1:  # the groups' statuses and lengths
        for sub, *_ in groups:
            sub.raise_on_error()
        comp_bytes = sum(int(sub.enc_len.sum().item()) for sub, *_ in groups)
    else:
        comp_bytes = int(bt.enc_len.sum().item())
    value = world * total * args.steps / dt / 2**30
    exch = _exchange_info(zd, comm, world)
    if comm is not None:
        comm.close()
    if diag:  # tools/*.sh read the kernel times; no metric from a diagnostic build
        return {"diagnostic": diag, "kernels_ms": kms, "ms_per_step": round(dt / args.steps * 1e3, 4),
                "timed_ms": {k: round(v, 4) for k, v in tms.items()}, "graph": graph}
    single = B == 1
    literal = single and N == 4096
    wl = "rans_literal" if literal else f"rans_n2e{N.bit_length() - 1}" if single else "rans"
    syms = dict(RANS_SYMS)  # the decode kernel this batch ran (zr_rans_decoder_kernel)
    if hasattr(L, "zr_rans_decoder_kernel"):
        syms["rans_decode"] = L.zr_rans_decoder_kernel(B, N).decode()
    rans_bytes = {"rans_encode": total + comp_bytes, "rans_decode": comp_bytes + total,
                  "rans_compact": 2 * comp_bytes, "histogram": total}

    res = {
        "metric": "GiB/s encode+decode (device-resident), rANS O0, 256 MiB, 1/2/4/8 MI355X",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (uniform xorshift64 bytes, tests/fse_tests.rs:711-717 generator)",
        "config": {"workload": (f"BASELINE configs[1] as written: rANS O0 encode+decode of ONE {n >> 20} MiB "
                                f"uniform buffer per GPU, {N}-way interleaved streams ({n // N} symbols per stream)"
                                if literal else
                                f"BASELINE.md C2 at N = {N}: rANS O0 encode+decode of ONE {n >> 20} MiB uniform "
                                f"buffer per GPU, {N}-way interleaved streams ({n // N} symbols per stream; the "
                                f"reference takes any N, rans.rs:165-168)"
                                if single else
                                f"rANS O0 encode+decode, {total >> 20} MiB uniform bytes per GPU as "
                                f"{B} x {n >> 20} MiB buffers, {N}-way interleaved streams each "
                                f"({B * N} streams), shared table (histogram all-reduce over ranks)"),
                   "buffers": B, "buffer_bytes": n, "n_streams": N, "parallelism": f"shard{world}",
                   "encoder_lanes": 64 if B * N <= 1 << 16 else 256,
                   **({"pipelined": "two distinct 256 MiB batches alternate; step k codes one batch (encode -> "
                                    "decode) while the histogram + table of the other run on a second HIP stream"}
                      if pipe else {})},
        # the dominant kernel's roofline (the encoder on the headline): algorithmic bytes
        # per launch = N_in read + C written (encode, decode), 2 C (compaction), N_in (histogram)
        "roofline": _roofline(dom, dom_ms, rans_bytes, wl, syms, kms),
        # the decoder's, from the instrumented pass (the decode half of the step)
        "roofline_decode": _roofline("rans_decode", tms["rans_decode"], rans_bytes, wl, syms, kms),
        # the whole step against the spec peak: (3 N_in + 2 C) / step time
        "step_frac": round((3 * total + 2 * comp_bytes) / (dt / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
        "kernels_ms": kms, "kernels_ms_source": KMS_SOURCE,
        "compressed_bytes": comp_bytes,
        "ratio": round(comp_bytes / total, 5),
    }
    res.update(exch)
    res["step_graph"] = graph  # untimed steps replayed a HIP graph of the step
    if rank == 0 and world == 1 and host_path and not args.no_host_path:
        res.update(host_pipe_rates(zr, bt, host[:total], [n] * B, N, args.steps))
    if rank == 0 and world == 1 and cpu and not args.no_cpu_baseline:
        # literal config: 16 MiB slices of the buffer, each its own x4096 stream set
        res["cpu_baseline"] = cpu_baseline(host, n, B, N, cpu_threads(args),
                                           sample_bytes=(16 << 20) if single else None)
    del raw, enc, out, bt
    return res


SECONDARY_KEYS = ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "config", "roofline",
                  "roofline_decode", "kernels_ms", "compressed_bytes", "ratio", "cpu_baseline",
                  "host_resident_gibps", "host_encode_gibps", "host_decode_gibps", "rccl_ranks",
                  "histogram_exchange")


def secondary_lines(args, torch, dist, world, rank, dev, zr, L, host):
    """The other BASELINE configs in the default run,
    each a short run of its own workload: configs[1] as written (one 256 MiB
    buffer x 4096 streams), configs[2] (FSE, 64 KiB blocks), configs[4] (the
    1 M x 1 KiB record batch), configs[3] (Huffman O1, the 128 MiB per-GPU shard
    of 1 GiB) and configs[0] (Huffman O0, 1 MiB, the CPU reference path). Not
    part of `value`."""
    import copy
    out = {}

    def sub(steps, warmup):
        a = copy.copy(args)
        a.steps, a.warmup = steps, warmup
        return a

    def slim(r):
        return {k: r[k] for k in SECONDARY_KEYS if k in r}

    out["rans_literal"] = slim(run_rans(sub(3, 1), torch, dist, world, rank, dev, zr, L, 1, 256 << 20, 4096,
                                        host=host, host_path=False))
    torch.cuda.empty_cache()
    # BASELINE.md C2's other stream count, N = 2^18, on ONE 256 MiB buffer
    out["rans_n2e18"] = slim(run_rans(sub(5, 2), torch, dist, world, rank, dev, zr, L, 1, 256 << 20, 1 << 18,
                                      host=host, host_path=False))
    torch.cuda.empty_cache()
    a = sub(3, 1)
    a.fse_block_kib = 64
    out["fse"] = slim(run_fse(a, torch, dist, world, rank, dev, zr, L))
    torch.cuda.empty_cache()
    a = sub(5, 2)
    a.records = 1 << 20
    out["blob"] = slim(run_blob(a, torch, dist, world, rank, dev, zr, L))
    torch.cuda.empty_cache()
    out["o1"] = slim(run_o1(sub(5, 2), torch, dist, world, rank, dev, zr, L))
    torch.cuda.empty_cache()
    if not args.no_cpu_baseline:
        out["huffman_o0"] = huffman_o0_line(zr)
    return out


def launch(args):
    """--gpus N > 1 without a launcher: start N rank processes (RANK/LOCAL_RANK/
    WORLD_SIZE/MASTER_* set as torch.distributed.run sets them, MASTER_ADDR
    127.0.0.1) as children of this process, which never touches a GPU; wait for
    them and exit with the first failure's code (the others are stopped). Only
    rank 0 prints the JSON line."""
    import socket
    import subprocess
    n = args.gpus
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    # (the port is free when probed; a process that takes it before rank 0
    # binds it makes rank 0's rendezvous fail, and the launch exits non-zero)
    import signal

    class _Stop(Exception):
        pass

    def _on_signal(signum, frame):
        raise _Stop(signum)

    old = {sig: signal.signal(sig, _on_signal) for sig in (signal.SIGTERM, signal.SIGINT)}
    procs = []
    rc, alive = 0, set()
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
            alive.add(r)
        while alive:
            for i in sorted(alive):
                c = procs[i].poll()
                if c is None:
                    continue
                alive.discard(i)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    print(f"bench.py: rank {i} exited with {c}; stopping the other ranks", file=sys.stderr)
                    for j in alive:
                        procs[j].terminate()
            time.sleep(0.1)
    except _Stop as e:
        print(f"bench.py: signal {e.args[0]}; stopping the ranks", file=sys.stderr)
        rc = 128 + int(e.args[0])
    finally:
        # no rank outlives the launcher (a killed parent would leave them holding GPUs)
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for sig, h in old.items():
            signal.signal(sig, h)
    return rc


def dry_run(world, rank):
    """The launcher path on a CPU box: a gloo group of `world` ranks, one empty
    timed step under the contract's barrier + max-over-ranks timing."""
    import torch
    import torch.distributed as dist
    from zipora_amd import dist as zd
    if world > 1:
        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    if world > 1:
        dist.barrier()
    dt = zd.max_over_ranks(time.perf_counter() - t0)
    seen = [(rank, os.getpid())]
    if world > 1:
        seen = [None] * world
        dist.all_gather_object(seen, (rank, os.getpid()))
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_seen": [r for r, _ in seen],
                          "processes": len({p for _, p in seen}),
                          "backend": dist.get_backend() if world > 1 else None, "max_s": dt}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        sys.exit(launch(args))
    if env_world is not None and args.gpus is not None and int(env_world) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}")
    if args.dry_run:
        return dry_run(int(env_world or 1), int(os.environ.get("RANK", "0")))
    from zipora_amd import _lib as _zl
    diag = _zl.diag_env()  # profiling ablations: garbage output, never a metric line
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import zipora_amd as zr
    L = zr.load()
    L.zr_set_device(local)

    copy_ceiling(torch, dev, L)
    if args.workload in ("fse", "o1", "blob"):
        fn = {"fse": run_fse, "o1": run_o1, "blob": run_blob}[args.workload]
        res = fn(args, torch, dist, world, rank, dev, zr, L)
        if diag:  # a diagnostic build or library override: kernel times only, never a metric line
            res = {"diagnostic": diag, "kernels_ms": res.get("kernels_ms"), "ms_per_step": res["ms_per_step"]}
        if rank == 0:
            print(json.dumps(res), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    B, n, N = args.buffers, args.buffer_mib << 20, args.streams
    host = zr.synth(args.kind, B * n, seed=0x9E3779B97F4A7C15 + rank)
    res = run_rans(args, torch, dist, world, rank, dev, zr, L, B, n, N, diag=diag, host=host)
    headline = (B, n, N) == (64, 4 << 20, 4096)
    if not diag and headline and world == 1 and not args.no_secondary:
        torch.cuda.empty_cache()
        res["secondary"] = secondary_lines(args, torch, dist, world, rank, dev, zr, L, host)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
