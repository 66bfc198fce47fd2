#!/usr/bin/env python3
"""Probe: headline step eager vs captured into a HIP graph (torch.cuda.CUDAGraph),
library timers off; and whether events recorded inside the capture time a kernel."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import zipora_amd as zr
from zipora_amd.device import RansDeviceBatch
dev = torch.device("cuda", 0)
L = zr.load()
B, n, N = 64, 4 << 20, 4096
host = zr.synth("u", B * n, seed=1)
raw = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(dev)
bt = RansDeviceBatch([n] * B, N, device=dev, shared_table=True)
enc, out = bt.new_enc(), bt.new_raw()
side = torch.cuda.Stream(dev)
res = {}
def step(s):
    bt.histogram(raw, s, zeroed=True)
    bt.tables_from_hist(s, consume=True)
    bt.encode(raw, enc, s)
    bt.decode(enc, out, s)
with torch.cuda.stream(side):
    for _ in range(3):
        step(side)
torch.cuda.synchronize()
assert torch.equal(out, raw)
K = 50
with torch.cuda.stream(side):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(K):
        step(side)
    torch.cuda.synchronize(); res["eager_ms"] = (time.perf_counter() - t0) / K * 1e3
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=side):
    step(torch.cuda.current_stream())
torch.cuda.synchronize()
out.zero_()
g.replay(); torch.cuda.synchronize()
res["graph_ok"] = bool(torch.equal(out, raw))
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(K):
    g.replay()
torch.cuda.synchronize(); res["graph_ms"] = (time.perf_counter() - t0) / K * 1e3
# events inside a capture around the encode call
try:
    e0, e1 = torch.cuda.Event(enable_timing=True, external=True), torch.cuda.Event(enable_timing=True, external=True)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, stream=side):
        s = torch.cuda.current_stream()
        bt.histogram(raw, s, zeroed=True)
        bt.tables_from_hist(s, consume=True)
        e0.record(s)
        bt.encode(raw, enc, s)
        e1.record(s)
        bt.decode(enc, out, s)
    torch.cuda.synchronize()
    tot = 0.0
    t0 = time.perf_counter()
    for _ in range(K):
        g2.replay()
        e1.synchronize()
        tot += e0.elapsed_time(e1)
    res["graph_ev_step_ms"] = (time.perf_counter() - t0) / K * 1e3
    res["graph_ev_encode_ms"] = tot / K
except Exception as ex:  # noqa
    res["graph_ev_error"] = repr(ex)[:300]
print(json.dumps(res), flush=True)
