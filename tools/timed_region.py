#!/usr/bin/env python3
"""Per-dispatch durations of the headline kernels in a kernel trace of the
default `python3 bench.py` run: the headline comes first (one first step,
W warmup steps, 4 x 8 instrumented steps, K timed steps, every kernel once
per step), so its dispatches of each kernel are the first 1 + W + 32 + K and
the timed region is the last K of them.
  timed_region.py <kernel_trace.csv> [W K]"""
import csv, sys
W = int(sys.argv[2]) if len(sys.argv) > 2 else 3
K = int(sys.argv[3]) if len(sys.argv) > 3 else 10
H = 1 + W + 32 + K
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
names = ["k_hist", "k_tab", "k_enc_xn<", "k_enc_compact", "k_dec_xn_fast<1024"]
print("kernel trace of `python3 bench.py` (the default command): per-dispatch durations, us")
print(f"headline: the first {H} dispatches of each kernel (1 first step + {W} warmup + 4x8 instrumented"
      f" + {K} timed); the timed region is dispatches {H - K + 1}-{H}")
for n in names:
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if n in r["Kernel_Name"]]
    k = next((r["Kernel_Name"] for r in rows if n in r["Kernel_Name"]), n)
    if len(d) < H:
        print(f"{k[:60]:60s} calls={len(d)} (fewer than {H})")
        continue
    h, t = d[:H], d[H - K:H]
    print(f"{k[:60]:60s} calls={len(d)} first{H} avg={sum(h) / H:8.1f} timed avg={sum(t) / K:8.1f}"
          f" min={min(t):6.1f} max={max(t):6.1f}")
