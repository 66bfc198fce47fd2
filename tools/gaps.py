#!/usr/bin/env python3
"""Per-kernel durations and the idle gaps before each, from a rocprofv3
kernel_trace.csv: gaps.py <kernel_trace.csv> [first-kernel-regex]"""
import csv, re, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = re.compile(sys.argv[2] if len(sys.argv) > 2 else "k_hist")
dur, gap, cnt = collections.defaultdict(float), collections.defaultdict(float), collections.Counter()
prev_end, steps, t0, spans = None, 0, None, []
for r in rows:
    name = re.sub(r"\(.*", "", r["Kernel_Name"])[:60]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if first.search(name):
        if t0 is not None:
            spans.append(s - t0)
        t0 = s
        steps += 1
    if prev_end is not None and steps > 1:
        gap[name] += max(0, s - prev_end)
        dur[name] += e - s
        cnt[name] += 1
    prev_end = e
n = max(1, steps - 1)
for k in dur:
    print(f"{k:60s} n/step={cnt[k] / n:4.1f} dur={dur[k] / n / 1e3:8.2f} us gap_before={gap[k] / n / 1e3:6.2f} us")
if spans:
    spans = spans[1:] or spans
    print(f"step span (first-kernel to first-kernel) median {sorted(spans)[len(spans) // 2] / 1e3:.1f} us;"
          f" sum dur {sum(dur.values()) / n / 1e3:.1f} us, sum gaps {sum(gap.values()) / n / 1e3:.1f} us")
