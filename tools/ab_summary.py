#!/usr/bin/env python3
"""Median step and timed kernel times per library of a tools/ab_multi.sh log."""
import collections
import json
import statistics as st
import sys

r = collections.defaultdict(list)
for line in open(sys.argv[1]):
    if "{" not in line:
        continue
    name = line.split(" :")[0].split(": {")[0]
    d = json.loads(line[line.index("{"):])
    r[name].append(d)
for name, ds in r.items():
    step = st.median(d["ms_per_step"] for d in ds)
    keys = ds[0].get("timed_ms") or ds[0].get("kernels_ms")
    src = "timed_ms" if ds[0].get("timed_ms") else "kernels_ms"
    ks = {k: round(st.median(d[src][k] for d in ds), 4) for k in keys}
    print(f"{name:48s} step {step:.4f}  {ks}  (n={len(ds)})")
