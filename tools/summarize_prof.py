#!/usr/bin/env python3
"""Summarise one round's rocprofv3 output directory (tools/profile_round.sh).

Prints per-kernel average duration (kernel-trace --stats) and per-dispatch HBM
traffic from the PMC passes, corrected as MI355X_MICROARCH.md (HBM section)
prescribes: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts
half of the bytes of 16-B-per-lane streaming reads, so it is doubled. Writes
<dir>/summary/traffic.json ({"source", "workloads": {workload: {kernel: {fetch_bytes,
write_bytes, hbm_bytes}}}}), the format bench.py reads from profiles/traffic.json.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_[A-Za-z0-9_]+)", name)
    return m.group(1) if m else name[:60]


def stats(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Name"])
                out.setdefault(os.path.relpath(f, d).split(os.sep)[0], {})[k] = {
                    "calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                    "pct": float(r["Percentage"])}
    return out


def counters(d, sub):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                vals[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    d = sys.argv[1]
    st = stats(d)
    for run, ks in sorted(st.items()):
        print(f"== kernel stats: {run}")
        for k, v in sorted(ks.items(), key=lambda kv: -kv[1]["pct"]):
            print(f"  {k:32s} calls={v['calls']:5d} avg={v['avg_us']:10.2f} us  {v['pct']:6.2f} %")
    traffic = {}
    for tag, fsub, wsub in (("rans", "pmc_fetch", "pmc_write"), ("rans_literal", "pmc_lit_fetch", "pmc_lit_write"),
                            ("fse64", "pmc_fse_fetch", "pmc_fse_write"), ("blob", "pmc_blob_fetch", "pmc_blob_write"),
                            ("o1", "pmc_o1_fetch", "pmc_o1_write"),
                            ("rans_n2e18", "pmc_n18_fetch", "pmc_n18_write")):
        fc, wc = counters(d, fsub), counters(d, wsub)
        ks = sorted({k for k, _ in fc} | {k for k, _ in wc})
        if ks:
            print(f"== HBM traffic per dispatch ({tag}; FETCH_SIZE x2 per the gfx950 rule)")
        for k in ks:
            fb = fc.get((k, "FETCH_SIZE"), 0.0) * 1024 * 2
            wb = wc.get((k, "WRITE_SIZE"), 0.0) * 1024
            traffic.setdefault(tag, {})[k] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb}
            print(f"  {k:32s} fetch={fb / 1e6:10.2f} MB  write={wb / 1e6:10.2f} MB  total={(fb + wb) / 1e6:10.2f} MB")
    os.makedirs(os.path.join(d, "summary"), exist_ok=True)
    with open(os.path.join(d, "summary", "traffic.json"), "w") as fh:
        json.dump({"source": os.path.basename(os.path.normpath(d)) + " PMC passes (FETCH_SIZE x2 + WRITE_SIZE)",
                   "workloads": traffic}, fh, indent=1)


if __name__ == "__main__":
    main()
