#!/usr/bin/env python3
"""Durations (us) of every dispatch of one kernel, in launch order, from a
rocprofv3 kernel_trace.csv: kdur.py <kernel_trace.csv> <kernel-substring>"""
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if sys.argv[2] in r["Kernel_Name"]]
print(len(d), "dispatches")
print(" ".join(f"{x:.1f}" for x in d))
