#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter_collection CSVs per kernel: pmc_sum.py <csv>..."""
import collections, csv, sys
for f in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(f, k, {c: round(sum(v) / len(v)) for c, v in d.items()})
