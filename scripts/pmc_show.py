#!/usr/bin/env python3
"""Summarise rocprofv3 counter_collection CSVs: per kernel, counter totals per dispatch."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:30]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    for k, v in acc.items():
        if "copyBuffer" in k:
            continue
        n = max(1, len(disp[k]))
        print(d.split("/")[-1], k, {c: f"{x / n:.4g}" for c, x in v.items()})
