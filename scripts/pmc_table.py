#!/usr/bin/env python3
"""Per-kernel mean of each counter in rocprofv3 --pmc counter_collection CSVs.
    python scripts/pmc_table.py gpurun_out/pmc_dir [...]"""
import csv, glob, os, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void amr::", "").replace("amr::", "")[:40]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.4g}  (n={len(v)})")
