#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv as name / calls / average ms."""
import csv
import glob
import sys

for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:48]:48s} calls={r['Calls']:>4} avg_ms={float(r['AverageNs']) / 1e6:9.3f}")
