"""Average of every counter of one kernel over its dispatches in a rocprofv3
counter-collection CSV: python tools/pmc_avg.py <dir-or-csv> <kernel substring>."""
import collections
import csv
import glob
import os
import sys

path, sub = sys.argv[1], sys.argv[2]
if os.path.isdir(path):
    path = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    if sub in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:28s} n={len(v):4d} avg={sum(v) / len(v):.6g}")
