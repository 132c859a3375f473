"""Median per-dispatch value of every counter collected for a kernel.

    python tools/pmc_counters.py PMC_DIR KERNEL_SUBSTRING [LAST]

Reads the rocprofv3 --pmc counter_collection.csv files under PMC_DIR and
prints one line per counter (sum over the XCD/SE instances of a dispatch,
median over the last LAST matching dispatches, default 20).
"""
import csv
import glob
import statistics
import sys


def main():
    d, sub = sys.argv[1], sys.argv[2]
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub not in r.get("Kernel_Name", ""):
                continue
            key = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
            c = vals.setdefault(r["Counter_Name"], {})
            c[key] = c.get(key, 0.0) + float(r["Counter_Value"])
    for name in sorted(vals):
        v = [vals[name][k] for k in sorted(vals[name])[-last:]]
        print(f"{name:32s} {statistics.median(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
