"""Per-launch HBM traffic of K5's adam_kernel launches (tools/r06/gpu_k5.sh),
grouped by grid (the early conv Adam and the late Adam are different
launches): FETCH_SIZE x 2 (gfx950's 64-B tally of 128-B requests) + WRITE_SIZE,
KiB per dispatch -> MB, median per grid.

    python tools/k5_adam_pmc.py FETCH_DIR WRITE_DIR
"""
import csv
import glob
import statistics
import sys
from collections import defaultdict


def per_grid(d, counter):
    out = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "adam_kernel" in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                out[r.get("Grid_Size", "")].append(float(r["Counter_Value"]))
    return out


def main():
    fd, wd = sys.argv[1:3]
    fe, wr = per_grid(fd, "FETCH_SIZE"), per_grid(wd, "WRITE_SIZE")
    for g in sorted(fe, key=lambda x: -int(x or 0)):
        f = statistics.median(fe[g]) * 2 * 1024 / 1e6
        w = statistics.median(wr.get(g, [0])) * 1024 / 1e6
        print(f"adam_kernel grid={g} n={len(fe[g])}: read {f:.2f} MB write {w:.2f} MB "
              f"total {f + w:.2f} MB")


if __name__ == "__main__":
    main()
