"""Per-launch HBM traffic of the dominant kernel from two rocprofv3 --pmc passes.

    python tools/pmc_summarize.py FETCH_DIR WRITE_DIR KERNEL_SUBSTRING OUT_JSON [DESC_JSON [ROUND]]

FETCH_SIZE is doubled (gfx950: wide coalesced reads are tallied at 64 B per
128-B request, MI355X_MICROARCH.md 'HBM'); WRITE_SIZE is taken as is.  Both
counters report KiB per dispatch.  The median over the matching dispatches
is written as hbm_bytes_per_launch, with what it measured: the full kernel
names (template arguments) and grid / workgroup sizes of those dispatches,
and -- given DESC_JSON from tools/pmc_dominant.py --desc-out -- the bench
line's kernel description, which bench.py requires to match before it
reports the file's bytes as roofline.traffic.
"""
import csv
import glob
import json
import statistics
import sys


def signatures(d, sub):
    """(kernel name, grid, workgroup) of the matching dispatches."""
    out = set()
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r.get("Kernel_Name", ""):
                out.add((r.get("Kernel_Name", ""), r.get("Grid_Size", ""),
                         r.get("Workgroup_Size", "")))
    return sorted(out)


def per_dispatch(d, counter, sub, last=20):
    """Counter value per matching dispatch, the last `last` dispatches only
    (tools/pmc_dominant.py launches the dominant kernel last, after warm-up
    updates that may run kernels with the same name)."""
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if sub in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                key = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)[-last:]]


def main():
    fdir, wdir, sub, out = sys.argv[1:5]
    f = per_dispatch(fdir, "FETCH_SIZE", sub)
    w = per_dispatch(wdir, "WRITE_SIZE", sub)
    fetch = 2.0 * statistics.median(f) * 1024.0
    write = statistics.median(w) * 1024.0
    res = {"kernel_substring": sub, "dispatches": [len(f), len(w)],
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "hbm_bytes_per_launch": fetch + write,
           "note": "FETCH_SIZE x2 (gfx950 wide-read tally) + WRITE_SIZE; KiB -> bytes",
           "kernels": [{"name": n, "grid": g, "workgroup": w} for n, g, w in signatures(fdir, sub)]}
    if len(sys.argv) > 5:
        res["bench_desc"] = json.load(open(sys.argv[5]))["desc"]
    if len(sys.argv) > 6:
        res["round"] = int(sys.argv[6])
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
