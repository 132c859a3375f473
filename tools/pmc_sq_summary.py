"""Per-kernel SQ counter summary of one rocprofv3 --pmc pass over tools/pmc_step.py
(SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES):
the median per dispatch over each kernel's dispatches, the wait / active
fractions of the wave cycles, and MFMA-busy cycles per SIMD (1,024 SIMDs).

    python tools/pmc_sq_summary.py PMC_DIR > profiles/r04_pmc_sq_step_cql.txt
    python tools/pmc_sq_summary.py PMC_DIR wide   # every counter's median, kernels matching "wide"
"""
import csv
import glob
import statistics
import sys


def main():
    files = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
    per = {}   # (kernel, dispatch) -> {counter: value}
    grid = {}
    order = []
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            key = (k, int(r.get("Dispatch_Id") or r.get("Correlation_Id")))
            d = per.setdefault(key, {})
            c = r["Counter_Name"]
            d[c] = d.get(c, 0.0) + float(r["Counter_Value"])
            grid[k] = r.get("Grid_Size", "")
            if k not in order:
                order.append(k)
    if len(sys.argv) > 2:
        for k in order:
            if sys.argv[2] not in k:
                continue
            ds = [v for (kk, _), v in per.items() if kk == k]
            print(k.split("(")[0][-60:], f"({len(ds)} dispatches)")
            for c in sorted({c for d in ds for c in d}):
                print(f"  {c:<28} {statistics.median([d.get(c, 0.0) for d in ds]):.4e}")
        return
    print("kernel grid wave_cycles wait_any_frac wait_inst_any_frac active_inst_frac "
          "mfma_busy_per_simd(k cycles)")
    for k in order:
        ds = [v for (kk, _), v in per.items() if kk == k]

        def med(c):
            return statistics.median([d.get(c, 0.0) for d in ds])
        wc = med("SQ_WAVE_CYCLES") or 1.0
        name = k.replace("(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0][-48:]
        print(f"{name:<50} {grid[k]:>8} {wc:.2e} {med('SQ_WAIT_ANY') / wc:.3f} "
              f"{med('SQ_WAIT_INST_ANY') / wc:.3f} {med('SQ_ACTIVE_INST_ANY') / wc:.3f} "
              f"{med('SQ_VALU_MFMA_BUSY_CYCLES') / 1024 / 1000:.2f}")


if __name__ == "__main__":
    main()
