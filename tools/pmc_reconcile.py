"""Reconcile one SQ counter pass of the K2 step's MFMA kernels (r02).

    python tools/pmc_reconcile.py PMC_DIR OUT_TXT

Per kernel (median over its dispatches): the SQ wave-cycle split
(WAIT_ANY = parked on s_waitcnt / barrier, WAIT_INST_ANY = issue stall,
ACTIVE_INST_ANY = issuing; quad-cycles, disjoint), SQ_VALU_MFMA_BUSY_CYCLES
against the kernel's MFMA count x 64 cycles (v_mfma_f32_32x32x2_f32 issue
interval per SIMD), and the effective clock (GRBM_GUI_ACTIVE / 8 / duration
is not available from one pass, so GRBM_GUI_ACTIVE is printed raw).
"""
import csv
import glob
import statistics
import sys

KERNELS = {  # substring -> (label, algorithmic FLOP per dispatch)
    "mlp_fwd_kernel": ("critic ensemble fused forward + target aux pass", 2 * 2 * 15872 * 69376),
    "gemm_f32_kernel<2, 2, 1, 1, 4, 4, 32>": ("critic layer-1 dW (split-K 32)", 2 * 2 * 7936 * 65536),
    "gemm_f32_kernel<1, 2, 1, 1, 4, 4, 32>": ("critic layer-1 dX + ReLU mask", 2 * 2 * 7936 * 65536),
}


def main():
    d, out = sys.argv[1], sys.argv[2]
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            for sub in KERNELS:
                if sub in r.get("Kernel_Name", ""):
                    key = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
                    c = vals.setdefault(sub, {}).setdefault(r["Counter_Name"], {})
                    c[key] = c.get(key, 0.0) + float(r["Counter_Value"])
    lines = []
    for sub, (label, flops) in KERNELS.items():
        if sub not in vals:
            continue
        med = {n: statistics.median(v.values()) for n, v in vals[sub].items()}
        n_mfma = flops / 4096.0
        wc = med.get("SQ_WAVE_CYCLES", float("nan"))
        lines.append(f"{sub}  ({label}; {len(next(iter(vals[sub].values())))} dispatches)")
        for n in sorted(med):
            lines.append(f"  {n:28s} {med[n]:16.0f}")
        if wc == wc and wc > 0:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if n in med:
                    lines.append(f"  {n:28s} {100 * med[n] / wc:6.1f} % of SQ_WAVE_CYCLES")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in med:
            lines.append(f"  MFMA instructions (FLOP/4096) {n_mfma:14.0f}; x 64 cyc = "
                         f"{64 * n_mfma:14.0f}; SQ_VALU_MFMA_BUSY_CYCLES / that = "
                         f"{med['SQ_VALU_MFMA_BUSY_CYCLES'] / (64 * n_mfma):.3f}")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
