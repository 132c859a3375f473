"""Launch sequence of one update step from a rocprofv3 kernel-trace CSV:
per launch its duration and the idle gap before it (the last complete step
of the trace, identified by the gather kernel that opens every step)."""
import csv
import sys

path = sys.argv[1]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "gather_" in r["Kernel_Name"]]
a, b = starts[-3], starts[-2]
prev_end = None
tot_k = tot_gap = 0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = 0 if prev_end is None else s - prev_end
    n = r["Kernel_Name"].replace("d3a::(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(")[0][:40]
    print(f"{n:40s} grid=({r['Grid_Size_X']},{r['Grid_Size_Y']},{r['Grid_Size_Z']}) "
          f"wg={r['Workgroup_Size_X']:>4s} dur={(e - s) / 1e3:7.2f}us gap={gap / 1e3:6.2f}us")
    tot_k += e - s
    tot_gap += max(gap, 0)
    prev_end = e
print(f"step: {(int(rows[b]['Start_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1e3:.1f} us, "
      f"kernels {tot_k / 1e3:.1f} us, gaps {tot_gap / 1e3:.1f} us, launches {b - a}")
