"""Per-(kernel, grid) breakdown of a rocprofv3 kernel-trace CSV, per update step."""
import collections
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 320
rows = list(csv.DictReader(open(path)))
g = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].replace("d3a::(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(")[0]
    key = (n[:44], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
    g[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = 0
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v)
    if sum(v) / steps / 1e3 < 0.5:
        continue
    print(f"{k[0]:44s} grid=({k[1]},{k[2]},{k[3]}) wg={k[4]:>4s} n={len(v):5d} "
          f"avg={sum(v)/len(v)/1e3:7.2f}us per-step={sum(v)/steps/1e3:7.2f}us")
print(f"total per step: {tot/steps/1e3:.1f} us")
