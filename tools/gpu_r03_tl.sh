# Kernel traces (timeline + per-shape breakdown) of the K2 fp32 and bf16 lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
for p in fp32 bf16; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tl_$p -o k2 --output-format csv -- python3 bench.py --precision $p --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 > gpurun_out/tl_$p.log 2>&1 || exit $?
  f=$(find gpurun_out/tl_$p -name '*kernel_trace.csv' -print -quit)
  python tools/prof_by_shape.py "$f" 320 > gpurun_out/tl_${p}_breakdown.txt 2>&1 || true
  python tools/prof_timeline.py "$f" > gpurun_out/tl_${p}_timeline.txt 2>&1 || true
done
