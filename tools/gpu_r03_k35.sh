# Kernel traces of the K3 (BCQ) and K5 (DiscreteCQL-IQN) steps: breakdown and timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
for a in bcq dcql; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/k35_$a -o run --output-format csv -- python3 bench.py --algo $a --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/k35_$a.log 2>&1 || exit $?
  f=$(find gpurun_out/k35_$a -name '*kernel_trace.csv' -print -quit)
  python tools/prof_by_shape.py "$f" 70 > gpurun_out/k35_${a}_breakdown.txt 2>&1 || true
  python tools/prof_timeline.py "$f" > gpurun_out/k35_${a}_timeline.txt 2>&1 || true
  rm -f "$f"
done
