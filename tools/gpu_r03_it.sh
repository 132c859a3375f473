# Iteration: full GPU suite, K2 bench line, K2 kernel trace (breakdown +
# timeline), launch-floor probe.  $1 = tag for the output files.
set -o pipefail
T=${1:-it}
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --steps 2000 --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o k2 --output-format csv -- python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 > gpurun_out/${T}_prof.log 2>&1 || exit $?
f=$(find gpurun_out/${T}_prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_by_shape.py "$f" 320 > gpurun_out/${T}_breakdown.txt 2>&1 || true
python tools/prof_timeline.py "$f" > gpurun_out/${T}_timeline.txt 2>&1 || true
rm -f "$f"
timeout -k 10 60 python tools/launch_floor.py > gpurun_out/${T}_floor.json 2>&1 || true
exit $rc
