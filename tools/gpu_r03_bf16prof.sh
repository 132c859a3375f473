# bf16 line: kernel trace of a short bench run -> breakdown + timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/bf16_prof -o bf16 --output-format csv -- python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 --precision bf16 > gpurun_out/bf16_prof.log 2>&1 || exit $?
f=$(find gpurun_out/bf16_prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_by_shape.py "$f" 320 > gpurun_out/bf16_breakdown.txt 2>&1 || true
python tools/prof_timeline.py "$f" > gpurun_out/bf16_timeline.txt 2>&1 || true
