# kernel-trace of a short bench ($ALGO, default cql) -> per-launch timeline of one step
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
A=${ALGO:-cql}
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_$A -o run --output-format csv -- python3 $R/bench.py --algo $A --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 > $R/gpurun_out/tl_$A.log 2>&1 || exit $?
cd $R && python tools/prof_timeline.py gpurun_out/tl_$A/run_kernel_trace.csv > gpurun_out/tl_$A.txt && python tools/prof_by_shape.py gpurun_out/tl_$A/run_kernel_trace.csv 320 > gpurun_out/tl_${A}_shape.txt
rm -f $R/gpurun_out/tl_$A/run_kernel_trace.csv
