# kernel-trace profiles of the K2 bench, default and with the fused backward
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_a -o run --output-format csv -- python3 $R/bench.py --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 > $R/gpurun_out/prof_a.log 2>&1 || exit $?
D3A_FUSED_BWD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_b -o run --output-format csv -- python3 $R/bench.py --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 > $R/gpurun_out/prof_b.log 2>&1 || exit $?
cd $R && python tools/prof_by_shape.py gpurun_out/prof_a/run_kernel_trace.csv 320 > gpurun_out/prof_a.txt && python tools/prof_by_shape.py gpurun_out/prof_b/run_kernel_trace.csv 320 > gpurun_out/prof_b.txt
