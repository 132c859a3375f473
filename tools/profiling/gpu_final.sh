# Round measurement: K2 bench (with CPU baseline), rocprofv3 kernel stats of the
# same command, PMC traffic of the dominant kernel, the other workloads' bench
# lines.  Everything lands in gpurun_out/; copy what is judged into profiles/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/final_bench_cql.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/final_prof -o run --output-format csv -- python3 $R/bench.py --steps 500 --warmup 20 --no-cpu-baseline --transitions 200000 > $R/gpurun_out/final_prof.log 2>&1 || exit $?
cd $R && python tools/prof_by_shape.py gpurun_out/final_prof/run_kernel_trace.csv 520 > gpurun_out/final_prof_breakdown.txt && rm -f gpurun_out/final_prof/run_kernel_trace.csv
bash tools/profiling/pmc_pass.sh cql mlp_fwd_kernel || exit $?
cd $R
for a in td3bc bcq dcql cqldp; do
  timeout -k 10 300 python bench.py --algo $a --cpu-seconds 10 > gpurun_out/final_bench_$a.log 2>&1 || exit $?
done
