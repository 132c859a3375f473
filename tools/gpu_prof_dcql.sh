# K5 DiscreteCQL-IQN kernel-trace profile + per-kernel breakdown
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dcql -o run --output-format csv -- python3 $R/bench.py --algo dcql --steps 100 --warmup 10 --no-cpu-baseline --transitions 200000 > $R/gpurun_out/prof_dcql.log 2>&1 || exit $?
cd $R && python tools/prof_by_shape.py gpurun_out/prof_dcql/run_kernel_trace.csv 110 > gpurun_out/prof_dcql_breakdown.txt
