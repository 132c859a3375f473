# full GPU suite, the four bench lines and a K2 kernel-trace profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_cql.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --algo td3bc --steps 4000 > gpurun_out/bench_td3bc.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --algo bcq --steps 1000 > gpurun_out/bench_bcq.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 > gpurun_out/bench_dcql.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 > $R/gpurun_out/prof.log 2>&1 || exit $?
cd $R && python tools/prof_by_shape.py gpurun_out/prof/run_kernel_trace.csv 320 > gpurun_out/prof_breakdown.txt
