# r04 iteration 20: uint8 conv weight gradient back on the fp32 kernel (32 splits),
# actor-head fusion off: K5 suites + bench + timeline, K2 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_arbiters.py -k dcql > gpurun_out/i20_arb.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_discrete_cql.py tests/test_gpu_dqn.py tests/test_gpu_conv.py tests/test_gpu_sampler.py tests/test_gpu_export.py > gpurun_out/i20_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/i20_bench.txt 2>/dev/null || exit $?
D3A_GATHER_BATCHED=0 timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline | sed "s/^/gather_batched 0: /" >> gpurun_out/i20_bench.txt 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline | sed "s/^/cql: /" >> gpurun_out/i20_bench.txt 2>/dev/null || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_dcql20 -o run --output-format csv -- python3 $R/bench.py --algo dcql --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $R/gpurun_out/tl_dcql20.log 2>&1 || exit $?
python tools/prof_timeline.py gpurun_out/tl_dcql20/run_kernel_trace.csv > gpurun_out/tl_dcql20.txt; rm -f gpurun_out/tl_dcql20/run_kernel_trace.csv
