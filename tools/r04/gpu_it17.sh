# r04 iteration 17: conv forward x6 (pixel scale on the sum), K5 suites + bench A/B +
# timeline; BCQ actor head change: BCQ suites + bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/i17_conv.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_discrete_cql.py tests/test_gpu_arbiters.py tests/test_gpu_dqn.py tests/test_gpu_export.py tests/test_gpu_bcq_parity.py tests/test_gpu_iqn_fused.py > gpurun_out/i17_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for x in 1 0; do D3A_CONV_X6=$x timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline | sed "s/^/conv_x6 $x: /" >> gpurun_out/i17_bench.txt 2>/dev/null || exit $?; done
timeout -k 10 300 python bench.py --algo bcq --no-cpu-baseline | sed "s/^/bcq: /" >> gpurun_out/i17_bench.txt 2>/dev/null || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_dcql17 -o run --output-format csv -- python3 $R/bench.py --algo dcql --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $R/gpurun_out/tl_dcql17.log 2>&1 || exit $?
python tools/prof_timeline.py gpurun_out/tl_dcql17/run_kernel_trace.csv > gpurun_out/tl_dcql17.txt; rm -f gpurun_out/tl_dcql17/run_kernel_trace.csv
