# r04 iteration 19: split-bf16 conv weight gradient (conv_bwd_w_x6_kernel):
# + implicit-GEMM conv input gradient (d3a_conv_bwd_x): conv tests, per-layer microbench A/B, K5 suites, K5 bench A/B + timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/i19_conv.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for x in 1 0; do D3A_CONV_BWD_X6=$x timeout -k 10 120 python tools/bench_conv_bwd.py >> gpurun_out/i19_convbench.jsonl 2>gpurun_out/i19_convbench.err || exit $?; done
D3A_CONV_BWD_X6=0 SPLITS=32 timeout -k 10 120 python tools/bench_conv_bwd.py >> gpurun_out/i19_convbench.jsonl 2>>gpurun_out/i19_convbench.err || exit $?
timeout -k 10 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_discrete_cql.py tests/test_gpu_arbiters.py tests/test_gpu_dqn.py > gpurun_out/i19_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for x in 1 0; do D3A_CONV_BWD_X6=$x D3A_CONV_BWD_X=$x timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline | sed "s/^/conv_bwd_x6+x $x: /" >> gpurun_out/i19_bench.txt 2>/dev/null || exit $?; done
D3A_CONV_BWD_X=0 timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline | sed "s/^/conv_bwd_x 0 only: /" >> gpurun_out/i19_bench.txt 2>/dev/null || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_dcql19 -o run --output-format csv -- python3 $R/bench.py --algo dcql --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $R/gpurun_out/tl_dcql19.log 2>&1 || exit $?
python tools/prof_timeline.py gpurun_out/tl_dcql19/run_kernel_trace.csv > gpurun_out/tl_dcql19.txt; rm -f gpurun_out/tl_dcql19/run_kernel_trace.csv
