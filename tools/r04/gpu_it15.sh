# r04 iteration 15: x6 critic mask as bits: kernel tests, CQL suites, forward
# microbench A/B, K2 benches + timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_x6.py > gpurun_out/i15_x6.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_cql_parity.py tests/test_gpu_production_path.py tests/test_gpu_dp.py tests/test_gpu_sac_parity.py tests/test_gpu_capture_gc.py > gpurun_out/i15_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for f in "" "--hmask" "" "--hmask"; do timeout -k 10 120 python tools/bench_fwd.py --x6 --reps 2000 $f >> gpurun_out/i15_fwd.jsonl 2>/dev/null || exit $?; done
for sw in "20 5" "2000 50" "20 5"; do set -- $sw; timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu-baseline >> gpurun_out/i15_bench.jsonl 2>/dev/null || exit $?; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_i15 -o run --output-format csv -- python3 $R/bench.py --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 > $R/gpurun_out/tl_i15.log 2>&1 || exit $?
python tools/prof_timeline.py gpurun_out/tl_i15/run_kernel_trace.csv > gpurun_out/tl_i15.txt; rm -f gpurun_out/tl_i15/run_kernel_trace.csv
timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/i16_conv.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_discrete_cql.py tests/test_gpu_arbiters.py tests/test_gpu_dqn.py tests/test_gpu_export.py > gpurun_out/i16_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for x in 1 0; do D3A_CONV_X6=$x timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline | sed "s/^/conv_x6 $x: /" >> gpurun_out/i16_bench.txt 2>/dev/null || exit $?; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_dcql16 -o run --output-format csv -- python3 $R/bench.py --algo dcql --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $R/gpurun_out/tl_dcql16.log 2>&1 || exit $?
python tools/prof_timeline.py gpurun_out/tl_dcql16/run_kernel_trace.csv > gpurun_out/tl_dcql16.txt; rm -f gpurun_out/tl_dcql16/run_kernel_trace.csv
