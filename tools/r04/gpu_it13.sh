# r04 iteration 13: fused IQN head forward (tests, K5 parity + bench A/B,
# timeline); x6 forward mask-image write A/B (microbench)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_iqn_fused.py > gpurun_out/i13_iqn.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_discrete_cql.py tests/test_gpu_arbiters.py tests/test_gpu_conv.py tests/test_gpu_export.py > gpurun_out/i13_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for f in "" "--hmask" "" "--hmask"; do timeout -k 10 120 python tools/bench_fwd.py --x6 --reps 2000 $f >> gpurun_out/i13_fwd.jsonl 2>/dev/null || exit $?; done
for m in 1 0; do D3A_IQN_FUSED=$m timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline >> gpurun_out/i13_bench.jsonl 2>/dev/null || exit $?; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_dcql13 -o run --output-format csv -- python3 $R/bench.py --algo dcql --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $R/gpurun_out/tl_dcql13.log 2>&1 || exit $?
python tools/prof_timeline.py gpurun_out/tl_dcql13/run_kernel_trace.csv > gpurun_out/tl_dcql13.txt; rm -f gpurun_out/tl_dcql13/run_kernel_trace.csv
bash tools/profiling/gpu_r04_measure.sh
