# r04 iteration 14: fused IQN head backward (tests, K5 parity), fused forward
# grid A/B, K5 bench + timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_iqn_fused.py > gpurun_out/i14_iqn.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_discrete_cql.py tests/test_gpu_arbiters.py tests/test_gpu_export.py > gpurun_out/i14_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for gsz in 256 512 1024 4096; do D3A_IQN_GRID=$gsz timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline | sed "s/^/grid $gsz: /" >> gpurun_out/i14_bench.txt 2>/dev/null || exit $?; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_dcql14 -o run --output-format csv -- python3 $R/bench.py --algo dcql --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $R/gpurun_out/tl_dcql14.log 2>&1 || exit $?
python tools/prof_timeline.py gpurun_out/tl_dcql14/run_kernel_trace.csv > gpurun_out/tl_dcql14.txt; rm -f gpurun_out/tl_dcql14/run_kernel_trace.csv
