# r04 iteration 12: x6 backward on the forward's mask image: kernel tests,
# microbench A/B, CQL parity suite, K2 benches (mask image on / off)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_x6.py > gpurun_out/i12_x6.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_cql_parity.py tests/test_gpu_production_path.py tests/test_gpu_dp.py tests/test_gpu_sac_parity.py > gpurun_out/i12_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for m in 1 0; do D3A_MASK_IMAGE=$m timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline >> gpurun_out/i12_bench.jsonl 2>/dev/null || exit $?; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_i12 -o run --output-format csv -- python3 $R/bench.py --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 > $R/gpurun_out/tl_i12.log 2>&1 || exit $?
python tools/prof_timeline.py gpurun_out/tl_i12/run_kernel_trace.csv > gpurun_out/tl_i12.txt; rm -f gpurun_out/tl_i12/run_kernel_trace.csv
