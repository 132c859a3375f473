# r04 iteration 10: in-kernel BCQ target rows (xg_*), tests + K3 bench + K3 timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_bcq_parity.py tests/test_gpu_arbiters.py > gpurun_out/i10_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --algo bcq --no-cpu-baseline >> gpurun_out/i10_bench.jsonl 2>/dev/null || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_bcq10 -o run --output-format csv -- python3 $R/bench.py --algo bcq --steps 100 --warmup 10 --no-cpu-baseline --transitions 200000 > $R/gpurun_out/tl_bcq10.log 2>&1 || exit $?
python tools/prof_timeline.py gpurun_out/tl_bcq10/run_kernel_trace.csv > gpurun_out/tl_bcq10.txt; rm -f gpurun_out/tl_bcq10/run_kernel_trace.csv
