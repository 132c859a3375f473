# r04 iteration 8: x6 default; narrow-head x6 forward + target means (K3);
# full GPU suite, smoke, benches (K2 20/5 and 2000/50, K3, bf16), K3 timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_x6.py > gpurun_out/i8_x6.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests > gpurun_out/i8_gpu_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/i8_smoke.log 2>&1 || exit $?
for sw in "20 5" "2000 50"; do set -- $sw; timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu-baseline >> gpurun_out/i8_bench.jsonl 2>/dev/null || exit $?; done
timeout -k 10 200 python bench.py --algo bcq --no-cpu-baseline >> gpurun_out/i8_bench.jsonl 2>/dev/null || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_bcq -o run --output-format csv -- python3 $R/bench.py --algo bcq --steps 100 --warmup 10 --no-cpu-baseline --transitions 200000 > $R/gpurun_out/tl_bcq.log 2>&1 || exit $?
python tools/prof_timeline.py gpurun_out/tl_bcq/run_kernel_trace.csv > gpurun_out/tl_bcq.txt; rm -f gpurun_out/tl_bcq/run_kernel_trace.csv
