# r04 iteration 28 (final tree, Adam lanes restored): full GPU suite, smoke, K2 and K5 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/i28
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_lines.jsonl 2>/dev/null || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/bench_lines.jsonl 2>/dev/null || exit $?
timeout -k 10 400 python bench.py --algo dcql --no-cpu-baseline >> $O/bench_lines.jsonl 2>/dev/null || exit $?
