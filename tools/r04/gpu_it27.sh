# r04 iteration 27 (final tree): Adam lanes per element by segment size; full GPU
# suite, smoke, K2 / K5 / K3 / K1 bench lines, K5 timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/i27
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench_lines.jsonl 2> $O/bench_cql.err || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/bench_lines.jsonl 2>/dev/null || exit $?
timeout -k 10 400 python bench.py --algo dcql --cpu-seconds 10 --cpu-seconds-1t 5 >> $O/bench_lines.jsonl 2>>$O/bench_err.log || exit $?
timeout -k 10 400 python bench.py --algo bcq --cpu-seconds 10 --cpu-seconds-1t 5 >> $O/bench_lines.jsonl 2>>$O/bench_err.log || exit $?
timeout -k 10 400 python bench.py --algo td3bc --cpu-seconds 10 --cpu-seconds-1t 5 >> $O/bench_lines.jsonl 2>>$O/bench_err.log || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tl_dcql -o run --output-format csv -- python3 $R/bench.py --algo dcql --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $O/tl_dcql.log 2>&1 || exit $?
python tools/prof_timeline.py $O/tl_dcql/run_kernel_trace.csv > $O/dcql_timeline.txt; rm -f $O/tl_dcql/run_kernel_trace.csv
