# r04 iteration 26: the step's conv weight copies in one launch (d3a_conv_pack_weights):
# conv + K5 suites, K5 bench A/B (2,000 steps), timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/i26
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_discrete_cql.py tests/test_gpu_arbiters.py tests/test_gpu_dqn.py tests/test_gpu_export.py > $O/tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for x in 1 0; do D3A_CONV_PREPACK=$x timeout -k 10 400 python bench.py --algo dcql --no-cpu-baseline | sed "s/^/prepack $x: /" >> $O/bench.txt 2>/dev/null || exit $?; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tl_dcql -o run --output-format csv -- python3 $R/bench.py --algo dcql --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $O/tl_dcql.log 2>&1 || exit $?
python tools/prof_timeline.py $O/tl_dcql/run_kernel_trace.csv > $O/dcql_timeline.txt; rm -f $O/tl_dcql/run_kernel_trace.csv
