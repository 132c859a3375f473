# r04 iteration 25: CQL logsumexp + loss stages in one launch (d3a_cql_loss ticket):
# CQL / SAC / DP suites, K2 bench A/B + 20-step window, K4 bench, K2 timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/i25
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_cql_parity.py -k "fused_lse or hopper or wide" > $O/cql.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_sac_parity.py tests/test_gpu_dp.py tests/test_gpu_production_path.py tests/test_gpu_api.py tests/test_gpu_capture_gc.py tests/test_gpu_actor_q.py tests/test_gpu_x6.py > $O/tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for x in 1 0 1; do D3A_LOSS_FUSED=$x timeout -k 10 300 python bench.py --no-cpu-baseline | sed "s/^/fused $x: /" >> $O/bench.txt 2>/dev/null || exit $?; done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline | sed "s/^/window: /" >> $O/bench.txt 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --algo cqldp --no-cpu-baseline | sed "s/^/cqldp: /" >> $O/bench.txt 2>/dev/null || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 500 --warmup 20 --no-cpu-baseline --transitions 200000 > $O/prof.log 2>&1 || exit $?
python tools/prof_timeline.py $O/prof/run_kernel_trace.csv > $O/cql_timeline.txt; rm -f $O/prof/run_kernel_trace.csv
