#!/bin/bash
# round 5: the IQN head backward recomputing phi from tau -- kernel tests,
# DiscreteCQL suites + K5 arbiters, K5 bench (recompute vs kept rows), timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5i
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_iqn_fused.py > $O/iqn_tests.log 2>&1 || { tail -30 $O/iqn_tests.log; exit 1; }
grep -E "passed|failed|recompute backward" $O/iqn_tests.log | tail -8
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_discrete_cql.py tests/test_gpu_arbiters.py > $O/dcql_tests.log 2>&1 || { tail -40 $O/dcql_tests.log; exit 1; }
tail -3 $O/dcql_tests.log
for nb in 4 2 8; do
  D3A_IQN_NB=$nb timeout -k 10 200 python -u bench.py --algo dcql --steps 100 --warmup 10 --no-cpu-baseline --transitions 100000 > $O/bench_nb$nb.json 2>$O/bench_nb$nb.err || exit 1
  echo "NB $nb"; cut -c1-300 $O/bench_nb$nb.json
done
D3A_IQN_RECOMPUTE=0 timeout -k 10 200 python -u bench.py --algo dcql --steps 100 --warmup 10 --no-cpu-baseline --transitions 100000 > $O/bench_keep.json 2>$O/bench_keep.err || exit 1
echo keep; cut -c1-300 $O/bench_keep.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --algo dcql --steps 50 --warmup 5 --no-cpu-baseline --transitions 100000 > $O/prof.log 2>&1 || exit 1
cd $R && python tools/prof_timeline.py $O/prof/run_kernel_trace.csv > $O/dcql_timeline.txt; rm -f $O/prof/run_kernel_trace.csv
cat $O/dcql_timeline.txt | tail -20
