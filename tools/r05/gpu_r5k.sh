#!/bin/bash
# round 5: first-layer conv weight gradient, IQN recompute + iqn_cos, deep
# critic backward on split-bf16 GEMMs -- kernel tests, parity suites, benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5k
cd $R && mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_conv.py tests/test_gpu_iqn_fused.py tests/test_gpu_cql_softmax.py > $O/k_tests.log 2>&1 || { tail -30 $O/k_tests.log; exit 1; }
grep -E "passed|failed|recompute backward|IS block|data rows|prior cos" $O/k_tests.log | tail -20
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_cql_parity.py tests/test_gpu_discrete_cql.py tests/test_gpu_arbiters.py tests/test_gpu_bcq_parity.py > $O/par_tests.log 2>&1 || { tail -40 $O/par_tests.log; exit 1; }
tail -3 $O/par_tests.log
B="timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --transitions 100000"
$B --algo dcql > $O/b_dcql.json 2>$O/b_dcql.err || exit 1; echo dcql; cut -c1-220 $O/b_dcql.json
D3A_K5_BRANCHES=0 $B --algo dcql > $O/b_dcql_br0.json 2>>$O/b.err || exit 1; echo dcql_branches_off; cut -c1-220 $O/b_dcql_br0.json
D3A_CONV1_U8S4=0 $B --algo dcql > $O/b_dcql_c1off.json 2>>$O/b.err || exit 1; echo dcql_conv1off; cut -c1-220 $O/b_dcql_c1off.json
$B --algo cqlrepro > $O/b_repro.json 2>$O/b_repro.err || exit 1; echo repro; cut -c1-220 $O/b_repro.json
D3A_X6_DEEP=0 $B --algo cqlrepro > $O/b_repro_off.json 2>>$O/b.err || exit 1; echo repro_x6deep_off; cut -c1-220 $O/b_repro_off.json
$B --algo bcq > $O/b_bcq.json 2>$O/b_bcq.err || exit 1; echo bcq; cut -c1-220 $O/b_bcq.json
D3A_BCQ_BRANCHES=0 $B --algo bcq > $O/b_bcq_off.json 2>>$O/b.err || exit 1; echo bcq_branches_off; cut -c1-220 $O/b_bcq_off.json
export TMPDIR=/tmp
for a in dcql cqlrepro bcq; do
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tl_$a -o run --output-format csv -- python3 $R/bench.py --algo $a --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $O/tl_$a.log 2>&1 || exit 1
  cd $R && python tools/prof_timeline.py $O/tl_$a/run_kernel_trace.csv > $O/${a}_timeline.txt; rm -f $O/tl_$a/run_kernel_trace.csv
  tail -1 $O/${a}_timeline.txt
done
