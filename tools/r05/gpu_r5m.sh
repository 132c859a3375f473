#!/bin/bash
# round 5: one-launch small-batch MLP backward (K3) -- kernel test, BCQ
# parity + arbiters, K3 bench A/B, timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5m
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_mlp_bwd_small.py > $O/sb_tests.log 2>&1 || { tail -30 $O/sb_tests.log; exit 1; }
grep -E "passed|failed|\{" $O/sb_tests.log | tail -8
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_bcq_parity.py tests/test_gpu_arbiters.py > $O/bcq_tests.log 2>&1 || { tail -40 $O/bcq_tests.log; exit 1; }
tail -3 $O/bcq_tests.log
B="timeout -k 10 200 python -u bench.py --steps 500 --warmup 20 --no-cpu-baseline --transitions 100000 --algo bcq"
$B > $O/b_bcq.json 2>$O/b_bcq.err || exit 1; echo bcq; cut -c1-200 $O/b_bcq.json
D3A_SMALL_BWD=0 $B > $O/b_bcq_off.json 2>>$O/b_bcq.err || exit 1; echo bcq_small_off; cut -c1-200 $O/b_bcq_off.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tl_bcq -o run --output-format csv -- python3 $R/bench.py --algo bcq --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $O/tl_bcq.log 2>&1 || exit 1
cd $R && python tools/prof_timeline.py $O/tl_bcq/run_kernel_trace.csv > $O/bcq_timeline.txt; rm -f $O/tl_bcq/run_kernel_trace.csv
cat $O/bcq_timeline.txt
