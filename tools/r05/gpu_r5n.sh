#!/bin/bash
# round 5: K3 with late-forked graph branches (A/B), BCQ parity with them on
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5n
cd $R && mkdir -p $O
D3A_BCQ_BRANCHES=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_bcq_parity.py > $O/bcq_tests.log 2>&1 || { tail -40 $O/bcq_tests.log; exit 1; }
tail -1 $O/bcq_tests.log
B="timeout -k 10 200 python -u bench.py --steps 500 --warmup 20 --no-cpu-baseline --transitions 100000 --algo bcq"
D3A_BCQ_BRANCHES=1 $B > $O/b_on.json 2>$O/b.err || exit 1; echo on; cut -c1-200 $O/b_on.json
$B > $O/b_off.json 2>>$O/b.err || exit 1; echo off; cut -c1-200 $O/b_off.json
D3A_BCQ_BRANCHES=1 $B > $O/b_on2.json 2>>$O/b.err || exit 1; echo on2; cut -c1-200 $O/b_on2.json
