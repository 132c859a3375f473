#!/bin/bash
# round 5: K5 early head/fc Adam on the weight-gradient branch -- DiscreteCQL
# parity + arbiters, bench A/B, timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5p2
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_discrete_cql.py tests/test_gpu_arbiters.py tests/test_gpu_dqn.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="timeout -k 10 200 python -u bench.py --steps 500 --warmup 20 --no-cpu-baseline --transitions 100000 --algo dcql"
$B > $O/b_on.json 2>$O/b.err || exit 1; echo early; cut -c1-200 $O/b_on.json
D3A_K5_EARLY_ADAM=0 $B > $O/b_off.json 2>>$O/b.err || exit 1; echo late; cut -c1-200 $O/b_off.json
