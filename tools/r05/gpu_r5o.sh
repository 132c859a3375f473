#!/bin/bash
# round 5: K3 small-net passes on the parts path -- BCQ parity + arbiters, bench A/B, timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5o
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_bcq_parity.py tests/test_gpu_arbiters.py > $O/bcq_tests.log 2>&1 || { tail -40 $O/bcq_tests.log; exit 1; }
tail -1 $O/bcq_tests.log
B="timeout -k 10 200 python -u bench.py --steps 500 --warmup 20 --no-cpu-baseline --transitions 100000 --algo bcq"
$B > $O/b_on.json 2>$O/b.err || exit 1; echo parts; cut -c1-200 $O/b_on.json
D3A_BCQ_PARTS=0 $B > $O/b_off.json 2>>$O/b.err || exit 1; echo small; cut -c1-200 $O/b_off.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tl_bcq -o run --output-format csv -- python3 $R/bench.py --algo bcq --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $O/tl_bcq.log 2>&1 || exit 1
cd $R && python tools/prof_timeline.py $O/tl_bcq/run_kernel_trace.csv > $O/bcq_timeline.txt; rm -f $O/tl_bcq/run_kernel_trace.csv
grep -E "mlp_parts|mlp_small|step:" $O/bcq_timeline.txt
