#!/bin/bash
# K2 bench after the Adam load batching + timelines of K2, the CQL
# reproduction config, K3 and K5
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5f
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 50 --no-cpu-baseline > $O/bench_k2.json 2>$O/bench.err || exit $?
cut -c1-200 $O/bench_k2.json
export TMPDIR=/tmp
for a in cql cqlrepro bcq dcql; do
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tl_$a -o run --output-format csv -- python3 $R/bench.py --algo $a --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $O/tl_$a.log 2>&1 || exit $?
  cd $R && python tools/prof_timeline.py $O/tl_$a/run_kernel_trace.csv > $O/${a}_timeline.txt; rm -f $O/tl_$a/run_kernel_trace.csv
  tail -1 $O/${a}_timeline.txt
done
