#!/bin/bash
# kernel timelines of one step of K3 (bcq) and the repro workload
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5tl
mkdir -p $O
export TMPDIR=/tmp
for a in ${ALGOS:-bcq}; do
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$a -o run --output-format csv -- python3 $R/bench.py --algo $a --steps 200 --warmup 20 --no-cpu-baseline > $O/prof_$a.log 2>&1 || exit 1
  cd $R && python tools/prof_timeline.py $O/prof_$a/run_kernel_trace.csv > $O/tl_$a.txt && rm -f $O/prof_$a/run_kernel_trace.csv && tail -1 $O/tl_$a.txt
done
