#!/bin/bash
# K3's final bench line (CPU baseline included) and step timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5bf
cd $R && mkdir -p $O
timeout -k 10 300 python -u bench.py --algo bcq --transitions 200000 > $O/bench_bcq.jsonl 2>$O/bench_bcq.err || exit 1
tail -1 $O/bench_bcq.jsonl | cut -c1-200
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bcq -o run --output-format csv -- python3 $R/bench.py --algo bcq --steps 200 --warmup 20 --no-cpu-baseline > $O/prof_bcq.log 2>&1 || exit 1
cd $R && python tools/prof_timeline.py $O/prof_bcq/run_kernel_trace.csv > $O/r05_bcq_timeline_final.txt; rm -f $O/prof_bcq/run_kernel_trace.csv
tail -1 $O/r05_bcq_timeline_final.txt
