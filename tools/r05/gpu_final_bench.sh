#!/bin/bash
# round 5: final bench lines (CPU baselines included) for every workload, the
# driver's 20-step window, and the K2 rocprof kernel summary
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5final
cd $R && mkdir -p $O
: > $O/bench_lines.jsonl
timeout -k 10 300 python -u bench.py >> $O/bench_lines.jsonl 2>$O/bench_cql.err || exit 1
tail -1 $O/bench_lines.jsonl | cut -c1-160
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/bench_lines.jsonl 2>>$O/bench_cql.err || exit 1
tail -1 $O/bench_lines.jsonl | cut -c1-160
for a in cqlrepro td3bc bcq dcql cqldp; do
  timeout -k 10 300 python -u bench.py --algo $a --transitions 200000 >> $O/bench_lines.jsonl 2>$O/bench_$a.err || exit 1
  tail -1 $O/bench_lines.jsonl | cut -c1-160
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cql -o run --output-format csv -- python3 $R/bench.py --steps 500 --warmup 20 --no-cpu-baseline > $O/prof_cql.log 2>&1 || exit 1
cd $R && cp $O/prof_cql/run_kernel_stats.csv $O/r05_cql_kernel_stats_final.csv && python tools/prof_timeline.py $O/prof_cql/run_kernel_trace.csv > $O/r05_cql_timeline_final.txt; rm -f $O/prof_cql/run_kernel_trace.csv
tail -14 $O/r05_cql_timeline_final.txt
# K3's step timeline on the final tree
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bcq -o run --output-format csv -- python3 $R/bench.py --algo bcq --steps 200 --warmup 20 --no-cpu-baseline > $O/prof_bcq.log 2>&1 || exit 1
cd $R && python tools/prof_timeline.py $O/prof_bcq/run_kernel_trace.csv > $O/r05_bcq_timeline_final.txt; rm -f $O/prof_bcq/run_kernel_trace.csv
tail -1 $O/r05_bcq_timeline_final.txt
