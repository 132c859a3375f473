#!/bin/bash
# copy the final GPU run's outputs (tools/r06/gpu_final6.sh, gpurun_out/r6final)
# into profiles/ under their round-6 names
set -e
O=gpurun_out/r6final
for n in cql cql_bf16 cqldp cqlrepro td3bc bcq dcql; do tail -1 $O/bench_$n.json; done > profiles/r06_bench_lines_final.jsonl
cp $O/gpu_tests.log profiles/r06_gpu_tests.log
cp $O/smoke.log profiles/r06_smoke.log
cp $O/arbiter_margins.log profiles/r06_arbiter_margins.log
cp $O/prof/run_kernel_stats.csv profiles/r06_cql_kernel_stats_final.csv
cp $O/cql_timeline.txt profiles/r06_cql_timeline_final.txt
cp $O/prof_breakdown.txt profiles/r06_cql_prof_breakdown_final.txt
