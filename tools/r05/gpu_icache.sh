#!/bin/bash
# instruction-cache counters of the small-batch backward (is its staging time cold-I$ fetch?)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5ic
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_WAVES -d $O/ic -o run --output-format csv -- python3 $R/tools/bench_small_bwd.py > $O/ic.log 2>&1 || { tail -5 $O/ic.log; exit 1; }
cd $R && python tools/pmc_sq_summary.py $O/ic small_a; python tools/pmc_sq_summary.py $O/ic small_b
find $O -name "*counter_collection.csv" -size +20M -delete
