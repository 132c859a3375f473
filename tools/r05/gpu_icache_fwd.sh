#!/bin/bash
# instruction-cache and stall counters of the K2 split-bf16 forward
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5icf
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_WAVES -d $O/ic -o run --output-format csv -- python3 $R/tools/bench_fwd.py --x6 --slice --reps 50 > $O/ic.log 2>&1 || { tail -5 $O/ic.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d $O/sq -o run --output-format csv -- python3 $R/tools/bench_fwd.py --x6 --slice --reps 50 > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
cd $R && python tools/pmc_sq_summary.py $O/ic q2x6_fwd; python tools/pmc_sq_summary.py $O/sq q2x6_fwd
find $O -name "*counter_collection.csv" -size +20M -delete
