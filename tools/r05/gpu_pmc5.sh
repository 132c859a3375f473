#!/bin/bash
# round 5: PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the dominant
# kernels of K5 (recomputing IQN head backward), K2 (x6 critic forward) and
# K3 (wide target pass), for bench.py's roofline.traffic
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5pmc
mkdir -p $O
export TMPDIR=/tmp
for spec in "dcql:iqn_head_bwd_rc" "cql:q2x6_fwd" "bcq:mlp_x6_wide"; do
  a=${spec%%:*}; k=${spec#*:}
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/${a}_f -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo $a --transitions 100000 > $O/${a}_f.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/${a}_w -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo $a --transitions 100000 > $O/${a}_w.log 2>&1 || exit 1
  cd $R && python tools/pmc_summarize.py $O/${a}_f $O/${a}_w $k $O/r05_pmc_traffic_${a}_x6.json && cat $O/r05_pmc_traffic_${a}_x6.json
  find $O -name "*counter_collection.csv" -size +20M -delete
done
# SQ stall / MFMA-busy counters of the same dominant kernels
for a in dcql bcq; do
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/${a}_sq -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo $a --transitions 100000 > $O/${a}_sq.log 2>&1 || exit 1
  cd $R && python tools/pmc_sq_summary.py $O/${a}_sq > $O/r05_pmc_sq_${a}.txt 2>&1; tail -4 $O/r05_pmc_sq_${a}.txt
  find $O -name "*counter_collection.csv" -size +20M -delete
done
