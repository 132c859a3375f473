#!/bin/bash
# SQ stall / MFMA-busy counters of K3's dominant kernel (the wide target pass)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5sq
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/bcq_sq -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo bcq --transitions 100000 > $O/bcq_sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_WAVES -d $O/bcq_sq2 -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo bcq --transitions 100000 > $O/bcq_sq2.log 2>&1 || exit 1
cd $R && python tools/pmc_sq_summary.py $O/bcq_sq > $O/sq.txt 2>&1; grep -i "wide\|kernel grid" $O/sq.txt
python tools/pmc_sq_summary.py $O/bcq_sq wide; python tools/pmc_sq_summary.py $O/bcq_sq2 wide
find $O -name "*counter_collection.csv" -size +20M -delete
