#!/bin/bash
# One rocprofv3 pass of SQ stall counters over the dominant kernel:
#   bash tools/profiling/pmc_sq.sh ALGO KERNEL_SUBSTRING TAG
R="${GRAFT_REPO_ROOT:-/root/repo}"
ALGO=${1:-cql}
SUB=${2:-mlp_fwd_kernel}
TAG=${3:-sq}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_${TAG}_$ALGO -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo $ALGO > $R/gpurun_out/pmc_${TAG}_$ALGO.log 2>&1 || exit $?
cd $R && python tools/pmc_counters.py gpurun_out/pmc_${TAG}_$ALGO $SUB > gpurun_out/pmc_${TAG}_${ALGO}.txt
