#!/bin/bash
# Two rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE) over the dominant
# kernel alone, then the per-launch summary -> profiles/r01_pmc_traffic.json
R="${GRAFT_REPO_ROOT:-/root/repo}"
ALGO=${1:-cql}
SUB=${2:-mlp_fwd_kernel}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$ALGO -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo $ALGO > $R/gpurun_out/pmc_fetch_$ALGO.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$ALGO -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo $ALGO > $R/gpurun_out/pmc_write_$ALGO.log 2>&1 || exit $?
cd $R && python tools/pmc_summarize.py gpurun_out/pmc_fetch_$ALGO gpurun_out/pmc_write_$ALGO $SUB gpurun_out/pmc_traffic_$ALGO.json
