#!/bin/bash
# round 6: PMC HBM traffic of a bench line's critic backward (the line's lead
# kernel when it outlasts the forward: the bf16 line) -> r06_pmc_traffic_<algo><sfx>_bwd.json
# usage: gpu_pmc_bwd.sh ALGO SUFFIX "PMC_DOMINANT_ARGS" KERNEL_SUBSTRING
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6pmc
mkdir -p $O
export TMPDIR=/tmp
a=$1; sfx=$2; px=$3; k=$4
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/${a}${sfx}_bwd_f -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo $a $px --backward --transitions 100000 --desc-out $O/${a}${sfx}_bwd_desc.json > $O/${a}${sfx}_bwd_f.log 2>&1 || { tail -5 $O/${a}${sfx}_bwd_f.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/${a}${sfx}_bwd_w -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo $a $px --backward --transitions 100000 > $O/${a}${sfx}_bwd_w.log 2>&1 || { tail -5 $O/${a}${sfx}_bwd_w.log; exit 1; }
cd $R && python tools/pmc_summarize.py $O/${a}${sfx}_bwd_f $O/${a}${sfx}_bwd_w $k $O/r06_pmc_traffic_${a}${sfx}_bwd.json $O/${a}${sfx}_bwd_desc.json 6 | cut -c1-400
find $O -name "*counter_collection.csv" -size +20M -delete
