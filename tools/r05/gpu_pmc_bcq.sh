#!/bin/bash
# PMC HBM traffic of K3's dominant kernel (the persistent wide target pass)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5pmcb
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/bcq_f -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo bcq --transitions 100000 > $O/bcq_f.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/bcq_w -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo bcq --transitions 100000 > $O/bcq_w.log 2>&1 || exit 1
cd $R && python tools/pmc_summarize.py $O/bcq_f $O/bcq_w mlp_x6_wide $O/r05_pmc_traffic_bcq_x6.json && cat $O/r05_pmc_traffic_bcq_x6.json
find $O -name "*counter_collection.csv" -size +20M -delete
