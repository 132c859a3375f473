# r04 iteration 29: PMC traffic of K3's and K4's dominant (split-bf16) kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/i29
cd $R && mkdir -p $O && cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_bcq_f -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo bcq --transitions 100000 > $O/pmc_bcq_f.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_bcq_w -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo bcq --transitions 100000 > $O/pmc_bcq_w.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_dp_f -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo cqldp --transitions 100000 > $O/pmc_dp_f.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_dp_w -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo cqldp --transitions 100000 > $O/pmc_dp_w.log 2>&1 || exit $?
cd $R
python tools/pmc_summarize.py $O/pmc_bcq_f $O/pmc_bcq_w mlp_x6_wide $O/r04_pmc_traffic_bcq_x6.json > $O/pmc_bcq.log 2>&1
python tools/pmc_summarize.py $O/pmc_dp_f $O/pmc_dp_w q2x6_fwd $O/r04_pmc_traffic_cqldp_x6.json > $O/pmc_dp.log 2>&1
find $O -name "*counter_collection.csv" -size +20M -delete
timeout -k 10 300 python bench.py --algo bcq --no-cpu-baseline > $O/bench.jsonl 2>/dev/null || exit $?
