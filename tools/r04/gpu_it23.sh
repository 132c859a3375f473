# r04 iteration 23: K5 with the fp32-MFMA conv input gradient (default again):
# K5 suites, bench (2,000 steps) + packed-forward A/B, timeline, PMC of the dominant kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4m_k5
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_arbiters.py tests/test_gpu_discrete_cql.py tests/test_gpu_conv.py tests/test_gpu_dqn.py > $O/k5_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --algo dcql --cpu-seconds 10 --cpu-seconds-1t 5 > $O/bench_dcql.jsonl 2>$O/bench_err.log || exit $?
D3A_CONV_FWD_PACK=1 timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline > $O/bench_dcql_fwdpack.jsonl 2>/dev/null || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tl_dcql -o run --output-format csv -- python3 $R/bench.py --algo dcql --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $O/tl_dcql.log 2>&1 || exit $?
python tools/prof_timeline.py $O/tl_dcql/run_kernel_trace.csv > $O/dcql_timeline.txt; rm -f $O/tl_dcql/run_kernel_trace.csv
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_dcql_f -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo dcql --transitions 100000 > $O/pmc_dcql_f.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_dcql_w -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo dcql --transitions 100000 > $O/pmc_dcql_w.log 2>&1 || exit $?
cd $R
python tools/pmc_summarize.py $O/pmc_dcql_f $O/pmc_dcql_w iqn_head_bwd_fused $O/r04_pmc_traffic_dcql_x6.json > $O/pmc_dcql.log 2>&1
find $O -name "*counter_collection.csv" -size +20M -delete
