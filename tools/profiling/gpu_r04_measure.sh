# Round-4 measurement of the committed tree: GPU suite, smoke(), every bench
# line (K2 headline with the live CPU baseline, the driver's 20-step window,
# the other workloads, precision / GEMM variants), rocprofv3 kernel trace +
# stats of the headline workload, PMC traffic of its dominant kernel and of
# every kernel of a step, K3 / K5 timelines.  Outputs: gpurun_out/r4m/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4m
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench_cql.jsonl 2> $O/bench_cql.err || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/bench_lines.jsonl 2>/dev/null || exit $?
for a in td3bc bcq dcql cqldp cqlrepro; do
  timeout -k 10 400 python bench.py --algo $a --cpu-seconds 10 --cpu-seconds-1t 5 >> $O/bench_lines.jsonl 2>>$O/bench_err.log || exit $?
done
for v in "--precision bf16" "--precision bf16h" "--critic-gemm fp32"; do
  timeout -k 10 200 python bench.py $v --no-cpu-baseline >> $O/bench_lines.jsonl 2>/dev/null || exit $?
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 500 --warmup 20 --no-cpu-baseline --transitions 200000 > $O/prof.log 2>&1 || exit $?
python tools/prof_timeline.py $O/prof/run_kernel_trace.csv > $O/cql_timeline.txt && python tools/prof_by_shape.py $O/prof/run_kernel_trace.csv 540 > $O/cql_breakdown.txt; rm -f $O/prof/run_kernel_trace.csv
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_dom_f -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo cql > $O/pmc_dom_f.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_dom_w -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo cql > $O/pmc_dom_w.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_dcql_f -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo dcql --transitions 100000 > $O/pmc_dcql_f.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_dcql_w -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo dcql --transitions 100000 > $O/pmc_dcql_w.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_step_f -o run --output-format csv -- python3 $R/tools/pmc_step.py > $O/pmc_step_f.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_step_w -o run --output-format csv -- python3 $R/tools/pmc_step.py > $O/pmc_step_w.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_sq -o run --output-format csv -- python3 $R/tools/pmc_step.py > $O/pmc_sq.log 2>&1 || exit $?
cd $R
python tools/pmc_summarize.py $O/pmc_dom_f $O/pmc_dom_w q2x6_fwd $O/r04_pmc_traffic_cql_x6.json > $O/pmc_dom.log 2>&1
python tools/pmc_summarize.py $O/pmc_dcql_f $O/pmc_dcql_w iqn_head_bwd_fused $O/r04_pmc_traffic_dcql_x6.json > $O/pmc_dcql.log 2>&1
python tools/pmc_step_kernels.py $O/pmc_step_f $O/pmc_step_w > $O/pmc_step_kernels_cql.txt 2>&1
find $O -name "*counter_collection.csv" -size +20M -delete
for a in bcq dcql; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tl_$a -o run --output-format csv -- python3 $R/bench.py --algo $a --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $O/tl_$a.log 2>&1 || exit $?
  python tools/prof_timeline.py $O/tl_$a/run_kernel_trace.csv > $O/${a}_timeline.txt; rm -f $O/tl_$a/run_kernel_trace.csv
done
