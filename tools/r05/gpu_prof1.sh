#!/bin/bash
# round 5 profile of the K2 step with the slice backward: kernel trace +
# timeline, per-kernel HBM bytes of a step (FETCH_SIZE / WRITE_SIZE passes),
# SQ stall counters of a step, and the x6 forward's probe variants / phase stamps
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5p
cd $R && mkdir -p $O
for v in 0 4 8 12 1; do
  D3A_X6_PROBE=$v timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice >> $O/fwd_probe.jsonl 2>>$O/fwd_probe.err || exit $?
done
D3A_X6_PROBE=16 timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --stamps --reps 1 >> $O/fwd_probe.jsonl 2>>$O/fwd_probe.err || exit $?
cat $O/fwd_probe.jsonl
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 500 --warmup 20 --no-cpu-baseline --transitions 200000 > $O/prof.log 2>&1 || exit $?
cd $R && python tools/prof_timeline.py $O/prof/run_kernel_trace.csv > $O/cql_timeline.txt && python tools/prof_by_shape.py $O/prof/run_kernel_trace.csv 540 > $O/cql_breakdown.txt; rm -f $O/prof/run_kernel_trace.csv
cat $O/cql_timeline.txt
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_step_f -o run --output-format csv -- python3 $R/tools/pmc_step.py > $O/pmc_step_f.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_step_w -o run --output-format csv -- python3 $R/tools/pmc_step.py > $O/pmc_step_w.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_sq -o run --output-format csv -- python3 $R/tools/pmc_step.py > $O/pmc_sq.log 2>&1 || exit $?
cd $R
python tools/pmc_step_kernels.py $O/pmc_step_f $O/pmc_step_w > $O/pmc_step_kernels_cql.txt 2>&1
python tools/pmc_sq_summary.py $O/pmc_sq > $O/pmc_sq_step_cql.txt 2>&1
find $O -name "*counter_collection.csv" -size +20M -delete
cat $O/pmc_step_kernels_cql.txt | head -20
cat $O/pmc_sq_step_cql.txt
