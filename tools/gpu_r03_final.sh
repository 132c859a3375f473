# Round-3 measurement of HEAD: K2 bench (with the CPU baseline), kernel trace
# of the same workload (stats, breakdown, timeline), PMC traffic and SQ split
# of the dominant kernel (q2_fwd), the SQ split of the critic backward
# (q2_bwd, via tools/bench_q2.py), HBM bytes of every kernel of an eager step
# (Adam traffic), and the other workloads' bench lines.  Outputs in gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/fin_bench_cql.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_prof -o k2 --output-format csv -- python3 bench.py --steps 500 --warmup 20 --no-cpu-baseline --transitions 200000 > gpurun_out/fin_prof.log 2>&1 || exit $?
f=$(find gpurun_out/fin_prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_by_shape.py "$f" 520 > gpurun_out/fin_breakdown.txt 2>&1 || true
python tools/prof_timeline.py "$f" > gpurun_out/fin_timeline.txt 2>&1 || true
rm -f "$f"
bash tools/pmc_pass.sh cql q2_fwd_kernel || exit $?
bash tools/pmc_sq.sh cql q2_fwd_kernel sq || exit $?
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_sq_q2bwd -o run --output-format csv -- python3 $R/tools/bench_q2.py --reps 20 > $R/gpurun_out/pmc_sq_q2bwd.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_step_fetch -o run --output-format csv -- python3 $R/tools/pmc_step.py > $R/gpurun_out/pmc_step_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_step_write -o run --output-format csv -- python3 $R/tools/pmc_step.py > $R/gpurun_out/pmc_step_write.log 2>&1 || exit $?
cd $R
python tools/pmc_counters.py gpurun_out/pmc_sq_q2bwd q2_bwd_kernel > gpurun_out/pmc_sq_q2bwd.txt 2>&1 || true
for a in td3bc bcq dcql cqldp; do
  timeout -k 10 300 python bench.py --algo $a --cpu-seconds 10 > gpurun_out/fin_bench_$a.log 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --precision bf16 --steps 2000 --no-cpu-baseline > gpurun_out/fin_bench_bf16.log 2>&1 || exit $?
timeout -k 10 60 ./tools/probes/pow_latency > gpurun_out/pow_latency.jsonl 2>&1 || true
