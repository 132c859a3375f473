# q2_bwd microbenchmark + one SQ counter pass over it (wave-cycle split, MFMA
# busy, LDS stalls).  Outputs in gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 120 python3 tools/bench_q2.py > gpurun_out/q2_bench.json 2>gpurun_out/q2_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_q2 -o run --output-format csv -- python3 $R/tools/bench_q2.py --reps 20 > $R/gpurun_out/pmc_q2.log 2>&1 || exit $?
