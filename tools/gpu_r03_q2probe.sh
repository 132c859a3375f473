# q2_bwd timing: normal vs staging-free probe, plus SQ counters of both.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 120 python3 tools/bench_q2.py > gpurun_out/q2_bench.json 2>gpurun_out/q2_bench.err || exit $?
D3A_Q2_PROBE=1 timeout -k 10 120 python3 tools/bench_q2.py > gpurun_out/q2_probe.json 2>gpurun_out/q2_probe.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_q2 -o run --output-format csv -- python3 $R/tools/bench_q2.py --reps 20 > $R/gpurun_out/pmc_q2.log 2>&1 || exit $?
