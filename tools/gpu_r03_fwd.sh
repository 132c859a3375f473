# d3a_mlp_fwd microbenchmark on the K2 critic shape (block_rows A/B) + two SQ
# counter passes over it.  Outputs in gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
for bm in 0 64 32; do
  timeout -k 10 120 python3 tools/bench_fwd.py --bm $bm >> gpurun_out/fwd_bench.json 2>gpurun_out/fwd_bench.err || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_fwd1 -o run --output-format csv -- python3 $R/tools/bench_fwd.py --reps 20 > $R/gpurun_out/pmc_fwd1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES -d $R/gpurun_out/pmc_fwd2 -o run --output-format csv -- python3 $R/tools/bench_fwd.py --reps 20 > $R/gpurun_out/pmc_fwd2.log 2>&1 || exit $?
cd $R && python3 tools/pmc_avg.py gpurun_out/pmc_fwd1 mlp_fwd > gpurun_out/pmc_fwd.txt && python3 tools/pmc_avg.py gpurun_out/pmc_fwd2 mlp_fwd >> gpurun_out/pmc_fwd.txt
