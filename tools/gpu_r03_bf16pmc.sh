set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
for p in 0 2; do
  D3A_BF16_PROBE=$p timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU -d $R/gpurun_out/pmc_bf16_$p -o run --output-format csv -- python3 $R/tools/bench_bf16.py > $R/gpurun_out/pmc_bf16_$p.log 2>&1 || exit $?
  python3 $R/tools/pmc_avg.py $R/gpurun_out/pmc_bf16_$p q2_bwd_bf16 > $R/gpurun_out/pmc_bf16_$p.txt || exit $?
done
