set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
: > gpurun_out/bf16d.json
for p in 0 2; do
  D3A_BF16_PROBE=$p timeout -k 10 120 python3 tools/bench_bf16.py >> gpurun_out/bf16d.json 2>>gpurun_out/bf16d.err || exit $?
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/bf16_tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VALU -d $R/gpurun_out/pmc_bf16f -o run --output-format csv -- python3 $R/tools/bench_fwd.py --bf16 --reps 20 > $R/gpurun_out/pmc_bf16f.log 2>&1 || exit $?
python3 $R/tools/pmc_avg.py $R/gpurun_out/pmc_bf16f q2_fwd_bf16 > $R/gpurun_out/pmc_bf16f.txt
