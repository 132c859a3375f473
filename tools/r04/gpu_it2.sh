# r04 iteration 2: x6 forward (producer prefetch) + x6 backward: tests, benches, one SQ PMC pass each;
# CQL parity suite after the softmax-weight change
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_x6.py > gpurun_out/r4i2_x6.log 2>&1 || exit $?
for f in "--x6" ""; do timeout -k 10 120 python tools/bench_fwd.py $f >> gpurun_out/r4i2_bench.jsonl 2>/dev/null || exit $?; done
for f in "--x6" ""; do timeout -k 10 120 python tools/bench_q2.py $f >> gpurun_out/r4i2_bench.jsonl 2>/dev/null || exit $?; done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/r4i2_pmc_fwd -o run --output-format csv -- python3 $R/tools/bench_fwd.py --x6 --reps 20 > $R/gpurun_out/r4i2_pmc_fwd.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/r4i2_pmc_bwd -o run --output-format csv -- python3 $R/tools/bench_q2.py --x6 --reps 20 > $R/gpurun_out/r4i2_pmc_bwd.log 2>&1 || exit $?
cd $R
for g in fp32 x6; do timeout -k 10 200 python bench.py --critic-gemm $g --no-cpu-baseline >> gpurun_out/r4i2_bench.jsonl 2>/dev/null || exit $?; done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/r4i2_bench.jsonl 2>/dev/null || exit $?
timeout -k 10 200 python bench.py --algo cqlrepro --no-cpu-baseline >> gpurun_out/r4i2_bench.jsonl 2>/dev/null || exit $?
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_production_path.py tests/test_gpu_cql_parity.py tests/test_gpu_dp.py tests/test_gpu_sac_parity.py > gpurun_out/r4i2_tests.log 2>&1
