# bf16 line evidence: accuracy log, kernel trace of the bf16
# bench line, SQ PMC of q2_fwd_bf16 / q2_bwd_bf16, FETCH / WRITE passes of the
# bf16 line's dominant kernel -> gpurun_out/r4_bf16_*
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bf16.py > gpurun_out/r4_bf16_accuracy.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_bf16_tl -o k2 --output-format csv -- python3 bench.py --precision bf16 --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 > gpurun_out/r4_bf16_tl.log 2>&1 || exit $?
f=$(find gpurun_out/r4_bf16_tl -name '*kernel_trace.csv' -print -quit)
python tools/prof_by_shape.py "$f" 320 > gpurun_out/r4_bf16_breakdown.txt 2>&1 || true
rm -f "$f"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/r4_bf16_pmc_sq -o run --output-format csv -- python3 tools/bench_bf16.py > gpurun_out/r4_bf16_pmc_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r4_bf16_fetch -o run --output-format csv -- python3 tools/pmc_dominant.py --precision bf16 > gpurun_out/r4_bf16_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r4_bf16_write -o run --output-format csv -- python3 tools/pmc_dominant.py --precision bf16 > gpurun_out/r4_bf16_write.log 2>&1 || exit $?
python tools/pmc_summarize.py gpurun_out/r4_bf16_fetch gpurun_out/r4_bf16_write q2_fwd_bf16 gpurun_out/r04_pmc_traffic_cql_bf16.json
